# v45 vs v44 over more shapes / rounds (dispatch threshold for the square raster).
set -e
OUT=gpurun_out/s6_sq
mkdir -p $OUT
timeout -k 10 600 python -u tools/gemm_sweep.py --shapes 8192,12288,16384x8192x8192,16384x16384x4096,16384,8192x8192x16384 --variants 44,45 --rounds 6 --iters 20 > $OUT/sweep2.jsonl 2> $OUT/sweep2.err
