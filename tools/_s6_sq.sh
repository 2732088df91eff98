# v45 (square cross-XCD raster) check + A/B against v44 and hipBLASLt.
set -e
OUT=gpurun_out/s6_sq
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "44 or 45" > $OUT/pytest_v45.log 2>&1
timeout -k 10 400 python -u tools/gemm_sweep.py --shapes 8192,16384,8192x8192x16384 --variants 44,45 --rounds 4 --iters 20 > $OUT/sweep.jsonl 2> $OUT/sweep.err
