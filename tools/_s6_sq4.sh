# Pinned A/B: bf16 v46 (= v44, no switch) vs v45; fp8 v14 (= v9, no switch) vs v13.
set -e
OUT=gpurun_out/s6_sq
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gemm2.log 2>&1
timeout -k 10 400 python -u tools/gemm_sweep.py --shapes 12288,16384x8192x8192,16384,16384x16384x8192 --variants 46,45 --rounds 6 --iters 20 > $OUT/sweep_ab_bf16.jsonl 2> $OUT/sweep_ab_bf16.err
timeout -k 10 400 python -u tools/gemm_sweep.py --dtype fp8 --shapes 12288,16384x8192x8192,16384,16384x16384x8192 --variants 14,13 --rounds 6 --iters 20 > $OUT/sweep_ab_fp8.jsonl 2> $OUT/sweep_ab_fp8.err
