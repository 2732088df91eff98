# v45 / fp8 v13 numerics (all GEMM GPU tests) + fp8 sweep with the default dispatch.
set -e
OUT=gpurun_out/s6_sq
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gemm.log 2>&1
timeout -k 10 400 python -u tools/gemm_sweep.py --dtype fp8 --shapes 8192,12288,16384x8192x8192,16384 --variants 5,9,13 --rounds 4 --iters 20 > $OUT/sweep_fp8.jsonl 2> $OUT/sweep_fp8.err
