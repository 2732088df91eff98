set -e
OUT=gpurun_out/s4_psp
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_fp8_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 400 python tools/gemm_sweep.py --dtype fp8 --shapes 8192,16384,16384x16384x1024 --variants 9,10,12 > $OUT/sweep_fp8.jsonl 2> $OUT/sweep_fp8.err
timeout -k 10 400 python tools/gemm_sweep.py --shapes 8192,16384,16384x16384x1024 --variants 44,25,27 > $OUT/sweep_bf16.jsonl 2> $OUT/sweep_bf16.err
