# Split-K asm frame: the fp8 and bf16 GEMM GPU tests (v24 / v57 numerics and dispatch).
OUT=gpurun_out/${SK_OUT:-r6s10}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log; exit $rc
