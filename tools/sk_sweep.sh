# Split-K asm frame (v57 / fp8 v24): the GEMM GPU tests, the ABFT naming / bitwise cases, then the automatic
# dispatch against hipBLASLt over the verdict's shapes and the 65-128-tile band.
OUT=gpurun_out/${SK_OUT:-r6s6}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_fp8_gpu.py tests/test_abft_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
S="timeout -k 10 280 python -u tools/gemm_sweep.py --rounds 3 --iters 30 --variants p0"
$S --shapes 2560,2048x2048x8192,2560x2560x8192,1024x1024x4096,2304x2304x8192,2048x4096x8192,2560x3072x8192,2560x2560x16384,8192 > $OUT/auto_bf16.jsonl 2>&1 &&
$S --dtype fp8 --shapes 2560,2560x2560x8192,1024x1024x16384,2560x2560x16384,2048x4096x16384,8192 > $OUT/auto_fp8.jsonl 2>&1
rc=$?; cat $OUT/auto*.jsonl | grep -v amdgpu.ids; exit $rc
