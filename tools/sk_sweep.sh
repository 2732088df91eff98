OUT=gpurun_out/r6s3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k "57" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
S="timeout -k 10 200 python -u tools/gemm_sweep.py --rounds 3 --iters 30"
$S --variants p0,p57s2b500,p57s2b520,p57s2b540,p57s2b560 --shapes 2560x2560x8192,2048x4096x8192 > $OUT/s2_long.jsonl 2>&1 &&
$S --variants p0,p57s2b500,p57s2b540,p57s2b580,p57s2b620 --shapes 2560,2048x2048x8192 > $OUT/s2_mid.jsonl 2>&1 &&
$S --variants p57s3b333,p57s3b400,p57s4b250,p57s4b300,p57s4b340 --shapes 2048x2048x8192 > $OUT/s34.jsonl 2>&1
rc=$?; cat $OUT/*.jsonl | grep -v amdgpu.ids; exit $rc
