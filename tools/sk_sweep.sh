# Split-K asm frame (v57): numerics, then the automatic dispatch on 33-64-tile grids with long K.
OUT=gpurun_out/${SK_OUT:-r6s8}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k "57 or automatic" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
S="timeout -k 10 280 python -u tools/gemm_sweep.py --rounds 3 --iters 30"
$S --variants p0,p60,p57s3b0 --shapes 2048x2048x16384,2048x2048x32768,1536x2560x16384,2048x1536x16384,1024x4096x16384 > $OUT/auto_s4.jsonl 2>&1
rc=$?; cat $OUT/*.jsonl | grep -v amdgpu.ids; exit $rc
