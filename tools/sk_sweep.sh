# 144-tile grids: split-K past one wave (3 pieces = 432 workgroups in two dispatch rounds of a third of K).
OUT=gpurun_out/${SK_OUT:-r6s18}; mkdir -p $OUT
timeout -k 10 500 python -u tools/gemm_sweep.py --rounds 3 --iters 30 --variants p0,p57s3b0,p57s3b0p,p57s4b0,p57s5b0 --shapes 3072x3072x8192,3072x3072x16384,3072x3072x4096 > $OUT/past_wave.jsonl 2>&1
rc=$?; cat $OUT/past_wave.jsonl | grep -v amdgpu.ids; exit $rc
