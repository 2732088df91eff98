OUT=gpurun_out/r6_final_b; mkdir -p $OUT
S=1024,1024x1024x4096,1024x1024x16384,512x512x8192,1536,2048,2048x2048x1024,2048x2048x8192,2048x2048x16384,2560,2560x2560x8192,2560x2560x16384,2048x4096x8192,3072x3072x1024,4096,8192,16384,16384x16384x1024
timeout -k 10 500 python -u tools/gemm_sweep.py --variants p0 --rounds 3 --iters 30 --shapes $S > $OUT/closing_sweep_bf16.jsonl 2>&1 &&
timeout -k 10 500 python -u tools/gemm_sweep.py --dtype fp8 --variants p0 --rounds 3 --iters 30 --shapes $S,2048x2048x32768 > $OUT/closing_sweep_fp8.jsonl 2>&1
rc=$?; grep -v amdgpu.ids $OUT/*.jsonl | wc -l; exit $rc
