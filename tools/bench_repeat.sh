# The headline bench N times on one box (each run: our GEMM and hipBLASLt in the same process), to show
# the spread of the ratio rather than one 20-step window. Stops at the first failing run.
OUT=gpurun_out/${1:-bench_repeat}; N=${2:-5}; mkdir -p $OUT
for i in $(seq 1 $N); do
  timeout -k 10 240 python bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/bench_$i.log 2>&1 || exit 1
  tail -1 $OUT/bench_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($i, d['value'], d['hipblaslt_tflops'], d['ratio_vs_hipblaslt'], d['fp8_ratio_vs_hipblaslt'])"
done
