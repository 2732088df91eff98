set -e
OUT=gpurun_out/s4_def
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python tools/gemm_sweep.py --shapes 4096,8192,16384,16384x16384x1024 --variants 18,44 > $OUT/sweep_bf16.jsonl 2> $OUT/sweep_bf16.err
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 50 --warmup 20 --no-extras > "$ROOT/$OUT/bench_prof.log" 2>&1
