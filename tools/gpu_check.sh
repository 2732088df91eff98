#!/bin/bash
# One GPU-box pass: GPU tests, smoke, GEMM variant sweep vs hipBLASLt, bench, rocprofv3 kernel stats.
# Usage (from the repo root, on the box): bash tools/gpu_check.sh <outdir> [variants]
set -e
OUT=${1:-gpurun_out/check}
VARIANTS=${2:-5,10,15,18}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python tools/gemm_sweep.py --shapes 4096,8192,16384 --variants "$VARIANTS" \
  > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 50 --warmup 20 --no-extras > "$ROOT/$OUT/bench_prof.log" 2>&1
