# One-call GPU confirmation: gpu tests, smoke, bench, rocprofv3 kernel stats.
# Usage (from the repo root on the GPU box): bash tools/gpu_round.sh [out-subdir]
set -e
OUT=gpurun_out/${1:-round}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 20 --no-extras > $GRAFT_REPO_ROOT/$OUT/bench_prof.log 2>&1
