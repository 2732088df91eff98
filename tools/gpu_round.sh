set -e
mkdir -p gpurun_out/round2
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q > gpurun_out/round2/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round2/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/round2/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/round2/prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 20 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/round2/bench_prof.log 2>&1
