set -e
mkdir -p gpurun_out/s5_final
timeout -k 10 600 python -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s5_final/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5_final/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/s5_final/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s5_final/prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 20 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s5_final/bench_prof.log 2>&1
