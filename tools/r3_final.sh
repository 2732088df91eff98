#!/bin/bash
# Final round-3 check: every GPU test, smoke(), the driver's bench invocation, bench defaults, kernel stats.
O=gpurun_out/${1:-r3_final}
mkdir -p $O
echo "pytest -m gpu"; timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo "smoke"; timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "bench (driver invocation)"; timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-300
echo "bench (defaults)"; timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
echo "rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 20 --no-extras > $GRAFT_REPO_ROOT/$O/bench_prof.log 2>&1
echo done
