#!/bin/bash
# GPU round: all GPU tests, the driver's bench invocation, a production shape sweep, kernel stats.
O=gpurun_out/${1:-r3s2_round}
mkdir -p $O
echo "pytest -m gpu"; timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "bench"; timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-600
echo "sweep bf16"; timeout -k 10 300 python -u tools/gemm_sweep.py --variants p0 --shapes 4096,8192,16384,4096x4096x16384,16384x16384x1024,12288,8192x8192x12288,12288x12288x10240 --rounds 2 > $O/sweep_bf16.jsonl 2> $O/sweep.err || exit 1
echo "sweep fp8"; timeout -k 10 300 python -u tools/gemm_sweep.py --dtype fp8 --variants p0 --shapes 4096,8192,16384,4096x4096x16384,16384x16384x1024,12288 --rounds 2 > $O/sweep_fp8.jsonl 2>> $O/sweep.err || exit 1
cd /tmp && export TMPDIR=/tmp
echo "rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 20 --no-extras > $GRAFT_REPO_ROOT/$O/bench_prof.log 2>&1
echo done
