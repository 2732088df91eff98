# One-call GPU confirmation: gpu tests, smoke, the driver's exact bench invocation, a longer bench,
# rocprofv3 kernel stats. Usage (from the repo root on the GPU box): bash tools/gpu_round.sh [out-subdir]
set -e
OUT=gpurun_out/${1:-round}
mkdir -p $OUT
# read-only evidence for the partition round trip (tests/test_node_agents_gpu.py): who we are, whether
# root is available without a password, and whether the compute-partition attributes are writable
{ id; sudo -n true 2>&1 && echo "sudo: ok" || echo "sudo: not available"
  for f in /sys/bus/pci/devices/*/current_compute_partition /sys/bus/pci/devices/*/current_memory_partition; do
    [ -e "$f" ] || continue; ls -l "$f"; echo "  value=$(cat "$f") writable=$([ -w "$f" ] && echo yes || echo no)"; done
} > $OUT/partition_permissions.log 2>&1 || true
echo "pytest -m gpu"; timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -3 $OUT/pytest_gpu.log
echo "smoke"; timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "bench (driver invocation)"; timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1
tail -1 $OUT/bench_driver.log
echo "bench (defaults)"; timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
echo "rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 20 --no-extras > $GRAFT_REPO_ROOT/$OUT/bench_prof.log 2>&1
echo "small-grid traces"
for spec in "bf16 1024" "fp8 1024" "bf16 1024x1024x8192" "fp8 1024x1024x16384" "bf16 2560" "bf16 2560x2560x8192" "fp8 2560x2560x16384"; do
  set -- $spec
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace_$1_$2 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --dtype $1 --variant p0 --size $2 --iters 100 > $GRAFT_REPO_ROOT/$OUT/trace_$1_$2.log 2>&1
done
[ "${SKIP_SWEEP:-0}" = 1 ] && { echo done; exit 0; }
echo "closing sweep"
cd $GRAFT_REPO_ROOT
S=1024,1024x1024x4096,1024x1024x16384,512x512x8192,1536,2048,2048x2048x1024,2048x2048x8192,2560,2560x2560x8192,2560x2560x16384,2048x4096x8192,3072x3072x1024,4096,8192,16384,16384x16384x1024
timeout -k 10 500 python -u tools/gemm_sweep.py --variants p0 --rounds 3 --iters 30 --shapes $S > $OUT/closing_sweep_bf16.jsonl 2>&1
timeout -k 10 500 python -u tools/gemm_sweep.py --dtype fp8 --variants p0 --rounds 3 --iters 30 --shapes $S > $OUT/closing_sweep_fp8.jsonl 2>&1
echo done
