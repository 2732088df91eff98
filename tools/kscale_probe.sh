# K-scaling probe of the production GEMM vs hipBLASLt (8192x8192xK, K=2k..32k) plus a
# kernel trace of the 8192^3 comparison.  Run on the GPU box: gpurun -- bash tools/kscale_probe.sh
# Output: gpurun_out/kp/sweep.jsonl (per-shape TFLOPS), gpurun_out/kp/tr (rocprofv3 CSV).
set -e
mkdir -p gpurun_out/kp
timeout -k 10 300 python3 tools/gemm_sweep.py --shapes 8192x8192x2048,8192x8192x4096,8192x8192x8192,8192x8192x16384,8192x8192x32768 --variants p0,p25 --iters 30 --rounds 3 > gpurun_out/kp/sweep.jsonl 2>gpurun_out/kp/sweep.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/kp/tr -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --size 8192 --iters 20 --blas > $GRAFT_REPO_ROOT/gpurun_out/kp/tr.log 2>&1
echo done
