set -e
mkdir -p gpurun_out/cmp
cd /tmp && export TMPDIR=/tmp
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 300 rocprofv3 --pmc $PMC --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/cmp/ours -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --variant 5 --size 8192 --iters 40 > $GRAFT_REPO_ROOT/gpurun_out/cmp/ours.log 2>&1
timeout -k 10 300 rocprofv3 --pmc $PMC --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/cmp/blas -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --blas --size 8192 --iters 40 > $GRAFT_REPO_ROOT/gpurun_out/cmp/blas.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/cmp/blas_trace -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --blas --size 8192 --iters 40 > $GRAFT_REPO_ROOT/gpurun_out/cmp/blas_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/cmp/ours_trace -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --variant 5 --size 8192 --iters 40 > $GRAFT_REPO_ROOT/gpurun_out/cmp/ours_trace.log 2>&1
