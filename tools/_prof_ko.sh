# Knock-out cycle accounting for the v10 GEMM (variants 20-24) vs v10 and hipBLASLt at 8192^3.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/ko
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in 10 20 21 22 23 24 5; do
  timeout -k 10 300 rocprofv3 --pmc $G1 --output-format csv -d $OUT/v$v -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --size 8192 --iters 30 --variant $v > $OUT/v$v.log 2>&1
done
timeout -k 10 300 rocprofv3 --pmc $G1 --output-format csv -d $OUT/blas -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --size 8192 --iters 30 --blas > $OUT/blas.log 2>&1
