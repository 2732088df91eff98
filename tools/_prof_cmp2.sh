# PMC comparison: GEMM variant(s) vs hipBLASLt at 8192^3 (one counter group per rocprofv3 run).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/cmp2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run() {  # tag pmc... -- args
  tag=$1; shift
  pmc=$1; shift
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $OUT/$tag -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --size 8192 --iters 30 "$@" > $OUT/$tag.log 2>&1
}
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for v in 5 10; do
  run v${v}_g1 "$G1" --variant $v
  run v${v}_g2 "$G2" --variant $v
done
run blas_g1 "$G1" --blas
run blas_g2 "$G2" --blas
