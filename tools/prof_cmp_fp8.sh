#!/bin/bash
# PMC comparison of fp8 GEMM variants vs hipBLASLt fp8 (torch._scaled_mm), one counter group per
# rocprofv3 run. Usage (on the box, repo root): bash tools/prof_cmp_fp8.sh <outdir> <size> <variant>...
set -e
OUT=$GRAFT_REPO_ROOT/$1; shift
SIZE=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # tag "pmc" args...
  tag=$1; shift
  pmc=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $OUT/$tag -- \
    python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --dtype fp8 --size $SIZE --iters 30 "$@" > $OUT/$tag.log 2>&1
}
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum"
G3="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_blas -- \
  python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --dtype fp8 --size $SIZE --iters 30 --blas > $OUT/trace_blas.log 2>&1
for v in "$@"; do
  run v${v}_g1 "$G1" --variant $v
  run v${v}_g2 "$G2" --variant $v
done
run blas_g1 "$G1" --blas
run blas_g2 "$G2" --blas
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/*_g1 > $OUT/summary_g1.txt
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/*_g2 > $OUT/summary_g2.txt
# address-translation / memory-request group last: a counter this ROCm does not know only loses it
for v in "$@"; do run v${v}_g3 "$G3" --variant $v; done
run blas_g3 "$G3" --blas
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/*_g3 > $OUT/summary_g3.txt
