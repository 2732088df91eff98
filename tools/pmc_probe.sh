#!/bin/bash
# Clock and cycle counters for several GEMM variants in one call: GRBM_GUI_ACTIVE (busy cycles, for
# the effective clock), wave cycles, MFMA busy and waitcnt/barrier waits, each run its own
# rocprofv3 process. Usage (on the box, repo root):
#   bash tools/pmc_probe.sh <outdir> <bf16|fp8> <size> <variant|blas> [...]
# variants as tools/gemm_prof.py takes them (p<v> = shipped library, <v> = lab library).
set -e
OUT=$GRAFT_REPO_ROOT/$1; DT=$2; SIZE=$3; shift 3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  extra="--variant $v"; [ $v = blas ] && extra="--blas"
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $OUT/${DT}_$v \
    -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --dtype $DT --size $SIZE --iters 40 $extra > $OUT/${DT}_$v.log 2>&1
done
python3 $GRAFT_REPO_ROOT/tools/clock_summary.py $OUT > $OUT/clock_summary.txt
cat $OUT/clock_summary.txt
