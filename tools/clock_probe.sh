#!/bin/bash
# Effective shader clock of a GEMM run: GRBM_GUI_ACTIVE (busy cycles) and the kernel duration from
# the same rocprofv3 run. Usage (on the box, repo root): bash tools/clock_probe.sh <outdir> <size>
set -e
OUT=$GRAFT_REPO_ROOT/$1
SIZE=$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for dt in bf16 fp8; do
  for who in ours blas; do
    extra=""; [ $who = blas ] && extra="--blas"
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv \
      -d $OUT/${dt}_${who} -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --dtype $dt --size $SIZE \
      --iters 30 --variant $([ $dt = bf16 ] && echo 44 || echo 9) $extra > $OUT/${dt}_${who}.log 2>&1
  done
done
python3 $GRAFT_REPO_ROOT/tools/clock_summary.py $OUT > $OUT/clock_summary.txt
