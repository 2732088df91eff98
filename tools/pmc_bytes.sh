#!/bin/bash
# HBM bytes per GEMM variant: FETCH_SIZE and WRITE_SIZE (KiB, derived TCC counters) in separate passes --
# one pass may hold 4 TCC counters and FETCH_SIZE alone takes 3. Usage (on the box, repo root):
#   bash tools/pmc_bytes.sh <outdir> <bf16|fp8> <size> <variant|blas> [...]
set -e
OUT=$GRAFT_REPO_ROOT/$1; DT=$2; SIZE=$3; shift 3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  extra="--variant $v"; [ $v = blas ] && extra="--blas"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/${DT}_${v}_$c \
      -- python3 $GRAFT_REPO_ROOT/tools/gemm_prof.py --dtype $DT --size $SIZE --iters 20 $extra > $OUT/${DT}_${v}_$c.log 2>&1
  done
done
