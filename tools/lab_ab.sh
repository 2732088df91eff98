#!/bin/bash
# GEMM A/B passes on the GPU box, one timed pass per spec, each under its own time limit; stops at
# the first failing pass. Replaces the one-off round-3 recipes (r3s2_*.sh).
#
#   bash tools/lab_ab.sh <out-subdir> <tool>:<dtype>:<shapes>:<variants>[:rounds] ...
#     tool     lab   = tools/asm_lab.py (lab kernels next to production, variant ids of the lab libraries)
#              sweep = tools/gemm_sweep.py (production dispatch, pN pins variant N, vs hipBLASLt)
#   e.g. bash tools/lab_ab.sh r4_zc lab:bf16:8192,16384:136,197:4 sweep:fp8:12288,4096x4096x32768:p0:2
set -eo pipefail
O=gpurun_out/${1:?out-subdir}
shift
mkdir -p "$O"
i=0
for spec in "$@"; do
  IFS=: read -r tool dt shapes variants rounds <<< "$spec"
  case "$tool" in
    lab) script=tools/asm_lab.py ;;
    sweep) script=tools/gemm_sweep.py ;;
    *) echo "unknown tool '$tool' in '$spec'" >&2; exit 2 ;;
  esac
  echo "pass $i: $spec"
  timeout -k 10 300 python -u "$script" --dtype "$dt" --shapes "$shapes" --variants "$variants" \
    --rounds "${rounds:-3}" > "$O/${i}_${tool}_${dt}.jsonl" 2>> "$O/err"
  i=$((i + 1))
done
echo done
