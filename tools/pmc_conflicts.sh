#!/bin/bash
# LDS bank-conflict / MFMA-op counters of the production GEMM kernels over a few shapes (one
# rocprofv3 --pmc pass per shape and dtype; counters only, no traces). Output: CSV per pass under
# gpurun_out/<dir>/ and a one-line-per-pass summary.
#   tools/pmc_conflicts.sh <outdir> <dtype> <shape>...
set -euo pipefail
out=$1; dtype=$2; shift 2
mkdir -p "$out"
BIN=gpu_operator_amd/_native/bin/amd-gemm-validate
for s in "$@"; do
  d="$out/${dtype}_$s"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --output-format csv -d "$d" -- "$BIN" --shapes "$s" --iters 1 --warmup 0 --no-stabilise --devices 0 \
    --check-rows 1 --dtype "$dtype" > "$d.log" 2>&1
  f=$(find "$d" -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$dtype" "$s" <<'PY'
import csv, sys
f, dtype, shape = sys.argv[1:]
agg = {}
for row in csv.DictReader(open(f)):
    if "gemm_" + ("fp8" if dtype == "fp8" else "bf16") + "_256x256" not in row["Kernel_Name"]:
        continue
    agg[row["Counter_Name"]] = agg.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    kern = row["Kernel_Name"][:90]
print(dtype, shape, {k: int(v) for k, v in sorted(agg.items())}, kern)
PY
done
