#!/bin/bash
# PMC passes (counters only, one rocprofv3 run per pass and implementation) of the asm-lab bf16
# kernels against hipBLASLt at one shape. Summary: per (impl, pass) the counter sums over the
# dispatches of the GEMM kernel, divided by the dispatch count.
#   tools/pmc_lab.sh <outdir> <shape> <impl>...     (impl: a tools/asm_lab.py variant number or blas)
set -euo pipefail
out=$1; shape=$2; shift 2
mkdir -p "$out"
PASSES=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
  "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum"
)
for impl in "$@"; do
  for i in "${!PASSES[@]}"; do
    d="$out/${impl}_p$i"
    timeout -s KILL 120 rocprofv3 --pmc ${PASSES[$i]} --output-format csv -d "$d" -- \
      python3 tools/asm_lab.py --shapes "$shape" --one "$impl" --iters 3 > "$d.log" 2>&1
    f=$(find "$d" -name '*counter_collection.csv' | head -1)
    python3 - "$f" "$impl" "$i" <<'PY'
import csv, sys
f, impl, p = sys.argv[1:]
agg, disp = {}, set()
for row in csv.DictReader(open(f)):
    k = row["Kernel_Name"]
    if not ("gemm_bf16_256x256" in k or k.startswith("Cijk") or "Cijk_" in k):
        continue
    disp.add(row["Dispatch_Id"])
    agg[row["Counter_Name"]] = agg.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
n = max(1, len(disp))
print(impl, "pass", p, "dispatches", len(disp), {k: round(v / n) for k, v in sorted(agg.items())})
PY
  done
done
