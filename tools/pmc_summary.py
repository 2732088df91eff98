#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per-dispatch mean of each counter for the GEMM kernel.

    python3 tools/pmc_summary.py gpurun_out/ko/v10 gpurun_out/ko/blas ...
"""
import collections
import csv
import glob
import sys


def summarise(d):
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if ("gemm" not in name and "Cijk" not in name) or "ref_rows" in name:
                continue
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (_, c), v in agg.items():
        per[c].append(v)
    return {c: sum(v) / len(v) for c, v in per.items()}


if __name__ == "__main__":
    rows = {d.rstrip("/").split("/")[-1]: summarise(d) for d in sys.argv[1:]}
    cols = sorted({c for r in rows.values() for c in r})
    print("run".ljust(8) + "".join(c.replace("SQ_", "")[:16].rjust(17) for c in cols))
    for k, r in rows.items():
        print(k.ljust(8) + "".join(f"{r.get(c, 0):17.4g}" for c in cols))
