#!/usr/bin/env python3
"""Per-run mean GEMM duration, GRBM_GUI_ACTIVE / GRBM_COUNT and the implied clock (cycles / time).

    python3 tools/clock_summary.py gpurun_out/clk      (subdirectories written by clock_probe.sh)
"""
import collections
import csv
import glob
import os
import sys


def gemm(name: str) -> bool:
    return ("gemm" in name or "Cijk" in name) and "ref_rows" not in name


def main(root: str) -> None:
    print(f"{'run':12s} {'dispatches':>10s} {'mean_us':>9s} {'GUI_ACTIVE':>12s} {'GRBM_COUNT':>12s} {'GHz(GUI/t)':>10s}")
    for d in sorted(glob.glob(os.path.join(root, "*/"))):
        ctr = collections.defaultdict(dict)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if gemm(r["Kernel_Name"]):
                    ctr[r["Dispatch_Id"]][r["Counter_Name"]] = ctr[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) \
                        + float(r["Counter_Value"])
        durs = {}
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if gemm(r["Kernel_Name"]):
                    durs[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        ids = [i for i in ctr if i in durs]
        if not ids:
            print(f"{os.path.basename(d.rstrip('/')):12s} no matched dispatches")
            continue
        t = sum(durs[i] for i in ids) / len(ids)
        gui = sum(ctr[i].get("GRBM_GUI_ACTIVE", 0) for i in ids) / len(ids)
        cnt = sum(ctr[i].get("GRBM_COUNT", 0) for i in ids) / len(ids)
        extra = sorted({c for i in ids for c in ctr[i]} - {"GRBM_GUI_ACTIVE", "GRBM_COUNT"})
        more = "  ".join(f"{c}={sum(ctr[i].get(c, 0) for i in ids) / len(ids):.4g}" for c in extra)
        print(f"{os.path.basename(d.rstrip('/')):12s} {len(ids):10d} {t * 1e6:9.1f} {gui:12.4g} {cnt:12.4g} "
              f"{gui / t / 1e9:10.3f}  {more}")


if __name__ == "__main__":
    main(sys.argv[1])
