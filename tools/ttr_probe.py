#!/usr/bin/env python3
"""Node time-to-ready on this box (validator/ttr.py): our light chain, the reference protocol and
our full chain (production HIP workload), with every barrier and mark. One JSON line per run.

    python tools/ttr_probe.py [--rounds 1] [--no-reference] [--no-full]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_operator_amd.validator import ttr  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--no-reference", action="store_true")
    ap.add_argument("--no-full", action="store_true")
    ap.add_argument("--gemm-shapes", default="8192")
    a = ap.parse_args()
    for i in range(a.rounds):
        runs = [("ours", False)] + ([] if a.no_full else [("ours", True)]) + ([] if a.no_reference else [("reference", False)])
        for proto, full in runs:
            h = ttr.Harness(hip_mode="local", gemm_shapes=a.gemm_shapes, timeout=180, hip_full=full)
            r = h.run(proto)
            print(json.dumps({"round": i, "protocol": proto, "full": full, "time_to_ready_s": r["time_to_ready_s"],
                              "barriers_s": r["barriers_s"], "marks_s": r["marks_s"], "errors": r["errors"]}),
                  flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
