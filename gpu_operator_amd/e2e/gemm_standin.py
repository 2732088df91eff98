"""A scripted stand-in for ``amd-gemm-validate`` (CPU rehearsals of the validation pods).

The e2e harness and the validation-pod tests run the real validator, the real workload entry
(``amd-validator-workload hip``) and a real kubelet's pod semantics on CPU; only the GEMM itself is
scripted. This program speaks the binary's protocol -- the same argv, the same JSON lines (``start``,
``hip-smoke``, one ``gemm`` line per GPU with its ``kind`` on failure, ``aggregate``, ``done``), the
same exit status, the same floor gate -- for the GPUs HIP_VISIBLE_DEVICES names (device numbers in
its output are visible indices, as the binary's are).

Script (environment):
  GEMM_STANDIN_SCRIPT   runs separated by ";" -- "fast", or "slow:3,5" (node GPUs 3 and 5 at 600
                        TF/s, the others at 1500), or "badtile:3@5.7.2" (node GPU 3 computes a wrong
                        output tile [5,7] on XCD 2: the ABFT failure line of the binary); run k uses
                        entry k, the last entry repeats
  GEMM_STANDIN_STATE    file counting the runs (also ``<state>.running`` exists while one runs)
  GEMM_STANDIN_RUNTIME_S  how long a run takes (default 1)
  GEMM_STANDIN_GPUS     GPUs without HIP_VISIBLE_DEVICES (default 8)
  GEMM_STANDIN_SLOW_FILE  a file of node GPU indices ("3" or "3,5") read when the run reports: those
                        GPUs are slow too (a tenant given the GPU mid-sweep shares it); the run waits
                        up to 60 s for the file to exist
"""

from __future__ import annotations

import json
import os
import sys
import time
from typing import List


def _arg(argv: List[str], name: str, default: str = "") -> str:
    return argv[argv.index(name) + 1] if name in argv and argv.index(name) + 1 < len(argv) else default


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    state = os.environ.get("GEMM_STANDIN_STATE", "")
    runs = 0
    if state and os.path.exists(state):
        with open(state) as f:
            runs = int(f.read().strip() or 0)
    if state:
        with open(state, "w") as f:
            f.write(str(runs + 1))
        open(state + ".running", "w").close()
    script = [x for x in os.environ.get("GEMM_STANDIN_SCRIPT", "fast").split(";") if x] or ["fast"]
    entry = script[min(runs, len(script) - 1)]
    slow = {int(x) for x in entry.split(":", 1)[1].split(",") if x} if entry.startswith("slow:") else set()
    bad = {}                                       # node GPU -> (tm, tn, xcd)
    if entry.startswith("badtile:"):
        for item in entry.split(":", 1)[1].split(","):
            gpu, where = item.split("@")
            tm, tn, xcd = (int(x) for x in where.split("."))
            bad[int(gpu)] = (tm, tn, xcd)
    vis = os.environ.get("HIP_VISIBLE_DEVICES", "")
    nodes = [int(x) for x in vis.split(",") if x.strip()] if vis else \
        list(range(int(os.environ.get("GEMM_STANDIN_GPUS", "8"))))
    m = n = k = int(_arg(argv, "--shapes", "8192").split(",")[0].split("x")[0])
    floor = float(_arg(argv, "--min-tflops", "0") or 0)
    floors_apply = m * n >= 256 * 65536 and k >= 4096
    print(json.dumps({"event": "start", "devices": len(nodes), "visible": len(nodes), "gcn_arch": "gfx950",
                      "cus": 256, "launch": "standin"}), flush=True)
    if "--smoke" in argv:
        print(json.dumps({"event": "hip-smoke", "devices": len(nodes), "elements": 50000, "ok": True}), flush=True)
    time.sleep(float(os.environ.get("GEMM_STANDIN_RUNTIME_S", "1")))
    slow_file = os.environ.get("GEMM_STANDIN_SLOW_FILE", "")
    if slow_file:
        end = time.monotonic() + 60
        while not os.path.exists(slow_file) and time.monotonic() < end:
            time.sleep(0.05)
        if os.path.exists(slow_file):
            with open(slow_file) as f:
                slow |= {int(x) for x in f.read().replace("\n", ",").split(",") if x.strip()}
    ok_all, total, lo = True, 0.0, None
    for i, node in enumerate(nodes):
        tf = 600.0 if node in slow else 1500.0
        ok = not (floors_apply and floor and tf < floor)
        line = {"event": "gemm", "dtype": "bf16", "device": i, "m": m, "n": n, "k": k, "tflops": tf,
                "max_rel_err": 1e-3, "checked_fraction": 1.0, "abft_worst_ratio": 0.3, "bad_tiles": 0, "variant": 50,
                "tile_m": 256, "tile_n": 256, "ok": ok}
        if not ok:
            line.update(kind="floor", error=f"below floor: {tf:.1f} < {floor:.1f} TFLOP/s")
        if node in bad:
            tm, tn, xcd = bad[node]
            ok = False
            line.update(ok=False, kind="correctness", bad_tiles=1, abft_worst_ratio=55.0, tile=[tm, tn],
                        workgroup=8 * tm + xcd, round=0, xcd=xcd, cu={"se": 1, "sh": 0, "cu": 4},
                        bad_tile_list=[[tm, tn, xcd]],
                        error=f"ABFT: 1 bad tile(s), first [{tm},{tn}] (workgroup {8 * tm + xcd}, XCD {xcd})")
        print(json.dumps(line), flush=True)
        ok_all = ok_all and ok
        total += tf
        lo = tf if lo is None else min(lo, tf)
    print(json.dumps({"event": "aggregate", "dtype": "bf16", "m": m, "n": n, "k": k, "gpus": len(nodes),
                      "total_tflops": total, "per_gpu_tflops": total / max(1, len(nodes)), "min_gpu_tflops": lo or 0.0,
                      "ok": ok_all}), flush=True)
    print(json.dumps({"event": "done", "ok": ok_all}), flush=True)
    if state and os.path.exists(state + ".running"):
        os.remove(state + ".running")
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
