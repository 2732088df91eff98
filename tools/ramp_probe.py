#!/usr/bin/env python3
"""How fast an MI355X gets its GEMM clock back after a host idle: stabilise (bench.py's protocol),
idle T ms, then time every one of the next N dispatches on events. Prints one JSON line per idle
length with the per-dispatch times (ms) in groups of 10. Used to size the re-ramp after a barrier
(bench.py Ctx.reramp, amd-gemm-validate --ramp-ms)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gpu_operator_amd.ops import gemm as G  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    a = G.fill_uniform_(torch.empty((m, m), dtype=torch.bfloat16, device=dev), 1)
    b = G.fill_uniform_(torch.empty((m, m), dtype=torch.bfloat16, device=dev), 2)
    c = torch.empty((m, m), dtype=torch.bfloat16, device=dev)
    n = 150
    for idle in (0, 20, 50, 200, 1000, 200, 0):
        for _ in range(100):
            G.gemm_bf16(a, b, c)
        torch.cuda.synchronize()
        time.sleep(idle / 1e3)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        ev[0].record()
        for i in range(n):
            G.gemm_bf16(a, b, c)
            ev[i + 1].record()
        torch.cuda.synchronize()
        t = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
        groups = [round(sum(t[i:i + 10]) / 10, 4) for i in range(0, n, 10)]
        steady = sorted(t[-50:])[25]
        slow = [i for i, x in enumerate(t) if x > 1.01 * steady]
        print(json.dumps({"idle_ms": idle, "steady_ms": round(steady, 4), "groups_ms": groups,
                          "last_slow_dispatch": max(slow) if slow else -1, "slow_count": len(slow)}), flush=True)


if __name__ == "__main__":
    main()
