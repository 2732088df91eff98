"""RCCL all-reduce fabric probe (one process per GPU, ``torch.distributed`` backend ``nccl``=RCCL).

The reference never exercises the GPU interconnect (no NCCL call sites). The
validator here proves the xGMI mesh of an 8xMI355X node by timing a sum all-reduce and
reporting algorithm bandwidth and bus bandwidth ``busBW = algBW * 2(n-1)/n``. On a fully
connected 8-GPU xGMI mesh each GPU has 7 links of ~153 GB/s; a single ring is bounded by one
link, so the reported busBW is compared against both the per-link and the 7-link bound.

The same protocol runs on CPU with the ``gloo`` backend for tests (correctness only).
"""

from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List, Optional

XGMI_LINK_GBPS = 153.0   # per direction, per link (MI355X)
XGMI_LINKS = 7


@dataclass
class AllReduceResult:
    nbytes: int
    ranks: int
    seconds: float
    algbw_gbps: float
    busbw_gbps: float
    ok: bool

    def as_dict(self) -> dict:
        return {"bytes": self.nbytes, "ranks": self.ranks, "time_us": self.seconds * 1e6,
                "algbw_gbps": self.algbw_gbps, "busbw_gbps": self.busbw_gbps, "ok": self.ok,
                "link_bound_gbps": XGMI_LINK_GBPS, "mesh_bound_gbps": XGMI_LINK_GBPS * XGMI_LINKS}


def bus_factor(ranks: int) -> float:
    return 2.0 * (ranks - 1) / ranks if ranks > 1 else 1.0


def measure_allreduce(nbytes: int, dtype=None, iters: int = 20, warmup: int = 5,
                      device=None, group=None) -> AllReduceResult:
    """Time ``iters`` all-reduces of ``nbytes`` and check the sum exactly.

    Every rank contributes ``rank + 1`` in every element, so the reduced value is
    ``n(n+1)/2`` — exactly representable in bf16 for n <= 8 (max 36).
    """
    import torch
    import torch.distributed as dist

    dtype = dtype or torch.float32
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    elem = torch.tensor([], dtype=dtype).element_size()
    numel = max(1, nbytes // elem)
    x = torch.empty(numel, dtype=dtype, device=device)
    is_gpu = x.is_cuda

    def sync():
        if is_gpu:
            torch.cuda.synchronize(x.device)

    for _ in range(warmup):
        x.fill_(rank + 1)
        dist.all_reduce(x, group=group)
    sync()
    x.fill_(rank + 1)
    sync()
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(x, group=group)
    sync()
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], dtype=torch.float64, device=device if is_gpu else None)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    dt = float(t.item())
    # After `iters` in-place reductions the value is s * world^(iters-1); check one fresh pass.
    x.fill_(rank + 1)
    dist.all_reduce(x, group=group)
    expect = world * (world + 1) / 2
    ok = bool(torch.all(x == expect).item())
    nb = numel * elem
    algbw = nb / dt / 1e9
    return AllReduceResult(nb, world, dt, algbw, algbw * bus_factor(world), ok)


def sweep(sizes: Optional[List[int]] = None, dtype=None, device=None, iters: int = 20,
          warmup: int = 5) -> List[AllReduceResult]:
    """Message-size sweep 8 B ... 8 GiB (x2 steps by default, capped by the caller)."""
    if sizes is None:
        sizes, s = [], 8
        while s <= (1 << 30):
            sizes.append(s)
            s *= 2
    return [measure_allreduce(s, dtype=dtype, device=device, iters=iters, warmup=warmup)
            for s in sizes]
