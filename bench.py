#!/usr/bin/env python3
"""Headline benchmark: validator HIP GEMM TFLOPS on 1/2/4/8 MI355X (+ RCCL all-reduce busBW).

BASELINE.json names the metric "node time-to-ready (driver->validator) + validator HIP GEMM
TFLOPS, 1/2/4/8 GPU". The reference publishes no number, so ``vs_baseline`` is
null. One *step* is one validator GEMM probe per GPU: C = A @ Bt^T, bf16 8192x8192x8192 on the
hand-written CDNA4 MFMA kernel (native/hip/gemm_bf16.hip), uniform [-1,1) synthetic operands.
Per-GPU work is fixed as N grows (weak scaling); ``value`` is the whole-job aggregate TFLOPS.

Launch: ``python bench.py`` (1 GPU) or, for N>1, one rank per GPU under
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N``.
After the timed region (and outside it) the job also measures, and reports as extra fields:
the RCCL all-reduce bus bandwidth over xGMI (N>1) and the node validation chain time
(driver/device checks -> hip-smoke -> GEMM check) that gates the validator's readiness.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--shape", default=None, help="MxNxK (overrides --m/--n/--k; safe under torchrun)")
    ap.add_argument("--allreduce-mib", type=int, default=256,
                    help="payload of the post-timing RCCL all-reduce probe (N>1)")
    ap.add_argument("--no-extras", action="store_true", help="skip the all-reduce/validation extras")
    ap.add_argument("--device", choices=["gpu", "cpu"], default="gpu",
                    help="cpu = rehearsal of the distributed plumbing (gloo, torch.matmul) for tests only")
    a = ap.parse_args(argv)
    if a.shape:
        a.m, a.n, a.k = (int(x) for x in a.shape.lower().split("x"))
    return a


def main(argv=None) -> int:
    args = parse_args(argv)
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gpu_operator_amd.ops import gemm as G

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    n_gpus = world
    cpu = args.device == "cpu"
    distributed = world > 1
    if cpu:
        dev = torch.device("cpu")
        if distributed:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
        if distributed:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if distributed:
            if cpu:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local_rank])

    def sync():
        if not cpu:
            torch.cuda.synchronize(dev)

    m, n, k = args.m, args.n, args.k
    a = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
    bt = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
    c = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    if cpu:
        g = torch.Generator().manual_seed(1000 + rank)
        a.copy_(torch.rand((m, k), generator=g) * 2 - 1)
        bt.copy_(torch.rand((n, k), generator=g) * 2 - 1)

        def step():
            torch.matmul(a, bt.t(), out=c)
    else:
        G.fill_uniform_(a, seed=1000 + rank)
        G.fill_uniform_(bt, seed=2000 + rank)

        def step():
            G.gemm_bf16(a, bt, c)

    if cpu:
        return _timed_and_report(args, torch, dist, dev, rank, n_gpus, distributed, barrier, sync, step, m, n, k,
                                 {"device": "cpu-rehearsal"})

    # Validation chain (what the validator pod does before reporting ready).
    t_chain0 = time.perf_counter()
    from gpu_operator_amd.ops import smoke as S
    smoke_ok = S.smoke(device=str(dev))
    G.gemm_bf16(a, bt, c)
    chk = G.verify(a, bt, c, nrows=32, seed=rank)
    torch.cuda.synchronize(dev)
    chain_s = time.perf_counter() - t_chain0
    if not (smoke_ok and chk.ok):
        print(f"rank {rank}: validation FAILED smoke={smoke_ok} gemm={chk}", file=sys.stderr)
        return 2

    extras = {"gemm_check_max_rel_err": chk.max_rel_err, "validation_chain_s": round(chain_s, 4)}
    return _timed_and_report(args, torch, dist, dev, rank, n_gpus, distributed, barrier, sync, step, m, n, k, extras)


def _r(x: float) -> float:
    """2 decimals for real GPU numbers; keep significant digits for tiny CPU rehearsals."""
    return round(x, 2) if abs(x) >= 1 else float(f"{x:.4g}")


def _fp8_extra(args, torch, dist, dev, rank, n_gpus, distributed, barrier, sync):
    """Same shape on the fp8 (OCP e4m3fn) block-scaled MFMA kernel, after and outside the timed
    bf16 region: the matrix cores at their fp8 rate, reported as extra fields only."""
    from gpu_operator_amd.ops import gemm as G
    m, n, k = args.m, args.n, args.k
    f8 = torch.float8_e4m3fn
    a = G.fill_uniform_fp8_(torch.empty((m, k), dtype=f8, device=dev), seed=3000 + rank)
    bt = G.fill_uniform_fp8_(torch.empty((n, k), dtype=f8, device=dev), seed=4000 + rank)
    c = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    steps = max(1, min(args.steps, 100))
    for _ in range(max(1, min(args.warmup, 50))):
        G.gemm_fp8(a, bt, c)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        G.gemm_fp8(a, bt, c)
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    chk = G.verify(a, bt, c, nrows=16, seed=rank)
    per_gpu = G.tflops(m, n, k, elapsed / steps)
    return {"fp8_per_gpu_tflops": _r(per_gpu), "fp8_total_tflops": _r(per_gpu * n_gpus),
            "fp8_check_ok": chk.ok, "fp8_steps": steps}


def _timed_and_report(args, torch, dist, dev, rank, n_gpus, distributed, barrier, sync, step, m, n, k, extras):
    from gpu_operator_amd.ops import gemm as G
    for _ in range(args.warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0

    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    per_gpu_tflops = G.tflops(m, n, k, elapsed / args.steps)
    total_tflops = per_gpu_tflops * n_gpus
    extras = dict(extras, per_gpu_tflops=_r(per_gpu_tflops))
    cpu = args.device == "cpu"
    if not cpu and not args.no_extras:
        extras.update(_fp8_extra(args, torch, dist, dev, rank, n_gpus, distributed, barrier, sync))
    if distributed and not args.no_extras:
        from gpu_operator_amd.parallel.allreduce import measure_allreduce
        nbytes = (64 << 10) if cpu else args.allreduce_mib * (1 << 20)
        r = measure_allreduce(nbytes, dtype=torch.bfloat16, iters=3 if cpu else 10, warmup=1 if cpu else 3,
                              device=dev)
        extras.update({"allreduce_bytes": r.nbytes, "allreduce_algbw_gbps": round(r.algbw_gbps, 2),
                       "allreduce_busbw_gbps": round(r.busbw_gbps, 2), "allreduce_ok": r.ok})

    if n_gpus == 1 and not args.no_extras and not cpu:
        # node time-to-ready (driver -> validator) on this GPU, outside the timed region
        try:
            from gpu_operator_amd.validator import ttr
            r = ttr.run_chain(gemm_shapes="8192", timeout=120)
            if r["time_to_ready_s"] is not None:
                extras["node_time_to_ready_s"] = round(r["time_to_ready_s"], 3)
                extras["reference_model_time_to_ready_s"] = ttr.reference_model(r["steps_s"])["time_to_ready_s"]
            else:
                extras["node_time_to_ready_error"] = "; ".join(r["errors"])[:300]
        except Exception as e:  # noqa: BLE001 - an extra must never fail the bench
            extras["node_time_to_ready_error"] = str(e)[:300]

    if rank == 0:
        line = {
            "metric": "validator HIP GEMM TFLOPS (bf16 8192^3, aggregate over GPUs)",
            "value": _r(total_tflops),
            "unit": "TFLOP/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform [-1,1) bf16 operands, random init)",
            "config": {"model": f"validator mfma-gemm bf16 M={m} N={n} K={k}",
                       "global_batch": n_gpus, "seq_len": None,
                       "parallelism": f"dp{n_gpus} (one GEMM per GPU, RCCL over xGMI)"},
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
