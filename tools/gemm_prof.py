#!/usr/bin/env python3
"""Run one GEMM variant repeatedly on random bf16 data (a target for rocprofv3 --pmc / --stats).

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/gemm_prof.py --variant p0 --size 8192 --iters 50

``--variant p<v>`` runs the shipped library (p0 = automatic dispatch); a plain number runs that
variant of the tools-only lab library (tools/gemm_lab.py).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_sweep import runner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="p0")
    ap.add_argument("--size", default="8192")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--blas", action="store_true", help="run hipBLASLt (torch.matmul / _scaled_mm) instead")
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16")
    a = ap.parse_args()
    if a.dtype == "fp8":
        return main_fp8(a)
    import torch
    from gpu_operator_amd.ops import gemm as G
    m, n, k = (map(int, a.size.split("x")) if "x" in a.size else [int(a.size)] * 3)
    dev = torch.device("cuda", 0)
    A = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
    Bt = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
    C = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    G.fill_uniform_(A, 1)
    G.fill_uniform_(Bt, 2)
    run = runner(G, a.variant, "bf16")
    run.select()
    for _ in range(a.iters):
        if a.blas:
            torch.matmul(A, Bt.t(), out=C)
        else:
            run(A, Bt, C)
    torch.cuda.synchronize()
    print("ok", G.verify(A, Bt, C, nrows=8).ok)


def main_fp8(a):
    import torch
    from gpu_operator_amd.ops import gemm as G
    m, n, k = (map(int, a.size.split("x")) if "x" in a.size else [int(a.size)] * 3)
    dev = torch.device("cuda", 0)
    f8 = torch.float8_e4m3fn
    A = G.fill_uniform_fp8_(torch.empty((m, k), dtype=f8, device=dev), 1)
    Bt = G.fill_uniform_fp8_(torch.empty((n, k), dtype=f8, device=dev), 2)
    C = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    one = torch.ones((), dtype=torch.float32, device=dev)
    run = runner(G, a.variant, "fp8")
    run.select()
    for _ in range(a.iters):
        if a.blas:
            C = torch._scaled_mm(A, Bt.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        else:
            run(A, Bt, C)
    torch.cuda.synchronize()
    print("ok", G.verify(A, Bt, C, nrows=8).ok)


if __name__ == "__main__":
    main()
