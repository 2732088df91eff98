#!/usr/bin/env python3
"""Run one GEMM variant repeatedly on random bf16 data (a target for rocprofv3 --pmc / --stats).

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/gemm_prof.py --variant 4 --size 8192 --iters 50
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=4)
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
    G.set_variant(a.variant)
    for _ in range(a.iters):
        if a.blas:
            torch.matmul(A, Bt.t(), out=C)
        else:
            G.gemm_bf16(A, Bt, C)
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
    G.set_fp8_variant(a.variant)
    for _ in range(a.iters):
        if a.blas:
            C = torch._scaled_mm(A, Bt.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        else:
            G.gemm_fp8(A, Bt, C)
    torch.cuda.synchronize()
    print("ok", G.verify(A, Bt, C, nrows=8).ok)


if __name__ == "__main__":
    main()
