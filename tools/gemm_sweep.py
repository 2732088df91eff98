#!/usr/bin/env python3
"""GEMM shape sweep: hand-written MFMA kernel vs hipBLASLt (torch.matmul) on the same random data.

Shapes follow SURVEY.md §7.5: M=N=K in {1024, 4096, 8192, 16384} plus skinny 16384x16384x1024.
Interleaves the two implementations in one process (methodology rule: A/B in one process); every
timed block follows ~0.1 s of back-to-back calls (the MI355X clock ramps over the first ~25 GEMMs)
and spans >= 0.05 s, so 1024^3 and 4096^3 are timed over hundreds of launches, not 20.
Prints one JSON line per shape. ``--variants`` takes production numbers (``p0`` = automatic
dispatch of the shipped library, ``p44`` = pinned) or lab numbers (plain integers: the tools-only
experiment library, tools/gemm_lab.py; build it with ``python -m gpu_operator_amd._build --lab``).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def time_fn(fn, iters, torch):
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / iters / 1e3


class _Pinned:
    """A callable (A, Bt, C) for a production ('p<v>') or lab ('<v>') variant. ``select()`` pins a
    production variant once before a timed block, so the timed launches carry no variant switch."""

    def __init__(self, G, spec: str, dtype: str):
        self.G, self.dtype = G, dtype
        self.split = None
        self.asm = None
        if spec.startswith("p") and "b" in spec[1:]:          # p57s2b540[p]: v57 / v24 in 2 pieces, the last 54 % of K
            v, rest = spec[1:].split("s")                     # (p: piece-major items; t, the default: tile-major)
            s, b = rest.split("b")
            pm = b.endswith("p")
            self.v, self.lab, self.asm = int(v), None, (int(s), int(b.rstrip("tp")), pm)
        elif spec.startswith("p") and "s" in spec[1:]:          # p61s2: v61 aiming at 2 workgroups per CU
            v, t = spec[1:].split("s")
            self.v, self.lab, self.split = int(v), None, int(t)
        elif spec.startswith("p"):
            self.v, self.lab = int(spec[1:]), None
        else:
            import gemm_lab
            self.v, self.lab = int(spec), gemm_lab

    def select(self):
        if self.lab is None:
            (self.G.set_variant if self.dtype == "bf16" else self.G.set_fp8_variant)(self.v)
            if self.dtype == "bf16":
                self.G.set_split_target(self.split or 1)
            self.G.set_asm_split(*(self.asm or (0, 0)))

    def __call__(self, A, Bt, C):
        if self.lab is not None:
            f = self.lab.gemm_bf16 if self.dtype == "bf16" else self.lab.gemm_fp8
            return f(self.v, A, Bt, C)
        return (self.G.gemm_bf16 if self.dtype == "bf16" else self.G.gemm_fp8)(A, Bt, C)


def runner(G, spec: str, dtype: str):
    return _Pinned(G, spec, dtype)


def timed(fn, a, torch, select=None):
    """Seconds per call: the clock ramped (~0.1 s of back-to-back calls first), then a block of at
    least ``a.iters`` calls and ~0.05 s, so a short kernel is timed over many launches."""
    if select:
        select()
    t = time_fn(fn, 5, torch)
    n = max(3, int(0.1 / max(t, 1e-6)))
    time_fn(fn, min(n, 5000), torch)
    return time_fn(fn, max(a.iters, min(5000, int(0.05 / max(t, 1e-6)))), torch)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1024,4096,8192,16384,16384x16384x1024")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="p0,44,45")
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16",
                    help="fp8: e4m3fn operands on gemm_fp8 vs hipBLASLt through torch._scaled_mm")
    a = ap.parse_args()
    if a.dtype == "fp8":
        return sweep_fp8(a)
    import torch
    from gpu_operator_amd.ops import gemm as G

    dev = torch.device("cuda", 0)
    for s in a.shapes.split(","):
        if "x" in s:
            m, n, k = map(int, s.split("x"))
        else:
            m = n = k = int(s)
        A = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
        Bt = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
        G.fill_uniform_(A, 1)
        G.fill_uniform_(Bt, 2)
        C = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
        variants = a.variants.split(",")
        run = {v: runner(G, v, "bf16") for v in variants}
        checks = {}
        for v in variants:
            C.zero_()
            run[v].select()
            run[v](A, Bt, C)
            checks[v] = G.verify(A, Bt, C, nrows=16)
        ours = {v: [] for v in variants}
        blas = []
        for _ in range(a.rounds):
            for v in variants:
                ours[v].append(timed(lambda: run[v](A, Bt, C), a, torch, run[v].select))
            blas.append(timed(lambda: torch.matmul(A, Bt.t(), out=C), a, torch))
        t_b = min(blas)
        rec = {"m": m, "n": n, "k": k, "hipblaslt_tflops": round(G.tflops(m, n, k, t_b), 1)}
        for v in variants:
            t_o = min(ours[v])
            rec[f"v{v}_tflops"] = round(G.tflops(m, n, k, t_o), 1)
            rec[f"v{v}_median_tflops"] = round(G.tflops(m, n, k, sorted(ours[v])[len(ours[v]) // 2]), 1)
            rec[f"v{v}_check_ok"] = checks[v].ok
        print(json.dumps(rec), flush=True)
        del A, Bt, C
        torch.cuda.empty_cache()


def sweep_fp8(a):
    import torch
    from gpu_operator_amd.ops import gemm as G

    dev = torch.device("cuda", 0)
    one = torch.ones((), dtype=torch.float32, device=dev)
    for s in a.shapes.split(","):
        m, n, k = map(int, s.split("x")) if "x" in s else (int(s),) * 3
        A = G.fill_uniform_fp8_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device=dev), 1)
        Bt = G.fill_uniform_fp8_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device=dev), 2)
        C = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
        variants = a.variants.split(",")
        run = {v: runner(G, v, "fp8") for v in variants}

        def blas():
            return torch._scaled_mm(A, Bt.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)

        try:
            blas()
            blas_ok = True
        except (RuntimeError, NotImplementedError) as e:          # no hipBLASLt fp8 path
            print(json.dumps({"m": m, "n": n, "k": k, "hipblaslt_error": str(e)[:200]}), flush=True)
            blas_ok = False
        checks = {}
        for v in variants:
            C.zero_()
            run[v].select()
            run[v](A, Bt, C)
            checks[v] = G.verify(A, Bt, C, nrows=16)
        ours = {v: [] for v in variants}
        tb = []
        for _ in range(a.rounds):
            for v in variants:
                ours[v].append(timed(lambda: run[v](A, Bt, C), a, torch, run[v].select))
            if blas_ok:
                tb.append(timed(blas, a, torch))
        rec = {"dtype": "fp8_e4m3fn", "m": m, "n": n, "k": k,
               "hipblaslt_tflops": round(G.tflops(m, n, k, min(tb)), 1) if tb else None}
        for v in variants:
            rec[f"f8v{v}_tflops"] = round(G.tflops(m, n, k, min(ours[v])), 1)
            rec[f"f8v{v}_median_tflops"] = round(G.tflops(m, n, k, sorted(ours[v])[len(ours[v]) // 2]), 1)
            rec[f"f8v{v}_check_ok"] = checks[v].ok
            rec[f"f8v{v}_max_rel_err"] = round(checks[v].max_rel_err, 5)
        print(json.dumps(rec), flush=True)
        del A, Bt, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
