#!/usr/bin/env python3
"""A/B of the hand-scheduled bf16 K pipeline (w4a, native/hip/gemm_bf16_asm_lab.hip) against the
production v44 and hipBLASLt (torch.matmul), in one process, on the same uniform [-1, 1) data.

1. exactness: every w4a variant's C is compared bit for bit with v44's (same MFMA order);
2. timing: ``--rounds`` rounds; in each round every implementation is clock-stabilised (back-to-back
   dispatches until 10 agree within 2 %, >= 30) and then ``--iters`` dispatches are timed between two
   events. Prints one JSON line per (shape, round) and a best/median summary per shape.

    python tools/asm_lab.py --shapes 8192,4096x4096x16384 --variants 44,100,101,102,103 --rounds 5
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class PowerMeter:
    """Average shader clock and socket power over a timed window, sampled from the PMFW gpu_metrics
    table (devices.read_gpu_metrics) every millisecond by a thread; None where it is unreadable."""

    def __init__(self):
        import threading
        self.threading = threading
        try:
            from gpu_operator_amd import devices
            self.read = lambda: devices.read_gpu_metrics("/")[0]
            self.read()
        except Exception:  # noqa: BLE001 - diagnostics only
            self.read = None

    def start(self):
        if self.read is None:
            return
        self.samples, self.stop_ev = [], self.threading.Event()

        def loop():
            while not self.stop_ev.is_set():
                try:
                    m = self.read()
                    clk = [c for c in m["gfxclk_mhz"] if c > 0] if isinstance(m["gfxclk_mhz"], list) else [m["gfxclk_mhz"]]
                    if clk:
                        self.samples.append((sum(clk) / len(clk), m["socket_power_w"]))
                except Exception:  # noqa: BLE001
                    pass
                self.stop_ev.wait(0.001)
        self.t = self.threading.Thread(target=loop, daemon=True)
        self.t.start()

    def stop(self):
        if self.read is None:
            return None
        self.stop_ev.set()
        self.t.join()
        s = [x for x in self.samples if x[0] > 0]
        if not s:
            return None
        return {"gfxclk_mhz": round(sum(x[0] for x in s) / len(s)), "socket_w": round(sum(x[1] for x in s) / len(s), 1),
                "samples": len(s)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8192")
    ap.add_argument("--variants", default="44,100,101,102,103")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16",
                    help="fp8: e4m3 operands through amdgo_asmlab_gemm_fp8, hipBLASLt via torch._scaled_mm")
    ap.add_argument("--one", default=None,
                    help="profiling mode: dispatch only this variant ('blas' = hipBLASLt) --iters times, no checks")
    a = ap.parse_args()
    import torch
    from gpu_operator_amd.ops import gemm as G
    lib = ctypes.CDLL(os.path.join(ROOT, "gpu_operator_amd", "_native", "libamdgo_gemm_asmlab.so"))
    f8 = a.dtype == "fp8"
    fn = lib.amdgo_asmlab_gemm_fp8 if f8 else lib.amdgo_asmlab_gemm_bf16
    fn.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    variants = [int(v) for v in a.variants.split(",")]
    pm = PowerMeter()

    def run(v, A, B, C):
        err = fn(v, A.data_ptr(), B.data_ptr(), C.data_ptr(), A.shape[0], B.shape[0], A.shape[1],
                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if err:
            raise RuntimeError(f"variant {v}: hipError {err}")

    for spec in a.shapes.split(","):
        m, n, k = (int(x) for x in spec.split("x")) if "x" in spec else (int(spec),) * 3
        if f8:
            A = G.fill_uniform_fp8_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device=dev), 11)
            B = G.fill_uniform_fp8_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device=dev), 12)
            one = torch.ones((), dtype=torch.float32, device=dev)

            def blas(out, Bt):
                return torch._scaled_mm(A, Bt, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        else:
            A = G.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=dev), 11)
            B = G.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=dev), 12)

            def blas(out, Bt):
                return torch.matmul(A, Bt, out=out)
        if a.one is not None:                 # rocprofv3 --pmc target: the dispatches and nothing else
            Cx = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
            Bt = B.t()
            for _ in range(a.iters):
                if a.one == "blas":
                    blas(Cx, Bt)
                else:
                    run(int(a.one), A, B, Cx)
            torch.cuda.synchronize()
            continue
        C = {v: torch.empty((m, n), dtype=torch.bfloat16, device=dev) for v in variants}
        Cb = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
        ref = None
        exact = {}
        for v in variants:
            run(v, A, B, C[v])
            torch.cuda.synchronize()
            if ref is None:
                ref = C[v]
                chk = G.verify(A, B, C[v], nrows=16, seed=1)
                exact["ref_check_ok"] = bool(chk.ok)
            exact[v] = bool(torch.equal(C[v], ref))
            if not exact[v]:          # another summation order (serpentine K on another raster): check it
                exact[f"{v}_ref_check_ok"] = bool(G.verify(A, B, C[v], nrows=16, seed=1).ok)
        print(json.dumps({"shape": spec, "bitwise_equal_to_first": exact}), flush=True)
        impls = [(str(v), (lambda v=v: run(v, A, B, C[v]))) for v in variants]
        if not a.no_blas:
            Bt = B.t()
            impls.append(("hipblaslt", lambda: blas(Cb, Bt)))
        flop = 2.0 * m * n * k
        res = {name: [] for name, _ in impls}
        power = {}
        for r in range(a.rounds):
            row, prow = {}, {}
            for name, f in impls:
                times = []
                for _ in range(12):                       # stabilise: batches of 10
                    evs = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
                    evs[0].record()
                    for i in range(10):
                        f()
                        evs[i + 1].record()
                    evs[-1].synchronize()
                    times += [evs[i].elapsed_time(evs[i + 1]) for i in range(10)]
                    last = sorted(times[-10:])
                    if len(times) >= 30 and (last[-1] - last[0]) / last[5] < 0.02:
                        break
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                pm.start()
                e0.record()
                for _ in range(a.iters):
                    f()
                e1.record()
                e1.synchronize()
                pw = pm.stop()
                tf = flop / (e0.elapsed_time(e1) / a.iters * 1e-3) / 1e12
                res[name].append(tf)
                row[name] = round(tf, 1)
                if pw:
                    power.setdefault(name, []).append(pw)
                    prow[name] = pw
            print(json.dumps({"shape": spec, "round": r, "tflops": row, "power": prow}), flush=True)
        summ = {name: {"best": round(max(v), 1), "median": round(statistics.median(v), 1)} for name, v in res.items()}
        if "hipblaslt" in res:
            for name in res:
                summ[name]["ratio_vs_hipblaslt_median"] = round(statistics.median(res[name]) /
                                                                statistics.median(res["hipblaslt"]), 4)
        for name, pws in power.items():
            summ[name]["gfxclk_mhz"] = round(statistics.median(p["gfxclk_mhz"] for p in pws))
            summ[name]["socket_w"] = round(statistics.median(p["socket_w"] for p in pws), 1)
            summ[name]["mj_per_gemm"] = round(statistics.median(p["socket_w"] for p in pws) * flop
                                              / (statistics.median(res[name]) * 1e12) * 1e3, 3)
        print(json.dumps({"shape": spec, "summary": summ}), flush=True)
        del A, B, C, Cb


if __name__ == "__main__":
    main()
