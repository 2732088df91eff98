"""Loader for the tools-only GEMM experiment library (``_native/libamdgo_gemm_lab.so``).

Build it with ``python -m gpu_operator_amd._build --lab``. It holds every superseded bf16/fp8 GEMM
generation, placement sweep and knock-out timing (native/hip/gemm_bf16_lab.hip, gemm_fp8_lab.hip)
under its historical variant number, for A/B sweeps and rocprofv3 runs. The validator never loads
it: the shipped ``libamdgo_hip.so`` dispatches only the production set.
"""

from __future__ import annotations

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

LAB_PATH = os.path.join(ROOT, "gpu_operator_amd", "_native", "libamdgo_gemm_lab.so")
KNOCKOUT_BF16 = range(20, 25)       # timings with deliberately wrong results
_LIB = None


def load() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LAB_PATH):
            raise FileNotFoundError(f"{LAB_PATH}: build it with `python -m gpu_operator_amd._build --lab`")
        lib = ctypes.CDLL(LAB_PATH)
        vp, i = ctypes.c_void_p, ctypes.c_int
        for f in ("amdgo_lab_gemm_bf16", "amdgo_lab_gemm_fp8"):
            getattr(lib, f).argtypes = [i, vp, vp, vp, i, i, i, vp]
            getattr(lib, f).restype = i
        _LIB = lib
    return _LIB


def _run(fn, v, a, bt, c):
    import torch

    m, k = a.shape
    n = bt.shape[0]
    err = fn(int(v), a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k,
             torch.cuda.current_stream(a.device).cuda_stream)
    if err:
        raise RuntimeError(f"lab variant {v} failed for {m}x{n}x{k}: hipError {err}")
    return c


def gemm_bf16(v: int, a, bt, c):
    return _run(load().amdgo_lab_gemm_bf16, v, a, bt, c)


def gemm_fp8(v: int, a, bt, c):
    return _run(load().amdgo_lab_gemm_fp8, v, a, bt, c)
