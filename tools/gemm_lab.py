"""Loader for the tools-only GEMM experiment libraries (``_native/libamdgo_gemm_lab_{bf16,fp8}.so``).

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

LAB_DIR = os.path.join(ROOT, "gpu_operator_amd", "_native")
KNOCKOUT_BF16 = tuple(range(20, 25))   # timings with deliberately wrong results
_LIBS = {}


def load(dtype: str = "bf16") -> ctypes.CDLL:
    if dtype not in _LIBS:
        path = os.path.join(LAB_DIR, f"libamdgo_gemm_lab_{dtype}.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path}: build it with `python -m gpu_operator_amd._build --lab`")
        lib = ctypes.CDLL(path)
        vp, i = ctypes.c_void_p, ctypes.c_int
        fn = getattr(lib, f"amdgo_lab_gemm_{dtype}")
        fn.argtypes = [i, vp, vp, vp, i, i, i, vp]
        fn.restype = i
        _LIBS[dtype] = lib
    return _LIBS[dtype]


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
    return _run(load("bf16").amdgo_lab_gemm_bf16, v, a, bt, c)


def gemm_fp8(v: int, a, bt, c):
    return _run(load("fp8").amdgo_lab_gemm_fp8, v, a, bt, c)
