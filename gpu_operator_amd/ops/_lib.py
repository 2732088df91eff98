"""Loader for the in-tree HIP shared library (``_native/libamdgo_hip.so``).

The library is built by :mod:`gpu_operator_amd._build` for gfx950. On a machine with a GPU the
ops refuse to fall back silently: if the library is missing they raise, so a GPU test can
never pass on an eager PyTorch path by accident.
"""

from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Optional

_NATIVE = Path(__file__).resolve().parent.parent / "_native"
_LOCK = threading.Lock()
_LIB: Optional[ctypes.CDLL] = None


class NativeLibraryMissing(RuntimeError):
    """Raised when the HIP library has not been built (run ``python -m gpu_operator_amd._build``)."""


def lib_path() -> Path:
    return Path(os.environ.get("AMDGO_HIP_LIB", str(_NATIVE / "libamdgo_hip.so")))


def load() -> ctypes.CDLL:
    global _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        p = lib_path()
        if not p.exists():
            raise NativeLibraryMissing(
                f"{p} not found: build it with `python -m gpu_operator_amd._build` (hipcc, gfx950)")
        # torch first: it ships its own libamdhip64. Loaded before it, this library would pull in
        # /opt/rocm's copy, torch would then run on a runtime it was not built with, and every HIP
        # call of the process failed with hipErrorNoDevice (a GPU test session whose collection
        # loaded this library first: 437 failures). With torch loaded, the dependency resolves to its
        # runtime, the one the tensors passed here live in.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(str(p))
        vp, i, sz, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint32
        lib.amdgo_gemm_bf16.argtypes = [vp, vp, vp, i, i, i, vp]
        lib.amdgo_gemm_bf16.restype = i
        lib.amdgo_gemm_bf16_generic.argtypes = [vp, vp, vp, i, i, i, vp]
        lib.amdgo_gemm_bf16_generic.restype = i
        lib.amdgo_gemm_ref_rows.argtypes = [vp, vp, vp, i, vp, i, i, vp]
        lib.amdgo_gemm_ref_rows.restype = i
        lib.amdgo_fill_uniform_bf16.argtypes = [vp, sz, u32, vp]
        lib.amdgo_fill_uniform_bf16.restype = i
        lib.amdgo_vector_add_f32.argtypes = [vp, vp, vp, sz, vp]
        lib.amdgo_vector_add_f32.restype = i
        lib.amdgo_gemm_fp8.argtypes = [vp, vp, vp, i, i, i, vp]
        lib.amdgo_gemm_fp8.restype = i
        lib.amdgo_gemm_fp8_generic.argtypes = [vp, vp, vp, i, i, i, vp]
        lib.amdgo_gemm_fp8_generic.restype = i
        lib.amdgo_gemm_fp8_ref_rows.argtypes = [vp, vp, vp, i, vp, i, i, vp]
        lib.amdgo_gemm_fp8_ref_rows.restype = i
        lib.amdgo_fill_uniform_fp8.argtypes = [vp, sz, u32, vp]
        lib.amdgo_fill_uniform_fp8.restype = i
        for f in ("amdgo_gemm_set_variant", "amdgo_gemm_fp8_set_variant"):
            getattr(lib, f).argtypes = [i]
            getattr(lib, f).restype = i
        for f in ("amdgo_gemm_resolve_variant", "amdgo_gemm_fp8_resolve_variant"):
            getattr(lib, f).argtypes = [i, i, i]
            getattr(lib, f).restype = i
        lib.amdgo_gemm_fp8_get_variant.restype = i
        lib.amdgo_gemm_get_variant.restype = i
        ip = ctypes.POINTER(ctypes.c_int)
        for f in ("amdgo_gemm_bf16_raster", "amdgo_gemm_fp8_raster"):
            getattr(lib, f).argtypes = [i, i, i, ip, ip, ip, i]
            getattr(lib, f).restype = i
        for f in ("amdgo_gemm_bf16_raster_for", "amdgo_gemm_fp8_raster_for"):
            getattr(lib, f).argtypes = [i, i, i, i, ip, ip, ip, i]
            getattr(lib, f).restype = i
        for f in ("amdgo_gemm_bf16_placed", "amdgo_gemm_fp8_placed"):
            getattr(lib, f).argtypes = [vp, vp, vp, i, i, i, vp, vp]
            getattr(lib, f).restype = i
        lib.amdgo_abft_workspace_bytes.argtypes = [i, i, i, i, i]
        lib.amdgo_abft_workspace_bytes.restype = ctypes.c_longlong
        lib.amdgo_abft_check.argtypes = [i, vp, vp, vp, i, i, i, i, i, vp, ctypes.c_longlong, ip,
                                         ctypes.POINTER(ctypes.c_float), vp]
        lib.amdgo_abft_check.restype = i
        lib.amdgo_abft_inject.argtypes = [vp, i, i, i, i, ctypes.c_float, vp]
        lib.amdgo_abft_inject.restype = i
        lib.amdgo_gemm_small_workspace_count.argtypes = [i]
        lib.amdgo_gemm_small_workspace_count.restype = i
        for f in ("amdgo_gemm_tile_m", "amdgo_gemm_tile_n", "amdgo_gemm_tile_k",
                  "amdgo_gemm_fp8_tile_m", "amdgo_gemm_fp8_tile_n", "amdgo_gemm_fp8_tile_k"):
            getattr(lib, f).restype = i
        _LIB = lib
        return lib


def check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"{what} failed with hipError {err}")
