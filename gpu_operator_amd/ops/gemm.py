"""Validator GEMMs: hand-written CDNA4 MFMA kernels.

``C[M,N] = A[M,K] @ Bt[N,K].T`` with fp32 accumulation and bf16 output, both operands K-major
(the layout the MFMA fragments read without a transpose):

* bf16 operands: ``native/hip/gemm_bf16.hip`` (``gemm_bf16``);
* fp8 OCP e4m3fn operands: ``native/hip/gemm_fp8.hip`` (``gemm_fp8``), the unscaled double-rate
  ``v_mfma_f32_16x16x128_f8f6f4`` (the block-scaled 32x32x64 form for short K), i.e. the matrix
  cores' fp8 rate;
* small grids, both dtypes: ``native/hip/gemm_small.h`` (variants 60 / 61 / 62: 128x128 tiles,
  their split-K form, 256x128 tiles).

Replaces the reference validator's ``vectorAdd`` pass/fail probe
(reference: validator/cuda-workload-validation.yaml:20) with a matrix-core
throughput probe whose result feeds ``amd_gpu_operator_validator_gemm_tflops``.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from . import _lib


def _stream_ptr(torch, device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _check_operand(t, name: str, rows: int, k: int, dtype=None) -> None:
    import torch

    dtype = dtype or torch.bfloat16
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if tuple(t.shape) != (rows, k) or not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous [{rows},{k}], got {tuple(t.shape)}")


def gemm_bf16(a, bt, out=None, *, generic: bool = False):
    """Compute ``a @ bt.T`` on the MFMA kernel. ``a``: [M,K], ``bt``: [N,K] (bf16, contiguous)."""
    import torch

    m, k = a.shape
    n = bt.shape[0]
    _check_operand(a, "a", m, k)
    _check_operand(bt, "bt", n, k)
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out", m, n)
    lib = _lib.load()
    fn = lib.amdgo_gemm_bf16_generic if generic else lib.amdgo_gemm_bf16
    err = fn(a.data_ptr(), bt.data_ptr(), out.data_ptr(), m, n, k, _stream_ptr(torch, a.device))
    _lib.check(err, "amdgo_gemm_bf16")
    return out


def gemm_fp8(a, bt, out=None, *, generic: bool = False):
    """Compute ``a @ bt.T`` with fp8 (``torch.float8_e4m3fn``) operands: [M,K] and [N,K], bf16 out."""
    import torch

    m, k = a.shape
    n = bt.shape[0]
    f8 = torch.float8_e4m3fn
    _check_operand(a, "a", m, k, f8)
    _check_operand(bt, "bt", n, k, f8)
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out", m, n)
    lib = _lib.load()
    fn = lib.amdgo_gemm_fp8_generic if generic else lib.amdgo_gemm_fp8
    err = fn(a.data_ptr(), bt.data_ptr(), out.data_ptr(), m, n, k, _stream_ptr(torch, a.device))
    _lib.check(err, "amdgo_gemm_fp8")
    return out


# Production variant sets (native/hip/gemm_bf16.hip, gemm_fp8.hip): 0 = automatic dispatch, any
# other member pins that kernel. Everything else lives in the tools-only lab library.
BF16_VARIANTS = (0, 18, 25, 42, 44, 45, 47, 48, 50, 51, 52, 53, 54, 55, 56, 57, 60, 61, 62)
FP8_VARIANTS = (0, 10, 15, 16, 17, 18, 20, 21, 22, 23, 24, 60, 61, 62)


def set_variant(v: int) -> None:
    """Pin a production bf16 kernel (see ``BF16_VARIANTS``; 0 restores automatic dispatch)."""
    if _lib.load().amdgo_gemm_set_variant(int(v)) != 0:
        raise ValueError(f"bf16 GEMM variant {v} is not in the production set {BF16_VARIANTS}")


def get_variant() -> int:
    return _lib.load().amdgo_gemm_get_variant()


def set_split_target(t: int) -> None:
    """v61 (split-K 128x128): aim for ``t`` workgroups per CU (1..8; per host thread)."""
    if _lib.load().amdgo_gemm_set_split_target(int(t)) != 0:
        raise ValueError(f"split target {t} outside 1..8")


def set_asm_split(splits: int = 0, last_permille: int = 0, piece_major: bool = False) -> None:
    """v57 / fp8 v24 (split-K in the 256x256 asm frame), per host thread: force ``splits`` K pieces per
    tile (0 = automatic), give the last piece ``last_permille`` of K (0 = the default 52 %, 500 = even),
    and order the items piece-major instead of tile-major (a tile's pieces on one XCD, the default)."""
    if _lib.load().amdgo_gemm_set_asm_split(int(splits), int(last_permille), int(bool(piece_major))) != 0:
        raise ValueError(f"asm split ({splits}, {last_permille}) outside 0..64 / 0..999")


def small_splits(m: int, n: int, k: int, cus: int = 256) -> int:
    """The K pieces per tile v61 uses for this bf16 shape on a device with ``cus`` CUs (1: none)."""
    return _lib.load().amdgo_gemm_small_splits(int(m), int(n), int(k), int(cus))


def resolve_variant(m: int, n: int, k: int) -> int:
    """The bf16 kernel ``gemm_bf16`` runs for this shape on the current device (0 = generic)."""
    return _lib.load().amdgo_gemm_resolve_variant(int(m), int(n), int(k))


def set_fp8_variant(v: int) -> None:
    """Pin a production fp8 kernel (see ``FP8_VARIANTS``; 0 restores automatic dispatch)."""
    if _lib.load().amdgo_gemm_fp8_set_variant(int(v)) != 0:
        raise ValueError(f"fp8 GEMM variant {v} is not in the production set {FP8_VARIANTS}")


def get_fp8_variant() -> int:
    return _lib.load().amdgo_gemm_fp8_get_variant()


def resolve_fp8_variant(m: int, n: int, k: int) -> int:
    return _lib.load().amdgo_gemm_fp8_resolve_variant(int(m), int(n), int(k))


def fp8_fast_path_supported(m: int, n: int, k: int) -> bool:
    lib = _lib.load()
    tk = lib.amdgo_gemm_fp8_tile_k()
    return m % lib.amdgo_gemm_fp8_tile_m() == 0 and n % lib.amdgo_gemm_fp8_tile_n() == 0 \
        and k % tk == 0 and k >= 2 * tk


def fast_path_supported(m: int, n: int, k: int) -> bool:
    lib = _lib.load()
    tk = lib.amdgo_gemm_tile_k()
    return m % lib.amdgo_gemm_tile_m() == 0 and n % lib.amdgo_gemm_tile_n() == 0 \
        and k % tk == 0 and k >= 2 * tk


def fill_uniform_(t, seed: int = 1234):
    """Fill a bf16 GPU tensor with deterministic uniform [-1, 1) values (native kernel)."""
    import torch

    if t.dtype != torch.bfloat16 or not t.is_cuda or not t.is_contiguous():
        raise ValueError("fill_uniform_ needs a contiguous bf16 GPU tensor")
    lib = _lib.load()
    _lib.check(lib.amdgo_fill_uniform_bf16(t.data_ptr(), t.numel(), seed & 0xFFFFFFFF,
                                           _stream_ptr(torch, t.device)), "fill_uniform")
    return t


def fill_uniform_fp8_(t, seed: int = 1234):
    """Fill an e4m3fn GPU tensor with uniform [-1, 1) values rounded by the hardware converter."""
    import torch

    if t.dtype != torch.float8_e4m3fn or not t.is_cuda or not t.is_contiguous():
        raise ValueError("fill_uniform_fp8_ needs a contiguous float8_e4m3fn GPU tensor")
    lib = _lib.load()
    _lib.check(lib.amdgo_fill_uniform_fp8(t.data_ptr(), t.numel(), seed & 0xFFFFFFFF,
                                          _stream_ptr(torch, t.device)), "fill_uniform_fp8")
    return t


def reference_rows(a, bt, rows):
    """fp32 reference of selected output rows, computed by an independent scalar HIP kernel
    (software e4m3 decode for fp8 operands)."""
    import torch

    rows_t = torch.as_tensor(rows, dtype=torch.int32, device=a.device).contiguous()
    n, k = bt.shape
    out = torch.empty((rows_t.numel(), n), dtype=torch.float32, device=a.device)
    lib = _lib.load()
    fn = lib.amdgo_gemm_fp8_ref_rows if a.dtype == torch.float8_e4m3fn else lib.amdgo_gemm_ref_rows
    _lib.check(fn(a.data_ptr(), bt.data_ptr(), rows_t.data_ptr(), rows_t.numel(), out.data_ptr(), n, k,
                  _stream_ptr(torch, a.device)), "gemm_ref_rows")
    return out


@dataclass
class GemmCheck:
    max_abs_err: float
    max_rel_err: float
    tol: float
    ok: bool


def verify(a, bt, c, nrows: int = 64, seed: int = 0, rows: Optional[list] = None) -> GemmCheck:
    """Compare sampled output rows of ``c`` with an fp32 reference (tolerance for bf16 output)."""
    import torch

    m, k = a.shape
    g = torch.Generator().manual_seed(seed)
    if rows is None:
        rows = torch.randint(0, m, (min(nrows, m),), generator=g).tolist()
    ref = reference_rows(a, bt, rows)
    got = c[torch.as_tensor(rows, device=c.device)].float()
    err = (got - ref).abs()
    scale = ref.abs().clamp_min(1.0)
    # bf16 output rounding (2^-8 relative) + fp32 accumulation-order differences.
    tol = 1.0 / 128
    max_rel = float((err / scale).max())
    return GemmCheck(float(err.max()), max_rel, tol, max_rel <= tol)


# ---------------------------------------------------------------------------------------------
# The dispatch's raster and the ABFT check (native/hip/gemm_raster_host.h, gemm_abft.hip)
# ---------------------------------------------------------------------------------------------
RASTER_KINDS = ("generic", "grid", "grid_sq", "persistent", "persistent_sq", "small", "split")


@dataclass
class Raster:
    """Which workgroup of a launch computes which output tile: ``owner[tm][tn][piece]`` is the linear
    block id, ``round`` the iteration of its tile loop (persistent grids)."""
    variant: int
    kind: str
    tile_m: int
    tile_n: int
    tiles_m: int
    tiles_n: int
    grid: int
    pieces: int
    owner: list
    round: list


def raster(m: int, n: int, k: int, dtype: str = "bf16", cus: Optional[int] = None) -> Raster:
    """The raster of the kernel the dispatch picks for this shape -- on a device with ``cus`` CUs
    (no GPU needed), or on the current device."""
    import ctypes

    lib = _lib.load()
    info = (ctypes.c_int * 8)()
    ip = ctypes.POINTER(ctypes.c_int)
    fn_for = lib.amdgo_gemm_fp8_raster_for if dtype == "fp8" else lib.amdgo_gemm_bf16_raster_for
    fn_cur = lib.amdgo_gemm_fp8_raster if dtype == "fp8" else lib.amdgo_gemm_bf16_raster

    def call(owners, rounds, cap):
        if cus is None:
            return fn_cur(m, n, k, info, owners, rounds, cap)
        return fn_for(m, n, k, cus, info, owners, rounds, cap)

    call(ctypes.cast(None, ip), ctypes.cast(None, ip), 0)
    cap = info[4] * info[5] * info[7]
    owners, rounds = (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
    if call(owners, rounds, cap) < 0:
        raise RuntimeError("raster: capacity")
    tm, tn, p = info[4], info[5], info[7]
    own = [[[owners[(a * tn + b) * p + q] for q in range(p)] for b in range(tn)] for a in range(tm)]
    rnd = [[[rounds[(a * tn + b) * p + q] for q in range(p)] for b in range(tn)] for a in range(tm)]
    return Raster(info[0], RASTER_KINDS[info[1]], info[2], info[3], tm, tn, info[6], p, own, rnd)


def gemm_placed(a, bt, out, placement, fp8: bool = False):
    """One GEMM through the placement-recording kernels: workgroup b writes its HW_REG_XCC_ID and
    HW_REG_HW_ID to ``placement[2b]``, ``[2b+1]`` (an int32 GPU tensor with room for the raster's grid)."""
    import torch

    m, k = a.shape
    n = bt.shape[0]
    lib = _lib.load()
    fn = lib.amdgo_gemm_fp8_placed if fp8 else lib.amdgo_gemm_bf16_placed
    _lib.check(fn(a.data_ptr(), bt.data_ptr(), out.data_ptr(), m, n, k, placement.data_ptr(),
                  _stream_ptr(torch, a.device)), "gemm_placed")
    return out


@dataclass
class AbftResult:
    tile_flags: list         # [tiles_m][tiles_n]: bit 0 a row sum failed, bit 1 a column sum
    worst_ratio: float       # max |sum - expected| / tolerance (< 1 when clean)

    @property
    def bad_tiles(self) -> list:
        return [(i, j) for i, row in enumerate(self.tile_flags) for j, f in enumerate(row) if f]


def abft_check(a, bt, c, tile_m: int, tile_n: int) -> AbftResult:
    """The ABFT check of ``c == a @ bt.T`` in ``tile_m`` x ``tile_n`` tiles (native/hip/gemm_abft.hip):
    every element covered by one row and one column checksum, the failing tiles named."""
    import ctypes
    import torch

    m, k = a.shape
    n = bt.shape[0]
    lib = _lib.load()
    nbytes = lib.amdgo_abft_workspace_bytes(m, n, k, tile_m, tile_n)
    ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=a.device)
    tm, tn = -(-m // tile_m), -(-n // tile_n)
    flags = (ctypes.c_int * (tm * tn))()
    worst = ctypes.c_float(0.0)
    dt = 1 if a.dtype == torch.float8_e4m3fn else 0
    _lib.check(lib.amdgo_abft_check(dt, a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, tile_m, tile_n,
                                    ws.data_ptr(), nbytes, flags, ctypes.byref(worst),
                                    _stream_ptr(torch, a.device)), "abft_check")
    return AbftResult([[flags[i * tn + j] for j in range(tn)] for i in range(tm)], float(worst.value))


def abft_inject_(c, row: int, col: int, delta: float) -> None:
    """Test hook: ``c[row, col] += delta`` on the GPU, ordered on the current stream."""
    import torch

    m, n = c.shape
    _lib.check(_lib.load().amdgo_abft_inject(c.data_ptr(), m, n, row, col, float(delta),
                                             _stream_ptr(torch, c.device)), "abft_inject")


def small_workspace_count(device: int) -> int:
    """v61 split-K workspace sets the library holds for ``device`` (capped, LRU)."""
    return _lib.load().amdgo_gemm_small_workspace_count(int(device))


def tflops(m: int, n: int, k: int, seconds: float) -> float:
    return 2.0 * m * n * k / seconds / 1e12
