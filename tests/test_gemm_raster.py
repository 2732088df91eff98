"""The host mirror of the GEMM dispatch's rasters (native/hip/gemm_raster_host.h), CPU only.

amd-gemm-validate names the workgroup behind a bad output tile from this mirror, so it must be a
bijection between (tile, K piece) and the launch's (workgroup, round) slots for every kernel the
dispatch can pick, and it must agree with the launch grid the dispatch uses."""

import itertools
import os

import pytest

from gpu_operator_amd.ops import _lib

# no load at import: collection must not load the HIP library (ops/_lib.py: torch's runtime first)
pytestmark = pytest.mark.skipif(not _lib.lib_path().exists(), reason="libamdgo_hip.so not built")

SHAPES = [
    (8192, 8192, 8192), (16384, 16384, 16384), (4096, 4096, 4096), (2560, 2560, 2560), (1024, 1024, 4096),
    (1024, 1024, 16384), (512, 512, 8192), (2048, 2048, 8192), (12288, 12288, 12288), (8192, 8192, 2048),
    (4096, 4096, 32768), (16384, 16384, 1024), (1000, 1000, 1000), (768, 512, 1024), (4096, 8192, 12288),
    (2816, 2816, 2816), (1536, 1536, 1536), (256, 256, 256), (3000, 200, 4096),
    (2560, 2560, 8192), (2560, 2560, 16384), (2048, 4096, 8192),     # v57 / fp8 v24: split-K asm frame
]


def _check_bijection(r):
    slots = set()
    for tm, tn, p in itertools.product(range(r.tiles_m), range(r.tiles_n), range(r.pieces)):
        b, rnd = r.owner[tm][tn][p], r.round[tm][tn][p]
        assert 0 <= b < r.grid, (r.variant, tm, tn, p, b, r.grid)
        assert rnd >= 0
        assert (b, rnd) not in slots, (r.variant, tm, tn, p, b, rnd)   # one tile per workgroup round
        slots.add((b, rnd))
    return slots


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_raster_is_a_bijection(dtype, shape):
    from gpu_operator_amd.ops import gemm as G

    m, n, k = shape
    r = G.raster(m, n, k, dtype, cus=256)
    slots = _check_bijection(r)
    assert len(slots) == r.tiles_m * r.tiles_n * r.pieces
    assert r.tile_n in (64, 128, 256, 512)            # the ABFT strip widths gemm_abft.hip supports
    if r.kind in ("generic", "grid", "grid_sq", "small", "split"):
        assert {b for b, _ in slots} == set(range(r.grid))          # every workgroup owns exactly one item
        assert all(rnd == 0 for _, rnd in slots)
    if r.kind == "persistent":
        # whole XCD groups; a workgroup's tiles all come from its XCD's contiguous run: the rounds of one
        # workgroup are consecutive and start at 0
        assert r.grid % 8 == 0
        per_wg = {}
        for b, rnd in slots:
            per_wg.setdefault(b, []).append(rnd)
        for rounds in per_wg.values():
            assert sorted(rounds) == list(range(len(rounds)))


@pytest.mark.parametrize("shape", [(2560, 2560, 2560), (2048, 2048, 8192), (1024, 1024, 4096), (512, 512, 8192),
                                   (2560, 2560, 8192), (4096, 4096, 4096), (1024, 1024, 1024)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("tile_major", [False, True])
def test_split_k_asm_raster_pinned(shape, tile_major):
    """v57 pinned: a bijection of (tile, piece) onto the grid; piece-major, each XCD's run of workgroups
    covers neighbouring tiles at one K range; tile-major, a tile's pieces are adjacent workgroups of one
    XCD. Shapes it cannot split fall back to v55."""
    from gpu_operator_amd.ops import gemm as G

    m, n, k = shape
    old = G.get_variant()
    G.set_variant(57)
    G.set_asm_split(0, 0, piece_major=not tile_major)
    try:
        r = G.raster(m, n, k, "bf16", cus=256)
    finally:
        G.set_asm_split()
        G.set_variant(old)
    tiles = (m // 256) * (n // 256)
    splits = min(256 // tiles, (k // 64) // 16, 2 if 4 * tiles > 256 else 4)
    if splits < 2:
        assert r.variant == 55 and r.kind == "persistent"
        return
    assert (r.variant, r.kind, r.pieces, r.grid) == (57, "split", splits, tiles * splits)
    slots = _check_bijection(r)
    assert {b for b, _ in slots} == set(range(r.grid))
    if tile_major:
        # every tile's pieces on one XCD (b % 8) whenever the XCD's run holds whole tiles
        if (tiles * splits) % 8 == 0 and ((tiles * splits) // 8) % splits == 0:
            for tm, tn in itertools.product(range(r.tiles_m), range(r.tiles_n)):
                assert len({b % 8 for b in r.owner[tm][tn]}) == 1
        return
    # the workgroups of one XCD (b % 8) hold one piece except where the piece-major order wraps
    pieces_of_xcd = {}
    for tm, tn, p in itertools.product(range(r.tiles_m), range(r.tiles_n), range(r.pieces)):
        pieces_of_xcd.setdefault(r.owner[tm][tn][p] % 8, set()).add(p)
    assert all(len(ps) <= 2 for ps in pieces_of_xcd.values())


def test_raster_kinds_follow_the_dispatch():
    from gpu_operator_amd.ops import gemm as G

    lib = _lib.load()
    for dtype, plan in (("bf16", lib.amdgo_gemm_plan_bf16), ("fp8", lib.amdgo_gemm_plan_fp8)):
        for m, n, k in SHAPES:
            r = G.raster(m, n, k, dtype, cus=256)
            assert r.variant == plan(m, n, k, 256, 0), (dtype, m, n, k)
            want = {60: "small", 61: "small", 62: "small", 0: "generic", 57: "split", 24: "split"}.get(r.variant)
            if want:
                assert r.kind == want, (dtype, m, n, k, r.variant, r.kind)
            if r.variant == 61:
                assert r.pieces == G.small_splits(m, n, k, 256) or dtype == "fp8"
    # the headline shape: v50 on 256 persistent workgroups, 4 rounds of 256x256 tiles
    r = G.raster(8192, 8192, 8192, "bf16", cus=256)
    assert (r.variant, r.kind, r.grid, r.tile_m, r.tiles_m) == (50, "persistent", 256, 256, 32)
    assert max(x[0] for row in r.round for x in row) == 3
    # a CPX partition (32 CUs) gets its own raster: a persistent grid of 32
    r = G.raster(8192, 8192, 8192, "bf16", cus=32)
    assert r.grid in (0, 32) or r.kind != "persistent"


def test_library_binds_to_torchs_hip_runtime_whatever_the_import_order():
    """Loaded before torch, libamdgo_hip.so pulled in /opt/rocm's libamdhip64 and torch then ran on a
    runtime it was not built with: every HIP call of that GPU test session failed with hipErrorNoDevice.
    _lib.load() imports torch first, so one runtime is mapped -- torch's."""
    import subprocess
    import sys
    code = ("from gpu_operator_amd.ops import _lib\n_lib.load()\n"
            "maps = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}\n"
            "import torch, os\nprint(len(maps), all(m.startswith(os.path.dirname(torch.__file__)) for m in maps))\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["1", "True"]
