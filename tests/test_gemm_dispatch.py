"""The GEMM dispatch tables (native/hip/gemm_bf16.hip kBf16Rules / kBf16Needs, gemm_fp8.hip
kFp8Rules / kFp8Needs) against the round-4 rule code they replaced, transcribed below: the same kernel
for every shape class, device size and pinned variant -- except where a new row (v60, the 128x128
kernel for small grids) was added on purpose. Pure functions of (M, N, K, CUs, pinned): no GPU."""

import itertools

import pytest

from gpu_operator_amd.ops import _lib

BM = BN = 256
BK = 64


def _r4_bf16(M, N, K, cus, g):
    """round 4's resolve_variant (gemm_bf16.hip at 5af2094), line for line."""
    if M % BM or N % BN or K % BK or K < 2 * BK:
        return 0
    nwg = (M // BM) * (N // BN)
    sq = (M // BM) % 16 == 0 and (N // BN) % 16 == 0

    def pg(n):
        return (min(n, cus) // 8) * 8
    v = g
    pow2k = (K & (K - 1)) == 0
    if v == 0 and cus == 256 and not pow2k and K % (2 * BK) == 0 and K >= 4 * BK and pg(nwg) >= 8:
        v = 54 if (sq and nwg >= 8 * cus) else 53
    elif v == 0 and cus == 256 and pow2k and K >= 4 * BK and pg(nwg) >= 8:
        v = 50
        if sq and nwg >= 8 * cus and K >= 128 * BK:
            v = 51
        elif nwg <= 2 * cus and K >= 512 * BK:
            v = 52
        elif sq and (K <= 32 * BK or nwg <= cus):
            v = 56
        elif nwg <= cus:
            v = 55
    elif v == 0:
        v = 44
        if K <= 64 * BK and nwg >= 2 * cus:
            v = 25
        elif sq and nwg >= 8 * cus and K >= 128 * BK:
            v = 45
    if v == 45 and not sq:
        v = 44
    if v == 48 and not sq:
        v = 47
    if v in (47, 48) and cus != 256:
        v = 42
    if v == 25 and pg(nwg) < 8:
        v = 44
    if v in (50, 51, 52, 53, 54, 55, 56) and (K % (2 * BK) != 0 or K < 4 * BK or pg(nwg) < 8):
        v = 44
    if v == 54 and (not sq or cus != 256):
        v = 53
    if v == 56 and (not sq or cus != 256):
        v = 55
    if v == 51 and (not sq or cus != 256):
        v = 50
    if v in (44, 45) and cus != 256:
        v = 42
    if g == 0 and not pow2k:
        if v == 44:
            v = 47
        elif v == 45:
            v = 48
    return v


def _splits(tiles, nk, cus, target=1):
    """v61's K pieces per tile (gemm_small_host.h small_splits): target x CUs / tiles, >= 16 K-tiles
    a piece, pieces of 16 only within half the chip, 1 = none."""
    s = min(target * cus // tiles, nk // 16)
    if s > 1 and nk // s <= 16:                 # 16-K-tile pieces only within half the chip
        s = min(s, target * cus // 2 // tiles)
    return max(1, s)


def _small(M, N, K, cus):
    """The round-5 rows: 128x128 tiles when the 256x256 grid fills at most a quarter of the CUs -- v61
    (split-K) when the 128x128 grid leaves pieces to give, else v60. None when neither applies."""
    tiles256 = M % BM == 0 and N % BN == 0 and K % BK == 0 and K >= 2 * BK
    tiles128 = M % 128 == 0 and N % 128 == 0 and K % 64 == 0 and K >= 64
    nwg = (M // BM) * (N // BN)
    if tiles256 and 4 * nwg > cus and 2 * nwg <= cus:
        if cus == 256 and K % 128 == 0 and K >= 4096:
            return 57                               # round 6: the asm frame in two K pieces
        return 62                                   # 256x128 tiles: one wave of the chip
    if tiles256 and 8 * nwg > cus and 4 * nwg <= cus and cus == 256 and K % 128 == 0 and K >= 16384:
        return 57                                   # round 6: the asm frame in up to four K pieces
    if not (tiles128 and (not tiles256 or 4 * nwg <= cus)):
        return None
    return 61 if _splits((M // 128) * (N // 128), K // 64, cus) > 1 else 60


DIMS = [128, 256, 384, 512, 1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384]
KS = [64, 128, 192, 256, 320, 512, 1024, 1536, 2048, 3072, 4096, 4160, 8192, 8256, 12288, 16384, 32768, 65536]
CUS = [256, 304, 80, 32, 4]
BF16_PINS = (0, 18, 25, 42, 44, 45, 47, 48, 50, 51, 52, 53, 54, 55, 56)   # 60, 61: tested below


@pytest.fixture(scope="module")
def lib():
    try:
        return _lib.load()
    except OSError as e:
        pytest.skip(f"libamdgo_hip.so not built: {e}")


def test_bf16_table_reproduces_the_round4_rules(lib):
    bad = []
    for M, N in itertools.product(DIMS, DIMS[::2]):
        for K, cus, pin in itertools.product(KS, CUS, BF16_PINS):
            got = lib.amdgo_gemm_plan_bf16(M, N, K, cus, pin)
            small = _small(M, N, K, cus) if pin == 0 else None
            want = small if small is not None else _r4_bf16(M, N, K, cus, pin)
            if got != want:
                bad.append((M, N, K, cus, pin, got, want))
    assert not bad, bad[:20]


def test_bf16_small_grid_row_and_its_evidence(lib):
    lib.amdgo_gemm_plan_bf16_evidence.restype = __import__("ctypes").c_char_p
    assert lib.amdgo_gemm_plan_bf16(1024, 1024, 1024, 256, 0) == 60
    assert lib.amdgo_gemm_plan_bf16(1152, 1152, 1024, 256, 0) == 60     # 128-tileable only
    assert lib.amdgo_gemm_plan_bf16(1000, 1000, 1000, 256, 0) == 0      # neither: the generic kernel
    assert lib.amdgo_gemm_plan_bf16(1024, 1024, 1024, 256, 60) == 60    # pinned
    assert lib.amdgo_gemm_plan_bf16(1000, 1024, 1024, 256, 60) == 0     # pinned, cannot run: generic
    assert lib.amdgo_gemm_plan_bf16(8192, 8192, 8192, 256, 0) == 50
    assert lib.amdgo_gemm_plan_bf16(1024, 1024, 8192, 256, 0) == 61     # split-K: 4 pieces of 32 K-tiles
    assert lib.amdgo_gemm_small_splits(1024, 1024, 8192, 256) == 4
    assert lib.amdgo_gemm_small_splits(1024, 1024, 1024, 256) == 1      # 16 K-tiles: no split
    assert lib.amdgo_gemm_plan_bf16(2560, 2560, 2560, 256, 0) == 62     # 100 256x256 tiles: 200 of 256x128
    ev = lib.amdgo_gemm_plan_bf16_evidence(1024, 1024, 1024, 256).decode()
    assert ev.startswith("profiles/r5_small/")
    assert lib.amdgo_gemm_plan_bf16_evidence(16384, 16384, 1024, 256).decode().startswith("profiles/r4_lean/")


def _r4_fp8(M, N, K, cus, g):
    """round 4's resolve_fp8_variant (gemm_fp8.hip at 5af2094), line for line."""
    if M % 256 or N % 256 or K % 128 or K < 256:
        return 0
    nwg = (M // 256) * (N // 256)
    pgrid = (min(nwg, cus) // 8) * 8
    sq = (M // 256) % 16 == 0 and (N // 256) % 16 == 0
    v = g
    ap_ok = cus == 256 and K % 256 == 0 and K >= 512 and pgrid >= 8
    if v == 0 and ap_ok:
        wide = M // 256 >= 32 and N // 256 >= 32
        if nwg <= cus:
            v = 22 if sq else 23
        elif sq and nwg >= 2 * cus:
            v = 22 if (wide or K >= 4096) else 21
        else:
            v = 20
    elif v == 0:
        v = 16 if sq else 15
        if K <= 12 * 128 and nwg >= 2 * cus:
            v = 10
        elif K <= 64 * 128 and nwg >= 4 * cus:
            v = 18
    if v in (20, 21, 22, 23) and not ap_ok:
        v = 16 if sq else 15
    if v in (21, 22) and not sq:
        v = 23 if v == 22 else 20
    if v == 16 and not sq:
        v = 15
    if v in (10, 18) and pgrid < 8:
        v = 15
    if v in (15, 16) and cus != 256:
        v = 17
    return v


FP8_PINS = (0, 10, 15, 16, 17, 18, 20, 21, 22, 23, 60, 61, 62)
FP8_KS = [128, 256, 384, 512, 640, 1024, 1536, 1664, 2048, 4096, 8192, 8320, 16384, 32768]


def _small_fp8(M, N, K, cus, pin):
    """The round-5 fp8 rows (the bf16 rule on 128-byte K-tiles of fp8) and the pins 60 / 61; None
    where round 4's rules apply unchanged."""
    tiles256 = M % 256 == 0 and N % 256 == 0 and K % 128 == 0 and K >= 256
    tiles128 = M % 128 == 0 and N % 128 == 0 and K % 128 == 0 and K >= 128
    if pin in (60, 61):
        return pin if tiles128 else 0
    if pin == 62:
        return 62 if tiles128 and M % 256 == 0 else 0
    nwg = (M // 256) * (N // 256)
    pgrid = (min(nwg, cus) // 8) * 8
    if (pin == 0 and tiles256 and 8 * nwg > cus and 4 * nwg <= cus and cus == 256 and K % 256 == 0 and K >= 32768
            and pgrid >= 8):
        return 24                                   # round 6: the asm frame in four K pieces
    if pin == 0 and tiles128 and (not tiles256 or 4 * nwg <= cus):
        return 61 if _splits((M // 128) * (N // 128), K // 128, cus) > 1 else 60
    if pin == 0 and tiles256 and 4 * nwg > cus and 2 * nwg <= cus:
        pgrid = (min(nwg, cus) // 8) * 8
        if cus == 256 and K % 256 == 0 and K >= 8192 and pgrid >= 8:
            return 24                               # round 6: the asm frame in two K pieces
        return 62
    return None


def test_fp8_table_reproduces_the_round4_rules(lib):
    bad = []
    for M, N in itertools.product(DIMS, DIMS[::2]):
        for K, cus, pin in itertools.product(FP8_KS, CUS, FP8_PINS):
            got = lib.amdgo_gemm_plan_fp8(M, N, K, cus, pin)
            small = _small_fp8(M, N, K, cus, pin)
            want = small if small is not None else _r4_fp8(M, N, K, cus, pin)
            if got != want:
                bad.append((M, N, K, cus, pin, got, want))
    assert not bad, bad[:20]


def test_the_pinned_variant_is_per_thread(lib):
    """amdgo_gemm_set_variant pins for the calling host thread only (thread_local): a sweep driving
    8 GPUs from 8 threads never sees another thread's pin."""
    import threading
    seen = {}

    def pin(v):
        lib.amdgo_gemm_set_variant(v)
        seen[v] = lib.amdgo_gemm_get_variant()
    ts = [threading.Thread(target=pin, args=(v,)) for v in (44, 56, 60)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert seen == {44: 44, 56: 56, 60: 60} and lib.amdgo_gemm_get_variant() == 0
    lib.amdgo_gemm_fp8_set_variant(22)
    got = []
    t = threading.Thread(target=lambda: got.append(lib.amdgo_gemm_fp8_get_variant()))
    t.start()
    t.join()
    assert got == [0] and lib.amdgo_gemm_fp8_get_variant() == 22
    lib.amdgo_gemm_fp8_set_variant(0)


def test_persistent_launch_grid_rounds_up_to_whole_xcd_groups(lib):
    """A grid of fewer tiles than CUs gets every tile in the first round: 100 tiles -> 104 workgroups
    (13 per XCD; rounding down to 96 had run 4 tiles in a second round at half the throughput)."""
    g = lib.amdgo_gemm_persistent_launch_grid
    assert g(100, 256) == 104 and g(81, 256) == 88 and g(64, 256) == 64 and g(1, 256) == 8
    assert g(256, 256) == 256 and g(1024, 256) == 256          # one workgroup per CU
    assert g(300, 304) == 304 and g(303, 304) == 304            # 304 CUs: 38 per XCD
    for nwg in range(1, 600):
        for cus in (80, 256, 304):
            n = g(nwg, cus)
            assert n % 8 == 0 and n <= cus
            if nwg <= (cus // 8) * 8:
                assert n // 8 >= -(-nwg // 8)           # workgroups per XCD >= its tiles: one round


def _asm_splits(tiles, nk, cus):
    """gemm_small_host.h asm_splits: the split-K asm form's pieces per 256x256 tile (>= 16 K-tiles)."""
    return max(1, min(cus // tiles, nk // 16, 2 if 4 * tiles > cus else 4)) if tiles else 1


def test_split_k_asm_pins_run_where_they_can_and_fall_back_otherwise(lib):
    """bf16 v57 / fp8 v24 (the asm frame's split-K form) pinned: they run on 256x256-tileable shapes
    with an even K-tile count and >= 2 pieces of >= 16 K-tiles within the CUs; otherwise they fall
    back to the one-wave asm kernels (v55 / v23) and on from there."""
    bad = []
    for M, N in itertools.product(DIMS, DIMS[::2]):
        for K, cus in itertools.product(KS, CUS):
            nwg = (M // 256) * (N // 256)
            tiles = M % 256 == 0 and N % 256 == 0 and K % 64 == 0 and K >= 128
            ok = tiles and K % 128 == 0 and _asm_splits(nwg, K // 64, cus) > 1
            got = lib.amdgo_gemm_plan_bf16(M, N, K, cus, 57)
            want = 57 if ok else lib.amdgo_gemm_plan_bf16(M, N, K, cus, 55)
            if got != want:
                bad.append(("bf16", M, N, K, cus, got, want))
        for K, cus in itertools.product(FP8_KS, CUS):
            nwg = (M // 256) * (N // 256)
            tiles = M % 256 == 0 and N % 256 == 0 and K % 128 == 0 and K >= 256
            pgrid = (min(nwg, cus) // 8) * 8
            ap = cus == 256 and K % 256 == 0 and K >= 512 and pgrid >= 8
            ok = tiles and ap and _asm_splits(nwg, K // 128, cus) > 1
            got = lib.amdgo_gemm_plan_fp8(M, N, K, cus, 24)
            want = 24 if ok else lib.amdgo_gemm_plan_fp8(M, N, K, cus, 23)
            if got != want:
                bad.append(("fp8", M, N, K, cus, got, want))
    assert not bad, bad[:20]
