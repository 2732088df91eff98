"""The ABFT check of the validator GEMM (native/hip/gemm_abft.hip), the placement record of the checked
dispatch and the tile naming of amd-gemm-validate, on a real MI355X.

Numerics: the check is compared with what it must accept -- our kernels' output and an independent
PyTorch fp32 product rounded to bf16 -- and with what it must reject: one element perturbed, one
element NaN, one tile left unwritten."""

import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "gpu_operator_amd", "_native", "bin")


def _operands(m, n, k, dtype, dev, seed=7):
    import torch
    from gpu_operator_amd.ops import gemm as G

    if dtype == "fp8":
        a = torch.empty((m, k), dtype=torch.float8_e4m3fn, device=dev)
        bt = torch.empty((n, k), dtype=torch.float8_e4m3fn, device=dev)
        G.fill_uniform_fp8_(a, seed)
        G.fill_uniform_fp8_(bt, seed + 1)
    else:
        a = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
        bt = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
        G.fill_uniform_(a, seed)
        G.fill_uniform_(bt, seed + 1)
    return a, bt


def _gemm(a, bt, dtype):
    from gpu_operator_amd.ops import gemm as G

    return G.gemm_fp8(a, bt) if dtype == "fp8" else G.gemm_bf16(a, bt)


CASES = [("bf16", (8192, 8192, 8192)), ("bf16", (1024, 1024, 4096)), ("bf16", (2560, 2560, 2560)),
         ("bf16", (1000, 768, 512)), ("fp8", (8192, 8192, 8192)), ("fp8", (1024, 1024, 16384)),
         ("fp8", (4096, 4096, 4096))]


@pytest.mark.parametrize("dtype,shape", CASES, ids=lambda x: x if isinstance(x, str) else "x".join(map(str, x)))
def test_abft_accepts_correct_products(cuda_device, dtype, shape):
    """Clean on our kernel's output and on an independent fp32 product rounded to bf16."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    m, n, k = shape
    a, bt = _operands(m, n, k, dtype, cuda_device)
    r = G.raster(m, n, k, dtype)
    c = _gemm(a, bt, dtype)
    res = G.abft_check(a, bt, c, r.tile_m, r.tile_n)
    assert not res.bad_tiles and res.worst_ratio < 1.0, (res.bad_tiles[:4], res.worst_ratio)
    if m * n * k <= 4096 ** 3:
        ref = (a.float() @ bt.float().t()).to(torch.bfloat16)
        res = G.abft_check(a, bt, ref, r.tile_m, r.tile_n)
        assert not res.bad_tiles and res.worst_ratio < 1.0, res.worst_ratio
    print(f"abft {dtype} {shape} v{r.variant} {r.tile_m}x{r.tile_n}: worst ratio {res.worst_ratio:.3f}")


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_abft_names_the_perturbed_tile_only(cuda_device, dtype):
    from gpu_operator_amd.ops import gemm as G

    m = n = k = 4096
    a, bt = _operands(m, n, k, dtype, cuda_device)
    r = G.raster(m, n, k, dtype)
    for (ti, tj), delta in (((3, 11), 64.0), ((0, 0), 16.0), ((r.tiles_m - 1, r.tiles_n - 1), float("nan")),
                            ((5, 2), -1e4)):
        c = _gemm(a, bt, dtype)
        G.abft_inject_(c, ti * r.tile_m + 17, tj * r.tile_n + r.tile_n - 3, delta)
        res = G.abft_check(a, bt, c, r.tile_m, r.tile_n)
        assert res.bad_tiles == [(ti, tj)], (delta, res.bad_tiles[:4])
        assert res.tile_flags[ti][tj] == 3        # its row sum and its column sum both failed


def test_abft_catches_an_unwritten_tile(cuda_device):
    import torch
    from gpu_operator_amd.ops import gemm as G

    m = n = k = 4096
    a, bt = _operands(m, n, k, "bf16", cuda_device)
    r = G.raster(m, n, k, "bf16")
    good = _gemm(a, bt, "bf16")
    c = good.clone()
    c[2 * r.tile_m:3 * r.tile_m, 9 * r.tile_n:10 * r.tile_n] = 0        # a tile a dead CU never stored
    assert G.abft_check(a, bt, c, r.tile_m, r.tile_n).bad_tiles == [(2, 9)]
    c = good.clone()
    c[7 * r.tile_m:8 * r.tile_m, 1 * r.tile_n:2 * r.tile_n] = \
        c[6 * r.tile_m:7 * r.tile_m, 1 * r.tile_n:2 * r.tile_n]           # a tile written with its neighbour's data
    assert G.abft_check(a, bt, c, r.tile_m, r.tile_n).bad_tiles == [(7, 1)]
    c = torch.full_like(good, float("nan"))                               # the poisoned buffer, no dispatch
    assert len(G.abft_check(a, bt, c, r.tile_m, r.tile_n).bad_tiles) == r.tiles_m * r.tiles_n


@pytest.mark.parametrize("variant", [50, 51, 52, 53, 54, 55, 56, 57, 25, 44, 45, 42, 18, 47, 48, 60, 61, 62, 0])
def test_placed_dispatch_is_bitwise_the_timed_one_bf16(cuda_device, variant):
    """Every production bf16 kernel's placement-recording instantiation computes bit-for-bit the timed
    kernel's C, and records one placement per workgroup of the raster's grid."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    m, n, k = {50: (8192, 8192, 4096), 51: (4096, 4096, 8192), 52: (2048, 2048, 32768), 53: (4096, 4096, 3072),
               54: (4096, 4096, 3072), 55: (2048, 2048, 2048), 56: (4096, 4096, 2048), 25: (4096, 4096, 1024),
               60: (1024, 1024, 1024), 61: (1024, 1024, 4096), 62: (2560, 2560, 2560), 0: (1000, 768, 512),
               57: (2560, 2560, 8192)}.get(variant, (4096, 4096, 4096))
    a, bt = _operands(m, n, k, "bf16", cuda_device, seed=3)
    G.set_variant(variant)
    try:
        r = G.raster(m, n, k, "bf16")
        c1 = G.gemm_bf16(a, bt)
        c2 = torch.full_like(c1, float("nan"))
        place = torch.full((2 * r.grid,), -1, dtype=torch.int32, device=cuda_device)
        G.gemm_placed(a, bt, c2, place)
        torch.cuda.synchronize()
    finally:
        G.set_variant(0)
    assert torch.equal(c1.view(torch.int16), c2.view(torch.int16)), f"v{r.variant}"
    xcc = (place[0::2] & 0xF).cpu().tolist()
    assert all(0 <= x < 8 for x in xcc) and -1 not in place.cpu().tolist(), f"v{r.variant}: {xcc[:16]}"


@pytest.mark.parametrize("variant", [20, 21, 22, 23, 24, 10, 18, 15, 16, 17, 60, 61, 62, 0])
def test_placed_dispatch_is_bitwise_the_timed_one_fp8(cuda_device, variant):
    import torch
    from gpu_operator_amd.ops import gemm as G

    m, n, k = {10: (8192, 8192, 512), 18: (8192, 8192, 2048), 60: (1024, 1024, 1024), 61: (1024, 1024, 16384),
               62: (2560, 2560, 2560), 0: (1000, 768, 512), 21: (8192, 8192, 2048), 22: (8192, 8192, 4096),
               24: (2560, 2560, 16384)}.get(
                   variant, (4096, 4096, 4096))
    a, bt = _operands(m, n, k, "fp8", cuda_device, seed=5)
    G.set_fp8_variant(variant)
    try:
        r = G.raster(m, n, k, "fp8")
        c1 = G.gemm_fp8(a, bt)
        c2 = torch.full_like(c1, float("nan"))
        place = torch.full((2 * r.grid,), -1, dtype=torch.int32, device=cuda_device)
        G.gemm_placed(a, bt, c2, place, fp8=True)
        torch.cuda.synchronize()
    finally:
        G.set_fp8_variant(0)
    assert torch.equal(c1.view(torch.int16), c2.view(torch.int16)), f"v{r.variant}"
    assert -1 not in place.cpu().tolist()


def test_placement_record_reads_the_hardware(cuda_device):
    """The headline dispatch (v50, 256 persistent workgroups): every workgroup reports an XCD 0-7,
    workgroups b and b + 8 share one (the round-robin the rasters are built on), each XCD holds 32
    workgroups, and the 256 workgroups sit on distinct CUs (one 160 KiB-LDS workgroup per CU)."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    m = n = k = 8192
    a, bt = _operands(m, n, k, "bf16", cuda_device)
    r = G.raster(m, n, k, "bf16")
    c = torch.empty((m, n), dtype=torch.bfloat16, device=cuda_device)
    place = torch.full((2 * r.grid,), -1, dtype=torch.int32, device=cuda_device)
    G.gemm_placed(a, bt, c, place)
    torch.cuda.synchronize()
    p = place.cpu().tolist()
    xcc = [p[2 * b] & 0xF for b in range(r.grid)]
    hw = [p[2 * b + 1] for b in range(r.grid)]
    assert r.grid == 256
    assert all(xcc[b] == xcc[b % 8] for b in range(r.grid)), xcc[:24]
    assert sorted(xcc.count(x) for x in set(xcc)) == [32] * 8
    cus = {(xcc[b], (hw[b] >> 13) & 7, (hw[b] >> 12) & 1, (hw[b] >> 8) & 0xF) for b in range(r.grid)}
    print(f"placement: XCD of block 0 = {xcc[0]}, distinct (xcd, se, sh, cu) = {len(cus)}, hw[0] = {hw[0]:#x}")
    assert len(cus) >= 200


def _validate(*args, timeout=600):
    p = subprocess.run([os.path.join(BIN, "amd-gemm-validate"), *args], capture_output=True, text=True,
                       timeout=timeout)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("dtype,shape,tile", [("bf16", "8192", (5, 7)), ("fp8", "8192", (31, 0)),
                                              ("bf16", "1024x1024x4096", (3, 6)), ("bf16", "2560", (9, 1)),
                                              ("bf16", "2560x2560x8192", (4, 8)), ("fp8", "2560x2560x16384", (2, 3))])
def test_validator_names_the_injected_tile(dtype, shape, tile):
    rc, lines, err = _validate("--shapes", shape, "--dtype", dtype, "--iters", "5", "--inject-fault",
                               f"{tile[0]},{tile[1]}")
    assert rc == 1, err
    g = [x for x in lines if x["event"] == "gemm"][0]
    assert not g["ok"] and g["kind"] == "correctness", g
    assert g["tile"] == list(tile) and g["bad_tiles"] == 1 and g["checked_fraction"] == 1.0, g
    assert g["xcd"] is None or 0 <= g["xcd"] < 8, g
    if g["variant"] not in (61, 57, 24):      # split-K: the pieces of a tile may sit on several XCDs
        assert isinstance(g["xcd"], int) and set(g["cu"]) == {"se", "sh", "cu"}, g
    assert g["bad_tile_list"][0][:2] == list(tile)
    print(json.dumps({k: g[k] for k in ("variant", "tile", "workgroup", "round", "xcd", "cu") if k in g}))


def test_validator_clean_run_checks_everything_cheaply():
    rc, lines, err = _validate("--shapes", "8192", "--dtype", "both", "--iters", "20")
    assert rc == 0, err
    for g in [x for x in lines if x["event"] == "gemm"]:
        assert g["ok"] and g["checked_fraction"] == 1.0 and g["bad_tiles"] == 0 and g["abft_worst_ratio"] < 1.0, g
        # the whole checked phase (poison, the recorded dispatch, ABFT, sampled rows) under 5 % of the probe
        assert g["check_ms"] < 0.05 * g["probe_ms"], g
        print(json.dumps({k: g[k] for k in ("dtype", "tflops", "abft_worst_ratio", "abft_ms", "check_ms", "probe_ms")}))


def test_split_k_workspaces_are_capped(cuda_device):
    """100 short-lived streams running v61: at most 16 workspace sets stay allocated and device memory
    stays flat once the cap is reached (a long-lived process cycling streams does not leak HBM)."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    m, n, k = 1024, 1024, 4096
    a, bt = _operands(m, n, k, "bf16", cuda_device)
    assert G.resolve_variant(m, n, k) == 61
    want = G.gemm_bf16(a, bt)
    free_at = {}
    for i in range(100):
        s = torch.cuda.Stream(device=cuda_device)
        with torch.cuda.stream(s):
            c = G.gemm_bf16(a, bt)
        s.synchronize()
        assert torch.equal(c, want)
        del s, c
        if i in (30, 99):
            torch.cuda.synchronize()
            free_at[i] = torch.cuda.mem_get_info(cuda_device)[0]
    assert G.small_workspace_count(cuda_device.index or 0) <= 16
    assert abs(free_at[99] - free_at[30]) < 64 << 20, free_at


def test_split_k_workspace_per_thread_stream(cuda_device):
    """the per-thread default stream handle names a different stream in every host
    thread; keyed by (device, handle) alone, two threads running v61 at once shared one set of fp32
    slabs and arrival counters. Two threads, each on hipStreamPerThread, each its own operands, 40
    launches each: every result equals its single-threaded reference."""
    import threading
    import torch
    from gpu_operator_amd.ops import _lib
    from gpu_operator_amd.ops import gemm as G

    m, n, k = 1024, 1024, 4096
    assert G.resolve_variant(m, n, k) == 61
    lib = _lib.load()
    per_thread = 2                                    # hipStreamPerThread
    jobs = []
    for seed in (11, 23):
        a, bt = _operands(m, n, k, "bf16", cuda_device, seed=seed)
        jobs.append((a, bt, G.gemm_bf16(a, bt), torch.empty((m, n), dtype=torch.bfloat16, device=cuda_device)))
    torch.cuda.synchronize()
    bad = []

    def run(j):
        a, bt, want, out = jobs[j]
        torch.cuda.set_device(cuda_device)
        for _ in range(40):
            err = lib.amdgo_gemm_bf16(a.data_ptr(), bt.data_ptr(), out.data_ptr(), m, n, k, per_thread)
            if err:
                bad.append(f"thread {j}: hipError {err}")
                return
            torch.cuda.synchronize()
            if not torch.equal(out, want):
                bad.append(f"thread {j}: result differs")
                return
    th = [threading.Thread(target=run, args=(j,)) for j in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not bad, bad
