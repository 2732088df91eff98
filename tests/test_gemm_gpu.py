"""Numerics of the hand-written CDNA4 MFMA GEMM against a plain PyTorch fp32 reference."""

import pytest

pytestmark = pytest.mark.gpu


def _ref(a, bt):
    return a.float() @ bt.float().t()


@pytest.fixture(params=[0, 18, 25, 42, 44, 45, 47, 48, 50, 51, 52, 53, 54, 55, 56, 57, 60, 61, 62])   # the production set (gemm.BF16_VARIANTS)
def variant(request):
    from gpu_operator_amd.ops import gemm as G
    old = G.get_variant()
    G.set_variant(request.param)
    yield request.param
    G.set_variant(old)


@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (512, 768, 256), (1024, 1024, 1024),
                                   (2048, 512, 4096), (768, 2304, 640), (256, 512, 128),
                                   (4608, 4608, 512),     # > 256 tiles: serpentine waves reverse K
                                   (4096, 8192, 256), (8192, 4096, 192)])   # 16x16-tile super-tiles (v45)
def test_fast_path_matches_fp32_reference(cuda_device, variant, m, n, k):
    import torch
    from gpu_operator_amd.ops import gemm as G

    assert G.fast_path_supported(m, n, k)
    g = torch.Generator(device=cuda_device).manual_seed(m + n + k)
    a = (torch.rand((m, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand((n, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
    c = G.gemm_bf16(a, bt)
    ref = _ref(a, bt)
    torch.testing.assert_close(c.float(), ref, atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)


@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (17, 33, 70), (300, 129, 65), (256, 256, 32)])
def test_generic_path_odd_shapes(cuda_device, m, n, k):
    import torch
    from gpu_operator_amd.ops import gemm as G

    a = (torch.rand((m, k), device=cuda_device) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand((n, k), device=cuda_device) * 2 - 1).to(torch.bfloat16)
    c = G.gemm_bf16(a, bt)
    torch.testing.assert_close(c.float(), _ref(a, bt), atol=3e-2, rtol=1e-2)


def test_identity_with_asymmetric_b_catches_transposes(cuda_device):
    """A = I with an asymmetric, exactly-representable B: C must equal B^T exactly."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    n = 512
    a = torch.eye(n, device=cuda_device, dtype=torch.bfloat16)
    idx = torch.arange(n, device=cuda_device)
    b = ((idx[:, None] * 3 + idx[None, :] * 7) % 61 - 30).to(torch.bfloat16)  # B[k][j]
    bt = b.t().contiguous()                                                     # Bt[j][k]
    for generic in (False, True):
        c = G.gemm_bf16(a, bt, generic=generic)
        assert torch.equal(c, b), f"generic={generic}"


def test_fast_and_generic_agree_on_8k_slice(cuda_device, variant):
    import torch
    from gpu_operator_amd.ops import gemm as G

    m, n, k = 1024, 2048, 8192
    a = torch.empty((m, k), dtype=torch.bfloat16, device=cuda_device)
    bt = torch.empty((n, k), dtype=torch.bfloat16, device=cuda_device)
    G.fill_uniform_(a, 1)
    G.fill_uniform_(bt, 2)
    c = G.gemm_bf16(a, bt)
    chk = G.verify(a, bt, c, nrows=64)
    assert chk.ok, chk
    torch.testing.assert_close(c.float(), _ref(a, bt), atol=0.15, rtol=1e-2)


def test_fill_uniform_range_and_determinism(cuda_device):
    import torch
    from gpu_operator_amd.ops import gemm as G

    t1 = G.fill_uniform_(torch.empty(1 << 20, dtype=torch.bfloat16, device=cuda_device), 5)
    t2 = G.fill_uniform_(torch.empty(1 << 20, dtype=torch.bfloat16, device=cuda_device), 5)
    assert torch.equal(t1, t2)
    assert float(t1.float().min()) >= -1.0 and float(t1.float().max()) <= 1.0
    assert abs(float(t1.float().mean())) < 0.01


def test_smoke_vector_add(cuda_device):
    from gpu_operator_amd.ops import smoke

    assert smoke.smoke(n=50_000, device=str(cuda_device))
    assert smoke.smoke(n=1_000_003, device=str(cuda_device))


def test_vp_square_raster_covers_every_tile(cuda_device):
    """12288x12288x10240 (K not a power of two; 48x48 tiles, 9 dispatch waves) takes the VP-form asm
    pipeline on the square raster (v54) under the default variant; one checked row per tile row."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    m = n = 12288
    k = 10240
    if torch.cuda.get_device_properties(cuda_device).multi_processor_count == 256:
        assert G.resolve_variant(m, n, k) == 54
    a = G.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=cuda_device), 13)
    bt = G.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=cuda_device), 14)
    c = G.gemm_bf16(a, bt)
    rows = torch.tensor([tm * 256 + (tm * 41) % 256 for tm in range(m // 256)], device=cuda_device)
    ref = a[rows].float() @ bt.float().t()
    torch.testing.assert_close(c[rows].float(), ref, atol=0.15, rtol=1e-2)


def test_short_k_square_raster_covers_every_tile(cuda_device):
    """12288x12288x2048 (48x48 tiles, 9 dispatch waves, short K) takes v56 -- VP + PA DMA rows, the
    pipelined LEAN epilogue, square raster -- under the default variant; one checked row per tile row
    (at varying residues of the PA row map) covers every output tile."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    m = n = 12288
    k = 2048
    if torch.cuda.get_device_properties(cuda_device).multi_processor_count == 256:
        assert G.resolve_variant(m, n, k) == 56
    a = G.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=cuda_device), 15)
    bt = G.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=cuda_device), 16)
    c = G.gemm_bf16(a, bt)
    rows = torch.tensor([tm * 256 + (tm * 43) % 256 for tm in range(m // 256)], device=cuda_device)
    ref = a[rows].float() @ bt.float().t()
    torch.testing.assert_close(c[rows].float(), ref, atol=0.15, rtol=1e-2)


def test_default_dispatch_square_raster_covers_every_tile(cuda_device):
    """12288x12288x8192 (48x48 tiles, 9 dispatch waves) takes the square cross-XCD raster (v51)
    under the default variant; one checked row per tile row covers every output tile."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    m = n = 12288
    k = 8192
    a = torch.empty((m, k), dtype=torch.bfloat16, device=cuda_device)
    bt = torch.empty((n, k), dtype=torch.bfloat16, device=cuda_device)
    G.fill_uniform_(a, 3)
    G.fill_uniform_(bt, 4)
    c = G.gemm_bf16(a, bt)
    rows = torch.tensor([tm * 256 + (tm * 37) % 256 for tm in range(m // 256)], device=cuda_device)
    ref = a[rows].float() @ bt.float().t()
    torch.testing.assert_close(c[rows].float(), ref, atol=0.15, rtol=1e-2)


def test_production_variant_set_is_closed(cuda_device):
    """Only exact, shipped kernels are reachable: lab/knock-out numbers are refused."""
    from gpu_operator_amd.ops import gemm as G

    assert tuple(G.BF16_VARIANTS) == (0, 18, 25, 42, 44, 45, 47, 48, 50, 51, 52, 53, 54, 55, 56, 57, 60, 61, 62)
    for bad in (1, 2, 10, 20, 24, 27, 40, 46, 99, -1):
        with pytest.raises(ValueError):
            G.set_variant(bad)
    assert G.get_variant() == 0


@pytest.mark.parametrize("m,n,k,want", [(8192, 8192, 8192, 50), (16384, 16384, 1024, 56), (8192, 8192, 4096, 50),
                                        (8192, 8192, 2048, 56), (4096, 8192, 1024, 56), (4096, 4096, 2048, 56), (2048, 4096, 512, 62),
                                        (12288, 12288, 12288, 54), (8192, 8192, 12288, 53), (8192, 8192, 8256, 47),
                                        (12288, 12288, 8256, 48),
                                        (12288, 12288, 8192, 51), (16384, 16384, 16384, 51),
                                        (4096, 4096, 16384, 56), (4096, 8192, 8192, 50), (4096, 4096, 32768, 52),
                                        (4096, 4096, 4096, 56),
                                        (8192, 8192, 128, 25), (256, 256, 64, 60), (300, 256, 256, 0),
                                        (1024, 1024, 1024, 60), (2048, 2048, 2048, 60), (1152, 1152, 1024, 60),
                                        (1024, 1024, 8192, 61), (1024, 1024, 2048, 61), (1024, 1024, 512, 60),
                                        (2560, 2560, 2560, 62), (4096, 2048, 4096, 57), (3072, 3072, 3072, 53),
                                        (2560, 2560, 8192, 57), (2560, 2560, 2048, 62), (2048, 2048, 16384, 57),
                                        (2048, 2048, 8192, 60)])
def test_automatic_dispatch_resolution(cuda_device, m, n, k, want):
    """The automatic dispatch picks the kernel documented in gemm_bf16.hip (256-CU MI355X)."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    if torch.cuda.get_device_properties(cuda_device).multi_processor_count != 256:
        want = {44: 42, 45: 42, 47: 42, 48: 42, 50: 42, 51: 42, 52: 42, 53: 42, 54: 42, 55: 42, 56: 42,
                57: 62}.get(want, want)
    assert G.get_variant() == 0
    assert G.resolve_variant(m, n, k) == want


@pytest.mark.parametrize("m,n,k", [(8192, 8192, 1024), (4096, 4096, 4096), (2048, 4096, 512), (4096, 4096, 3072)])
def test_asm_pipeline_is_bitwise_v44(cuda_device, m, n, k):
    """v50 (the hand-scheduled asm K pipeline, persistent) issues the MFMAs of v44 in the same
    per-accumulator order, with the same serpentine K per dispatch wave: the outputs are equal bit
    for bit, not only within tolerance."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    a = G.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=cuda_device), 5)
    bt = G.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=cuda_device), 6)
    old = G.get_variant()
    try:
        G.set_variant(44)
        c44 = G.gemm_bf16(a, bt)
        G.set_variant(50)
        assert G.resolve_variant(m, n, k) == 50
        c50 = G.gemm_bf16(a, bt)
        G.set_variant(53)            # the same pipeline in the VP DMA form: same MFMA order
        assert G.resolve_variant(m, n, k) == 53
        c53 = G.gemm_bf16(a, bt)
        G.set_variant(55)            # VP + PA rows + LEAN epilogue: permuted staging, same sums
        assert G.resolve_variant(m, n, k) == 55
        c55 = G.gemm_bf16(a, bt)
    finally:
        G.set_variant(old)
    torch.cuda.synchronize()
    assert torch.equal(c44, c50)
    assert torch.equal(c44, c53)
    assert torch.equal(c44, c55)


@pytest.mark.parametrize("m,n,k", [(4096, 8192, 256), (8192, 8192, 1024), (4096, 4096, 2048)])
def test_asm_square_raster_is_bitwise_v45(cuda_device, m, n, k):
    """v51 (persistent asm pipeline on the square cross-XCD raster) walks the tiles of v45 in the
    same rounds of 256 with the same serpentine K per round: bitwise-equal outputs."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    if torch.cuda.get_device_properties(cuda_device).multi_processor_count != 256:
        pytest.skip("square raster needs the 256-CU MI355X")
    a = G.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=cuda_device), 7)
    bt = G.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=cuda_device), 8)
    old = G.get_variant()
    try:
        G.set_variant(45)
        c45 = G.gemm_bf16(a, bt)
        G.set_variant(51)
        assert G.resolve_variant(m, n, k) == 51
        c51 = G.gemm_bf16(a, bt)
        G.set_variant(52)
        c52 = G.gemm_bf16(a, bt)
        G.set_variant(50)
        c50 = G.gemm_bf16(a, bt)
        G.set_variant(54)            # v51 in the VP DMA form
        c54 = G.gemm_bf16(a, bt)
        G.set_variant(56)            # v54 with PA rows and the LEAN epilogue
        c56 = G.gemm_bf16(a, bt)
    finally:
        G.set_variant(old)
    torch.cuda.synchronize()
    assert torch.equal(c45, c51)
    assert torch.equal(c45, c54)
    assert torch.equal(c45, c56)
    assert torch.equal(c50, c52)      # same pipeline, different instruction placement


@pytest.mark.parametrize("v", [60])
@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (128, 128, 128), (1024, 1024, 1024), (1152, 1280, 576),
                                   (2048, 2048, 2048), (384, 640, 4160), (1024, 1024, 8192)])
def test_small_grid_kernel_v60_matches_fp32_reference(cuda_device, v, m, n, k):
    """v60 (128x128 tiles, gemm_small.h) on shapes only it or the generic kernel can run, and on the
    small grids the automatic dispatch now sends it; A = I checks its C mapping exactly."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    old = G.get_variant()
    G.set_variant(v)
    try:
        assert G.resolve_variant(m, n, k) == v
        g = torch.Generator(device=cuda_device).manual_seed(m * 3 + n + k)
        a = (torch.rand((m, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand((n, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        c = G.gemm_bf16(a, bt)
        torch.testing.assert_close(c.float(), _ref(a, bt), atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)
        eye = torch.eye(m, k, device=cuda_device, dtype=torch.bfloat16)      # C = Bt^T rows (exact)
        idx = torch.arange(k, device=cuda_device)
        bt2 = ((torch.arange(n, device=cuda_device)[:, None] * 5 + idx[None, :] * 3) % 41 - 20).to(torch.bfloat16)
        assert torch.equal(G.gemm_bf16(eye, bt2), (eye.float() @ bt2.float().t()).to(torch.bfloat16))
    finally:
        G.set_variant(old)
    assert G.resolve_variant(1024, 1024, 1024) == 60          # the automatic choice for a 16-tile grid


@pytest.mark.parametrize("m,n,k,splits", [(2560, 2560, 2560, 2), (2048, 2048, 8192, 4), (1024, 1024, 4096, 4),
                                          (512, 512, 8192, 4), (2048, 512, 4096, 4), (1536, 2560, 3072, 3)])
def test_split_k_asm_v57_matches_fp32_reference_on_repeat(cuda_device, m, n, k, splits):
    """v57: the asm 256x256 frame, one (tile, K piece) per workgroup; each tile's last arriving waves
    sum the fp32 slabs in piece order. Repeated launches on one stream (the counters must be reset),
    one on a side stream, all against the fp32 reference and bitwise equal to each other."""
    import torch
    from gpu_operator_amd.ops import gemm as G
    from gpu_operator_amd.ops import _lib

    old = G.get_variant()
    G.set_variant(57)
    try:
        assert G.resolve_variant(m, n, k) == 57
        info = G.raster(m, n, k, "bf16")
        assert info.pieces == splits and info.grid == (m // 256) * (n // 256) * splits
        g = torch.Generator(device=cuda_device).manual_seed(m + 5 * n + k)
        a = (torch.rand((m, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand((n, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        ref = _ref(a, bt)
        outs = [G.gemm_bf16(a, bt) for _ in range(3)]
        side = torch.cuda.Stream(device=cuda_device)
        with torch.cuda.stream(side):
            outs.append(G.gemm_bf16(a, bt))
        torch.cuda.synchronize()
        for c in outs:
            torch.testing.assert_close(c.float(), ref, atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)
        assert all(torch.equal(outs[0], c) for c in outs[1:])     # piece order fixed: arrival order is not
    finally:
        G.set_variant(old)


@pytest.mark.parametrize("m,n,k,splits,permille,tile_major", [
    (2560, 2560, 8192, 2, 540, False), (2048, 2048, 8192, 4, 340, False), (2048, 2048, 8192, 3, 400, True),
    (1024, 1024, 4096, 2, 700, False), (2048, 4096, 8192, 2, 540, True), (2048, 2048, 8192, 4, 0, True)])
def test_split_k_asm_v57_uneven_pieces(cuda_device, m, n, k, splits, permille, tile_major):
    """v57 with forced piece counts, a longer last piece (the first pieces' slabs stored under the last
    one's K-loop) and either item order: against the fp32 reference, repeated launches bitwise equal."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    old = G.get_variant()
    G.set_variant(57)
    G.set_asm_split(splits, permille, piece_major=not tile_major)
    try:
        assert G.raster(m, n, k, "bf16").pieces == splits
        g = torch.Generator(device=cuda_device).manual_seed(m + 3 * n + k + permille)
        a = (torch.rand((m, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand((n, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        ref = _ref(a, bt)
        outs = [G.gemm_bf16(a, bt) for _ in range(3)]
        torch.cuda.synchronize()
        for c in outs:
            torch.testing.assert_close(c.float(), ref, atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)
        assert all(torch.equal(outs[0], c) for c in outs[1:])
    finally:
        G.set_asm_split(0, 0)
        G.set_variant(old)


@pytest.mark.parametrize("v", [61])
@pytest.mark.parametrize("m,n,k,target", [(1024, 1024, 1024, 1), (1024, 1024, 8192, 1), (128, 128, 4096, 1),
                                          (2048, 2048, 2048, 2), (1152, 1280, 4160, 4), (256, 384, 64, 1)])
def test_split_k_kernel_v61_matches_fp32_reference_on_repeat(cuda_device, v, m, n, k, target):
    """v61: the K splits of a tile meet at a per-tile counter; the last one adds the others' fp32
    partials. Three launches in a row on one stream (each must find the counters reset) and a launch
    on a second stream, all against the fp32 reference."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    old = G.get_variant()
    G.set_variant(v)
    G.set_split_target(target)
    try:
        assert G.resolve_variant(m, n, k) == v
        g = torch.Generator(device=cuda_device).manual_seed(m + 7 * n + k)
        a = (torch.rand((m, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand((n, k), generator=g, device=cuda_device) * 2 - 1).to(torch.bfloat16)
        ref = _ref(a, bt)
        outs = [G.gemm_bf16(a, bt) for _ in range(3)]
        side = torch.cuda.Stream(device=cuda_device)
        with torch.cuda.stream(side):
            outs.append(G.gemm_bf16(a, bt))
        torch.cuda.synchronize()
        for c in outs:
            torch.testing.assert_close(c.float(), ref, atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)
        assert all(torch.equal(outs[0], c) for c in outs[1:3])     # same splits, same summation order
    finally:
        G.set_split_target(1)
        G.set_variant(old)
