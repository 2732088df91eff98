"""Numerics of the hand-written CDNA4 fp8 (OCP e4m3fn) MFMA GEMM against a PyTorch fp32 reference.

The reference decodes the same fp8 operands with PyTorch (``.float()``) and multiplies in fp32;
the kernel accumulates in fp32 and rounds to bf16, so the tolerance is a bf16 ulp of the output
plus accumulation-order slack.
"""

import pytest

pytestmark = pytest.mark.gpu


def _ref(a, bt):
    return a.float() @ bt.float().t()


def _rand_fp8(shape, gen, dev):
    import torch

    return (torch.rand(shape, generator=gen, device=dev) * 2 - 1).to(torch.float8_e4m3fn)


@pytest.fixture(params=[0, 10, 15, 16, 17, 18, 20, 21, 22, 23, 24, 60, 61, 62])   # the production set (gemm.FP8_VARIANTS)
def fp8_variant(request):
    from gpu_operator_amd.ops import gemm as G

    old = G.get_fp8_variant()
    G.set_fp8_variant(request.param)
    yield request.param
    G.set_fp8_variant(old)


@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (512, 768, 512), (1024, 1024, 1024),
                                   (2048, 512, 4096), (768, 2304, 640), (256, 512, 384),
                                   (4608, 4608, 512),     # > 256 tiles: serpentine waves reverse K
                                   (4096, 8192, 256), (8192, 4096, 384),    # 16x16-tile super-tiles (v16)
                                   (4096, 8192, 512), (8192, 8192, 768)])   # v21: 2 / 4 dispatch waves, 4 / 6 K-tiles
def test_fp8_fast_path_matches_fp32_reference(cuda_device, fp8_variant, m, n, k):
    import torch
    from gpu_operator_amd.ops import gemm as G

    assert G.fp8_fast_path_supported(m, n, k)
    g = torch.Generator(device=cuda_device).manual_seed(m + 3 * n + 7 * k)
    a = _rand_fp8((m, k), g, cuda_device)
    bt = _rand_fp8((n, k), g, cuda_device)
    c = G.gemm_fp8(a, bt)
    ref = _ref(a, bt)
    torch.testing.assert_close(c.float(), ref, atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)


@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (17, 33, 70), (300, 129, 65), (256, 256, 128)])
def test_fp8_generic_path_odd_shapes(cuda_device, m, n, k):
    import torch
    from gpu_operator_amd.ops import gemm as G

    g = torch.Generator(device=cuda_device).manual_seed(7)
    a = _rand_fp8((m, k), g, cuda_device)
    bt = _rand_fp8((n, k), g, cuda_device)
    assert not G.fp8_fast_path_supported(m, n, k)
    c = G.gemm_fp8(a, bt)
    torch.testing.assert_close(c.float(), _ref(a, bt), atol=3e-2, rtol=1e-2)


def test_fp8_identity_with_asymmetric_b_catches_transposes(cuda_device):
    """A = I with an asymmetric B of small integers (exact in e4m3 and bf16): C must equal B."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    n = 512
    a = torch.eye(n, device=cuda_device).to(torch.float8_e4m3fn)
    idx = torch.arange(n, device=cuda_device)
    b = ((idx[:, None] * 3 + idx[None, :] * 7) % 17 - 8).float()      # B[k][j]
    bt = b.t().contiguous().to(torch.float8_e4m3fn)                     # Bt[j][k]
    for generic in (False, True):
        c = G.gemm_fp8(a, bt, generic=generic)
        assert torch.equal(c.float(), b), f"generic={generic}"


def test_fp8_fast_and_reference_rows_agree_on_8k_k(cuda_device):
    import torch
    from gpu_operator_amd.ops import gemm as G

    m, n, k = 1024, 2048, 8192
    a = G.fill_uniform_fp8_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device=cuda_device), 1)
    bt = G.fill_uniform_fp8_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device=cuda_device), 2)
    c = G.gemm_fp8(a, bt)
    chk = G.verify(a, bt, c, nrows=64)
    assert chk.ok, chk
    torch.testing.assert_close(c.float(), _ref(a, bt), atol=0.15, rtol=1e-2)


def test_fp8_software_decoder_matches_torch_on_every_code(cuda_device):
    """The reference kernel's e4m3 decoder (A row x unit Bt) reproduces torch's decode of all codes."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    codes = torch.arange(256, dtype=torch.int32)
    codes = codes[(codes & 0x7F) != 0x7F].to(torch.uint8)               # drop the two NaNs
    k = codes.numel()
    a = codes.view(torch.float8_e4m3fn).reshape(1, k).to(cuda_device)
    bt = torch.eye(k, device=cuda_device).to(torch.float8_e4m3fn)
    got = G.reference_rows(a, bt, [0])[0]
    assert torch.equal(got, a.float()[0])


def test_fill_uniform_fp8_range_and_determinism(cuda_device):
    import torch
    from gpu_operator_amd.ops import gemm as G

    f8 = torch.float8_e4m3fn
    t1 = G.fill_uniform_fp8_(torch.empty(1 << 20, dtype=f8, device=cuda_device), 5)
    t2 = G.fill_uniform_fp8_(torch.empty(1 << 20, dtype=f8, device=cuda_device), 5)
    assert torch.equal(t1.view(torch.uint8), t2.view(torch.uint8))
    f = t1.float()
    assert float(f.min()) >= -1.0 and float(f.max()) <= 1.0
    assert abs(float(f.mean())) < 0.01
    assert torch.unique(t1.view(torch.uint8)).numel() > 100


@pytest.mark.parametrize("variant", [16, 21, 22])
def test_fp8_square_raster_covers_every_tile(cuda_device, variant):
    """The square cross-XCD raster (q16 v16, persistent asm q16ap v21, its VP + PA + LEAN form v22) over
    12288x12288x8192 (48x48 tiles, 9 dispatch waves, snaking super-rows); one checked row per tile row
    covers every output tile (and, for v22, every residue of the PA row map)."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    old = G.get_fp8_variant()
    G.set_fp8_variant(variant)
    try:
        _check_square_raster_fp8(cuda_device, G, torch)
    finally:
        G.set_fp8_variant(old)


def _check_square_raster_fp8(cuda_device, G, torch):
    m = n = 12288
    k = 8192
    g = torch.Generator(device=cuda_device).manual_seed(99)
    a = _rand_fp8((m, k), g, cuda_device)
    bt = _rand_fp8((n, k), g, cuda_device)
    c = G.gemm_fp8(a, bt)
    rows = torch.tensor([tm * 256 + (tm * 53) % 256 for tm in range(m // 256)], device=cuda_device)
    ref = a[rows].float() @ bt.float().t()
    torch.testing.assert_close(c[rows].float(), ref, atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)


def test_fp8_production_variant_set_is_closed(cuda_device):
    import torch
    from gpu_operator_amd.ops import gemm as G

    for bad in (1, 2, 3, 4, 5, 6, 7, 8, 9, 11, 12, 13, 14, 19, 25, 28, 40, 99):
        with pytest.raises(ValueError):
            G.set_fp8_variant(bad)
    assert G.get_fp8_variant() == 0
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    if cus == 256:       # MI355X: the persistent asm pipeline
        assert G.resolve_fp8_variant(8192, 8192, 8192) == 22
        assert G.resolve_fp8_variant(8192, 8192 + 256, 8192) == 20     # not 16x16-tile multiples
        assert G.resolve_fp8_variant(16384, 16384, 16384) == 22
        assert G.resolve_fp8_variant(16384, 16384, 1024) == 22
        assert G.resolve_fp8_variant(12288, 12288, 12288) == 22
        assert G.resolve_fp8_variant(12288, 4096, 1024) == 21            # a 16-tile side keeps v21
        assert G.resolve_fp8_variant(4096, 4096, 4096) == 22                # one dispatch wave
        assert G.resolve_fp8_variant(2048, 4096, 4096) == 62                # 128 tiles: 256x128 tiles fill the chip
        assert G.resolve_fp8_variant(2048, 4096, 16384) == 24               # 128 tiles, long K: two K pieces
        assert G.resolve_fp8_variant(2048, 2048, 32768) == 24               # 64 tiles, K >= 32768: four pieces
        assert G.resolve_fp8_variant(4096, 8192, 4096) == 22                # a 16-tile side, K >= 4096
        assert G.resolve_fp8_variant(4096 + 256, 4096, 4096) == 20
        assert G.resolve_fp8_variant(8192, 8192, 8192 + 128) in (16, 18)   # odd K-tile count
    assert G.resolve_fp8_variant(300, 256, 256) == 0


@pytest.mark.parametrize("m,n,k,pieces", [(2560, 2560, 16384, 2), (2048, 2048, 32768, 4), (1536, 2560, 32768, 4)])
def test_fp8_split_k_asm_v24_matches_fp32_reference_on_repeat(cuda_device, m, n, k, pieces):
    """fp8 v24 (the q16ap frame's split-K form) as the automatic dispatch runs it: two pieces on a
    100-tile grid, four on 60-64 tiles; sampled rows of every tile row against the fp32 reference,
    repeated launches bitwise equal (the pieces are summed in a fixed tree)."""
    import torch
    from gpu_operator_amd.ops import gemm as G

    if torch.cuda.get_device_properties(cuda_device).multi_processor_count != 256:
        pytest.skip("the asm frame runs on the 256-CU MI355X")
    assert G.resolve_fp8_variant(m, n, k) == 24
    assert G.raster(m, n, k, "fp8").pieces == pieces
    g = torch.Generator(device=cuda_device).manual_seed(m + n + k)
    a = _rand_fp8((m, k), g, cuda_device)
    bt = _rand_fp8((n, k), g, cuda_device)
    outs = [G.gemm_fp8(a, bt) for _ in range(3)]
    torch.cuda.synchronize()
    rows = torch.tensor([tm * 256 + (tm * 37) % 256 for tm in range(m // 256)], device=cuda_device)
    ref = a[rows].float() @ bt.float().t()
    torch.testing.assert_close(outs[0][rows].float(), ref, atol=2e-2 * (k ** 0.5) / 8, rtol=1e-2)
    assert all(torch.equal(outs[0], c) for c in outs[1:])
