"""hip-smoke: fp32 vector add with full host verification.

The functional analogue of the reference's CUDA-samples ``vectorAdd`` (50,000 elements,
reference: validator/cuda-workload-validation.yaml:20). It gates the ``hip-ready`` barrier
quickly, before the heavier GEMM and all-reduce probes.
"""

from __future__ import annotations

from . import _lib


def vector_add(a, b, out=None):
    import torch

    for name, t in (("a", a), ("b", b)):
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous fp32 GPU tensor")
    if a.shape != b.shape:
        raise ValueError("shape mismatch")
    if out is None:
        out = torch.empty_like(a)
    lib = _lib.load()
    err = lib.amdgo_vector_add_f32(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(),
                                   torch.cuda.current_stream(a.device).cuda_stream)
    _lib.check(err, "amdgo_vector_add_f32")
    return out


def smoke(n: int = 50_000, device: str = "cuda:0") -> bool:
    """Run the smoke kernel and verify every element on the host (like vectorAdd)."""
    import torch

    g = torch.Generator().manual_seed(7)
    a_h = torch.rand(n, generator=g)
    b_h = torch.rand(n, generator=g)
    c = vector_add(a_h.to(device), b_h.to(device))
    torch.cuda.synchronize(device)
    return bool(torch.equal(c.cpu(), a_h + b_h))
