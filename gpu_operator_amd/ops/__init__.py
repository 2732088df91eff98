"""GPU compute ops of the validator workloads (hand-written HIP kernels for gfx950)."""

from .gemm import gemm_bf16, fill_uniform_, verify, tflops  # noqa: F401
from .smoke import vector_add  # noqa: F401
