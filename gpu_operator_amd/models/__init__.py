"""GPU model catalog: the AMD Instinct product families the operator supports.

One table drives everything that depends on the GPU model: node labels (family, product
short name), the sandbox device plugin's resource names (PF and VF device ids), which nodes
get the partition manager (compute/memory partition modes), and the validator's expectations
(dense matrix peaks, HBM per device, xGMI fabric). Numbers are dense (no 2:1 sparsity) at the
spec peak clock; the validator's pass/fail floor is a fraction of them because the sustained
clock under MFMA load is lower (MI355X_MICROARCH.md 'DVFS give-back').
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple


@dataclass(frozen=True)
class GPUModel:
    name: str                      # short product name (resource / label value)
    product: str                   # marketing name
    family: str                    # cdna4 / cdna3 / cdna2
    gfx: str                       # gfx target
    device_ids: Tuple[int, ...]    # PF PCI device ids
    vf_device_ids: Tuple[int, ...] = ()
    cus: int = 0
    xcds: int = 0
    hbm_gib: int = 0
    lds_kib: int = 64
    xgmi_links: int = 0            # per GPU in an 8-GPU hive
    xgmi_link_gbps: float = 0.0    # per link, per direction (GB/s)
    bf16_dense_tflops: float = 0.0
    fp8_dense_tflops: float = 0.0
    compute_partitions: Tuple[str, ...] = ("SPX",)
    memory_partitions: Tuple[str, ...] = ("NPS1",)

    @property
    def partition_capable(self) -> bool:
        return len(self.compute_partitions) > 1

    def gemm_floor_tflops(self, fraction: float = 0.35) -> float:
        """Validator floor for the bf16 GEMM probe (per GPU)."""
        return round(self.bf16_dense_tflops * fraction, 1)


CATALOG: Tuple[GPUModel, ...] = (
    GPUModel("MI355X", "AMD Instinct MI355X", "cdna4", "gfx950", (0x75A3,), (0x75B3,), cus=256, xcds=8, hbm_gib=288,
             lds_kib=160, xgmi_links=7, xgmi_link_gbps=153.6, bf16_dense_tflops=2516.6, fp8_dense_tflops=5033.2,
             compute_partitions=("SPX", "DPX", "QPX", "CPX"), memory_partitions=("NPS1", "NPS2")),
    GPUModel("MI350X", "AMD Instinct MI350X", "cdna4", "gfx950", (0x75A0,), (0x75B0,), cus=256, xcds=8, hbm_gib=288,
             lds_kib=160, xgmi_links=7, xgmi_link_gbps=153.6, bf16_dense_tflops=2306.9, fp8_dense_tflops=4613.7,
             compute_partitions=("SPX", "DPX", "QPX", "CPX"), memory_partitions=("NPS1", "NPS2")),
    GPUModel("MI325X", "AMD Instinct MI325X", "cdna3", "gfx942", (0x74A5,), (0x74B9,), cus=304, xcds=8, hbm_gib=256,
             lds_kib=64, xgmi_links=7, xgmi_link_gbps=128.0, bf16_dense_tflops=1307.4, fp8_dense_tflops=2614.9,
             compute_partitions=("SPX", "DPX", "QPX", "CPX"), memory_partitions=("NPS1", "NPS4")),
    GPUModel("MI300X", "AMD Instinct MI300X", "cdna3", "gfx942", (0x74A1,), (0x74B5,), cus=304, xcds=8, hbm_gib=192,
             lds_kib=64, xgmi_links=7, xgmi_link_gbps=128.0, bf16_dense_tflops=1307.4, fp8_dense_tflops=2614.9,
             compute_partitions=("SPX", "DPX", "QPX", "CPX"), memory_partitions=("NPS1", "NPS4")),
    GPUModel("MI308X", "AMD Instinct MI308X", "cdna3", "gfx942", (0x74A2,), (), cus=80, xcds=4, hbm_gib=192,
             lds_kib=64, xgmi_links=7, xgmi_link_gbps=128.0, bf16_dense_tflops=343.0,
             compute_partitions=("SPX", "CPX"), memory_partitions=("NPS1",)),
    GPUModel("MI300A", "AMD Instinct MI300A", "cdna3", "gfx942", (0x74A0,), (), cus=228, xcds=6, hbm_gib=128,
             lds_kib=64, xgmi_links=4, xgmi_link_gbps=128.0, bf16_dense_tflops=980.6, fp8_dense_tflops=1961.2,
             compute_partitions=("SPX", "TPX", "CPX"), memory_partitions=("NPS1",)),
    GPUModel("MI250X", "AMD Instinct MI250X", "cdna2", "gfx90a", (0x740C,), (), cus=220, xcds=2, hbm_gib=128,
             lds_kib=64, xgmi_links=8, xgmi_link_gbps=50.0, bf16_dense_tflops=383.0),
    GPUModel("MI210", "AMD Instinct MI210", "cdna2", "gfx90a", (0x740F,), (), cus=104, xcds=1, hbm_gib=64,
             lds_kib=64, xgmi_links=3, xgmi_link_gbps=50.0, bf16_dense_tflops=181.0),
)

GFX_FAMILY: Dict[str, str] = {m.gfx: m.family for m in CATALOG}
GFX_FAMILY.update({"gfx940": "cdna3", "gfx941": "cdna3", "gfx908": "cdna1", "gfx1100": "rdna3", "gfx1101": "rdna3",
                   "gfx1030": "rdna2"})
PARTITION_CAPABLE_FAMILIES = frozenset(m.family for m in CATALOG if m.partition_capable)

_BY_ID: Dict[int, Tuple[GPUModel, bool]] = {}
for _m in CATALOG:
    for _d in _m.device_ids:
        _BY_ID[_d] = (_m, False)
    for _d in _m.vf_device_ids:
        _BY_ID[_d] = (_m, True)


def by_device_id(device_id: int) -> Optional[Tuple[GPUModel, bool]]:
    """(model, is_virtual_function) for a PCI device id, or None."""
    return _BY_ID.get(device_id)


def by_name(name: str) -> Optional[GPUModel]:
    return next((m for m in CATALOG if m.name == name), None)


def family_of_gfx(gfx: str) -> str:
    return GFX_FAMILY.get(gfx, "unknown")
