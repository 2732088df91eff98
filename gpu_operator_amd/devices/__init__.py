"""Node-local view of AMD GPUs (discovery, driver state, partitions, telemetry, barriers).

Thin Python layer over the native ``_amdnode`` extension (native/node/amdnode.cpp). Paths are
resolved under ``root`` (``/`` on the host, ``/host`` in a container that mounts it, a
fake sysfs tree in tests — see :mod:`gpu_operator_amd.devices.fakesys`).
"""

from __future__ import annotations

import importlib
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Sequence

_NATIVE = None


def native():
    """The compiled extension; raises if it was not built (no silent Python fallback)."""
    global _NATIVE
    if _NATIVE is None:
        try:
            _NATIVE = importlib.import_module("gpu_operator_amd._native._amdnode")
        except ImportError as e:  # pragma: no cover - exercised only on a broken install
            raise ImportError("gpu_operator_amd._native._amdnode is not built: run "
                              "`python -m gpu_operator_amd._build`") from e
    return _NATIVE


def sys_root() -> str:
    return os.environ.get("AMD_SYSFS_ROOT", "/")


XGMI_LINK_TYPE = 11
PCIE_LINK_TYPE = 2

GPU_FIELDS = ("index", "kfd_node", "gpu_id", "unique_id", "gfx_target", "gfx_target_version", "simd_count",
              "cu_count", "simd_per_cu", "max_waves_per_simd", "lds_size_kib", "drm_render_minor", "drm_card",
              "numa_node", "pci_bdf", "vendor_id", "device_id", "subsystem_device", "pci_class", "driver",
              "vram_total", "vram_used", "product_name", "vbios_version", "compute_partition",
              "memory_partition", "available_compute_partitions", "available_memory_partitions",
              "xgmi_hive_id", "xgmi_links", "pcie_links", "device_path", "partition_capable")


def gpu_dict(g) -> Dict:
    d = {f: getattr(g, f) for f in GPU_FIELDS}
    d["available_compute_partitions"] = list(d["available_compute_partitions"])
    d["available_memory_partitions"] = list(d["available_memory_partitions"])
    d["links"] = [{"type": l.type, "node_from": l.node_from, "node_to": l.node_to, "weight": l.weight}
                  for l in g.links]
    return d


def enumerate_gpus(root: Optional[str] = None) -> List[Dict]:
    return [gpu_dict(g) for g in native().enumerate_gpus(root or sys_root())]


def driver_state(root: Optional[str] = None, dev_root: Optional[str] = None) -> Dict:
    s = native().driver_state(root or sys_root(), dev_root or os.environ.get("AMD_DEV_ROOT", "/"))
    return {"module_loaded": s.module_loaded, "live": s.live, "kfd_present": s.kfd_present,
            "version": s.version, "kfd_gpu_nodes": s.kfd_gpu_nodes}


def scan_pci(root: Optional[str] = None, vendor: int = 0x1002, gpu_classes_only: bool = True) -> List[Dict]:
    out = []
    for f in native().scan_pci(root or sys_root(), vendor, gpu_classes_only):
        out.append({k: getattr(f, k) for k in ("bdf", "vendor_id", "device_id", "pci_class", "driver",
                                               "iommu_group", "sriov_totalvfs", "sriov_numvfs",
                                               "is_virtfn", "physfn")})
    return out


def read_telemetry(root: Optional[str] = None) -> List[Dict]:
    out = []
    for t in native().read_telemetry(root or sys_root()):
        out.append({k: getattr(t, k) for k in ("index", "power_w", "temp_edge_c", "temp_junction_c",
                                               "temp_mem_c", "gpu_busy_pct", "mem_busy_pct", "vram_used",
                                               "vram_total", "sclk_mhz", "mclk_mhz", "ecc_correctable",
                                               "ecc_uncorrectable", "pcie_bw_bytes", "ras_ue_total", "ras_ce_total",
                                               "ras_ue_blocks", "bad_pages_retired", "bad_pages_pending")})
    return out


GPU_METRICS_FIELDS = ("index", "pci_bdf", "valid", "error", "format_revision", "content_revision", "structure_size",
                      "temp_hotspot_c", "temp_mem_c", "temp_vrsoc_c", "socket_power_w", "gfx_activity_pct",
                      "umc_activity_pct", "energy_acc", "system_clock_ns", "firmware_timestamp",
                      "accumulation_counter", "ppt_residency_acc", "pcie_link_width", "pcie_link_speed",
                      "xgmi_link_width", "xgmi_link_speed", "pcie_bandwidth_acc", "pcie_bandwidth_inst",
                      "mem_max_bandwidth", "xgmi_read_kb", "xgmi_write_kb", "xgmi_link_status", "gfxclk_mhz",
                      "uclk_mhz")
ENERGY_UNIT_J = 15.259e-6           # gpu_metrics energy_accumulator unit (2^-16 J)


def _metrics_dict(m) -> Dict:
    d = {f: getattr(m, f) for f in GPU_METRICS_FIELDS}
    for f in ("xgmi_read_kb", "xgmi_write_kb", "xgmi_link_status", "gfxclk_mhz"):
        d[f] = list(d[f])
    return d


def read_gpu_metrics(root: Optional[str] = None) -> List[Dict]:
    """Per GPU agent: the decoded sysfs ``gpu_metrics`` table (xGMI per-link KiB read/written,
    link status/width/speed, energy, PCIe bandwidth, clocks). ``valid`` is False (with ``error``)
    for a table revision whose layout has not been pinned on hardware."""
    return [_metrics_dict(m) for m in native().read_gpu_metrics(root or sys_root())]


def parse_gpu_metrics(blob: bytes) -> Dict:
    return _metrics_dict(native().parse_gpu_metrics(blob))


def set_partition(bdf: str, kind: str, mode: str, root: Optional[str] = None) -> None:
    err = native().set_partition(root or sys_root(), bdf, kind, mode)
    if err:
        raise ValueError(err)


def wait_files(directory: str, names: Sequence[str], any_of: bool = False,
               timeout: Optional[float] = None) -> List[str]:
    """inotify-driven wait for barrier files; returns the present names ([] on timeout)."""
    ms = -1 if timeout is None else int(timeout * 1000)
    return list(native().wait_files(directory, list(names), any_of, ms))


def xgmi_topology(gpus: List[Dict]) -> Dict[int, List[int]]:
    """GPU index -> GPU indices it has a direct xGMI link to."""
    by_node = {g["kfd_node"]: g["index"] for g in gpus}
    topo: Dict[int, List[int]] = {}
    for g in gpus:
        topo[g["index"]] = sorted(by_node[l["node_to"]] for l in g["links"]
                                  if l["type"] == XGMI_LINK_TYPE and l["node_to"] in by_node)
    return topo


def single_hive(gpus: List[Dict]) -> bool:
    hives = {g["xgmi_hive_id"] for g in gpus}
    return len(gpus) > 0 and len(hives) == 1 and 0 not in hives
