"""Build fake sysfs/KFD trees of AMD GPU nodes for tests and dry runs.

Mirrors the files libamdnode reads on a real MI355X node: KFD topology nodes (one CPU agent
per socket + one GPU agent per XCP partition) with xGMI/PCIe io_links, PCI device
directories with VRAM, partition and hwmon files, the amdgpu module state and /dev/kfd.
The reference ships no fake GPU or sysfs for its validator.
"""

from __future__ import annotations

import os
import struct
from pathlib import Path
from typing import Dict, Optional, Sequence

MI355X_DEVICE_ID = 0x75A3
MI355X_CUS = 256
MI355X_VRAM = 288 * (1 << 30)          # 288 GiB HBM3E
PARTITION_XCDS = {"SPX": 8, "DPX": 4, "QPX": 2, "CPX": 1}
GFX950 = 90500


GPU_METRICS_V18_SIZE = 3872


def encode_gpu_metrics_v18(*, xgmi_read_kb: Sequence[int] = (0,) * 8, xgmi_write_kb: Sequence[int] = (0,) * 8,
                           xgmi_link_status: Sequence[int] = (-1, 1, 1, 1, 1, 1, 1, 1), clock_ns: int = 10 ** 15,
                           energy_acc: int = 1 << 40, socket_power_w: int = 750, temp_hotspot_c: int = 61,
                           temp_mem_c: int = 52, xgmi_link_width: int = 16, xgmi_link_speed: int = 38,
                           gfxclk_mhz: Sequence[int] = (2100,) * 8) -> bytes:
    """A gpu_metrics table in the MI355X layout (format 1, content 8) with every field the native
    decoder reads; everything else holds the PMFW's N/A pattern (0xFF bytes)."""
    b = bytearray(b"\xff" * GPU_METRICS_V18_SIZE)
    struct.pack_into("<HBB", b, 0, GPU_METRICS_V18_SIZE, 1, 8)
    struct.pack_into("<HHHHHH", b, 4, temp_hotspot_c, temp_mem_c, 40, socket_power_w, 37, 12)
    struct.pack_into("<QQQ", b, 16, 8192, energy_acc, clock_ns)
    struct.pack_into("<IIIIIII", b, 40, 1000, 0, 0, 0, 0, 0, 0)
    struct.pack_into("<HHHH", b, 68, 16, 320, xgmi_link_width, xgmi_link_speed)
    struct.pack_into("<QQ", b, 88, 1 << 30, 20)
    struct.pack_into("<8Q", b, 136, *xgmi_read_kb)
    struct.pack_into("<8Q", b, 200, *xgmi_write_kb)
    struct.pack_into("<8H", b, 264, *[0xFFFF if x < 0 else x for x in xgmi_link_status])
    struct.pack_into("<Q", b, 288, clock_ns // 10)
    struct.pack_into("<8H", b, 296, *gfxclk_mhz)
    struct.pack_into("<H", b, 336, 1900)
    return bytes(b)


def write_gpu_metrics(root, bdf: str, blob: bytes) -> None:
    p = Path(root) / "sys/bus/pci/devices" / bdf / "gpu_metrics"
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_bytes(blob)


def _w(p: Path, content) -> None:
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(f"{content}\n")


def _group_member(grp: Path, dev: Path) -> None:
    link = grp / "devices" / dev.name
    link.parent.mkdir(parents=True, exist_ok=True)
    if not link.is_symlink():
        os.symlink(os.path.relpath(dev, link.parent), link)


def _props(p: Path, kv: Dict[str, int]) -> None:
    _w(p, "\n".join(f"{k} {v}" for k, v in kv.items()))


def make_node(root, n_gpus: int = 8, compute: str = "SPX", memory: str = "NPS1", driver: str = "amdgpu",
              live: bool = True, kfd: bool = True, hive_id: int = 0x5A5A_0001, device_id: int = MI355X_DEVICE_ID,
              driver_version: str = "6.12.12", sriov_totalvfs: int = 0, vfio_bound: bool = False,
              product: Optional[str] = "AMD Instinct MI355X", companion_audio: bool = False) -> Path:
    """Create a fake node under ``root``; returns the root path."""
    root = Path(root)
    nparts = 8 // PARTITION_XCDS[compute]
    cus = MI355X_CUS // nparts
    vram_per_part = MI355X_VRAM // (nparts if memory != "NPS1" else 1) if memory != "NPS1" else MI355X_VRAM
    if live:
        _w(root / "sys/module/amdgpu/initstate", "live")
        if driver_version:
            _w(root / "sys/module/amdgpu/version", driver_version)
    if kfd:
        (root / "dev").mkdir(parents=True, exist_ok=True)
        (root / "dev/kfd").write_text("")
    topo = root / "sys/class/kfd/kfd/topology/nodes"
    _props(topo / "0/properties", {"cpu_cores_count": 128, "simd_count": 0, "mem_banks_count": 1})
    _w(topo / "0/gpu_id", 0)
    node = 1
    gpu_nodes = []
    for g in range(n_gpus):
        bus = 0x05 + 0x10 * g
        bdf = f"0000:{bus:02x}:00.0"
        dev = root / "sys/bus/pci/devices" / bdf
        _w(dev / "vendor", "0x1002")
        _w(dev / "device", f"0x{device_id:04x}")
        _w(dev / "subsystem_device", "0x0b00")
        _w(dev / "class", "0x120000")
        _w(dev / "numa_node", g // 4)
        _w(dev / "mem_info_vram_total", MI355X_VRAM)
        _w(dev / "mem_info_vram_used", 1 << 30)
        if product:
            _w(dev / "product_name", product)
        _w(dev / "vbios_version", "113-MI355X-001")
        _w(dev / "current_compute_partition", compute)
        _w(dev / "available_compute_partition", "SPX, DPX, QPX, CPX")
        _w(dev / "current_memory_partition", memory)
        _w(dev / "available_memory_partition", "NPS1, NPS2")
        _w(dev / "xgmi_hive_info/xgmi_hive_id", hive_id)
        _w(dev / "gpu_busy_percent", 37)
        _w(dev / "mem_busy_percent", 12)
        _w(dev / "pp_dpm_sclk", "0: 500Mhz\n1: 2100Mhz *\n2: 2400Mhz")
        _w(dev / "pp_dpm_mclk", "0: 900Mhz\n1: 1900Mhz *")
        _w(dev / "ras/umc_err_count", "ue: 0\nce: 3")
        _w(dev / "ras/gfx_err_count", "ue: 0\nce: 0")
        _w(dev / "ras/sdma_err_count", "ue: 0\nce: 0")
        _w(dev / "ras/gpu_vram_bad_pages", "")
        (dev / "gpu_metrics").write_bytes(encode_gpu_metrics_v18())
        hw = dev / "hwmon/hwmon3"
        _w(hw / "power1_average", 750_000_000)
        for i, (label, t) in enumerate((("edge", 45000), ("junction", 61000), ("mem", 52000)), start=1):
            _w(hw / f"temp{i}_label", label)
            _w(hw / f"temp{i}_input", t)
        (dev / "drm" / f"card{g}").mkdir(parents=True, exist_ok=True)
        (dev / "drm" / f"renderD{128 + g}").mkdir(parents=True, exist_ok=True)
        drv_dir = root / "sys/bus/pci/drivers" / ("vfio-pci" if vfio_bound else driver)
        drv_dir.mkdir(parents=True, exist_ok=True)
        link = dev / "driver"
        if link.is_symlink() or link.exists():
            link.unlink()
        os.symlink(os.path.relpath(drv_dir, dev), link)
        grp = root / "sys/kernel/iommu_groups" / str(10 + g)
        grp.mkdir(parents=True, exist_ok=True)
        ig = dev / "iommu_group"
        if not ig.exists():
            os.symlink(os.path.relpath(grp, dev), ig)
        _group_member(grp, dev)
        if companion_audio:
            # a second endpoint in the GPU's IOMMU group (HD-audio class), bound to snd_hda_intel
            adev = root / "sys/bus/pci/devices" / f"0000:{bus:02x}:00.1"
            _w(adev / "vendor", "0x1002")
            _w(adev / "device", "0xab38")
            _w(adev / "class", "0x040300")
            adrv = root / "sys/bus/pci/drivers/snd_hda_intel"
            adrv.mkdir(parents=True, exist_ok=True)
            if not (adev / "driver").is_symlink():
                os.symlink(os.path.relpath(adrv, adev), adev / "driver")
            if not (adev / "iommu_group").exists():
                os.symlink(os.path.relpath(grp, adev), adev / "iommu_group")
            _group_member(grp, adev)
        if sriov_totalvfs:
            _w(dev / "sriov_totalvfs", sriov_totalvfs)
            _w(dev / "sriov_numvfs", 0)
        for p in range(nparts):
            nd = topo / str(node)
            _props(nd / "properties", {
                "cpu_cores_count": 0, "simd_count": cus * 4, "mem_banks_count": 1,
                "simd_per_cu": 4, "max_waves_per_simd": 8, "lds_size_in_kb": 160,
                "gfx_target_version": GFX950, "vendor_id": 0x1002, "device_id": device_id,
                "location_id": bus << 8, "domain": 0, "drm_render_minor": 128 + g * nparts + p,
                "unique_id": 0x1000_0000_0000_0000 + g * 16 + p, "num_xcc": PARTITION_XCDS[compute],
                "hive_id": hive_id,
            })
            _w(nd / "gpu_id", 40000 + node)
            if kfd:
                (root / "dev/dri").mkdir(parents=True, exist_ok=True)
                (root / "dev/dri" / f"renderD{128 + g * nparts + p}").write_text("")
            gpu_nodes.append(node)
            node += 1
    # io links: every GPU agent has a PCIe link to the CPU and xGMI links to every GPU agent
    # of the other physical GPUs (fully connected 8-GPU mesh)
    for i, a in enumerate(gpu_nodes):
        links = [(2, 0, 20)]
        for j, b in enumerate(gpu_nodes):
            if a != b and (i // nparts) != (j // nparts):
                links.append((11, b, 15))
        for li, (t, to, w) in enumerate(links):
            _props(topo / str(a) / "io_links" / str(li) / "properties",
                   {"type": t, "node_from": a, "node_to": to, "weight": w,
                    "min_bandwidth": 50000 if t == 11 else 32000, "max_bandwidth": 153000 if t == 11 else 64000})
    return root


def _bdf_of(root, gpu: int) -> str:
    return f"0000:{0x05 + 0x10 * gpu:02x}:00.0"       # make_node's numbering


def set_ras(root, gpu: int, block: str = "umc", ue: int = 0, ce: int = 0) -> None:
    """The RAS error counts of one block of GPU ``gpu`` (ras/<block>_err_count)."""
    _w(Path(root) / "sys/bus/pci/devices" / _bdf_of(root, gpu) / f"ras/{block}_err_count", f"ue: {ue}\nce: {ce}")


def add_bad_pages(root, gpu: int, n: int, flag: str = "R") -> None:
    """Append ``n`` entries to GPU ``gpu``'s ras/gpu_vram_bad_pages (R retired, P pending, F failed)."""
    p = Path(root) / "sys/bus/pci/devices" / _bdf_of(root, gpu) / "ras/gpu_vram_bad_pages"
    old = p.read_text() if p.exists() else ""
    start = old.count("\n")
    rows = "".join(f"0x{0x1000 + start + i:08x} : 0x00001000 : {flag}\n" for i in range(n))
    p.write_text(old + rows)


def set_compute_partition(root, compute: str, memory: Optional[str] = None) -> None:
    """Re-enumerate the fake node as the driver does after a partition change."""
    import shutil
    root = Path(root)
    pci = root / "sys/bus/pci/devices"
    n = len([d for d in pci.iterdir()]) if pci.exists() else 8
    mem = memory or (root / "sys/bus/pci/devices").iterdir().__next__().joinpath(
        "current_memory_partition").read_text().strip()
    shutil.rmtree(root / "sys/class/kfd", ignore_errors=True)
    make_node(root, n_gpus=n, compute=compute, memory=mem)


MI355X_VF_DEVICE_ID = 0x75B3


def create_vfs(root, pf_bdf: str, n: int, driver: str = "", device_id: int = MI355X_VF_DEVICE_ID) -> list:
    """Instantiate ``n`` SR-IOV virtual functions of ``pf_bdf`` as the PF driver (GIM) does
    after a write to ``sriov_numvfs``: VF devices with ``physfn`` links, ``virtfn<i>`` links on
    the PF, own IOMMU groups; optionally pre-bound to ``driver``. Returns the VF BDFs."""
    root = Path(root)
    pci = root / "sys/bus/pci/devices"
    pf = pci / pf_bdf
    dom, bus, rest = pf_bdf.split(":")
    out = []
    for i in range(n):
        bdf = f"{dom}:{int(bus, 16) + 1:02x}:{i // 8:02x}.{i % 8}"
        vf = pci / bdf
        _w(vf / "vendor", "0x1002")
        _w(vf / "device", f"0x{device_id:04x}")
        _w(vf / "class", "0x120000")
        if not (vf / "physfn").is_symlink():
            os.symlink(os.path.relpath(pf, vf), vf / "physfn")
        link = pf / f"virtfn{i}"
        if not link.is_symlink():
            os.symlink(os.path.relpath(vf, pf), link)
        grp = root / "sys/kernel/iommu_groups" / str(100 + int(bus, 16) * 8 + i)
        grp.mkdir(parents=True, exist_ok=True)
        if not (vf / "iommu_group").is_symlink():
            os.symlink(os.path.relpath(grp, vf), vf / "iommu_group")
        if driver:
            drv_dir = root / "sys/bus/pci/drivers" / driver
            drv_dir.mkdir(parents=True, exist_ok=True)
            if (vf / "driver").is_symlink():
                (vf / "driver").unlink()
            os.symlink(os.path.relpath(drv_dir, vf), vf / "driver")
        out.append(bdf)
    _w(pf / "sriov_numvfs", n)
    return out


def remove_vfs(root, pf_bdf: str) -> None:
    import shutil
    root = Path(root)
    pci = root / "sys/bus/pci/devices"
    pf = pci / pf_bdf
    for link in sorted(pf.glob("virtfn*")):
        vf = (pf / os.readlink(link)).resolve()
        shutil.rmtree(vf, ignore_errors=True)
        link.unlink()
    _w(pf / "sriov_numvfs", 0)


def bind_driver(root, bdf: str, driver: str) -> None:
    """Re-point ``bdf``'s driver link (what a write to drivers/<drv>/bind does)."""
    root = Path(root)
    dev = root / "sys/bus/pci/devices" / bdf
    drv_dir = root / "sys/bus/pci/drivers" / driver
    drv_dir.mkdir(parents=True, exist_ok=True)
    if (dev / "driver").is_symlink():
        (dev / "driver").unlink()
    if driver:
        os.symlink(os.path.relpath(drv_dir, dev), dev / "driver")
