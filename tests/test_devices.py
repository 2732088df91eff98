"""libamdnode (native) against fake sysfs/KFD trees of an 8x MI355X node."""

import os
import subprocess
import threading
import time

import pytest

from gpu_operator_amd import devices as D
from gpu_operator_amd.devices import fakesys

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu_operator_amd", "_native", "bin")


@pytest.fixture
def node(tmp_path):
    return str(fakesys.make_node(tmp_path / "root"))


def test_enumerate_spx_node(node):
    gpus = D.enumerate_gpus(node)
    assert len(gpus) == 8
    g = gpus[0]
    assert g["gfx_target"] == "gfx950" and g["cu_count"] == 256 and g["lds_size_kib"] == 160
    assert g["vendor_id"] == 0x1002 and g["device_id"] == 0x75A3
    assert g["pci_bdf"] == "0000:05:00.0" and g["driver"] == "amdgpu"
    assert g["vram_total"] == 288 * (1 << 30)
    assert g["compute_partition"] == "SPX" and g["memory_partition"] == "NPS1"
    assert g["available_compute_partitions"] == ["SPX", "DPX", "QPX", "CPX"]
    assert g["partition_capable"] and g["xgmi_links"] == 7
    assert g["product_name"] == "AMD Instinct MI355X" and g["drm_card"] == 0
    assert D.single_hive(gpus)
    topo = D.xgmi_topology(gpus)
    assert topo[0] == [1, 2, 3, 4, 5, 6, 7]


def test_enumerate_cpx_node_has_64_partitions(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", compute="CPX"))
    gpus = D.enumerate_gpus(root)
    assert len(gpus) == 64
    assert {g["cu_count"] for g in gpus} == {32}
    assert {g["compute_partition"] for g in gpus} == {"CPX"}
    # partitions of one physical GPU share the PCI function
    assert len({g["pci_bdf"] for g in gpus}) == 8


def test_product_name_fallback_from_device_id(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=1, product=None, device_id=0x74A1))
    assert D.enumerate_gpus(root)[0]["product_name"] == "AMD Instinct MI300X"


def test_driver_state(node, tmp_path):
    s = D.driver_state(node, node)
    assert s == {"module_loaded": True, "live": True, "kfd_present": True, "version": "6.12.12",
                 "kfd_gpu_nodes": 8}
    empty = tmp_path / "empty"
    empty.mkdir()
    s = D.driver_state(str(empty), str(empty))
    assert not s["live"] and not s["kfd_present"] and s["kfd_gpu_nodes"] == 0


def test_scan_pci_and_vfio_binding(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=2, vfio_bound=True, sriov_totalvfs=8))
    fs = D.scan_pci(root)
    assert [f["bdf"] for f in fs] == ["0000:05:00.0", "0000:15:00.0"]
    assert all(f["driver"] == "vfio-pci" and f["sriov_totalvfs"] == 8 and f["iommu_group"] >= 10 for f in fs)


def test_telemetry(node):
    t = D.read_telemetry(node)[0]
    assert t["power_w"] == pytest.approx(750.0)
    assert (t["temp_edge_c"], t["temp_junction_c"], t["temp_mem_c"]) == (45.0, 61.0, 52.0)
    assert t["gpu_busy_pct"] == 37 and t["sclk_mhz"] == 2100 and t["mclk_mhz"] == 1900
    assert t["ecc_correctable"] == 3 and t["ecc_uncorrectable"] == 0


def test_set_partition_validates_modes(node):
    bdf = D.enumerate_gpus(node)[0]["pci_bdf"]
    D.set_partition(bdf, "compute", "cpx", root=node)
    assert D.enumerate_gpus(node)[0]["compute_partition"] == "CPX"
    with pytest.raises(ValueError, match="not in available_memory_partition"):
        D.set_partition(bdf, "memory", "NPS8", root=node)
    with pytest.raises(ValueError, match="no such PCI device"):
        D.set_partition("0000:ff:00.0", "compute", "SPX", root=node)


def test_wait_files_is_event_driven(tmp_path):
    d = tmp_path / "validations"
    d.mkdir()

    def writer():
        time.sleep(0.2)
        (d / "driver-ready").write_text("")
    threading.Thread(target=writer).start()
    t0 = time.monotonic()
    got = D.wait_files(str(d), ["driver-ready"], timeout=5)
    dt = time.monotonic() - t0
    assert got == ["driver-ready"] and 0.15 < dt < 1.0


def test_wait_files_any_all_and_timeout(tmp_path):
    d = tmp_path / "v"
    d.mkdir()
    (d / "host-driver-ready").write_text("")
    assert D.wait_files(str(d), ["driver-ready", "host-driver-ready"], any_of=True, timeout=1) == \
        ["host-driver-ready"]
    t0 = time.monotonic()
    assert D.wait_files(str(d), ["driver-ready", "host-driver-ready"], any_of=False, timeout=0.3) == []
    assert time.monotonic() - t0 >= 0.25


def test_wait_files_directory_created_later(tmp_path):
    d = tmp_path / "later"

    def writer():
        time.sleep(0.2)
        d.mkdir()
        time.sleep(0.1)
        (d / "toolkit-ready").write_text("")
    threading.Thread(target=writer).start()
    assert D.wait_files(str(d), ["toolkit-ready"], timeout=5) == ["toolkit-ready"]


def test_barrier_wait_cli(tmp_path):
    d = tmp_path / "v"
    d.mkdir()
    exe = os.path.join(BIN, "amd-barrier-wait")
    p = subprocess.Popen([exe, "--dir", str(d), "--all", "a,b", "--timeout", "10"], stdout=subprocess.PIPE, text=True)
    time.sleep(0.1)
    (d / "a").write_text("")
    time.sleep(0.1)
    (d / "b").write_text("")
    out, _ = p.communicate(timeout=10)
    assert p.returncode == 0 and "a b" in out
    r = subprocess.run([exe, "--dir", str(d), "--all", "zzz", "--timeout", "0"], capture_output=True)
    assert r.returncode == 1


def test_node_probe_cli(node):
    import json
    out = subprocess.run([os.path.join(BIN, "amd-node-probe"), "--root", node, "--dev-root", node],
                         capture_output=True, text=True, check=True).stdout
    j = json.loads(out)
    assert j["driver"]["live"] and len(j["gpus"]) == 8 and j["gpus"][3]["gfx"] == "gfx950"


def test_gpus_hidden_by_the_device_cgroup_still_count_as_xgmi_peers(tmp_path):
    """In a container that may access one GPU, KFD refuses to show the other GPU agents'
    properties (EPERM, read as empty). Their xGMI links are still physical GPU links: a GPU of an
    8-GPU hive reports 7, as on the MI355X box."""
    from pathlib import Path

    from gpu_operator_amd import devices as D
    from gpu_operator_amd.devices import fakesys

    root = fakesys.make_node(tmp_path, n_gpus=8)
    topo = Path(root) / "sys/class/kfd/kfd/topology/nodes"
    for n in range(2, 9):
        (topo / str(n) / "properties").write_text("")
    gpus = D.enumerate_gpus(str(root))
    assert len(gpus) == 1 and gpus[0]["xgmi_links"] == 7 and gpus[0]["pcie_links"] == 1
    from gpu_operator_amd.operands import node_labeller as NL
    assert NL.compute_labels(str(root))["amd.com/gpu.xgmi.links"] == "7"
