"""The node agents on a real MI355X node, read-only: device plugin discovery and Allocate, the
feature labeller, the metrics exporter (hwmon + PMFW gpu_metrics incl. per-link xGMI counters),
the partition manager's view of the partition modes, and the OCI runtime shim against the real
/dev/kfd and render nodes. Nothing here writes to sysfs or changes the GPU.

Reference bar: the e2e checks of tests/scripts/checks.sh:3-36 (operands up, GPU advertised).
"""

import json
import os
import stat
import subprocess
import time

import pytest

from gpu_operator_amd import devices as D

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "gpu_operator_amd", "_native", "bin", "amd-container-runtime")


@pytest.fixture(scope="module")
def gpus():
    g = D.enumerate_gpus("/")
    if not g:
        pytest.skip("no KFD GPU agent visible")
    return g


def _torch_cus():
    import torch

    return torch.cuda.get_device_properties(0).multi_processor_count


def test_kfd_agents_match_drm_render_nodes(gpus):
    for g in gpus:
        assert g["gfx_target"] == "gfx950" and g["driver"] == "amdgpu"
        node = f"/dev/dri/renderD{g['drm_render_minor']}"
        assert stat.S_ISCHR(os.stat(node).st_mode), node
        # the PCI device behind the render node is the one KFD reports
        real = os.path.realpath(f"/sys/class/drm/renderD{g['drm_render_minor']}/device")
        assert os.path.basename(real) == g["pci_bdf"]
    assert D.driver_state("/", "/")["live"] and D.driver_state("/", "/")["kfd_present"]


def test_device_plugin_discover_and_allocate(gpus, tmp_path):
    from gpu_operator_amd.operands import device_plugin as DP
    from gpu_operator_amd.operands import kubeletapi as K

    cfg = DP.Config()
    devs = DP.discover(cfg, "/")
    assert len(devs) == len(gpus) and all(d.resource == "amd.com/gpu" for d in devs)
    assert {d.render_minor for d in devs} == {g["drm_render_minor"] for g in gpus}
    assert all(d.id.startswith("amdgpu-") and d.healthy and d.partition == "SPX" for d in devs)
    plugin = DP.DevicePlugin(cfg, "/", plugin_dir=str(tmp_path))
    plugin.devices = devs
    srv = DP.ResourceServer("amd.com/gpu", plugin)
    req = K.DP["AllocateRequest"]()
    req.container_requests.add(devicesIDs=[devs[0].id])
    resp = srv.Allocate(req, None)
    paths = [d.host_path for d in resp.container_responses[0].devices]
    assert paths == ["/dev/kfd", f"/dev/dri/renderD{devs[0].render_minor}"]
    assert all(os.path.exists(p) for p in paths)
    assert resp.container_responses[0].envs["AMD_VISIBLE_DEVICES"] == devs[0].id
    # health check sees the live driver: nothing flips
    assert plugin.check_health() is False and all(d.healthy for d in plugin.devices)


def test_node_labeller_on_real_sysfs(gpus):
    from gpu_operator_amd.operands import node_labeller as NL

    lb = NL.compute_labels("/")
    assert lb["amd.com/gpu.gfx"] == "gfx950" and lb["amd.com/gpu.family"] == "cdna4"
    assert int(lb["amd.com/gpu.cu-count"]) == _torch_cus() == 256
    assert lb["amd.com/gpu.vram"] == "288G"                       # 288 GiB HBM3E per GPU
    assert lb["amd.com/gpu.lds-kib"] == "160"
    assert int(lb["amd.com/gpu.xgmi.hive-id"], 16) != 0
    assert lb["amd.com/gpu.xgmi.links"] == "7"                     # 8-GPU fully connected hive
    assert "MI355" in lb["amd.com/gpu.product"]
    assert lb["amd.com/gpu.compute-partition"] in ("SPX", "DPX", "QPX", "CPX")
    assert lb["amd.com/gpu.partition.capable"] == "true"
    assert all(len(v) <= 63 for v in lb.values())


def _scrape(reg):
    out = {}
    for fam in reg.collect():
        for s in fam.samples:
            out.setdefault(s.name, []).append((s.labels, s.value))
    return out


def test_metrics_exporter_scrape_on_real_hardware(gpus):
    from gpu_operator_amd.operands import metrics_exporter as ME

    reg = ME.build_registry(ME.load_fields(None), root="/", hostname="box")
    s1 = _scrape(reg)
    g0 = gpus[0]
    mine = lambda name: [v for lbl, v in s1.get(name, []) if lbl["bdf"] == g0["pci_bdf"]]  # noqa: E731
    assert mine("amd_gpu_power_watts")[0] > 50 or mine("amd_gpu_socket_power_watts")[0] > 50
    assert 10 < mine("amd_gpu_temperature_junction_celsius")[0] < 110
    with open(f"/sys/bus/pci/devices/{g0['pci_bdf']}/mem_info_vram_total") as f:
        assert mine("amd_gpu_vram_total_bytes")[0] == float(f.read())
    assert mine("amd_gpu_energy_joules_total")[0] > 0
    assert mine("amd_gpu_xgmi_link_speed_gbps")[0] > 0
    up = [v for lbl, v in s1["amd_gpu_xgmi_link_up"] if lbl["bdf"] == g0["pci_bdf"]]
    assert len(up) == 7 and all(v == 1 for v in up)
    rd = [v for lbl, v in s1["amd_gpu_xgmi_read_bytes_total"] if lbl["bdf"] == g0["pci_bdf"]]
    assert len(rd) == 7 and sum(rd) > 0                            # accumulated since boot
    time.sleep(1.2)                                                # PMFW table refreshes ~1 ms..1 s
    s2 = _scrape(reg)
    thr = [v for lbl, v in s2.get("amd_gpu_xgmi_read_throughput_bytes_per_second", [])
           if lbl["bdf"] == g0["pci_bdf"]]
    assert len(thr) == 7 and all(v >= 0 for v in thr)


def test_gpu_metrics_table_is_the_pinned_layout(gpus):
    ms = D.read_gpu_metrics("/")
    assert ms and all(m["valid"] for m in ms), [m["error"] for m in ms]
    for m in ms:
        assert (m["format_revision"], m["content_revision"]) == (1, 8)
        assert m["xgmi_link_width"] > 0 and m["pcie_link_width"] > 0
        assert sum(1 for s in m["xgmi_link_status"] if s == 1) == 7
        assert 0 < m["socket_power_w"] < 2000 and m["uclk_mhz"] > 0


def test_gpu_metrics_agrees_with_amdsmi(gpus):
    amdsmi = pytest.importorskip("amdsmi")
    amdsmi.amdsmi_init()
    try:
        by_bdf = {amdsmi.amdsmi_get_gpu_device_bdf(h): h for h in amdsmi.amdsmi_get_processor_handles()}
        for m in D.read_gpu_metrics("/"):
            h = by_bdf.get(m["pci_bdf"])
            if h is None:
                continue
            ref = amdsmi.amdsmi_get_gpu_metrics_info(h)
            assert m["xgmi_link_width"] == ref["xgmi_link_width"]
            assert m["xgmi_link_speed"] == ref["xgmi_link_speed"]
            assert m["pcie_link_width"] == ref["pcie_link_width"]
            for ours, theirs in zip(m["xgmi_read_kb"], ref["xgmi_read_data_acc"]):
                if theirs != "N/A":
                    assert ours <= theirs <= ours + (1 << 30)          # ours read first; counters only grow
    finally:
        amdsmi.amdsmi_shut_down()


def test_partition_manager_reads_real_modes_without_writing(gpus):
    from gpu_operator_amd.operands import partition_manager as PM

    phys = PM.physical_gpus("/")
    assert phys
    for g in phys:
        assert g["compute_partition"] in g["available_compute_partitions"]
        assert g["memory_partition"] in g["available_memory_partitions"]
        assert {"SPX", "CPX"} <= set(g["available_compute_partitions"])
        assert "NPS1" in g["available_memory_partitions"]
    want = PM.desired_layout([{"devices": "all", "compute": "SPX", "memory": "NPS1"}], len(phys))
    assert want == {i: ("SPX", "NPS1") for i in range(len(phys))}
    before = [(g["compute_partition"], g["memory_partition"]) for g in PM.physical_gpus("/")]
    assert before == [(g["compute_partition"], g["memory_partition"]) for g in phys]   # nothing written
    with pytest.raises(PM.PartitionError):
        PM.desired_layout([{"devices": [len(phys)], "compute": "CPX"}], len(phys))


def test_oci_shim_injects_real_device_nodes(gpus, tmp_path):
    b = tmp_path / "bundle"
    (b / "rootfs").mkdir(parents=True)
    spec = {"ociVersion": "1.1.0", "process": {"args": ["sh"], "env": ["PATH=/usr/bin", "AMD_VISIBLE_DEVICES=all"]},
            "root": {"path": "rootfs"}, "linux": {"resources": {"devices": [{"allow": False, "access": "rwm"}]}}}
    (b / "config.json").write_text(json.dumps(spec))
    env = dict(os.environ, AMD_CONTAINER_RUNTIME_RUNTIMES="/bin/echo", AMD_CONTAINER_RUNTIME_MODE="legacy",
               AMD_CONTAINER_RUNTIME_CDI_SPEC_DIRS="/nonexistent")
    p = subprocess.run([SHIM, "create", "--bundle", str(b), "c1"], capture_output=True, text=True, env=env,
                       timeout=30)
    assert p.returncode == 0, p.stderr
    out = json.loads((b / "config.json").read_text())
    devs = {d["path"]: d for d in out["linux"]["devices"]}
    want = ["/dev/kfd"] + [f"/dev/dri/renderD{g['drm_render_minor']}" for g in gpus]
    assert sorted(devs) == sorted(want)
    for path, d in devs.items():
        st = os.stat(path)
        assert (d["type"], d["major"], d["minor"]) == ("c", os.major(st.st_rdev), os.minor(st.st_rdev)), path
    rules = out["linux"]["resources"]["devices"]
    assert rules[0] == {"allow": False, "access": "rwm"} and len(rules) == 1 + len(want)


def test_node_probe_reports_the_hive(gpus):
    p = subprocess.run([os.path.join(ROOT, "gpu_operator_amd", "_native", "bin", "amd-node-probe")],
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    j = json.loads(p.stdout.splitlines()[0])
    g = [x for x in j["gpus"] if x["gfx"] == "gfx950"][0]
    assert g["xgmi_links"] == 7 and g["xgmi_hive_id"] != 0


def _other_kfd_clients():
    """PIDs other than this one holding /dev/kfd open (readable /proc entries only)."""
    me, out = os.getpid(), []
    for pid in os.listdir("/proc"):
        if not pid.isdigit() or int(pid) == me:
            continue
        try:
            for fd in os.listdir(f"/proc/{pid}/fd"):
                if os.readlink(f"/proc/{pid}/fd/{fd}") == "/dev/kfd":
                    out.append(int(pid))
                    break
        except OSError:
            continue
    return out


def test_partition_round_trip_spx_cpx_spx(gpus, tmp_path):
    """SPX -> CPX -> SPX on the leased GPU through the partition manager (BASELINE config 5,
    reference assets/state-mig-manager/0600_daemonset.yaml:26-104). Runs only where the compute
    partition is writable and no other process has the GPU open; NPS is never touched on a shared
    box. Asserts KFD agents 1 -> 8 -> 1, the device plugin's 8 partition devices with their
    sysfs VRAM, and the labeller's compute-partition label."""
    from gpu_operator_amd.k8s.fake import FakeClient
    from gpu_operator_amd.operands import device_plugin as DP
    from gpu_operator_amd.operands import node_labeller as NL
    from gpu_operator_amd.operands import partition_manager as PM

    phys = PM.physical_gpus("/")
    g0 = phys[0]
    attr = f"/sys/bus/pci/devices/{g0['pci_bdf']}/current_compute_partition"
    if not os.path.exists(attr) or not os.access(attr, os.W_OK):
        pytest.skip(f"{attr} is not writable by this user (partition changes need root on the node)")
    if g0["compute_partition"] != "SPX" or "CPX" not in g0["available_compute_partitions"]:
        pytest.skip(f"GPU is in {g0['compute_partition']}, CPX available: {g0['available_compute_partitions']}")
    others = _other_kfd_clients()
    if others:
        pytest.skip(f"other KFD clients hold the GPU: {others[:8]}")
    cfg = tmp_path / "config.yaml"
    cfg.write_text("version: v1\npartition-configs:\n"
                   "  spx: [{devices: all, compute: SPX, memory: " + g0["memory_partition"] + "}]\n"
                   "  cpx: [{devices: all, compute: CPX, memory: " + g0["memory_partition"] + "}]\n")
    node = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n", "labels": {}}}
    c = FakeClient([node])
    pm = PM.PartitionManager(c, "n", str(cfg), root="/", barrier_dir=str(tmp_path / "v"), enum_timeout=120)
    agents0 = len(D.enumerate_gpus("/"))
    try:
        c.patch("v1", "Node", "n", {"metadata": {"labels": {PM.CONFIG_LABEL: "cpx"}}})
        assert pm.reconcile() == "applied"
        cpx = D.enumerate_gpus("/")
        assert len(cpx) == agents0 - 1 + 8
        devs = [d for d in DP.discover(DP.Config(), "/") if d.bdf == g0["pci_bdf"]]
        assert len(devs) == 8 and {d.partition for d in devs} == {"CPX"}
        sysfs_vram = {g["index"]: g["vram_total"] for g in cpx if g["pci_bdf"] == g0["pci_bdf"]}
        assert all(d.vram_bytes > 0 for d in devs) and sorted(d.vram_bytes for d in devs) == sorted(sysfs_vram.values())
        assert NL.compute_labels("/")["amd.com/gpu.compute-partition"] == "CPX"
    finally:
        c.patch("v1", "Node", "n", {"metadata": {"labels": {PM.CONFIG_LABEL: "spx"}}})
        assert pm.reconcile() in ("applied", "in-sync")
    assert len(D.enumerate_gpus("/")) == agents0
    assert NL.compute_labels("/")["amd.com/gpu.compute-partition"] == "SPX"
