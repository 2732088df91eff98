"""Node labeller, partition manager and metrics exporter against fake MI355X sysfs trees."""

import json
import os
import threading
import time

import pytest
import yaml

from gpu_operator_amd import devices as D
from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.operands import metrics_exporter as me
from gpu_operator_amd.operands import node_labeller as nl
from gpu_operator_amd.operands import partition_manager as pm

from k8s_helpers import gpu_node


@pytest.fixture
def spx(tmp_path):
    return str(fakesys.make_node(tmp_path / "root"))


# -- node labeller ---------------------------------------------------------------------------------

def test_labels_spx(spx):
    L = nl.compute_labels(spx)
    assert L["amd.com/gpu.product"] == "AMD-Instinct-MI355X"
    assert L["amd.com/gpu.family"] == "cdna4" and L["amd.com/gpu.gfx"] == "gfx950"
    assert L["amd.com/gpu.device-id"] == "75a3"
    assert L["amd.com/gpu.count"] == "8" and L["amd.com/gpu.partition.count"] == "8"
    assert L["amd.com/gpu.cu-count"] == "256" and L["amd.com/gpu.lds-kib"] == "160"
    assert L["amd.com/gpu.vram"] == "288G"
    assert L["amd.com/gpu.compute-partition"] == "SPX" and L["amd.com/gpu.memory-partition"] == "NPS1"
    assert L["amd.com/gpu.xgmi.links"] == "7" and L["amd.com/gpu.xgmi.fully-connected"] == "true"
    assert L["amd.com/gpu.numa-nodes"] == "2" and L["amd.com/gpu.driver-version"] == "6.12.12"
    assert L["amd.com/gpu.partition.capable"] == "true"
    for k, v in L.items():
        assert len(v) <= 63 and nl.OWNED.match(k), k


def test_labels_cpx(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", compute="CPX", memory="NPS2"))
    L = nl.compute_labels(root)
    assert L["amd.com/gpu.count"] == "8" and L["amd.com/gpu.partition.count"] == "64"
    assert L["amd.com/gpu.cu-count"] == "256"          # per physical GPU, not per partition
    assert L["amd.com/gpu.compute-partition"] == "CPX" and L["amd.com/gpu.memory-partition"] == "NPS2"
    assert L["amd.com/gpu.xgmi.links"] == "7"


def test_labels_no_gpu(tmp_path):
    os.makedirs(tmp_path / "empty")
    assert nl.compute_labels(str(tmp_path / "empty")) == {}


def test_label_patch_removes_stale_owned_only():
    cur = {"amd.com/gpu.product": "x", "amd.com/gpu.vram": "1G", "amd.com/gpu.present": "true", "foo": "bar"}
    want = {"amd.com/gpu.product": "x"}
    assert nl.label_patch(cur, want) == {"amd.com/gpu.vram": None}


def test_apply_node_and_nfd(spx, tmp_path):
    c = FakeClient([gpu_node("n1", extra_labels={"amd.com/gpu.vram": "1G"})])
    want = nl.compute_labels(spx)
    patch = nl.apply_node(c, "n1", want)
    assert patch["amd.com/gpu.vram"] == "288G"
    labels = o.get_labels(c.get("v1", "Node", "n1"))
    assert all(labels[k] == v for k, v in want.items())
    assert nl.apply_node(c, "n1", want) == {}                    # idempotent
    f = tmp_path / "features.d" / "amd-gpu"
    nl.write_nfd(str(f), want)
    lines = f.read_text().splitlines()
    assert "amd.com/gpu.gfx=gfx950" in lines and len(lines) == len(want)


def test_labeller_main_oneshot_nfd(spx, tmp_path, monkeypatch):
    monkeypatch.setenv("AMD_SYSFS_ROOT", spx)
    f = tmp_path / "out" / "amd-gpu"
    assert nl.main(["--oneshot", "--output", "nfd", "--nfd-file", str(f)]) == 0
    assert "amd.com/gpu.family=cdna4" in f.read_text()


def test_wait_for_change_wakes_on_barrier(tmp_path):
    d = tmp_path / "validations"
    d.mkdir()
    path = d / "partition-applied"
    stop = threading.Event()
    t0 = time.monotonic()
    threading.Timer(0.3, lambda: path.write_text("{}")).start()
    assert nl.wait_for_change(str(path), 10.0, stop)
    assert time.monotonic() - t0 < 5.0
    assert not nl.wait_for_change(str(path), 1.0, stop)           # exists, unchanged -> period expires


def test_parse_duration():
    assert nl.parse_duration("60s") == 60 and nl.parse_duration("2m") == 120
    assert nl.parse_duration("500ms") == 0.5 and nl.parse_duration("5") == 5
    with pytest.raises(ValueError):
        nl.parse_duration("soon")


# -- partition manager -----------------------------------------------------------------------------

CONFIG = {"version": "v1", "partition-configs": {
    "all-spx": [{"devices": "all", "compute": "SPX", "memory": "NPS1"}],
    "all-cpx": [{"devices": "all", "compute": "CPX", "memory": "NPS2"}],
    "bad-mode": [{"devices": "all", "compute": "XPX"}],
    "bad-dev": [{"devices": [9], "compute": "CPX"}],
    "unavailable": [{"devices": "all", "compute": "CPX", "memory": "NPS4"}],
}}


@pytest.fixture
def cfg(tmp_path):
    p = tmp_path / "config.yaml"
    p.write_text(yaml.safe_dump(CONFIG))
    return str(p)


def _cluster(config_label=None):
    extra = {"amd.com/gpu.deploy.device-plugin": "true", "amd.com/gpu.deploy.metrics-exporter": "true",
             "amd.com/gpu.deploy.rdc": "false"}
    if config_label:
        extra[pm.CONFIG_LABEL] = config_label
    return FakeClient([gpu_node("n1", extra_labels=extra)])


def _mgr(c, spx, cfg, tmp_path, **kw):
    kw.setdefault("reload_driver", lambda: None)        # the fake driver applies NPS writes at once
    return pm.PartitionManager(c, "n1", cfg, root=spx, barrier_dir=str(tmp_path / "barriers"),
                               enum_timeout=3.0, pods_timeout=3.0, reload_timeout=3.0, **kw)


def test_desired_layout():
    assert pm.desired_layout(CONFIG["partition-configs"]["all-cpx"], 2) == {0: ("CPX", "NPS2"), 1: ("CPX", "NPS2")}
    with pytest.raises(pm.PartitionError):
        pm.desired_layout(CONFIG["partition-configs"]["bad-mode"], 8)
    with pytest.raises(pm.PartitionError):
        pm.desired_layout(CONFIG["partition-configs"]["bad-dev"], 8)


def test_partition_in_sync_marks_success(spx, cfg, tmp_path):
    c = _cluster("all-spx")
    assert _mgr(c, spx, cfg, tmp_path).reconcile() == "in-sync"
    n = c.get("v1", "Node", "n1")
    assert o.get_labels(n)[pm.STATE_LABEL] == "success"
    assert o.get_annotations(n)[pm.APPLIED_ANNOTATION] == "all-spx"
    assert (tmp_path / "barriers" / "partition-applied").exists()


def test_partition_no_config(spx, cfg, tmp_path):
    assert _mgr(_cluster(), spx, cfg, tmp_path).reconcile() == "no-config"


def test_partition_apply_cpx(spx, cfg, tmp_path):
    c = _cluster("all-cpx")
    seen = []

    def on_node(ev):
        seen.append(dict(o.get_labels(ev.obj)))
    c.watch("v1", "Node", on_node)
    m = _mgr(c, spx, cfg, tmp_path, reenumerate=lambda: fakesys.set_compute_partition(spx, "CPX", "NPS2"))
    assert m.reconcile() == "applied"
    gpus = D.enumerate_gpus(spx)
    assert len(gpus) == 64 and {g["compute_partition"] for g in gpus} == {"CPX"}
    assert {g["memory_partition"] for g in gpus} == {"NPS2"}
    labels = o.get_labels(c.get("v1", "Node", "n1"))
    assert labels[pm.STATE_LABEL] == "success"
    # clients were paused during the change and restored afterwards; disabled ones untouched
    assert any(s.get("amd.com/gpu.deploy.device-plugin") == pm.PAUSED for s in seen)
    assert any(s.get(pm.STATE_LABEL) == "pending" for s in seen)
    assert labels["amd.com/gpu.deploy.device-plugin"] == "true"
    assert labels["amd.com/gpu.deploy.metrics-exporter"] == "true"
    assert labels["amd.com/gpu.deploy.rdc"] == "false"
    # second pass is a no-op
    assert m.reconcile() == "in-sync"


def test_partition_waits_for_client_pods(spx, cfg, tmp_path):
    c = _cluster("all-cpx")
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "dp-1", "namespace": "gpu",
                                                               "labels": {"app": "amd-device-plugin-daemonset"}},
              "spec": {"nodeName": "n1"}})
    threading.Timer(0.5, lambda: c.delete("v1", "Pod", "dp-1", "gpu")).start()
    m = _mgr(c, spx, cfg, tmp_path, reenumerate=lambda: fakesys.set_compute_partition(spx, "CPX", "NPS2"))
    assert m.reconcile() == "applied"


def test_partition_failures(spx, cfg, tmp_path):
    for name in ("missing-config", "bad-mode", "unavailable"):
        c = _cluster(name)
        assert _mgr(c, spx, cfg, tmp_path).reconcile() == "failed", name
        assert o.get_labels(c.get("v1", "Node", "n1"))[pm.STATE_LABEL] == "failed"
        assert any(e["reason"] == "PartitionFailed" for e in c.events)
        # deploy labels restored even on failure
        assert o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.deploy.device-plugin"] == "true"


def test_partition_reenumeration_timeout(spx, cfg, tmp_path):
    c = _cluster("all-cpx")
    m = _mgr(c, spx, cfg, tmp_path)
    m.enum_timeout = 0.5
    assert m.reconcile() == "failed"                              # driver never re-enumerated
    ev = [e for e in c.events if e["reason"] == "PartitionFailed"]
    assert "re-enumeration" in ev[0]["message"]


def test_partition_host_services(spx, cfg, tmp_path):
    calls = []
    c = _cluster("all-cpx")
    m = _mgr(c, spx, cfg, tmp_path, host_services=["amd-smi-exporter"],
             run=lambda argv, **kw: calls.append(argv[-2:]),
             reenumerate=lambda: fakesys.set_compute_partition(spx, "CPX", "NPS2"))
    assert m.reconcile() == "applied"
    assert calls == [["stop", "amd-smi-exporter"], ["start", "amd-smi-exporter"]]


def test_partition_client_pod_that_never_exits_restores_labels(spx, cfg, tmp_path):
    """a timed-out wait for a client pod must still restore the paused deploy labels."""
    c = _cluster("all-cpx")
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "dp-stuck", "namespace": "gpu",
                                                               "labels": {"app": "amd-device-plugin-daemonset"}},
              "spec": {"nodeName": "n1"}})
    m = _mgr(c, spx, cfg, tmp_path)
    m.pods_timeout = 0.3
    assert m.reconcile() == "failed"
    labels = o.get_labels(c.get("v1", "Node", "n1"))
    assert labels["amd.com/gpu.deploy.device-plugin"] == "true"
    assert labels["amd.com/gpu.deploy.metrics-exporter"] == "true"
    assert labels["amd.com/gpu.deploy.rdc"] == "false"
    assert "still running" in [e for e in c.events if e["reason"] == "PartitionFailed"][0]["message"]


def test_partition_restores_labels_a_crashed_run_left_paused(spx, cfg, tmp_path):
    c = _cluster("all-spx")
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.deploy.device-plugin": pm.PAUSED}}})
    assert _mgr(c, spx, cfg, tmp_path).reconcile() == "in-sync"
    assert o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.deploy.device-plugin"] == "true"


def test_partition_nps_change_reloads_the_driver(spx, cfg, tmp_path):
    """NPS1 -> NPS2: memory modes written, then amdgpu reloaded (reload-required -> reloading),
    then the compute modes, then re-enumeration; clients paused throughout and restored."""
    c = _cluster("all-cpx")
    order, states = [], []
    c.watch("v1", "Node", lambda ev: states.append(o.get_labels(ev.obj).get(pm.STATE_LABEL)))
    real_set = D.set_partition

    def spy_set(bdf, kind, mode, root=None):
        order.append(kind)
        real_set(bdf, kind, mode, root=root)

    def reload():
        order.append("reload")
        dp = o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.deploy.device-plugin"]
        assert dp == pm.PAUSED                         # no GPU client across the reload
    import unittest.mock as um
    with um.patch.object(pm.devices, "set_partition", spy_set):
        m = _mgr(c, spx, cfg, tmp_path, reload_driver=reload,
                 reenumerate=lambda: fakesys.set_compute_partition(spx, "CPX", "NPS2"))
        assert m.reconcile() == "applied"
    assert order.index("reload") > max(i for i, k in enumerate(order) if k == "memory")
    assert order.index("reload") < min(i for i, k in enumerate(order) if k == "compute")
    assert order.count("reload") == 1 and order.count("memory") == 8
    seen = [s for i, s in enumerate(states) if s and (i == 0 or states[i - 1] != s)]
    assert seen[:4] == ["pending", "reload-required", "reloading", "success"], seen
    assert o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.deploy.device-plugin"] == "true"


def test_partition_compute_only_change_needs_no_reload(spx, cfg, tmp_path):
    cfgd = yaml.safe_load(open(cfg))
    cfgd["partition-configs"]["cpx-nps1"] = [{"devices": "all", "compute": "CPX", "memory": "NPS1"}]
    open(cfg, "w").write(yaml.safe_dump(cfgd))
    reloads = []
    m = _mgr(_cluster("cpx-nps1"), spx, cfg, tmp_path, reload_driver=lambda: reloads.append(1),
             reenumerate=lambda: fakesys.set_compute_partition(spx, "CPX", "NPS1"))
    assert m.reconcile() == "applied" and reloads == []


def test_partition_reload_failure_fails_and_restores_clients(spx, cfg, tmp_path):
    c = _cluster("all-cpx")
    calls = []

    def run(argv, **kw):
        calls.append(argv)
        import subprocess as sp
        return sp.CompletedProcess(argv, 1 if "-r" in argv else 0, "", "modprobe: FATAL: Module amdgpu is in use.")
    m = _mgr(c, spx, cfg, tmp_path, run=run)
    m.reload_driver = m._reload_driver                   # the real modprobe sequence, faked run()
    assert m.reconcile() == "failed"
    assert calls[0] == ["chroot", "/host", "modprobe", "-r", "amdgpu"] and len(calls) == 1
    labels = o.get_labels(c.get("v1", "Node", "n1"))
    assert labels[pm.STATE_LABEL] == "failed" and labels["amd.com/gpu.deploy.device-plugin"] == "true"
    msg = [e for e in c.events if e["reason"] == "PartitionFailed"][0]["message"]
    assert "in use" in msg and "modprobe -r amdgpu" in msg


def test_partition_reload_cmd_override(spx, cfg, tmp_path):
    calls = []
    import subprocess as sp
    m = _mgr(_cluster("all-cpx"), spx, cfg, tmp_path, run=lambda argv, **kw: (calls.append(argv),
                                                                             sp.CompletedProcess(argv, 0))[1],
             reload_cmd="chroot /host /usr/local/bin/amdgpu-reload --nps; true",
             reenumerate=lambda: fakesys.set_compute_partition(spx, "CPX", "NPS2"))
    m.reload_driver = m._reload_driver
    assert m.reconcile() == "applied"
    assert calls == [["chroot", "/host", "/usr/local/bin/amdgpu-reload", "--nps"], ["true"]]


def test_partition_driver_not_live_after_reload_fails(spx, cfg, tmp_path):
    from pathlib import Path
    c = _cluster("all-cpx")

    def reload_broken():
        (Path(spx) / "sys/module/amdgpu/initstate").write_text("coming\n")
    m = _mgr(c, spx, cfg, tmp_path, reload_driver=reload_broken)
    m.reload_timeout = 0.5
    assert m.reconcile() == "failed"
    assert "did not come back live" in [e for e in c.events if e["reason"] == "PartitionFailed"][0]["message"]
    assert o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.deploy.device-plugin"] == "true"


# -- metrics exporter ------------------------------------------------------------------------------

def test_metrics_registry(spx):
    from prometheus_client import generate_latest
    reg = me.build_registry(me.load_fields(None), root=spx, hostname="n1")
    text = generate_latest(reg).decode()
    assert 'amd_gpu_power_watts{bdf="0000:05:00.0"' in text
    assert "amd_gpu_temperature_junction_celsius" in text
    assert "amd_gpu_ecc_correctable_total" in text
    samples = {(s.name, s.labels["gpu"]): s.value for m in reg.collect() for s in m.samples}
    assert samples[("amd_gpu_power_watts", "0")] == pytest.approx(750.0)
    assert samples[("amd_gpu_temperature_junction_celsius", "3")] == pytest.approx(61.0)
    assert samples[("amd_gpu_utilization_percent", "7")] == 37
    assert samples[("amd_gpu_ecc_correctable_total", "0")] == 3
    assert samples[("amd_gpu_vram_total_bytes", "0")] == 288 * (1 << 30)
    assert samples[("amd_gpu_xgmi_link_count", "0")] == 7


def test_metrics_field_file(spx, tmp_path):
    f = tmp_path / "fields.csv"
    f.write_text("# comment\ngpu_power_watts, gauge\nnot_a_field\n")
    assert me.load_fields(str(f)) == ["gpu_power_watts"]
    reg = me.build_registry(me.load_fields(str(f)), root=spx)
    assert [m.name for m in reg.collect()] == ["amd_gpu_power_watts"]


def test_metrics_pod_attribution(spx, tmp_path):
    import grpc
    from concurrent import futures
    from gpu_operator_amd.operands import kubeletapi as K
    gpus = D.enumerate_gpus(spx)
    did = f"amdgpu-{gpus[2]['unique_id']:016x}"

    def list_fn(req, ctx):
        r = K.PR["ListPodResourcesResponse"]()
        p = r.pod_resources.add(name="train-0", namespace="ml")
        cnt = p.containers.add(name="worker")
        cnt.devices.add(resource_name="amd.com/gpu", device_ids=[did])
        cnt.devices.add(resource_name="example.com/nic", device_ids=["x"])
        return r
    sock = str(tmp_path / "pr.sock")
    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
    srv.add_generic_rpc_handlers((K.pod_resources_handler(list_fn),))
    srv.add_insecure_port("unix://" + sock)
    srv.start()
    try:
        assert me.pod_attribution(sock) == {did: ("ml", "train-0", "worker")}
        reg = me.build_registry(["gpu_power_watts"], root=spx, kubernetes=True, pod_socket=sock)
        s = {x.labels["gpu"]: x.labels for m in reg.collect() for x in m.samples}
        assert s["2"]["pod"] == "train-0" and s["2"]["namespace"] == "ml" and s["0"]["pod"] == ""
    finally:
        srv.stop(0)


def test_labeller_sharing_labels_follow_advertised_replicas(spx):
    """GFD's gpu.replicas / sharing-strategy / product -SHARED, read from what the device plugin
    advertises (allocatable amd.com/gpu over the partition count)."""
    want = nl.compute_labels(spx)
    parts = int(want["amd.com/gpu.partition.count"])
    node = lambda n: {"status": {"allocatable": {"amd.com/gpu": str(n)}}}  # noqa: E731
    assert nl.sharing_labels({"status": {}}, want) == {}                    # plugin not registered yet
    assert nl.sharing_labels(node(parts), want) == {"amd.com/gpu.replicas": "1",
                                                     "amd.com/gpu.sharing-strategy": "none"}
    s = nl.sharing_labels(node(parts * 10), want)
    assert s["amd.com/gpu.replicas"] == "10" and s["amd.com/gpu.sharing-strategy"] == "time-slicing"
    assert s["amd.com/gpu.product"].endswith("-SHARED")
    # both labels are owned: dropping sharing removes/reverts them
    assert nl.OWNED.match("amd.com/gpu.replicas") and nl.OWNED.match("amd.com/gpu.sharing-strategy")


def test_config_manager_finds_the_plugin_under_any_launcher(tmp_path):
    from gpu_operator_amd.operands import config_manager as cm
    proc = tmp_path / "proc"
    for pid, argv in {"11": ["/usr/bin/python3", "/usr/local/bin/amd-device-plugin", "--x"],
                      "12": ["amd-device-plugin"],
                      "13": ["/usr/bin/python3", "-m", "gpu_operator_amd.cmd.entry", "amd-device-plugin"],
                      "14": ["/bin/sh", "-c", "/bin/entrypoint.sh"],
                      "15": ["/usr/bin/python3", "-m", "gpu_operator_amd.cmd.entry", "amd-node-labeller"]}.items():
        (proc / pid).mkdir(parents=True)
        (proc / pid / "cmdline").write_bytes(b"\0".join(a.encode() for a in argv) + b"\0")
    assert sorted(cm.find_pids("amd-device-plugin", str(proc))) == [11, 12, 13]


def test_partition_nps_change_reloads_through_the_driver_container(spx, cfg, tmp_path):
    """with driver.enabled the partition manager asks the driver container (the
    only holder of the module tree that loaded amdgpu) through /run/amd/driver/reload-request; the
    container rmmods its precompiled modules, insmods them again, rewrites .driver-ctr and answers
    reload-result. The NPS change then completes (state success)."""
    import shutil
    import threading
    from pathlib import Path
    from gpu_operator_amd.operands import driver_container as dcm
    kernel = "6.8.0-45-generic"
    img = tmp_path / "image"
    d = img / "opt/amdgpu/precompiled" / kernel
    d.mkdir(parents=True)
    for m in ("amdgpu", "amdxcp", "amdttm", "amdkcl"):
        (d / f"{m}.ko.xz").write_text("x")
    root = Path(spx)
    for m in ("amdxcp", "amdttm", "amdkcl"):
        (root / "sys/module" / m).mkdir(parents=True, exist_ok=True)
    calls = []

    def run(argv, **kw):
        import subprocess as sp
        calls.append([argv[0], dcm._mod_name(argv[1])])
        mod = root / "sys/module" / dcm._mod_name(argv[1])
        if argv[0] == "rmmod":
            shutil.rmtree(mod, ignore_errors=True)
        elif argv[0] == "insmod":
            mod.mkdir(parents=True, exist_ok=True)
            if dcm._mod_name(argv[1]) == "amdgpu":       # the module comes back in the new NPS mode
                (mod / "initstate").write_text("live\n")
                fakesys.set_compute_partition(spx, "SPX", "NPS2")
        return sp.CompletedProcess(argv, 0, "", "")
    run_dir = tmp_path / "run"
    dc = dcm.DriverContainer(sys_root=spx, dev_root=spx, image_root=str(img), host_etc=str(tmp_path / "etc"),
                             run_dir=str(run_dir), firmware_dir=str(tmp_path / "fw"),
                             params_file=str(tmp_path / "none.conf"), kernel=kernel, run=run, ready_timeout=3.0)
    dc._write_marker({"mode": "precompiled"})
    stop = threading.Event()
    t = threading.Thread(target=dc.serve_reloads, args=(stop, 0.2), daemon=True)
    t.start()
    try:
        c = _cluster("all-cpx")
        m = pm.PartitionManager(c, "n1", cfg, root=spx, barrier_dir=str(tmp_path / "barriers"), enum_timeout=3.0,
                                pods_timeout=3.0, reload_timeout=5.0, reload_via="driver-container",
                                driver_dir=str(run_dir / "driver"),
                                reenumerate=lambda: fakesys.set_compute_partition(spx, "CPX", "NPS2"))
        assert m.reconcile() == "applied"
    finally:
        stop.set()
        t.join(5)
    assert calls[:4] == [["rmmod", "amdgpu"], ["rmmod", "amdxcp"], ["rmmod", "amdttm"], ["rmmod", "amdkcl"]]
    assert [c[1] for c in calls[4:]] == ["amdkcl", "amdttm", "amdxcp", "amdgpu"]
    res = json.loads((run_dir / "driver" / dcm.RELOAD_RESULT).read_text())
    assert res["ok"] and res["info"]["unloaded"][0] == "amdgpu"
    assert json.loads((run_dir / "driver/.driver-ctr").read_text())["reload_s"] >= 0
    assert o.get_labels(c.get("v1", "Node", "n1"))[pm.STATE_LABEL] == "success"


def test_partition_driver_container_reload_timeout_fails(spx, cfg, tmp_path):
    c = _cluster("all-cpx")
    m = pm.PartitionManager(c, "n1", cfg, root=spx, barrier_dir=str(tmp_path / "b"), enum_timeout=1.0,
                            pods_timeout=1.0, reload_timeout=0.5, reload_via="driver-container",
                            driver_dir=str(tmp_path / "driver"))
    assert m.reconcile() == "failed"
    msg = [e for e in c.events if e["reason"] == "PartitionFailed"][0]["message"]
    assert "did not answer reload request" in msg
    # the unanswered request is withdrawn -- a driver container starting later must not
    # unload amdgpu for it
    assert not (tmp_path / "driver" / "reload-request").exists()


def _driver_container(tmp_path, spx, run, **kw):
    from gpu_operator_amd.operands import driver_container as dcm
    return dcm.DriverContainer(sys_root=spx, dev_root=spx, image_root=str(tmp_path / "image"),
                               host_etc=str(tmp_path / "etc"), run_dir=str(tmp_path / "run"),
                               firmware_dir=str(tmp_path / "fw"), params_file=str(tmp_path / "none.conf"),
                               kernel="6.8.0-45-generic", run=run, ready_timeout=3.0, **kw)


def _serve_once(dc, timeout=5.0):
    import threading
    from gpu_operator_amd.operands import driver_container as dcm
    res = os.path.join(dc.driver_dir, dcm.RELOAD_RESULT)
    if os.path.exists(res):
        os.unlink(res)
    stop = threading.Event()
    t = threading.Thread(target=dc.serve_reloads, args=(stop, 0.1), daemon=True)
    t.start()
    deadline = time.monotonic() + timeout
    while not os.path.exists(res) and time.monotonic() < deadline:
        time.sleep(0.05)
    stop.set()
    t.join(5)
    return json.loads(open(res).read())


def test_driver_container_ignores_a_stale_reload_request(spx, tmp_path):
    """a request left from before this container started (its requester timed out, or
    the manager restarted) is answered stale and never unloads the driver."""
    calls = []
    dc = _driver_container(tmp_path, spx, lambda argv, **kw: calls.append(argv))
    os.makedirs(dc.driver_dir, exist_ok=True)
    with open(os.path.join(dc.driver_dir, "reload-request"), "w") as f:
        json.dump({"id": "old", "ts": dc.started - 60, "deadline": dc.started + 540}, f)
    res = _serve_once(dc)
    assert res["id"] == "old" and res["stale"] and not res["ok"] and calls == []
    # ... and one whose requester's deadline has passed
    with open(os.path.join(dc.driver_dir, "reload-request"), "w") as f:
        json.dump({"id": "late", "ts": time.time(), "deadline": time.time() - 1}, f)
    res = _serve_once(dc)
    assert res["id"] == "late" and res["stale"] and calls == []


def test_driver_container_reload_never_rebuilds_and_always_answers(spx, tmp_path):
    """a DKMS reload is modprobe -r / modprobe (no `dkms install` under a 1800 s timeout),
    bounded by the request's deadline; an unexpected exception still writes a result."""
    import subprocess as sp
    calls = []

    def run(argv, timeout=None, **kw):
        calls.append((argv, timeout))
        return sp.CompletedProcess(argv, 0, "", "")
    dc = _driver_container(tmp_path, spx, run, driver_version="6.12.12")
    os.makedirs(dc.driver_dir, exist_ok=True)
    now = time.time()
    with open(os.path.join(dc.driver_dir, "reload-request"), "w") as f:
        json.dump({"id": "r1", "ts": now, "deadline": now + 30}, f)
    res = _serve_once(dc)
    assert res["id"] == "r1" and res["ok"], res
    assert [c[0][:2] for c in calls] == [["modprobe", "-r"], ["modprobe", "amdgpu"]]
    assert all(c[1] <= 30 for c in calls)                      # within the requester's deadline

    def boom(argv, **kw):
        raise sp.TimeoutExpired(argv, 1)
    dc2 = _driver_container(tmp_path, spx, boom, driver_version="6.12.12")
    with open(os.path.join(dc2.driver_dir, "reload-request"), "w") as f:
        json.dump({"id": "r2", "ts": time.time(), "deadline": time.time() + 30}, f)
    res = _serve_once(dc2)
    assert res["id"] == "r2" and not res["ok"] and "did not finish" in res["error"]


def test_partition_entrypoint_drops_the_driver_container_reload_on_a_host_driver():
    text = open(os.path.join(os.path.dirname(pm.__file__), "..", "assets", "state-partition-manager",
                             "0420_configmap.yaml")).read()
    host = text[text.index("host-driver-ready ]; then"):text.index("else")]
    assert "unset DRIVER_RELOAD_VIA" in host


def test_metrics_device_level_series_once_per_physical_gpu_under_cpx(tmp_path):
    """CPX enumerates 8 agents per GPU that share the PMFW gpu_metrics table and
    the hwmon sensors; energy, power, per-link xGMI bytes and temperatures are emitted once per
    physical device (its lowest-index agent), per-partition series stay per agent."""
    from prometheus_client import generate_latest
    root = str(fakesys.make_node(tmp_path / "cpx", n_gpus=2, compute="CPX"))
    text = generate_latest(me.build_registry(me.load_fields(None), root=root, hostname="n1")).decode()

    def series(name):
        return [ln for ln in text.splitlines() if ln.startswith(name + "{")]
    assert len(series("amd_gpu_energy_joules_total")) == 2
    assert len(series("amd_gpu_power_watts")) == 2
    assert len(series("amd_gpu_temperature_junction_celsius")) == 2
    assert {ln.split('gpu="')[1].split('"')[0] for ln in series("amd_gpu_power_watts")} == {"0", "8"}
    links = series("amd_gpu_xgmi_read_bytes_total")
    assert links and {ln.split('gpu="')[1].split('"')[0] for ln in links} == {"0", "8"}
    assert len(series("amd_gpu_vram_total_bytes")) == 16 and len(series("amd_gpu_sclk_mhz")) == 16
