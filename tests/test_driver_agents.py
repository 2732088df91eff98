"""amdgpu driver container entrypoint and the driver manager (unload before reinstall)."""

import json
import os
import subprocess
import threading
from types import SimpleNamespace

import pytest

from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.operands import driver_container as dcm
from gpu_operator_amd.operands import driver_manager as dmm

from k8s_helpers import gpu_node


def _ok(stdout=""):
    return SimpleNamespace(returncode=0, stdout=stdout, stderr="")


# -- driver container -----------------------------------------------------------------------------

def test_module_params_and_os_release(tmp_path):
    p = tmp_path / "amdgpu.conf"
    p.write_text("# tuning\noptions amdgpu ras_enable=1 vm_update_mode=0\noptions other x=1\nmes=1\n")
    assert dcm.module_params(str(p)) == ["ras_enable=1", "vm_update_mode=0", "mes=1"]
    assert dcm.module_params(str(tmp_path / "none")) == []
    r = tmp_path / "os-release"
    r.write_text('ID=ubuntu\nVERSION_ID="22.04"\n')
    assert dcm.os_release(str(r)) == {"ID": "ubuntu", "VERSION_ID": "22.04"}


def _image(tmp_path, kernel, mods=("amdgpu", "amdxcp", "amdttm", "amdkcl", "extra_helper")):
    img = tmp_path / "image"
    d = img / "opt/amdgpu/precompiled" / kernel
    d.mkdir(parents=True)
    for m in mods:
        (d / f"{m}.ko.xz").write_text("x")
    fw = img / "opt/amdgpu/firmware"
    fw.mkdir(parents=True)
    (fw / "gc_9_5_0_mec.bin").write_bytes(b"\0" * 16)
    (fw / "psp_14_0_2_sos.bin").write_bytes(b"\1" * 8)
    return img


def _dc(tmp_path, root, img, run, **kw):
    return dcm.DriverContainer(sys_root=str(root), dev_root=str(root), image_root=str(img),
                               host_etc=str(tmp_path / "etc"), run_dir=str(tmp_path / "run"),
                               firmware_dir=str(tmp_path / "fw"), params_file=str(tmp_path / "amdgpu.conf"),
                               kernel="6.8.0-45-generic", run=run, ready_timeout=2.0, **kw)


def test_precompiled_init(tmp_path):
    root = tmp_path / "root"
    os.makedirs(root)
    (tmp_path / "amdgpu.conf").write_text("options amdgpu ras_enable=1\n")
    img = _image(tmp_path, "6.8.0-45-generic")
    calls = []

    def run(argv, **kw):
        calls.append(argv)
        if argv[0] == "insmod" and argv[1].endswith("amdgpu.ko.xz"):
            fakesys.make_node(root, n_gpus=8)          # the driver comes up
        return _ok()
    dc = _dc(tmp_path, root, img, run)
    info = dc.init()
    assert [dcm._mod_name(c[1]) for c in calls] == ["extra_helper", "amdkcl", "amdttm", "amdxcp", "amdgpu"]
    assert calls[-1][2:] == ["ras_enable=1"]
    assert info["mode"] == "precompiled" and info["firmware_files"] == 2
    assert "8 GPU(s)" in info["state"]
    assert (tmp_path / "fw/updates/amdgpu/gc_9_5_0_mec.bin").exists()
    marker = json.loads((tmp_path / "run/driver/.driver-ctr").read_text())
    assert marker["kernel"] == "6.8.0-45-generic"
    assert dc.ready()[0]
    assert dc.install_firmware() == 0                     # idempotent copy


def test_dkms_fallback_and_errors(tmp_path):
    root = tmp_path / "root"
    os.makedirs(root)
    img = tmp_path / "empty-image"
    img.mkdir()
    calls = []

    def run(argv, **kw):
        calls.append(argv[:2])
        if argv[0] == "modprobe":
            fakesys.make_node(root, n_gpus=2)
        return _ok()
    dc = _dc(tmp_path, root, img, run, driver_version="6.12.12")
    assert dc.init()["mode"] == "dkms"
    assert calls == [["dkms", "install"], ["modprobe", "amdgpu"]]
    # no precompiled + no version -> error; failing command -> error
    root2 = tmp_path / "root2"
    os.makedirs(root2)
    with pytest.raises(dcm.DriverError, match="DRIVER_VERSION"):
        _dc(tmp_path, root2, img, run).load()
    bad = _dc(tmp_path, root2, img, lambda a, **k: SimpleNamespace(returncode=1, stdout="", stderr="no headers"),
              driver_version="6.12.12")
    with pytest.raises(dcm.DriverError, match="no headers"):
        bad.load()


def test_host_driver_refused_and_timeout(tmp_path):
    root = fakesys.make_node(tmp_path / "root", n_gpus=1)        # loaded, but no container marker
    dc = _dc(tmp_path, root, tmp_path, lambda a, **k: _ok())
    with pytest.raises(dcm.DriverError, match="pre-installed"):
        dc.init()
    root2 = tmp_path / "r2"
    os.makedirs(root2)
    img = _image(tmp_path, "6.8.0-45-generic")
    never = _dc(tmp_path, root2, img, lambda a, **k: _ok())
    never.ready_timeout = 0.2
    with pytest.raises(dcm.DriverError, match="did not become ready"):
        never.init()


def test_probe_and_daemon_shutdown(tmp_path):
    root = tmp_path / "root"
    os.makedirs(root)
    img = _image(tmp_path, "6.8.0-45-generic")
    calls = []

    def run(argv, **kw):
        calls.append(argv[:2])
        if argv[0] == "insmod" and "amdgpu" in argv[1]:
            fakesys.make_node(root, n_gpus=2)
        return _ok()
    dc = _dc(tmp_path, root, img, run)
    assert dcm.main(["probe"], dc=dc) == 1
    stop = threading.Event()
    t = threading.Thread(target=dcm.main, args=(["init"], stop, dc))
    t.start()
    for _ in range(200):
        if (tmp_path / "run/driver/.driver-ctr").exists():
            break
        threading.Event().wait(0.02)
    assert dcm.main(["probe"], dc=dc) == 0
    stop.set()
    t.join(5)
    assert calls[-1] == ["modprobe", "-r"]
    assert not (tmp_path / "run/driver/.driver-ctr").exists()


# -- driver manager ---------------------------------------------------------------------------------

def _pod(name, node="n1", app=None, gpu=False, owner="ReplicaSet", ns="default", empty_dir=False):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": ns, "labels": {"app": app} if app else {}},
         "spec": {"nodeName": node, "containers": [{"name": "c", "resources": {
             "limits": {"amd.com/gpu": "1"} if gpu else {}}}]},
         "status": {"phase": "Running"}}
    if owner:
        p["metadata"]["ownerReferences"] = [{"kind": owner, "name": "o", "uid": "u-" + name, "controller": True,
                                             "apiVersion": "apps/v1"}]
    if empty_dir:
        p["spec"]["volumes"] = [{"name": "s", "emptyDir": {}}]
    return p


def _dm(tmp_path, client, root, calls=None, **kw):
    run_dir = tmp_path / "run"
    (run_dir / "validations").mkdir(parents=True, exist_ok=True)

    def run(argv, **k):
        if calls is not None:
            calls.append(argv)
        return _ok()
    return dmm.DriverManager(client, "n1", "gpu-operator", sys_root=str(root), run_dir=str(run_dir),
                             pods_timeout=2.0, poll=0.05, run=run, **kw)


def _labels():
    return {"amd.com/gpu.deploy.device-plugin": "true", "amd.com/gpu.deploy.metrics-exporter": "true",
            "amd.com/gpu.deploy.driver": "true", "amd.com/gpu.deploy.rdc": "false"}


def test_manager_fast_paths(tmp_path):
    c = FakeClient([gpu_node("n1", extra_labels=_labels())])
    empty = tmp_path / "none"
    empty.mkdir()
    dm = _dm(tmp_path, c, empty)
    (tmp_path / "run/validations/driver-ready").write_text("{}")
    assert dm.uninstall_driver() == "not-loaded"
    assert not (tmp_path / "run/validations/driver-ready").exists()
    host = fakesys.make_node(tmp_path / "host", n_gpus=1)
    assert _dm(tmp_path, c, host).uninstall_driver() == "host-driver"


def test_manager_unload_with_eviction(tmp_path):
    root = fakesys.make_node(tmp_path / "root", n_gpus=1)
    c = FakeClient([gpu_node("n1", extra_labels=_labels()),
                    _pod("dp", app="amd-device-plugin-daemonset", owner="DaemonSet", ns="gpu-operator"),
                    _pod("train", gpu=True), _pod("web"), _pod("other-node-train", node="n2", gpu=True)])
    calls = []
    dm = _dm(tmp_path, c, root, calls)
    os.makedirs(tmp_path / "run/driver")
    (tmp_path / "run/driver/.driver-ctr").write_text("{}")
    seen = []
    c.watch("v1", "Node", lambda ev: seen.append(dict(o.get_labels(ev.obj))))

    def on_pause(ev):            # the DaemonSet controller removes the paused operand's pod
        if o.get_labels(ev.obj).get("amd.com/gpu.deploy.device-plugin") == dmm.PAUSED:
            try:
                c.delete("v1", "Pod", "dp", "gpu-operator")
            except Exception:
                pass
    c.watch("v1", "Node", on_pause)
    assert dm.uninstall_driver() == "unloaded"
    names = {o.name(p) for p in c.objects("Pod")}
    assert names == {"web", "other-node-train"}                         # only local GPU pods evicted
    assert calls and calls[0][:4] == ["chroot", "/host", "modprobe", "-r"] and "amdgpu" in calls[0]
    assert any(s.get("amd.com/gpu.deploy.device-plugin") == dmm.PAUSED for s in seen)
    labels = o.get_labels(c.get("v1", "Node", "n1"))
    assert labels["amd.com/gpu.deploy.device-plugin"] == "true" and labels["amd.com/gpu.deploy.rdc"] == "false"
    assert labels["amd.com/gpu.deploy.driver"] == "true"                # never paused


def test_manager_eviction_blocked_then_drain(tmp_path):
    root = fakesys.make_node(tmp_path / "root", n_gpus=1)
    c = FakeClient([gpu_node("n1", extra_labels=_labels()), _pod("bare", gpu=True, owner=None),
                    _pod("cache", empty_dir=True)])
    os.makedirs(tmp_path / "run/driver")
    (tmp_path / "run/driver/.driver-ctr").write_text("{}")
    dm = _dm(tmp_path, c, root)
    with pytest.raises(dmm.DriverManagerError, match="auto drain is disabled"):
        dm.uninstall_driver()
    assert o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.deploy.device-plugin"] == "true"
    dm2 = _dm(tmp_path, c, root, auto_drain=True, drain_force=True, drain_empty_dir=True)
    assert dm2.uninstall_driver() == "unloaded"
    assert c.objects("Pod") == []
    assert not (c.get("v1", "Node", "n1").get("spec") or {}).get("unschedulable")     # uncordoned


def test_manager_refuses_busy_module(tmp_path):
    root = fakesys.make_node(tmp_path / "root", n_gpus=1)
    (root / "sys/module/amdgpu/refcnt").write_text("3\n")
    c = FakeClient([gpu_node("n1", extra_labels=_labels())])
    os.makedirs(tmp_path / "run/driver")
    (tmp_path / "run/driver/.driver-ctr").write_text("{}")
    with pytest.raises(dmm.DriverManagerError, match="refcnt 3"):
        _dm(tmp_path, c, root).uninstall_driver()


def test_manager_from_env(monkeypatch):
    monkeypatch.setenv("NODE_NAME", "n9")
    monkeypatch.setenv("DRAIN_TIMEOUT_SECONDS", "90s")
    monkeypatch.setenv("ENABLE_AUTO_DRAIN", "true")
    dm = dmm.DriverManager.from_env(FakeClient([]))
    assert dm.node == "n9" and dm.drain_timeout == 90 and dm.auto_drain and dm.evict_gpu_pods
