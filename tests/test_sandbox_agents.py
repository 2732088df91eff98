"""Config-manager sidecar, KubeVirt sandbox device plugin, MxGPU VF manager, kata manager."""

import os
import signal
import threading
import time
from concurrent import futures

import grpc
import pytest
import tomli
import yaml

from gpu_operator_amd import devices as D
from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.operands import config_manager as cm
from gpu_operator_amd.operands import kata_manager as km
from gpu_operator_amd.operands import kubeletapi as K
from gpu_operator_amd.operands import mxgpu_device_manager as mx
from gpu_operator_amd.operands import sandbox_device_plugin as sdp

from k8s_helpers import gpu_node


# -- config manager -------------------------------------------------------------------------------

@pytest.fixture
def configs(tmp_path):
    d = tmp_path / "available"
    d.mkdir()
    (d / "default").write_text("version: v1\nsharing: {}\n")
    (d / "ts-4").write_text("version: v1\nsharing: {timeSlicing: {resources: [{name: amd.com/gpu, replicas: 4}]}}\n")
    return d


def test_select_strategies(configs, tmp_path):
    assert cm.select("ts-4", str(configs), "default", ["named"])[0] == "ts-4"
    assert cm.select(None, str(configs), "default", ["named", "single"])[0] == "default"
    with pytest.raises(cm.ConfigError):
        cm.select("nope", str(configs), "default", ["named"])
    with pytest.raises(cm.ConfigError):
        cm.select(None, str(configs), "", ["named", "single"])          # two configs, no default
    single = tmp_path / "single"
    single.mkdir()
    (single / "only").write_text("x")
    assert cm.select(None, str(single), "", ["named", "single"]) == ("only", "x")
    assert cm.select(None, str(configs), "", ["single", "empty"]) == ("", "")


def test_config_manager_signals_on_change(configs, tmp_path):
    c = FakeClient([gpu_node("n1")])
    sent = []
    m = cm.ConfigManager(c, "n1", "amd.com/device-plugin.config", str(configs), str(tmp_path / "out/config.yaml"),
                         default="default", process="amd-device-plugin", kill=lambda p, s: sent.append((p, s)),
                         pids=lambda name: [4242], resync=30)
    stop = threading.Event()
    t = threading.Thread(target=m.run, args=(stop,))
    t.start()
    try:
        for _ in range(100):
            if (tmp_path / "out/config.yaml").exists():
                break
            time.sleep(0.02)
        assert "sharing: {}" in (tmp_path / "out/config.yaml").read_text()
        assert sent == []                                              # first write: no signal
        c.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/device-plugin.config": "ts-4"}}})
        for _ in range(200):
            if sent:
                break
            time.sleep(0.02)
        assert sent == [(4242, signal.SIGHUP)]
        assert "replicas: 4" in (tmp_path / "out/config.yaml").read_text()
        c.patch("v1", "Node", "n1", {"metadata": {"labels": {"unrelated": "x"}}})
        time.sleep(0.2)
        assert len(sent) == 1
    finally:
        stop.set()
        c.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/device-plugin.config": "default"}}})
        t.join(5)


def test_config_manager_oneshot_env(configs, tmp_path, monkeypatch):
    c = FakeClient([gpu_node("n1", extra_labels={"amd.com/device-plugin.config": "ts-4"})])
    monkeypatch.setenv("NODE_NAME", "n1")
    monkeypatch.setenv("CONFIG_FILE_SRCDIR", str(configs))
    monkeypatch.setenv("CONFIG_FILE_DST", str(tmp_path / "c.yaml"))
    monkeypatch.setenv("ONESHOT", "true")
    assert cm.main(client=c) == 0
    assert "replicas: 4" in (tmp_path / "c.yaml").read_text()
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/device-plugin.config": "bad"}}})
    assert cm.main(client=c) == 1


def test_find_pids_matches_console_scripts(tmp_path):
    proc = tmp_path / "proc"
    for pid, argv in ((11, [b"/usr/bin/amd-device-plugin", b"--x"]), (12, [b"python3", b"/usr/local/bin/amd-device-plugin"]),
                      (13, [b"sleep", b"1"])):
        (proc / str(pid)).mkdir(parents=True)
        (proc / str(pid) / "cmdline").write_bytes(b"\0".join(argv) + b"\0")
    assert sorted(cm.find_pids("amd-device-plugin", str(proc))) == [11, 12]


# -- sandbox device plugin ----------------------------------------------------------------------

def test_resource_and_env_names():
    assert sdp.resource_name(0x75A3, False) == "amd.com/MI355X"
    assert sdp.resource_name(0x75B3, True) == "amd.com/MI355X_VF"
    assert sdp.resource_name(0x1234, True) == "amd.com/DEVICE_1234_VF"
    assert sdp.env_name("amd.com/MI355X_VF") == "PCI_RESOURCE_AMD_COM_MI355X_VF"


def test_sandbox_plugin_passthrough_and_vfs(tmp_path):
    root = fakesys.make_node(tmp_path / "r", n_gpus=2, vfio_bound=True, live=False, sriov_totalvfs=4)
    fakesys.bind_driver(root, "0000:15:00.0", "amdgpu")                   # PF 1 hosts VFs instead
    vfs = fakesys.create_vfs(root, "0000:15:00.0", 2, driver="vfio-pci")
    devs = sdp.discover(str(root))
    assert [(d.resource, d.bdf) for d in devs] == [("amd.com/MI355X", "0000:05:00.0"),
                                                   ("amd.com/MI355X_VF", vfs[0]), ("amd.com/MI355X_VF", vfs[1])]
    dev_root = tmp_path / "dev"
    (dev_root / "dev/vfio").mkdir(parents=True)
    for d in devs:
        (dev_root / "dev/vfio" / str(d.iommu_group)).write_text("")
    plugin_dir = tmp_path / "dp"
    plugin_dir.mkdir()
    registered = []
    kubelet = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
    kubelet.add_generic_rpc_handlers((K.registration_handler(lambda r: registered.append(r.resource_name)),))
    kubelet.add_insecure_port("unix://" + str(plugin_dir / "kubelet.sock"))
    kubelet.start()
    p = sdp.SandboxDevicePlugin(str(root), dev_root=str(dev_root), plugin_dir=str(plugin_dir))
    try:
        p.start()
        assert sorted(registered) == ["amd.com/MI355X", "amd.com/MI355X_VF"]
        s = p.servers["amd.com/MI355X_VF"]
        with grpc.insecure_channel("unix://" + s.socket) as ch:
            stub = K.device_plugin_stub(ch)
            it = stub["ListAndWatch"](K.DP["Empty"]())
            first = next(it)
            assert sorted(d.ID for d in first.devices) == vfs
            req = K.DP["AllocateRequest"]()
            req.container_requests.add(devicesIDs=vfs)
            resp = stub["Allocate"](req)
            car = resp.container_responses[0]
            assert car.envs["PCI_RESOURCE_AMD_COM_MI355X_VF"] == ",".join(vfs)
            paths = [d.host_path for d in car.devices]
            assert paths[0] == "/dev/vfio/vfio" and len(paths) == 3
            bad = K.DP["AllocateRequest"]()
            bad.container_requests.add(devicesIDs=["0000:99:00.0"])
            with pytest.raises(grpc.RpcError) as ei:
                stub["Allocate"](bad)
            assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
            # VF rebound away from vfio-pci -> unhealthy, streamed
            fakesys.bind_driver(root, vfs[1], "amdgpu")
            assert p.check_health()
            upd = next(it)
            assert {d.ID: d.health for d in upd.devices}[vfs[1]] == K.UNHEALTHY
            it.cancel()
    finally:
        p.stop()
        kubelet.stop(0)


# -- MxGPU device manager -----------------------------------------------------------------------

class FakeKernel:
    """Simulates GIM + the PCI core: numvfs writes create/remove VFs, binds re-point links."""

    def __init__(self, root, autobind=None):
        self.root = root
        self.autobind = autobind
        self.calls = []

    def set_numvfs(self, pf, n):
        self.calls.append(("numvfs", pf, n))
        fakesys.remove_vfs(self.root, pf)
        if n:
            fakesys.create_vfs(self.root, pf, n, driver=self.autobind or "")

    def bind(self, bdf, driver):
        self.calls.append(("bind", bdf, driver))
        fakesys.bind_driver(self.root, bdf, driver)


MX_CFG = {"version": "v1", "mxgpu-configs": {"default": [{"devices": "all", "vfs": 1}],
                                             "quad": [{"devices": "all", "vfs": 4}],
                                             "too-many": [{"devices": [0], "vfs": 99}]}}


def _mx(tmp_path, label=None, default="default"):
    root = fakesys.make_node(tmp_path / "r", n_gpus=2, sriov_totalvfs=8, live=False)
    f = tmp_path / "mx.yaml"
    f.write_text(yaml.safe_dump(MX_CFG))
    c = FakeClient([gpu_node("n1", extra_labels={mx.CONFIG_LABEL: label} if label else {})])
    k = FakeKernel(root)
    return root, c, k, mx.MxGPUDeviceManager(c, "n1", str(f), root=str(root), default_config=default,
                                            kernel=k, vf_timeout=1.0, poll=0.01)


def test_mxgpu_default_then_relayout(tmp_path):
    root, c, k, m = _mx(tmp_path)
    assert m.reconcile() == "applied"
    vfs = [f for f in D.scan_pci(str(root)) if f["is_virtfn"]]
    assert len(vfs) == 2 and all(f["driver"] == "vfio-pci" for f in vfs)
    assert o.get_labels(c.get("v1", "Node", "n1"))[mx.STATE_LABEL] == "success"
    assert m.reconcile() == "in-sync"
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {mx.CONFIG_LABEL: "quad"}}})
    k.calls.clear()
    assert m.reconcile() == "applied"
    assert ("numvfs", "0000:05:00.0", 0) in k.calls and ("numvfs", "0000:05:00.0", 4) in k.calls
    assert len([f for f in D.scan_pci(str(root)) if f["is_virtfn"]]) == 8


def test_mxgpu_failures(tmp_path):
    _, c, _, m = _mx(tmp_path, label="too-many")
    assert m.reconcile() == "failed"
    assert o.get_labels(c.get("v1", "Node", "n1"))[mx.STATE_LABEL] == "failed"
    assert "99 VFs requested" in c.events[-1]["message"]
    _, c2, _, m2 = _mx(tmp_path / "b", label="missing")
    assert m2.reconcile() == "failed"
    _, _, _, m3 = _mx(tmp_path / "c", default="")
    assert m3.reconcile() == "no-config"


def test_mxgpu_sysfs_kernel_writes(tmp_path):
    root = fakesys.make_node(tmp_path / "r", n_gpus=1, sriov_totalvfs=8, live=False)
    vfs = fakesys.create_vfs(root, "0000:05:00.0", 1, driver="amdgpu")
    (root / "sys/bus/pci/drivers/amdgpu/unbind").write_text("")
    k = mx.SysfsKernel(str(root))
    k.bind(vfs[0], "vfio-pci")
    dev = root / "sys/bus/pci/devices" / vfs[0]
    assert (dev / "driver_override").read_text() == "vfio-pci"
    assert (root / "sys/bus/pci/drivers_probe").read_text() == vfs[0]
    assert (root / "sys/bus/pci/drivers/amdgpu/unbind").read_text() == vfs[0]
    k.set_numvfs("0000:05:00.0", 3)
    assert (root / "sys/bus/pci/devices/0000:05:00.0/sriov_numvfs").read_text() == "3"


# -- kata manager --------------------------------------------------------------------------------

def test_kata_manager_local_artifacts(tmp_path):
    art = tmp_path / "src"
    art.mkdir()
    (art / "vmlinuz-6.8-amd").write_text("k")
    (art / "kata-rootfs.img").write_text("i")
    ctrd = tmp_path / "config.toml"
    ctrd.write_text('version = 2\n[plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc]\n'
                    'runtime_type = "io.containerd.runc.v2"\n')
    reloads = []
    cfg = {"artifactsDir": str(tmp_path / "artifacts"),
           "runtimeClasses": [{"name": "kata-qemu-amd-gpu", "artifacts": {"url": f"file://{art}"}}]}
    root = fakesys.make_node(tmp_path / "r", n_gpus=8, vfio_bound=True, live=False)
    m = km.KataManager(cfg, str(ctrd), reload=lambda: reloads.append(1), sys_root=str(root))
    assert m.install() is True
    doc = tomli.loads(ctrd.read_text())
    rts = doc["plugins"]["io.containerd.grpc.v1.cri"]["containerd"]["runtimes"]
    h = rts["kata-qemu-amd-gpu"]
    assert h["runtime_type"] == "io.containerd.kata.v2" and "runc" in rts
    conf = open(h["options"]["ConfigPath"]).read()
    assert "pcie_root_port = 8" in conf and "kata-rootfs.img" in conf and "vmlinuz-6.8-amd" in conf
    assert m.install() is False and reloads == [1]                    # idempotent, no extra reload
    assert m.uninstall() is True and reloads == [1, 1]
    assert "kata-qemu-amd-gpu" not in tomli.loads(ctrd.read_text())["plugins"]["io.containerd.grpc.v1.cri"][
        "containerd"]["runtimes"]


def test_kata_manager_pull_command_and_errors(tmp_path):
    calls = []

    class P:
        returncode = 0
        stderr = ""

    def run(argv, **kw):
        calls.append(argv)
        os.makedirs(argv[-1], exist_ok=True)
        with open(os.path.join(argv[-1], "configuration-x.toml"), "w") as f:
            f.write("[hypervisor.qemu]\n")
        return P()
    cfg = {"artifactsDir": str(tmp_path / "a"),
           "runtimeClasses": [{"name": "kata-x", "artifacts": {"url": "registry.example.com/kata:1"}}]}
    m = km.KataManager(cfg, str(tmp_path / "c.toml"), run=run)
    h = m.handlers()
    assert calls == [["oras", "pull", "registry.example.com/kata:1", "-o", str(tmp_path / "a/kata-x")]]
    assert h["kata-x"]["options"]["ConfigPath"].endswith("configuration-x.toml")
    with pytest.raises(km.KataError):
        km.KataManager({"runtimeClasses": [{"name": "y", "artifacts": {}}]}, str(tmp_path / "c.toml"),
                       artifacts_dir=str(tmp_path / "a")).handlers()


# -- vfio-manage.sh executed against a fake sysfs with a simulated PCI core ------------------------
def _vfio_script():
    import yaml
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "gpu_operator_amd/assets/state-vfio-manager/0400_configmap.yaml")) as f:
        return yaml.safe_load(f)["data"]["vfio-manage.sh"]


class _FakePciCore:
    """Serves sysfs bus/pci/drivers_probe as a FIFO: binds a device to its driver_override, or
    back to its original driver when the override is cleared (what the kernel's probe does)."""

    def __init__(self, root):
        import threading
        self.root = root
        self.pci = os.path.join(root, "sys/bus/pci")
        self.orig = {b: os.path.basename(os.readlink(os.path.join(self.pci, "devices", b, "driver")))
                     for b in os.listdir(os.path.join(self.pci, "devices"))
                     if os.path.islink(os.path.join(self.pci, "devices", b, "driver"))}
        self.fifo = os.path.join(self.pci, "drivers_probe")
        os.mkfifo(self.fifo)
        self.stop = False
        self.t = threading.Thread(target=self.run, daemon=True)
        self.t.start()

    def run(self):
        while not self.stop:
            with open(self.fifo) as f:
                data = f.read()
            for bdf in data.split():
                dev = os.path.join(self.pci, "devices", bdf)
                try:
                    ov = open(os.path.join(dev, "driver_override")).read().strip()
                except OSError:
                    ov = ""
                drv = ov or self.orig.get(bdf, "")
                link = os.path.join(dev, "driver")
                if os.path.islink(link):
                    os.unlink(link)
                if drv:
                    d = os.path.join(self.pci, "drivers", drv)
                    os.makedirs(d, exist_ok=True)
                    os.symlink(os.path.relpath(d, dev), link)

    def close(self):
        self.stop = True
        with open(self.fifo, "w") as f:
            f.write("\n")
        self.t.join(5)


def _driver(root, bdf):
    return os.path.basename(os.readlink(os.path.join(root, "sys/bus/pci/devices", bdf, "driver")))


def test_vfio_manage_binds_gpus_with_their_iommu_group_companions(tmp_path):
    import subprocess
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=2, companion_audio=True))
    script = tmp_path / "vfio-manage.sh"
    script.write_text(_vfio_script())
    core = _FakePciCore(root)
    env = dict(os.environ, SYSFS_ROOT=os.path.join(root, "sys"))
    try:
        p = subprocess.run(["bash", str(script), "bind", "--all"], env=env, capture_output=True, text=True, timeout=60)
        assert p.returncode == 0, p.stdout + p.stderr
        for bus in ("05", "15"):
            assert _driver(root, f"0000:{bus}:00.0") == "vfio-pci"
            assert _driver(root, f"0000:{bus}:00.1") == "vfio-pci"      # the audio companion followed
        assert p.stdout.count("bound") == 4
        p = subprocess.run(["bash", str(script), "bind", "--all"], env=env, capture_output=True, text=True, timeout=60)
        assert p.returncode == 0 and "already bound" in p.stdout
        p = subprocess.run(["bash", str(script), "unbind", "--all"], env=env, capture_output=True, text=True,
                           timeout=60)
        assert p.returncode == 0, p.stdout + p.stderr
        assert _driver(root, "0000:05:00.0") == "amdgpu" and _driver(root, "0000:05:00.1") == "snd_hda_intel"
    finally:
        core.close()


def _foreign_nic(root, group=10, bdf="0000:06:00.0"):
    """A host NIC (Mellanox, class 0x0200) in the IOMMU group of the first GPU: a platform
    without ACS isolation."""
    from pathlib import Path
    r = Path(root)
    dev = r / "sys/bus/pci/devices" / bdf
    dev.mkdir(parents=True)
    (dev / "vendor").write_text("0x15b3\n")
    (dev / "class").write_text("0x020000\n")
    (dev / "driver_override").write_text("\n")
    drv = r / "sys/bus/pci/drivers/mlx5_core"
    drv.mkdir(parents=True, exist_ok=True)
    os.symlink(os.path.relpath(drv, dev), dev / "driver")
    grp = r / "sys/kernel/iommu_groups" / str(group)
    os.symlink(os.path.relpath(grp, dev), dev / "iommu_group")
    os.symlink(os.path.relpath(dev, grp / "devices"), grp / "devices" / bdf)
    return bdf


def test_vfio_manage_refuses_a_group_with_a_foreign_device(tmp_path):
    """an IOMMU group that also holds a host NIC is refused -- the NIC keeps its
    driver and gets no driver_override, the GPU stays on amdgpu -- while other GPUs still bind."""
    import subprocess
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=2, companion_audio=True))
    nic = _foreign_nic(root)
    script = tmp_path / "vfio-manage.sh"
    script.write_text(_vfio_script())
    core = _FakePciCore(root)
    env = dict(os.environ, SYSFS_ROOT=os.path.join(root, "sys"))
    try:
        p = subprocess.run(["bash", str(script), "bind", "--all"], env=env, capture_output=True, text=True, timeout=60)
        assert p.returncode == 1 and "refusing to bind 0000:05:00.0" in p.stderr and nic in p.stderr
        assert _driver(root, nic) == "mlx5_core"
        assert open(os.path.join(root, "sys/bus/pci/devices", nic, "driver_override")).read().strip() == ""
        assert _driver(root, "0000:05:00.0") == "amdgpu" and _driver(root, "0000:05:00.1") == "snd_hda_intel"
        assert _driver(root, "0000:15:00.0") == "vfio-pci" and _driver(root, "0000:15:00.1") == "vfio-pci"
    finally:
        core.close()


def test_vfio_manage_rolls_back_a_failed_companion(tmp_path):
    """A companion that cannot take the override: it is re-probed to its host driver, and the
    GPU is left on amdgpu (never half a group on vfio-pci)."""
    import shutil
    import subprocess
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=1, companion_audio=True))
    ov = os.path.join(root, "sys/bus/pci/devices/0000:05:00.1/driver_override")
    if os.path.exists(ov):
        os.remove(ov)
    os.makedirs(ov)                                       # writes to it fail, even as root
    script = tmp_path / "vfio-manage.sh"
    script.write_text(_vfio_script())
    core = _FakePciCore(root)
    env = dict(os.environ, SYSFS_ROOT=os.path.join(root, "sys"))
    try:
        p = subprocess.run(["bash", str(script), "bind", "--all"], env=env, capture_output=True, text=True, timeout=60)
        assert p.returncode == 1 and "left 0000:05:00.0 with its host driver" in p.stderr
        assert _driver(root, "0000:05:00.1") == "snd_hda_intel" and _driver(root, "0000:05:00.0") == "amdgpu"
    finally:
        core.close()
        shutil.rmtree(ov, ignore_errors=True)
