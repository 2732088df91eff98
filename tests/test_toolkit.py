"""Container toolkit: CDI generation, runtime config edits and the native OCI runtime shim."""

import json
import os
import socket
import subprocess
import threading

import pytest
import tomli

from gpu_operator_amd import devices as D
from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.toolkit import cdi, ctk, runtime_config as rc, tomlw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "gpu_operator_amd", "_native", "bin", "amd-container-runtime")

CONTAINERD_V2 = """
version = 2
root = "/var/lib/containerd"

[grpc]
  address = "/run/containerd/containerd.sock"

[plugins."io.containerd.grpc.v1.cri"]
  sandbox_image = "registry.k8s.io/pause:3.9"
  [plugins."io.containerd.grpc.v1.cri".containerd]
    default_runtime_name = "runc"
    [plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc]
      runtime_type = "io.containerd.runc.v2"
      [plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options]
        SystemdCgroup = true

[[proxy_plugins_list]]
  name = "a"
"""


def _fake_dev(tmp_path, n_render):
    """Device tree whose nodes are symlinks to /dev/null (a real character device)."""
    dev = tmp_path / "devroot"
    (dev / "dev/dri").mkdir(parents=True)
    os.symlink("/dev/null", dev / "dev/kfd")
    for i in range(n_render):
        os.symlink("/dev/null", dev / f"dev/dri/renderD{128 + i}")
    return str(dev)


# -- TOML -----------------------------------------------------------------------------------

def test_toml_roundtrip():
    doc = tomli.loads(CONTAINERD_V2)
    assert tomli.loads(tomlw.dumps(doc)) == doc
    weird = {"a": {"b.c": {"x": "q\"uote", "l": [1, 2], "f": 1.5, "t": False}}, "top": "v"}
    assert tomli.loads(tomlw.dumps(weird)) == weird


# -- runtime config -------------------------------------------------------------------------

def test_containerd_configure_and_revert(tmp_path):
    cfg = tmp_path / "config.toml"
    cfg.write_text(CONTAINERD_V2)
    before = tomli.loads(CONTAINERD_V2)
    bins = rc.handler_binaries("/usr/local/amd/toolkit", "amd", cdi=True)
    rc.configure("containerd", str(cfg), bins, default="amd", cdi=True)
    doc = tomli.loads(cfg.read_text())
    c = doc["plugins"]["io.containerd.grpc.v1.cri"]
    rts = c["containerd"]["runtimes"]
    assert set(rts) == {"runc", "amd", "amd-cdi", "amd-legacy"}
    assert rts["amd"]["options"] == {"SystemdCgroup": True,
                                     "BinaryName": "/usr/local/amd/toolkit/amd-container-runtime"}
    assert rts["amd-cdi"]["options"]["BinaryName"].endswith(".cdi")
    assert c["containerd"]["default_runtime_name"] == "amd"
    assert c["enable_cdi"] is True and "/var/run/cdi" in c["cdi_spec_dirs"]
    assert doc["grpc"]["address"] == "/run/containerd/containerd.sock"
    # idempotent
    rc.configure("containerd", str(cfg), bins, default="amd", cdi=True)
    assert tomli.loads(cfg.read_text()) == doc
    rc.revert("containerd", str(cfg))
    assert tomli.loads(cfg.read_text()) == before
    assert not (tmp_path / "config.toml.amd-state.json").exists()


def test_containerd_v3_and_empty(tmp_path):
    cfg = tmp_path / "c3.toml"
    cfg.write_text('version = 3\n')
    rc.configure("containerd", str(cfg), {"amd": "/x/amd-container-runtime"})
    doc = tomli.loads(cfg.read_text())
    assert doc["plugins"]["io.containerd.cri.v1.runtime"]["containerd"]["runtimes"]["amd"]["runtime_type"] == \
        "io.containerd.runc.v2"
    fresh = tmp_path / "new" / "config.toml"
    rc.configure("containerd", str(fresh), {"amd": "/x/amd-container-runtime"})
    assert tomli.loads(fresh.read_text())["version"] == 2


def test_docker_configure_and_revert(tmp_path):
    cfg = tmp_path / "daemon.json"
    orig = {"log-driver": "json-file", "default-runtime": "runc"}
    cfg.write_text(json.dumps(orig))
    rc.configure("docker", str(cfg), rc.handler_binaries("/opt/amd", "amd", cdi=False), default="amd", cdi=True)
    doc = json.loads(cfg.read_text())
    assert doc["runtimes"]["amd"]["path"] == "/opt/amd/amd-container-runtime"
    assert doc["default-runtime"] == "amd" and doc["features"]["cdi"] is True
    rc.revert("docker", str(cfg))
    assert json.loads(cfg.read_text()) == orig


def test_crio_dropin(tmp_path):
    f = tmp_path / "crio.conf.d" / "99-amd.conf"
    rc.configure("crio", str(f), rc.handler_binaries("/opt/amd", "amd", cdi=True), default="amd")
    doc = tomli.loads(f.read_text())
    rt = doc["crio"]["runtime"]
    assert rt["default_runtime"] == "amd"
    assert rt["runtimes"]["amd-legacy"]["runtime_path"] == "/opt/amd/amd-container-runtime.legacy"
    rc.revert("crio", str(f))
    assert not f.exists()


def test_unknown_runtime(tmp_path):
    with pytest.raises(ValueError):
        rc.configure("podman", str(tmp_path / "x"), {})


# -- CDI ------------------------------------------------------------------------------------

def test_cdi_generate_spx(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r"))
    dev = _fake_dev(tmp_path, 8)
    spec = cdi.generate(root, dev)
    assert spec["kind"] == "amd.com/gpu" and spec["cdiVersion"] == "0.6.0"
    kfd = spec["containerEdits"]["deviceNodes"][0]
    assert kfd["path"] == "/dev/kfd" and kfd["type"] == "c" and (kfd["major"], kfd["minor"]) == (1, 3)
    names = [d["name"] for d in spec["devices"]]
    assert names[:2] == ["0", f"amdgpu-{D.enumerate_gpus(root)[0]['unique_id']:016x}"]
    assert names[-1] == "all" and len(names) == 8 * 2 + 1
    assert len(spec["devices"][-1]["containerEdits"]["deviceNodes"]) == 8
    p = cdi.write(spec, str(tmp_path / "cdi"))
    assert json.load(open(p)) == spec
    assert cdi.list_devices(str(tmp_path / "cdi"))[0] == "amd.com/gpu=0"


def test_cdi_generate_cpx_partitions(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", compute="CPX"))
    spec = cdi.generate(root, str(tmp_path / "nodev"), strategy="index")
    assert len(spec["devices"]) == 65
    assert spec["devices"][63]["containerEdits"]["deviceNodes"][0]["path"] == "/dev/dri/renderD191"
    assert "major" not in spec["devices"][0]["containerEdits"]["deviceNodes"][0]   # resolved at create


def test_dev_char_symlinks(tmp_path):
    dev = _fake_dev(tmp_path, 2)
    links = cdi.create_dev_char_symlinks(dev, str(tmp_path / "char"))
    assert links and os.readlink(links[0]).startswith("/dev/")
    assert os.path.basename(links[0]) == "1:3"


def test_ctk_cli_cdi_stdout(tmp_path, capsys):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=2))
    assert ctk.main(["cdi", "generate", "--stdout", "--sys-root", root]) == 0
    assert json.loads(capsys.readouterr().out)["devices"][-1]["name"] == "all"


# -- native OCI runtime shim ----------------------------------------------------------------

def _bundle(tmp_path, env=None, annotations=None, name="b"):
    b = tmp_path / name
    b.mkdir()
    spec = {"ociVersion": "1.1.0", "process": {"user": {"uid": 0, "gid": 0}, "args": ["sh"],
                                               "env": ["PATH=/usr/bin"] + (env or [])},
            "root": {"path": "rootfs"},
            "linux": {"resources": {"devices": [{"allow": False, "access": "rwm"}],
                                    "memory": {"limit": 18446744073709551615}},
                      "namespaces": [{"type": "pid"}]}}
    if annotations:
        spec["annotations"] = annotations
    (b / "config.json").write_text(json.dumps(spec))
    return b


def _run_shim(args, root, dev, extra_env=None, cdi_dirs="/nonexistent"):
    env = dict(os.environ, AMD_CONTAINER_RUNTIME_RUNTIMES="/bin/echo", AMD_CONTAINER_RUNTIME_SYS_ROOT=root,
               AMD_CONTAINER_RUNTIME_DEV_ROOT=dev, AMD_CONTAINER_RUNTIME_CDI_SPEC_DIRS=cdi_dirs)
    env.update(extra_env or {})
    return subprocess.run([SHIM] + args, capture_output=True, text=True, env=env, timeout=30)


@pytest.fixture
def node(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=4))
    return root, _fake_dev(tmp_path, 4)


def test_shim_legacy_injects_selected_gpus(tmp_path, node):
    root, dev = node
    uid = f"amdgpu-{D.enumerate_gpus(root)[2]['unique_id']:016x}"
    b = _bundle(tmp_path, env=[f"AMD_VISIBLE_DEVICES=0,{uid}"])
    p = _run_shim(["--root", "/run/runc", "--log", "/tmp/l", "create", "--bundle", str(b), "ctr1"], root, dev,
                  {"AMD_CONTAINER_RUNTIME_MODE": "legacy"})
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["--root", "/run/runc", "--log", "/tmp/l", "create", "--bundle", str(b), "ctr1"]
    spec = json.loads((b / "config.json").read_text())
    paths = [d["path"] for d in spec["linux"]["devices"]]
    assert paths == ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/renderD130"]
    assert all((d["type"], d["major"], d["minor"]) == ("c", 1, 3) for d in spec["linux"]["devices"])
    rules = spec["linux"]["resources"]["devices"]
    assert rules[0] == {"allow": False, "access": "rwm"} and len(rules) == 4 and rules[1]["access"] == "rwm"
    # untouched fields survive bit-exactly (64-bit number, order)
    assert spec["linux"]["resources"]["memory"]["limit"] == 18446744073709551615
    assert list(spec) == ["ociVersion", "process", "root", "linux"]


def test_shim_passthrough(tmp_path, node):
    root, dev = node
    b = _bundle(tmp_path)
    before = (b / "config.json").read_text()
    assert _run_shim(["create", "-b", str(b), "c"], root, dev).returncode == 0
    assert (b / "config.json").read_text() == before               # no GPU requested
    b2 = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=all"], name="b2")
    before2 = (b2 / "config.json").read_text()
    p = _run_shim(["state", "c"], root, dev)                        # not `create`: untouched
    assert p.returncode == 0 and p.stdout.strip() == "state c"
    assert (b2 / "config.json").read_text() == before2
    b3 = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=none"], name="b3")
    before3 = (b3 / "config.json").read_text()
    assert _run_shim(["create", f"--bundle={b3}", "c"], root, dev).returncode == 0
    assert (b3 / "config.json").read_text() == before3


def test_shim_all_and_unknown(tmp_path, node):
    root, dev = node
    b = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=all"])
    assert _run_shim(["create", "--bundle", str(b), "c"], root, dev).returncode == 0
    assert len(json.loads((b / "config.json").read_text())["linux"]["devices"]) == 5
    b2 = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=7"], name="b2")
    p = _run_shim(["create", "--bundle", str(b2), "c"], root, dev)
    assert p.returncode == 1 and "matches no GPU" in p.stderr


def test_shim_cdi_annotations(tmp_path, node):
    root, dev = node
    spec_dir = tmp_path / "cdi"
    cdi.write(cdi.generate(root, dev), str(spec_dir))
    b = _bundle(tmp_path, annotations={"amd.cdi.k8s.io/amd-device-plugin": "amd.com/gpu=1,amd.com/gpu=3",
                                       "other": "x"})
    p = _run_shim(["create", "--bundle", str(b), "c"], root, dev, cdi_dirs=str(spec_dir))
    assert p.returncode == 0, p.stderr
    spec = json.loads((b / "config.json").read_text())
    assert [d["path"] for d in spec["linux"]["devices"]] == ["/dev/dri/renderD129", "/dev/kfd",
                                                             "/dev/dri/renderD131"]
    assert any(e.startswith("AMD_GPU_UUID_1=amdgpu-") for e in spec["process"]["env"])
    # auto mode picks CDI when a spec exists: env names map to amd.com/gpu=<name>
    b2 = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=all"], name="b2")
    assert _run_shim(["create", "--bundle", str(b2), "c"], root, dev, cdi_dirs=str(spec_dir)).returncode == 0
    assert len(json.loads((b2 / "config.json").read_text())["linux"]["devices"]) == 5
    b3 = _bundle(tmp_path, annotations={"amd.cdi.k8s.io/x": "amd.com/gpu=9"}, name="b3")
    p = _run_shim(["create", "--bundle", str(b3), "c"], root, dev, cdi_dirs=str(spec_dir))
    assert p.returncode == 1 and "unresolvable CDI device amd.com/gpu=9" in p.stderr


def test_shim_mode_pinned_by_name(tmp_path, node):
    root, dev = node
    link = tmp_path / "amd-container-runtime.legacy"
    os.symlink(SHIM, link)
    spec_dir = tmp_path / "cdi"
    cdi.write(cdi.generate(root, dev), str(spec_dir))
    b = _bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=1"])
    env = dict(os.environ, AMD_CONTAINER_RUNTIME_RUNTIMES="/bin/echo", AMD_CONTAINER_RUNTIME_SYS_ROOT=root,
               AMD_CONTAINER_RUNTIME_DEV_ROOT=dev, AMD_CONTAINER_RUNTIME_CDI_SPEC_DIRS=str(spec_dir))
    p = subprocess.run([str(link), "create", "--bundle", str(b), "c"], env=env, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    spec = json.loads((b / "config.json").read_text())
    assert "AMD_GPU_UUID_1" not in " ".join(spec["process"]["env"])     # legacy: no CDI env edits


def test_shim_bad_json(tmp_path, node):
    root, dev = node
    b = tmp_path / "bad"
    b.mkdir()
    (b / "config.json").write_text('{"process": {"env": ["AMD_VISIBLE_DEVICES=0"]')
    p = _run_shim(["create", "--bundle", str(b), "c"], root, dev)
    assert p.returncode == 1 and "invalid" in p.stderr


# -- install daemon -------------------------------------------------------------------------

def test_installer_roundtrip(tmp_path, node):
    root, dev = node
    cfg = tmp_path / "etc" / "config.toml"
    cfg.parent.mkdir()
    cfg.write_text(CONTAINERD_V2)
    sock_path = str(tmp_path / "ctrd.sock")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(sock_path)
    srv.listen(4)
    calls = []
    inst = ctk.Installer(root=str(tmp_path / "usr-local-amd"), runtime="containerd", runtime_config=str(cfg),
                         runtime_socket=sock_path, cdi_enabled=True, mode="auto", cdi_dir=str(tmp_path / "cdi"),
                         sys_root=root, dev_root=dev, restart_mode="systemd", shim=SHIM,
                         run=lambda argv, **kw: calls.append(argv), socket_timeout=5)
    try:
        out = inst.install()
    finally:
        srv.close()
    assert calls == [["chroot", "/host", "systemctl", "restart", "containerd"]]
    dest = tmp_path / "usr-local-amd" / "toolkit"
    assert os.access(dest / "amd-container-runtime", os.X_OK)
    assert os.readlink(dest / "amd-container-runtime.cdi") == "amd-container-runtime"
    assert "mode = auto" in (dest / "amd-container-runtime.conf").read_text()
    assert out["handlers"] == ["amd", "amd-cdi", "amd-legacy"] and out["cdi_spec"]
    rts = tomli.loads(cfg.read_text())["plugins"]["io.containerd.grpc.v1.cri"]["containerd"]["runtimes"]
    assert rts["amd"]["options"]["BinaryName"] == str(dest / "amd-container-runtime")
    inst.restart_mode = "none"
    inst.uninstall()
    assert tomli.loads(cfg.read_text()) == tomli.loads(CONTAINERD_V2)
    assert not dest.exists() and not (tmp_path / "cdi" / cdi.SPEC_NAME).exists()


def test_installer_socket_timeout(tmp_path):
    inst = ctk.Installer(root=str(tmp_path), runtime="docker", runtime_config=str(tmp_path / "d.json"),
                         runtime_socket=str(tmp_path / "none.sock"), socket_timeout=0.3)
    assert inst.wait_socket() is False


def test_install_daemon_cleans_up_on_stop(tmp_path, node, monkeypatch):
    root, dev = node
    cfg = tmp_path / "daemon.json"
    cfg.write_text("{}")
    monkeypatch.setenv("RUNTIME", "docker")
    monkeypatch.setenv("RUNTIME_CONFIG", str(cfg))
    monkeypatch.setenv("ROOT", str(tmp_path / "amd"))
    monkeypatch.setenv("RESTART_MODE", "none")
    stop = threading.Event()
    t = threading.Thread(target=ctk.main, args=(["install", "--daemon"], stop))
    t.start()
    for _ in range(100):
        if cfg.read_text() != "{}":
            break
        threading.Event().wait(0.05)
    assert "amd" in json.loads(cfg.read_text())["runtimes"]
    stop.set()
    t.join(10)
    assert json.loads(cfg.read_text()) == {}
