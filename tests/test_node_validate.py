"""amd-node-validate (native/node/node_validate.cpp) against validator/components.py on fake sysfs:
the same decisions, barrier names and payloads for driver, toolkit and the no-fabric rccl path."""

import json
import os
import subprocess
import time

import pytest

from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.validator import components as comp
from gpu_operator_amd.validator import status as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "gpu_operator_amd", "_native", "bin", "amd-node-validate")

pytestmark = pytest.mark.skipif(not os.path.exists(BIN), reason="native binaries not built")
VOLATILE = {"ts", "revalidated_ts", "validator"}


def native(component, root, out, env=None, *args):
    e = {k: v for k, v in os.environ.items() if k not in ("AMD_MOUNTS", "DRIVER_ROOT_MODE")}
    e.update({"AMD_SYSFS_ROOT": root, "AMD_DEV_ROOT": root, "OUTPUT_DIR": str(out), "HOST_ROOT": str(out) + "-host"})
    e.update(env or {})
    p = subprocess.run([BIN, component, *args], capture_output=True, text=True, timeout=30, env=e)
    return p.returncode, p.stdout, p.stderr


def python(component, root, out, env=None, **kw):
    ctx = comp.Context(status=S.StatusDir(str(out)), sys_root=root, dev_root=root, host_root=str(out) + "-host",
                       env=dict(env or {}), **kw)
    try:
        return 0, comp.COMPONENTS[component](ctx)
    except comp.ValidationError as e:
        return 1, str(e)


def barriers(out):
    return {n: {k: v for k, v in json.load(open(os.path.join(out, n))).items() if k not in VOLATILE}
            for n in sorted(os.listdir(out)) if not n.startswith(".")} if os.path.isdir(out) else {}


@pytest.fixture
def node(tmp_path):
    return str(fakesys.make_node(tmp_path / "root"))


@pytest.mark.parametrize("mode", ["host", "container"])
def test_driver_matches_the_python_validator(tmp_path, node, mode):
    env = {"DRIVER_ROOT_MODE": mode}
    for d in ("n", "p"):
        if mode == "container":                          # the driver pod's startup probe has run
            S.StatusDir(str(tmp_path / d)).create(S.DRIVER_CTR_READY)
    rc, out, err = native("driver", node, tmp_path / "n", env)
    assert rc == 0, err
    line = json.loads(out)
    assert python("driver", node, tmp_path / "p", env)[0] == 0
    assert barriers(tmp_path / "n") == barriers(tmp_path / "p")
    name = "host-driver-ready" if mode == "host" else "driver-ready"
    assert line["component"] == "driver" and line["info"]["mode"] == mode and name in barriers(tmp_path / "n")
    assert json.load(open(tmp_path / "n" / name))["validator"] == "native"


def test_driver_failures_match(tmp_path):
    dead = str(fakesys.make_node(tmp_path / "dead", live=False))
    rc, _, err = native("driver", dead, tmp_path / "n", {"DRIVER_ROOT_MODE": "host"})
    prc, msg = python("driver", dead, tmp_path / "p", {"DRIVER_ROOT_MODE": "host"})
    assert rc == prc == 1 and "not loaded" in err and "not loaded" in msg
    good = str(fakesys.make_node(tmp_path / "good"))
    rc, _, err = native("driver", good, tmp_path / "n2", {"DRIVER_ROOT_MODE": "container"})
    assert rc == 1 and ".driver-ctr-ready missing" in err and not barriers(tmp_path / "n2")
    t = time.monotonic()                                   # bounded wait for the driver container
    rc, _, err = native("driver", good, tmp_path / "n3", {"DRIVER_ROOT_MODE": "container", "WITH_WAIT": "true",
                                                          "WAIT_TIMEOUT_SECONDS": "0.5"})
    assert rc == 1 and "timed out" in err and time.monotonic() - t < 5


def test_driver_revalidation_keeps_the_first_ready_time(tmp_path, node):
    env = {"DRIVER_ROOT_MODE": "host"}
    assert native("driver", node, tmp_path / "n", env)[0] == 0
    first = json.load(open(tmp_path / "n" / "host-driver-ready"))
    time.sleep(0.05)
    assert native("driver", node, tmp_path / "n", env)[0] == 0
    again = json.load(open(tmp_path / "n" / "host-driver-ready"))
    assert again["ts"] == first["ts"] and again["revalidated_ts"] > first["ts"]
    # the Python validator does the same on the same barrier
    python("driver", node, tmp_path / "n", env)
    assert json.load(open(tmp_path / "n" / "host-driver-ready"))["ts"] == first["ts"]


def test_toolkit_matches_the_python_validator(tmp_path, node):
    rc, out, err = native("toolkit", node, tmp_path / "n")
    assert rc == 0, err
    assert python("toolkit", node, tmp_path / "p")[0] == 0
    assert barriers(tmp_path / "n") == barriers(tmp_path / "p") == {"toolkit-ready": {"render_nodes": 8, "kfd": True}}
    os.remove(os.path.join(node, "dev/dri/renderD131"))
    rc, _, err = native("toolkit", node, tmp_path / "n4")
    assert rc == 1 and "renderD131" in err


def test_rccl_without_a_fabric_is_native_and_with_one_is_not(tmp_path):
    one = str(fakesys.make_node(tmp_path / "one", n_gpus=1))
    rc, out, err = native("rccl", one, tmp_path / "n")
    assert rc == 0, err
    assert barriers(tmp_path / "n")["rccl-ready"] == {"skipped": "1 physical GPU(s): no fabric to validate",
                                                      "ok": True}
    eight = str(fakesys.make_node(tmp_path / "eight"))
    rc, out, _ = native("rccl", eight, tmp_path / "n8")
    assert rc == 3 and out == "" and not barriers(tmp_path / "n8")         # amd-validator takes over
    cpx = str(fakesys.make_node(tmp_path / "cpx", n_gpus=1, compute="CPX"))  # 8 agents, 1 physical GPU
    assert native("rccl", cpx, tmp_path / "nc")[0] == 0


def test_mount_table_maps_the_default_paths(tmp_path, node):
    """In a process-level harness AMD_MOUNTS carries the pod's volumes; the binary's default barrier
    dir (/run/amd/validations) resolves through it like utils/mounts.py."""
    e = {k: v for k, v in os.environ.items() if k not in ("OUTPUT_DIR", "HOST_ROOT")}
    e.update(AMD_SYSFS_ROOT=node, AMD_DEV_ROOT=node, DRIVER_ROOT_MODE="host",
             AMD_MOUNTS=json.dumps([["/run/amd/validations", str(tmp_path / "v")], ["/host", str(tmp_path / "h")]]))
    p = subprocess.run([BIN, "driver"], capture_output=True, text=True, timeout=30, env=e)
    assert p.returncode == 0, p.stderr
    assert os.path.exists(tmp_path / "v" / "host-driver-ready")


def _api(tmp_path, node_caps, tls=False):
    """The fake API server (HTTP, or HTTPS with a self-signed certificate for 127.0.0.1) holding one
    Node; returns (server, kubeconfig path)."""
    import ssl
    from gpu_operator_amd.k8s.apiserver import FakeAPIServer
    from gpu_operator_amd.k8s.fake import FakeClient
    node = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1"},
            "status": {"capacity": dict(node_caps), "allocatable": dict(node_caps)}}
    backing = FakeClient([node])
    srv = FakeAPIServer(backing)
    url = srv.url
    ca = ""
    if tls:
        key, crt = tmp_path / "key.pem", tmp_path / "crt.pem"
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=api",
                        "-addext", "subjectAltName=IP:127.0.0.1", "-keyout", str(key), "-out", str(crt)],
                       check=True, capture_output=True, timeout=60)
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(str(crt), str(key))
        srv.httpd.socket = ctx.wrap_socket(srv.httpd.socket, server_side=True)
        url = url.replace("http://", "https://")
        ca = f"    certificate-authority: {crt}\n"
    srv.start()
    kc = tmp_path / "kubeconfig"
    kc.write_text(f"apiVersion: v1\nkind: Config\ncurrent-context: t\nclusters:\n- cluster:\n    server: {url}\n{ca}"
                  "  name: t\ncontexts:\n- context:\n    cluster: t\n    user: t\n  name: t\nusers:\n- name: t\n"
                  "  user:\n    token: abc\n")
    return srv, backing, str(kc)


@pytest.mark.parametrize("tls", [False, True])
def test_plugin_reads_node_capacity_over_the_api(tmp_path, node, tls):
    srv, backing, kc = _api(tmp_path, {}, tls=tls)
    try:
        def advertise():
            time.sleep(0.5)                      # the device plugin registers after the check starts
            backing.patch("v1", "Node", "n1", {"status": {"capacity": {"amd.com/gpu": "8", "cpu": "96"}}})
        import threading
        threading.Thread(target=advertise, daemon=True).start()
        env = {"KUBECONFIG": kc, "NODE_NAME": "n1", "WITH_WORKLOAD": "false"}
        t = time.monotonic()
        rc, out, err = native("plugin", node, tmp_path / "n", env)
        assert rc == 0, err
        assert 0.4 < time.monotonic() - t < 10
        assert barriers(tmp_path / "n")["plugin-ready"] == {"resources": {"amd.com/gpu": 8}, "devices": 8}
        # the same barrier as the Python validator's
        from gpu_operator_amd.k8s.rest import Config, RestClient
        cl = RestClient(Config.from_kubeconfig(kc))
        ctx = comp.Context(status=S.StatusDir(str(tmp_path / "p")), node_name="n1", client=cl, env={})
        comp.validate_plugin(ctx)
        assert barriers(tmp_path / "p") == barriers(tmp_path / "n")
    finally:
        srv.stop()


def test_plugin_hands_over_what_it_does_not_handle(tmp_path, node):
    srv, backing, kc = _api(tmp_path, {"amd.com/gpu": "8", "amd.com/partition-cpx": "8"})
    try:
        base = {"KUBECONFIG": kc, "NODE_NAME": "n1", "WITH_WORKLOAD": "false"}
        assert native("plugin", node, tmp_path / "a", dict(base, WITH_WORKLOAD="true"))[0] == 3
        assert native("plugin", node, tmp_path / "b", dict(base, VALIDATOR_WAIT_MODE="poll"))[0] == 3
        assert native("plugin", node, tmp_path / "c", dict(base, NODE_NAME=""))[0] == 3
        assert native("plugin", node, tmp_path / "d", dict(base, KUBECONFIG=str(tmp_path / "none")))[0] == 3
        rc, _, err = native("plugin", node, tmp_path / "e", dict(base, PARTITION_STRATEGY="mixed"))
        assert rc == 0, err
        assert barriers(tmp_path / "e")["plugin-ready"]["devices"] == 16
        assert not any(os.listdir(tmp_path / d) for d in "abcd" if os.path.isdir(tmp_path / d))
    finally:
        srv.stop()


def test_plugin_watches_instead_of_polling(tmp_path, node):
    """capacity that appears 10 s after the check starts costs one GET and one
    watch on a kept-alive connection -- not a TLS connection every 100 ms (10 QPS per node)."""
    srv, backing, kc = _api(tmp_path, {})
    try:
        import threading

        def advertise():
            time.sleep(10.0)
            backing.patch("v1", "Node", "n1", {"status": {"capacity": {"amd.com/gpu": "8"}}})
        threading.Thread(target=advertise, daemon=True).start()
        t = time.monotonic()
        rc, out, err = native("plugin", node, tmp_path / "n", {"KUBECONFIG": kc, "NODE_NAME": "n1",
                                                               "WITH_WORKLOAD": "false"})
        took = time.monotonic() - t
        assert rc == 0, err
        assert 9.5 < took < 13, took                         # the watch event, not a poll tick
        assert srv.connections <= 5, srv.connections
        assert len(srv.requests) <= 5, srv.requests
        assert barriers(tmp_path / "n")["plugin-ready"]["devices"] == 8
    finally:
        srv.stop()


def test_kubeconfig_current_context_selects_the_user(tmp_path, node):
    """with two users the native check authenticates as the current context's user (the
    Python client's choice), not as whichever token line came last; an unknown context is handed over."""
    srv, backing, kc = _api(tmp_path, {"amd.com/gpu": "8"})
    try:
        text = open(kc).read().replace("current-context: t", "current-context: second")
        text = text.replace("contexts:\n", "contexts:\n- context:\n    cluster: t\n    user: u2\n  name: second\n")
        text += "- name: u2\n  user:\n    token: second-token\n- name: u3\n  user:\n    token: last-token\n"
        (tmp_path / "kc2").write_text(text)
        env = {"KUBECONFIG": str(tmp_path / "kc2"), "NODE_NAME": "n1", "WITH_WORKLOAD": "false"}
        rc, out, err = native("plugin", node, tmp_path / "n", env)
        assert rc == 0, err
        assert set(srv.authorization) == {"Bearer second-token"}, srv.authorization
        from gpu_operator_amd.k8s.rest import Config
        assert Config.from_kubeconfig(str(tmp_path / "kc2")).bearer() == "second-token"    # the same choice
        (tmp_path / "kc3").write_text(text.replace("current-context: second", "current-context: nope"))
        assert native("plugin", node, tmp_path / "m", dict(env, KUBECONFIG=str(tmp_path / "kc3")))[0] == 3
    finally:
        srv.stop()
