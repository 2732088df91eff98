"""The production REST client and the operator process against an in-process HTTP API server
(the envtest tier the reference never used)."""

import os
import signal
import subprocess
import sys
import threading
import time

import pytest
import yaml

from gpu_operator_amd.k8s import errors
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.apiserver import FakeAPIServer, plural
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.k8s.rest import Config, RestClient
from gpu_operator_amd.k8s.sim import ClusterSim

from k8s_helpers import NS, cluster, gpu_node, namespace, reconciler

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def api():
    srv = FakeAPIServer(FakeClient([namespace(), gpu_node("n1"), gpu_node("n2", gpu=False)]),
                        unserved=("ServiceMonitor",)).start()
    yield srv, RestClient(Config(srv.url, verify=False), timeout=10)
    srv.stop()


def _pod(name, node="n1", labels=None):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": NS, "labels": labels or {}},
            "spec": {"nodeName": node, "containers": [{"name": "c", "image": "x"}]}}


def test_plural_rules():
    assert [plural(k) for k in ("ClusterPolicy", "RuntimeClass", "SecurityContextConstraints", "Pod", "Ingress")] == \
        ["clusterpolicies", "runtimeclasses", "securitycontextconstraints", "pods", "ingresses"]


def test_crud_selectors_and_errors(api):
    srv, c = api
    assert c.server_version() == "v1.29.2"
    assert c.has_kind("apps/v1", "DaemonSet") and not c.has_kind("monitoring.coreos.com/v1", "ServiceMonitor")
    with pytest.raises(errors.NoKindMatch):
        c.get("monitoring.coreos.com/v1", "ServiceMonitor", "x", NS)
    p = c.create(_pod("a", labels={"app": "x"}))
    assert p["metadata"]["uid"] and p["metadata"]["namespace"] == NS
    c.create(_pod("b", node="n2", labels={"app": "y"}))
    with pytest.raises(errors.AlreadyExists):
        c.create(_pod("a"))
    assert [o.name(x) for x in c.list("v1", "Pod", NS, label_selector="app in (x,z)")] == ["a"]
    assert [o.name(x) for x in c.list("v1", "Pod", NS, label_selector={"app": "y"})] == ["b"]
    assert [o.name(x) for x in c.list("v1", "Pod", field_selector="spec.nodeName=n2")] == ["b"]
    assert {o.name(n) for n in c.list("v1", "Node")} == {"n1", "n2"}
    # optimistic concurrency over the wire
    cur = c.get("v1", "Pod", "a", NS)
    cur["metadata"]["labels"]["v"] = "1"
    c.update(cur)
    cur["metadata"]["labels"]["v"] = "2"
    with pytest.raises(errors.Conflict):
        c.update(cur)                                   # stale resourceVersion
    # merge patch + status subresource
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {"amd.com/gpu.present": "true", "gone": None}}})
    assert o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.present"] == "true"
    c.patch("v1", "Node", "n1", {"status": {"capacity": {"amd.com/gpu": "8"}}})
    assert c.get("v1", "Node", "n1")["status"]["capacity"]["amd.com/gpu"] == "8"
    c.delete("v1", "Pod", "b", NS)
    with pytest.raises(errors.NotFound):
        c.get("v1", "Pod", "b", NS)
    c.evict("a", NS)
    assert c.list("v1", "Pod", NS) == []
    c.create_event(c.get("v1", "Node", "n1"), "Test", "hello")
    evs = srv.client.objects("Event")
    assert evs and evs[0]["reason"] == "Test" and o.name(evs[0]).startswith("n1.")
    assert ("POST", f"/api/v1/namespaces/{NS}/pods/a/eviction") in srv.requests


def test_watch_stream(api):
    srv, c = api
    seen = []
    got = threading.Event()

    def cb(ev):
        seen.append((ev.type, o.name(ev.obj), o.get_labels(ev.old).get("x") if ev.old else None))
        if ev.type == "DELETED":
            got.set()
    stop = c.watch("v1", "Pod", cb, NS)
    try:
        time.sleep(0.5)                                   # initial list + watch established
        c.create(_pod("w"))
        time.sleep(0.2)
        c.patch("v1", "Pod", "w", {"metadata": {"labels": {"x": "1"}}}, NS)
        time.sleep(0.2)
        c.delete("v1", "Pod", "w", NS)
        assert got.wait(10)
    finally:
        stop()
    assert [s[:2] for s in seen] == [("ADDED", "w"), ("MODIFIED", "w"), ("DELETED", "w")]
    assert seen[2][2] == "1"                              # DELETED carries the last known object


def test_reconciler_over_http_reaches_ready():
    backing = cluster([gpu_node(f"n{i}") for i in range(3)])
    with FakeAPIServer(backing, unserved=("ServiceMonitor", "PrometheusRule")) as srv:
        rc = RestClient(Config(srv.url, verify=False), timeout=10)
        rec = reconciler(rc)
        sim = ClusterSim(backing)
        state = None
        for _ in range(6):
            rec.reconcile(("", "cluster-policy"))
            sim.sync()
            state = rc.get("amd.com/v1", "ClusterPolicy", "cluster-policy").get("status", {}).get("state")
            if state == "ready":
                break
        assert state == "ready"
        assert any(p.startswith("/apis/apps/v1/namespaces/") for _, p in srv.requests)


def test_operator_process_end_to_end(tmp_path):
    """`amd-gpu-operator` as a real process: kubeconfig -> HTTP API, leader election Lease,
    watches, reconcile to ready while a simulated kubelet/DaemonSet controller runs."""
    backing = cluster([gpu_node("n1"), gpu_node("n2")])
    with FakeAPIServer(backing, unserved=("ServiceMonitor", "PrometheusRule")) as srv:
        kc = tmp_path / "kubeconfig"
        kc.write_text(yaml.safe_dump({
            "apiVersion": "v1", "kind": "Config", "current-context": "t",
            "clusters": [{"name": "t", "cluster": {"server": srv.url}}],
            "contexts": [{"name": "t", "context": {"cluster": "t", "user": "u"}}],
            "users": [{"name": "u", "user": {}}]}))
        env = dict(os.environ, OPERATOR_NAMESPACE=NS, PYTHONPATH=ROOT)
        proc = subprocess.Popen([sys.executable, "-m", "gpu_operator_amd.cmd.operator", "--kubeconfig", str(kc),
                                 "--leader-elect", "--metrics-bind-address", "127.0.0.1:0",
                                 "--health-probe-bind-address", "127.0.0.1:0"],
                                env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        sim = ClusterSim(backing)
        state = None
        try:
            deadline = time.monotonic() + 90
            while time.monotonic() < deadline and proc.poll() is None:
                sim.sync()
                state = (backing.get("amd.com/v1", "ClusterPolicy", "cluster-policy").get("status") or {}).get("state")
                if state == "ready":
                    break
                time.sleep(0.5)
            leases = backing.objects("Lease")
        finally:
            proc.send_signal(signal.SIGTERM)
            try:
                out, _ = proc.communicate(timeout=20)
            except subprocess.TimeoutExpired:
                proc.kill()
                out, _ = proc.communicate()
        assert state == "ready", out[-3000:]
        assert leases and o.name(leases[0]) == "53822513.amd.com"
        labels = o.get_labels(backing.get("v1", "Node", "n1"))
        assert labels.get("amd.com/gpu.present") == "true" and labels.get("amd.com/gpu.deploy.device-plugin") == "true"


def test_watch_with_field_selector_sees_only_its_node(api):
    """node agents watch their own Node (metadata.name=<node>) -- the selector
    reaches the API server on the list and on the watch, so other nodes' updates never arrive."""
    srv, c = api
    for n in ("a", "b"):
        c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": n, "labels": {}}})
    seen = []
    got = threading.Event()

    def cb(ev):
        seen.append((ev.type, o.name(ev.obj)))
        if o.get_labels(ev.obj).get("x") == "2":
            got.set()
    stop = c.watch("v1", "Node", cb, field_selector="metadata.name=b")
    try:
        time.sleep(0.5)
        c.patch("v1", "Node", "a", {"metadata": {"labels": {"x": "1"}}})
        c.patch("v1", "Node", "b", {"metadata": {"labels": {"x": "2"}}})
        assert got.wait(10)
    finally:
        stop()
    assert seen == [("ADDED", "b"), ("MODIFIED", "b")]


class _ScriptedServer:
    """A raw HTTP/1.1 server whose every request follows a script: "ok" (200, kept alive), "drop"
    (the connection closes with no response byte, as a server closing an idle kept-alive
    connection does) or "hang" (no response until the client gives up)."""

    def __init__(self, script, idle_close_s=None):
        import socket as so
        self.script, self.seen = list(script), []
        self.idle_close_s = idle_close_s        # close a kept-alive connection idle this long (a proxy)
        self.sock = so.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(8)
        self.url = f"http://127.0.0.1:{self.sock.getsockname()[1]}"
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while True:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._conn, args=(c,), daemon=True).start()

    def _conn(self, c):
        import socket as so
        buf = b""
        c.settimeout(self.idle_close_s)
        while True:
            while b"\r\n\r\n" not in buf:
                try:
                    d = c.recv(65536)
                except so.timeout:
                    d = b""
                if not d:
                    c.close()
                    return
                buf += d
            head, buf = buf.split(b"\r\n\r\n", 1)
            n = 0
            for ln in head.split(b"\r\n")[1:]:
                if ln.lower().startswith(b"content-length:"):
                    n = int(ln.split(b":")[1])
            while len(buf) < n:
                buf += c.recv(65536)
            buf = buf[n:]
            self.seen.append(head.split(b" ")[0].decode())
            what = self.script.pop(0) if self.script else "ok"
            if what == "drop":
                c.close()
                return
            if what == "hang":
                time.sleep(3)
                c.close()
                return
            body = b'{"kind":"Status","apiVersion":"v1","metadata":{"name":"x"}}'
            c.sendall(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: " +
                      str(len(body)).encode() + b"\r\n\r\n" + body)

    def stop(self):
        self.sock.close()


def test_transport_retries_only_idempotent_requests_on_a_dropped_keepalive(monkeypatch):
    """a dropped kept-alive connection is retried once for GET/PUT/DELETE; a POST is never
    sent twice (it goes out on a fresh connection when the kept one may have gone stale); a timeout is
    never retried (the request may have been applied)."""
    from gpu_operator_amd.k8s import rest
    srv = _ScriptedServer(["ok", "drop", "ok"])
    t = rest._Transport(Config(srv.url, verify=False))
    assert t.request("GET", "/api/v1/nodes/a", None, {}, 5).status_code == 200
    assert t.request("GET", "/api/v1/nodes/a", None, {}, 5).status_code == 200     # dropped, retried once
    assert srv.seen == ["GET", "GET", "GET"]
    srv.stop()
    # POST on a connection idle past the trust window: a fresh connection, one send
    monkeypatch.setattr(rest, "_KEEPALIVE_TRUST_S", 0.0)
    srv = _ScriptedServer(["ok", "ok"])
    t = rest._Transport(Config(srv.url, verify=False))
    t.request("GET", "/x", None, {}, 5)
    assert t.request("POST", "/x", b"{}", {"Content-Type": "application/json"}, 5).status_code == 200
    assert srv.seen == ["GET", "POST"]
    srv.stop()
    # a dropped POST is an error, not a second POST
    monkeypatch.setattr(rest, "_KEEPALIVE_TRUST_S", 60.0)
    srv = _ScriptedServer(["ok", "drop", "ok"])
    t = rest._Transport(Config(srv.url, verify=False))
    t.request("GET", "/x", None, {}, 5)
    with pytest.raises(OSError):
        t.request("POST", "/x", b"{}", {"Content-Type": "application/json"}, 5)
    assert srv.seen == ["GET", "POST"]
    srv.stop()
    # a timed-out GET is not re-sent
    srv = _ScriptedServer(["ok", "hang", "ok"])
    t = rest._Transport(Config(srv.url, verify=False))
    t.request("GET", "/x", None, {}, 5)
    with pytest.raises(OSError):
        t.request("GET", "/x", None, {}, 0.5)
    time.sleep(0.2)
    assert srv.seen == ["GET", "GET"]
    srv.stop()


def test_merge_patch_and_post_survive_a_proxy_that_closes_idle_connections_after_1s():
    """with a proxy closing idle kept-alive connections after 1 s (sooner than the 5 s we
    trust one), a label merge-PATCH on the reused connection used to raise to its caller (the upgrade
    FSM does not retry). A merge patch is safe to re-send: it is retried once on a fresh connection.
    A POST always takes a fresh connection, so it is sent once and succeeds."""
    from gpu_operator_amd.k8s import rest
    srv = _ScriptedServer([], idle_close_s=1.0)
    t = rest._Transport(Config(srv.url, verify=False))
    merge = {"Content-Type": "application/merge-patch+json"}
    assert t.request("GET", "/api/v1/nodes/a", None, {}, 5).status_code == 200
    time.sleep(1.5)                                  # the proxy has closed the kept-alive connection
    assert t.request("PATCH", "/api/v1/nodes/a", b'{"metadata":{"labels":{"x":"1"}}}', merge, 5).status_code == 200
    time.sleep(1.5)
    assert t.request("POST", "/api/v1/namespaces/d/pods", b"{}", {"Content-Type": "application/json"},
                     5).status_code == 200
    assert srv.seen == ["GET", "PATCH", "POST"]       # each applied exactly once
    # a JSON patch (not idempotent) inside the trust window on a dropped connection: an error, sent once
    srv.stop()
    srv = _ScriptedServer(["ok", "drop", "ok"])
    t = rest._Transport(Config(srv.url, verify=False))
    t.request("GET", "/x", None, {}, 5)
    with pytest.raises(OSError):
        t.request("PATCH", "/x", b"[]", {"Content-Type": "application/json-patch+json"}, 5)
    assert srv.seen == ["GET", "PATCH"]
    srv.stop()
