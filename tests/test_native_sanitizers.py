"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5.2:
the reference has no race/sanitizer tier; its Go equivalent would be `go test -race`).

libamdnode (sysfs/KFD parsing), the barrier waiter, the OCI runtime shim (JSON parser, bundle
rewrite) and amd-node-validate (a hand-rolled HTTP/TLS client: chunked transfer, watch stream,
kubeconfig reader) are rebuilt with -fsanitize=address,undefined and driven over fake sysfs trees,
partition re-enumeration, malformed inputs and bundles, and a scripted API server that splits chunked
bodies at every byte, truncates and oversizes chunks, sends malformed JSON and 410 Gone mid-watch; two
random-input loops cover minijson.h and amd-gemm-validate's launcher <-> worker line protocol
(tests/native/fuzz_*.cpp). Any sanitizer report fails the test."""

import json
import os
import shutil
import subprocess
import threading
import time

import pytest

from gpu_operator_amd.devices import fakesys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "native")
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


@pytest.fixture(scope="module")
def bins(tmp_path_factory):
    out = tmp_path_factory.mktemp("asan")
    tests_native = os.path.join(ROOT, "tests", "native")
    targets = {
        "probe": (["node/node_probe.cpp", "node/amdnode.cpp"], []),
        "wait": (["node/barrier_wait.cpp", "node/amdnode.cpp"], []),
        "shim": (["toolkit/amd_container_runtime.cpp", "node/amdnode.cpp"], []),
        "nodeval": (["node/node_validate.cpp", "node/amdnode.cpp"], ["-lssl", "-lcrypto", "-ldl", "-lpthread"]),
        "fuzz_json": ([os.path.join(tests_native, "fuzz_minijson.cpp")], []),
        "fuzz_proto": ([os.path.join(tests_native, "fuzz_protocol.cpp")], []),
    }
    paths = {}
    procs = {}
    for name, (srcs, libs) in targets.items():
        exe = str(out / name)
        cmd = ["g++", "-std=c++17", f"-I{NATIVE}/include"] + SAN + [os.path.join(NATIVE, s) for s in srcs] + \
            ["-o", exe] + libs
        procs[name] = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        paths[name] = exe
    for name, p in procs.items():
        _, err = p.communicate(timeout=300)
        assert p.returncode == 0, err[-3000:]
    return paths


def _run(cmd, **kw):
    p = subprocess.run(cmd, capture_output=True, text=True, env=kw.pop("env", ENV), timeout=60, **kw)
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    return p


@pytest.mark.parametrize("compute,memory", [("SPX", "NPS1"), ("CPX", "NPS2"), ("QPX", "NPS1")])
def test_node_probe_clean(bins, tmp_path, compute, memory):
    root = fakesys.make_node(tmp_path / "n", compute=compute, memory=memory, sriov_totalvfs=4)
    fakesys.create_vfs(root, "0000:05:00.0", 2, driver="vfio-pci")
    p = _run([bins["probe"], "--root", str(root)])
    assert p.returncode == 0
    doc = json.loads(p.stdout)
    assert len(doc["gpus"]) == 8 * {"SPX": 1, "QPX": 4, "CPX": 8}[compute]


def test_node_probe_malformed_tree(bins, tmp_path):
    root = fakesys.make_node(tmp_path / "n", n_gpus=2)
    props = root / "sys/class/kfd/kfd/topology/nodes/1/properties"
    props.write_text("simd_count\nlocation_id not-a-number\n" + "x" * 5000 + "\n\n  \n")
    (root / "sys/bus/pci/devices/0000:05:00.0/current_compute_partition").write_text("")
    (root / "sys/bus/pci/devices/0000:15:00.0/hwmon/hwmon3/power1_average").write_text("garbage")
    p = _run([bins["probe"], "--root", str(root)])
    assert p.returncode == 0
    empty = tmp_path / "empty"
    empty.mkdir()
    assert _run([bins["probe"], "--root", str(empty)]).returncode == 0


def test_barrier_wait_clean(bins, tmp_path):
    d = tmp_path / "v"
    d.mkdir()
    threading.Timer(0.3, lambda: (d / "toolkit-ready").write_text("{}")).start()
    assert _run([bins["wait"], "--dir", str(d), "--all", "toolkit-ready", "--timeout", "10"]).returncode == 0
    assert _run([bins["wait"], "--dir", str(d), "--any", "nope,also-nope", "--timeout", "1"]).returncode == 1
    assert _run([bins["wait"], "--bogus"]).returncode == 2


def test_runtime_shim_clean(bins, tmp_path):
    root = fakesys.make_node(tmp_path / "n", n_gpus=2)
    dev = tmp_path / "dev"
    (dev / "dev/dri").mkdir(parents=True)
    os.symlink("/dev/null", dev / "dev/kfd")
    for i in range(2):
        os.symlink("/dev/null", dev / f"dev/dri/renderD{128 + i}")
    env = dict(ENV, AMD_CONTAINER_RUNTIME_RUNTIMES="/bin/true", AMD_CONTAINER_RUNTIME_SYS_ROOT=str(root),
               AMD_CONTAINER_RUNTIME_DEV_ROOT=str(dev), AMD_CONTAINER_RUNTIME_CDI_SPEC_DIRS=str(tmp_path / "cdi"))
    cases = {
        "ok": {"process": {"env": ["AMD_VISIBLE_DEVICES=all", "X=\"q\\u00e9\\ud83d\\ude00\""]},
               "linux": {"resources": {"memory": {"limit": 1.5e20}}}, "annotations": {"a": "b"}},
        "nested": {"a": [[[[{"b": [1, -2.5e-3, True, False, None, "\\n\\t"]}]]]],
                   "process": {"env": ["AMD_VISIBLE_DEVICES=0"]}},
    }
    for name, spec in cases.items():
        b = tmp_path / name
        b.mkdir()
        (b / "config.json").write_text(json.dumps(spec))
        p = _run([bins["shim"], "--root", "/r", "create", "--bundle", str(b), "c"], env=env)
        assert p.returncode == 0, p.stderr
        json.loads((b / "config.json").read_text())
    for bad in ('{"process": {"env": ["AMD_VISIBLE_DEVICES=0"]', '{"a": "\\uZZZZ"}', "[" * 300 + "]" * 300,
                '{"a": 1,}', ""):
        b = tmp_path / f"bad{abs(hash(bad))}"
        b.mkdir()
        (b / "config.json").write_text(bad)
        p = _run([bins["shim"], "create", "--bundle", str(b), "c"], env=env)
        assert p.returncode in (0, 1)



# ------------------------------------------------------------------------------ random-input loops
@pytest.mark.parametrize("name,seed", [("fuzz_json", 1), ("fuzz_json", 2), ("fuzz_proto", 1), ("fuzz_proto", 2)])
def test_random_input_loops(bins, name, seed):
    p = _run([bins[name], "30000", str(seed)])
    assert p.returncode == 0, p.stderr[-3000:]
    assert json.loads(p.stdout.strip().splitlines()[-1])["failures"] == 0


# ------------------------------------------------------------------------------ amd-node-validate vs a hostile API
class RawAPI:
    """A raw HTTP/1.1 server: each request gets the next scripted reply -- raw bytes, framing exactly
    as given -- and the connection is closed after it when the entry says so. Records each request's
    first line and Authorization header."""

    def __init__(self, replies):
        import socket as so
        self.replies, self.seen = list(replies), []
        self.sock = so.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(16)
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
        buf = b""
        try:
            while True:
                while b"\r\n\r\n" not in buf:
                    d = c.recv(65536)
                    if not d:
                        return
                    buf += d
                head, buf = buf.split(b"\r\n\r\n", 1)
                lines = head.split(b"\r\n")
                auth = [ln.split(b":", 1)[1].strip().decode() for ln in lines[1:] if ln.lower().startswith(b"authorization:")]
                self.seen.append((lines[0].decode(), auth[0] if auth else ""))
                if not self.replies:
                    return
                raw, close = self.replies.pop(0)
                for piece in (raw if isinstance(raw, list) else [raw]):
                    c.sendall(piece)
                    time.sleep(0.001)
                if close:
                    return
        except OSError:
            return
        finally:
            c.close()

    def stop(self):
        self.sock.close()


def _node(caps):
    return json.dumps({"kind": "Node", "metadata": {"name": "n1", "resourceVersion": "7"},
                       "status": {"capacity": caps}}).encode()


def _event(kind, caps=None, code=None):
    obj = {"kind": "Status", "code": code, "reason": "Expired"} if code else json.loads(_node(caps or {}))
    return json.dumps({"type": kind, "object": obj}).encode() + b"\n"


def _chunked(body, sizes=None):
    out, i = [], 0
    sizes = sizes or [1] * len(body)
    for n in sizes:
        if i >= len(body):
            break
        piece = body[i:i + n]
        out.append(b"%x\r\n" % len(piece) + piece + b"\r\n")
        i += n
    if i < len(body):
        out.append(b"%x\r\n" % (len(body) - i) + body[i:] + b"\r\n")
    return b"".join(out) + b"0\r\n\r\n"


def _resp(body, chunked=None, status=b"200 OK", extra=b""):
    if chunked is not None:
        return b"HTTP/1.1 " + status + b"\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n" + extra + \
            b"\r\n" + _chunked(body, chunked)
    return b"HTTP/1.1 " + status + b"\r\nContent-Type: application/json\r\nContent-Length: " + \
        str(len(body)).encode() + b"\r\n" + extra + b"\r\n" + body


def _kubeconfig(tmp_path, url, two_users=False):
    kc = tmp_path / "kubeconfig"
    text = (f"apiVersion: v1\nkind: Config\ncurrent-context: {'second' if two_users else 't'}\nclusters:\n- cluster:\n"
            f"    server: {url}\n  name: t\ncontexts:\n- context:\n    cluster: t\n    user: t\n  name: t\n")
    if two_users:
        text += "- context:\n    cluster: t\n    user: u2\n  name: second\n"
    text += "users:\n- name: t\n  user:\n    token: first-token\n"
    if two_users:
        text += "- name: u2\n  user:\n    token: second-token\n"
    kc.write_text(text)
    return str(kc)


def _plugin(bins, tmp_path, api, two_users=False, timeout_s="20"):
    out = tmp_path / "out"
    env = dict(ENV, KUBECONFIG=_kubeconfig(tmp_path, api.url, two_users), NODE_NAME="n1", WITH_WORKLOAD="false",
               OUTPUT_DIR=str(out), RESOURCE_TIMEOUT_SECONDS=timeout_s)
    env.pop("KUBERNETES_SERVICE_HOST", None)
    p = _run([bins["nodeval"], "plugin"], env=env)
    ready = out / "plugin-ready"
    return p, json.loads(ready.read_text()) if ready.exists() else None


def test_node_validate_chunked_node_split_at_every_byte(bins, tmp_path):
    body = _node({"amd.com/gpu": "8", "cpu": "96"})
    api = RawAPI([(_resp(body, chunked=[1] * len(body)), False)])
    try:
        p, ready = _plugin(bins, tmp_path, api)
        assert p.returncode == 0, p.stderr[-2000:]
        assert ready["devices"] == 8
    finally:
        api.stop()


@pytest.mark.parametrize("split", ["every-byte", "random-a", "random-b", "one-chunk"])
def test_node_validate_watch_events_split_anywhere(bins, tmp_path, split):
    import random
    events = _event("ADDED", {"cpu": "96"}) + _event("MODIFIED", {"cpu": "96"}) + \
        _event("MODIFIED", {"amd.com/gpu": "4"})
    if split == "every-byte":
        sizes = [1] * len(events)
    elif split == "one-chunk":
        sizes = [len(events)]
    else:
        rng = random.Random(split)
        sizes = [rng.randint(1, 40) for _ in range(len(events))]
    api = RawAPI([(_resp(_node({"cpu": "96"})), False), (_resp(events, chunked=sizes), False)])
    try:
        p, ready = _plugin(bins, tmp_path, api)
        assert p.returncode == 0, p.stderr[-2000:]
        assert ready["devices"] == 4
        assert [r[0].split(" ")[1].split("?")[0] for r in api.seen] == ["/api/v1/nodes/n1", "/api/v1/nodes"]
    finally:
        api.stop()


def test_node_validate_410_gone_mid_watch_lists_again(bins, tmp_path):
    watch = _event("ADDED", {"cpu": "96"}) + _event("ERROR", code=410)
    api = RawAPI([(_resp(_node({})), False), (_resp(watch, chunked=[7] * 40), True),
                  (_resp(_node({"amd.com/gpu": "8"}), chunked=[13] * 40), False)])
    try:
        p, ready = _plugin(bins, tmp_path, api)
        assert p.returncode == 0, p.stderr[-2000:]
        assert ready["devices"] == 8
        assert len(api.seen) == 3 and "watch=1" in api.seen[1][0]
    finally:
        api.stop()


@pytest.mark.parametrize("case", ["truncated-chunk", "oversized-chunk", "bad-chunk-size", "malformed-json",
                                  "bad-status-line", "negative-length", "huge-length", "endless-header",
                                  "json-wrong-types", "garbage-watch"])
def test_node_validate_hostile_replies_hand_over_cleanly(bins, tmp_path, case):
    """Malformed API replies: the native check hands over (exit 3) or keeps waiting until its budget --
    never a crash, a sanitizer report, or a barrier written from a broken reply."""
    body = _node({"amd.com/gpu": "8"})
    replies = {
        "truncated-chunk": [(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n100\r\n" + body[:10], True)],
        "oversized-chunk": [(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nffffffffffffffff\r\n" + body, True)],
        "bad-chunk-size": [(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n" + body + b"\r\n0\r\n\r\n",
                            True)],
        "malformed-json": [(_resp(b'{"kind":"Node","status":{"capacity":{"amd.com/gpu":8'), False)],
        "bad-status-line": [(b"HTTP/1.1\r\n\r\n", True)],
        "negative-length": [(b"HTTP/1.1 200 OK\r\nContent-Length: -5\r\n\r\n" + body, True)],
        "huge-length": [(b"HTTP/1.1 200 OK\r\nContent-Length: 99999999999999999999\r\n\r\n" + body, True)],
        "endless-header": [(b"HTTP/1.1 200 OK\r\nX: " + b"a" * (1 << 20), True)],
        "json-wrong-types": [(_resp(b'{"status":{"capacity":{"amd.com/gpu":{"x":[1,2]}}},"metadata":[]}'), False),
                             (_resp(b'{"type":7,"object":"x"}\n', chunked=[3] * 10), True)],
        "garbage-watch": [(_resp(_node({})), False),
                          (_resp(b"\xff\xfe\x00not json\n{\"type\":\n", chunked=[2] * 20), True)],
    }[case]
    api = RawAPI(replies)
    try:
        p, ready = _plugin(bins, tmp_path, api, timeout_s="3")
        # negative-length reads the body up to the close: a valid Node, so the check may pass
        if case == "negative-length" and p.returncode == 0:
            assert ready["devices"] == 8
        else:
            assert p.returncode in (1, 3), (p.returncode, p.stderr[-2000:])
            assert ready is None
    finally:
        api.stop()


def test_node_validate_two_user_kubeconfig_uses_the_current_context(bins, tmp_path):
    api = RawAPI([(_resp(_node({"amd.com/gpu": "2"})), False)])
    try:
        p, ready = _plugin(bins, tmp_path, api, two_users=True)
        assert p.returncode == 0, p.stderr[-2000:]
        assert ready["devices"] == 2 and [a for _, a in api.seen] == ["Bearer second-token"]
    finally:
        api.stop()
