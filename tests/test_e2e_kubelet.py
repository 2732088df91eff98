"""The e2e harness's process kubelet (gpu_operator_amd/e2e/kubelet.py) on its own: pod lifecycle
semantics the e2e flow relies on -- restart policies, init-container ordering, termination
messages, readiness probes, ConfigMap volumes with subPath, env from fieldRef/ConfigMap, the
runtime-class gate, deletion killing the process group, scheduling by nodeSelector."""

import os
import time

import pytest

from gpu_operator_amd.e2e.kubelet import ProcessKubelet
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.k8s import objects as o

NODE = "kl-node"


@pytest.fixture
def kl(tmp_path):
    c = FakeClient([{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "t"}},
                    {"apiVersion": "v1", "kind": "Node",
                     "metadata": {"name": NODE, "labels": {"kubernetes.io/hostname": NODE}}, "status": {}}])
    base = f"/tmp/kl-{os.getpid()}-{int(time.time() * 1000) % 100000}"
    k = ProcessKubelet(c, NODE, base, dict(os.environ), host_links={}).start()
    yield c, k
    k.stop()
    k.cleanup()


def _pod(name, containers, init=None, policy="Never", **spec):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "t"},
            "spec": dict({"nodeName": NODE, "restartPolicy": policy, "containers": containers,
                          "initContainers": init or []}, **spec)}


def _wait(fn, timeout=20.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        v = fn()
        if v:
            return v
        time.sleep(0.05)
    raise AssertionError("timed out")


def _phase(c, name):
    return (c.get("v1", "Pod", name, "t").get("status") or {}).get("phase")


def test_init_order_env_configmap_subpath_and_termination_message(kl):
    c, k = kl
    c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm", "namespace": "t"},
              "data": {"run.sh": "echo from-script $MY_NODE $FROM_CM > /out/result\ncat /out/first\n",
                       "val": "cm-value"}})
    vol = [{"name": "s", "configMap": {"name": "cm", "defaultMode": 0o755}},
           {"name": "out", "emptyDir": {}}]
    init = [{"name": "first", "command": ["sh", "-c", "echo init-ran > /out/first"],
             "volumeMounts": [{"name": "out", "mountPath": "/out"}]}]
    main = [{"name": "main", "command": ["sh", "-c", "/bin/run.sh > /dev/termination-log"],
             "env": [{"name": "MY_NODE", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
                     {"name": "FROM_CM", "valueFrom": {"configMapKeyRef": {"name": "cm", "key": "val"}}}],
             "volumeMounts": [{"name": "s", "mountPath": "/bin/run.sh", "subPath": "run.sh"},
                              {"name": "out", "mountPath": "/out"}]}]
    c.create(_pod("p1", main, init, volumes=vol))
    _wait(lambda: _phase(c, "p1") == "Succeeded")
    st = c.get("v1", "Pod", "p1", "t")["status"]
    assert st["containerStatuses"][0]["state"]["terminated"]["message"].strip() == "init-ran"
    assert st["initContainerStatuses"][0]["state"]["terminated"]["exitCode"] == 0
    run = [d for d in os.listdir(os.path.join(k.base, "pods")) if "_p1_" in d][0]
    with open(os.path.join(k.base, "pods", run, "volumes", "out", "result")) as f:
        assert f.read().strip() == f"from-script {NODE} cm-value"


def test_restart_policies(kl):
    c, k = kl
    c.create(_pod("never", [{"name": "m", "command": ["sh", "-c", "exit 3"]}]))
    _wait(lambda: _phase(c, "never") == "Failed")
    # OnFailure: the first run fails (no marker yet), the restart succeeds
    flag = os.path.join(k.base, "flag")
    c.create(_pod("onfail", [{"name": "m", "command": ["sh", "-c", f"test -f {flag} || {{ touch {flag}; exit 1; }}"]}],
                  policy="OnFailure"))
    _wait(lambda: _phase(c, "onfail") == "Succeeded")
    assert c.get("v1", "Pod", "onfail", "t")["status"]["containerStatuses"][0]["restartCount"] == 1
    # a failing init container of a Never pod fails the pod; its main container never starts
    c.create(_pod("badinit", [{"name": "m", "command": ["sh", "-c", "sleep 30"]}],
                  init=[{"name": "i", "command": ["false"]}]))
    _wait(lambda: _phase(c, "badinit") == "Failed")
    assert "m" not in k.running().get("badinit").procs


def test_readiness_probe_gates_ready_and_deletion_kills_the_process_group(kl):
    c, k = kl
    ready_file = os.path.join(k.base, "ready-now")
    c.create(_pod("svc", [{"name": "m", "command": ["sh", "-c", "sleep 300 & wait"],
                           "readinessProbe": {"exec": {"command": ["test", "-f", ready_file]}}}], policy="Always"))
    _wait(lambda: _phase(c, "svc") == "Running")
    time.sleep(1.0)
    conds = {x["type"]: x["status"] for x in c.get("v1", "Pod", "svc", "t")["status"]["conditions"]}
    assert conds["Ready"] == "False"
    open(ready_file, "w").close()
    _wait(lambda: {x["type"]: x["status"] for x in c.get("v1", "Pod", "svc", "t")["status"]["conditions"]}
          ["Ready"] == "True")
    pids = k.all_pids()
    assert pids
    c.delete("v1", "Pod", "svc", "t")
    _wait(lambda: not k.all_pids())
    for pid in pids:
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


def test_runtime_class_gate_and_scheduling_by_node_selector(kl):
    c, k = kl
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "gated", "namespace": "t"},
              "spec": {"runtimeClassName": "amd", "restartPolicy": "Never",
                       "nodeSelector": {"kubernetes.io/hostname": NODE},
                       "containers": [{"name": "m", "command": ["true"]}]}})
    _wait(lambda: c.get("v1", "Pod", "gated", "t")["spec"].get("nodeName") == NODE)    # bound by the scheduler
    time.sleep(0.8)
    assert _phase(c, "gated") in (None, "Pending")              # no runtime handler yet: no sandbox
    cfg = k.host_path("/etc/containerd/config.toml")
    os.makedirs(os.path.dirname(cfg), exist_ok=True)
    with open(cfg, "w") as f:
        f.write('[plugins."io.containerd.grpc.v1.cri".containerd.runtimes.amd]\n  runtime_type = "x"\n')
    _wait(lambda: _phase(c, "gated") == "Succeeded")
    # a pod for another node is left alone
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "elsewhere", "namespace": "t"},
              "spec": {"nodeSelector": {"kubernetes.io/hostname": "other"}, "restartPolicy": "Never",
                       "containers": [{"name": "m", "command": ["true"]}]}})
    time.sleep(0.8)
    assert not c.get("v1", "Pod", "elsewhere", "t")["spec"].get("nodeName")
    assert o.name(c.get("v1", "Pod", "elsewhere", "t")) == "elsewhere"
