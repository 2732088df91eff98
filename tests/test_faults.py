"""Fault injection (SURVEY.md §5.3 build list): API errors mid-reconcile, a driver pod that
crashes after being ready, a barrier file removed mid-flight, a partition change while GPU
clients are still running, and an operator restart in the middle of a driver upgrade."""

import os
import threading
import time

from gpu_operator_amd.controllers import consts as C
from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.k8s import errors
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.sim import ClusterSim
from gpu_operator_amd.validator import components as comp
from gpu_operator_amd.validator import metrics as M
from gpu_operator_amd.validator import status as S

from k8s_helpers import cluster, gpu_node, reconciler, run_until_ready


def _state(c):
    return (c.get("amd.com/v1", "ClusterPolicy", "cluster-policy").get("status") or {})


def test_driver_pod_crash_flips_policy_not_ready_then_recovers():
    c = cluster([gpu_node("n1"), gpu_node("n2")])
    crashed = {"on": False}

    def ready(pod, node):
        return not (crashed["on"] and o.get_labels(pod).get("app") == C.DS_DRIVER and o.name(node) == "n2")
    sim = ClusterSim(c, ready_fn=ready)
    rec = reconciler(c)
    _, st = run_until_ready(c, rec, sim)
    assert st == "ready"
    crashed["on"] = True
    sim.sync()
    res = rec.reconcile(("", "cluster-policy"))
    assert _state(c)["state"] == "notReady" and "state-driver" in _state(c)["notReadyStates"]
    assert res.requeue_after == 5.0
    crashed["on"] = False
    _, st = run_until_ready(c, rec, sim)
    assert st == "ready"


def test_api_errors_on_every_kind_once_still_converge():
    c = cluster()
    rec = reconciler(c)
    for kind in ("DaemonSet", "ServiceAccount", "ConfigMap", "Node"):
        c.fail_on("create" if kind != "Node" else "patch", kind, errors.ApiError("etcd timeout", 500), times=1)
    c.fail_on("update_status", "ClusterPolicy", errors.Conflict("stale"), times=1)
    sim = ClusterSim(c)
    states = []
    for _ in range(8):
        try:
            rec.reconcile(("", "cluster-policy"))
        except errors.ApiError:
            pass
        sim.sync()
        states.append(_state(c).get("state"))
        if states[-1] == "ready":
            break
    assert states[-1] == "ready", states


def test_barrier_removed_mid_flight_reblocks_dependants(tmp_path):
    root = fakesys.make_node(tmp_path / "n", n_gpus=2)
    sd = S.StatusDir(str(tmp_path / "v"))
    ctx = comp.Context(status=sd, node_name="n1", sys_root=str(root), dev_root=str(root),
                       env={"DRIVER_ROOT_MODE": "host"})
    comp.validate_driver(ctx)
    sd.create(S.TOOLKIT_READY)
    m = M.NodeMetrics(ctx)
    m.refresh_status()
    assert m.barrier["driver"].labels("n1")._value.get() == 1
    # the driver pod's preStop removes its barriers (driver restart): dependants must block again
    sd.delete(S.HOST_DRIVER_READY)
    sd.delete(S.TOOLKIT_READY)
    m.refresh_status()
    assert m.barrier["driver"].labels("n1")._value.get() == 0
    got = {}

    def waiter():
        got["r"] = sd.wait([S.TOOLKIT_READY], timeout=10)
    t = threading.Thread(target=waiter)
    t.start()
    time.sleep(0.3)
    assert t.is_alive()                      # blocked on inotify, not polling a stale file
    comp.validate_driver(ctx)
    sd.create(S.TOOLKIT_READY)
    t.join(5)
    assert got["r"] == [S.TOOLKIT_READY]


def test_partition_change_under_load_waits_for_clients_then_applies(tmp_path):
    import yaml
    from gpu_operator_amd.operands import partition_manager as pm
    root = str(fakesys.make_node(tmp_path / "n", n_gpus=2))
    cfg = tmp_path / "c.yaml"
    cfg.write_text(yaml.safe_dump({"version": "v1", "partition-configs": {
        "cpx": [{"devices": "all", "compute": "CPX", "memory": "NPS1"}]}}))
    c = cluster([gpu_node("n1", extra_labels={pm.CONFIG_LABEL: "cpx",
                                               "amd.com/gpu.deploy.metrics-exporter": "true"})])
    # a telemetry pod holds the GPUs and only goes away after its DaemonSet's label flips
    c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "exp", "namespace": "gpu",
                                                               "labels": {"app": "amd-metrics-exporter"}},
              "spec": {"nodeName": "n1"}})

    def on_node(ev):
        if o.get_labels(ev.obj).get("amd.com/gpu.deploy.metrics-exporter") == pm.PAUSED:
            threading.Timer(0.3, lambda: c.delete("v1", "Pod", "exp", "gpu")).start()
    c.watch("v1", "Node", on_node)
    mgr = pm.PartitionManager(c, "n1", str(cfg), root=root, barrier_dir=str(tmp_path / "b"),
                              reenumerate=lambda: fakesys.set_compute_partition(root, "CPX", "NPS1"),
                              enum_timeout=5, pods_timeout=5)
    t0 = time.monotonic()
    assert mgr.reconcile() == "applied"
    assert time.monotonic() - t0 >= 0.3      # waited for the client to leave
    assert o.get_labels(c.get("v1", "Node", "n1"))["amd.com/gpu.deploy.metrics-exporter"] == "true"


def test_operator_restart_mid_upgrade_resumes_from_node_labels():
    """The upgrade FSM state lives on the Node: a fresh reconciler picks it up."""
    from gpu_operator_amd.controllers import upgrade as U
    c = cluster([gpu_node("n1")])
    rec = reconciler(c)
    run_until_ready(c, rec)
    c.patch("v1", "Node", "n1", {"metadata": {"labels": {U.UPGRADE_STATE_LABEL: U.CORDON_REQUIRED}}})
    # "restart": brand-new reconciler objects, same API state
    rec2 = reconciler(c)
    rec2.reconcile(("", "cluster-policy"))
    assert o.get_labels(c.get("v1", "Node", "n1"))[U.UPGRADE_STATE_LABEL] == U.CORDON_REQUIRED
