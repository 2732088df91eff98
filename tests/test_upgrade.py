"""Rolling driver upgrade FSM, end to end over a simulated multi-node cluster."""

import pytest

from gpu_operator_amd.controllers import consts as C
from gpu_operator_amd.controllers import upgrade as U
from gpu_operator_amd.controllers.upgrade_controller import UpgradeReconciler
from gpu_operator_amd.k8s import errors
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.sim import ClusterSim
from k8s_helpers import NS, cluster, gpu_node, reconciler, run_until_ready, sample_cp


def gpu_workload(node, name, owner=True, emptydir=False):
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": name, "namespace": "default"},
           "spec": {"nodeName": node, "containers": [{"name": "train", "image": "rocm/pytorch",
                                                      "resources": {"limits": {"amd.com/gpu": 8}}}]},
           "status": {"phase": "Running"}}
    if owner:
        pod["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs",
                                               "uid": "rs-uid", "controller": True}]
    if emptydir:
        pod["spec"]["volumes"] = [{"name": "scratch", "emptyDir": {}}]
    return pod


def setup(n_nodes=3, **policy):
    cp = sample_cp()
    cp["spec"]["driver"]["upgradePolicy"].update(policy)
    c = cluster([gpu_node(f"n{i}") for i in range(n_nodes)], cp)
    rec = reconciler(c)
    sim = ClusterSim(c)
    run_until_ready(c, rec, sim)
    up = UpgradeReconciler(c, NS, rec.sm.snapshot, rec.metrics, run_async=False)
    return c, rec, sim, up


def bump_driver(c, version="6.13.1"):
    cp = c.get("amd.com/v1", "ClusterPolicy", "cluster-policy")
    cp["spec"]["driver"]["version"] = version
    c.update(cp)


def states(c):
    return {o.name(n): o.get_labels(n).get(U.UPGRADE_STATE_LABEL, "") for n in c.list("v1", "Node")}


def step(c, rec, sim, up, max_in_progress=None):
    up.reconcile(("", "cluster-policy"))
    sim.sync()
    rec.reconcile(("", "cluster-policy"))
    if max_in_progress is not None:
        in_prog = [s for s in states(c).values() if s in U.IN_PROGRESS]
        assert len(in_prog) <= max_in_progress, states(c)


def test_initial_pass_marks_nodes_done():
    c, rec, sim, up = setup()
    up.reconcile(("", "cluster-policy"))
    assert set(states(c).values()) == {U.DONE}


def test_rolling_upgrade_one_node_at_a_time_evicts_gpu_pods():
    c, rec, sim, up = setup(maxParallelUpgrades=1, maxUnavailable="100%")
    up.reconcile(("", "cluster-policy"))
    c.create(gpu_workload("n0", "job-0"))
    c.create(gpu_workload("n1", "job-1"))
    cpu_pod = gpu_workload("n0", "web")
    cpu_pod["spec"]["containers"][0]["resources"] = {}
    c.create(cpu_pod)
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    seen = set()
    for _ in range(60):
        step(c, rec, sim, up, max_in_progress=1)
        seen.update(states(c).values())
        if set(states(c).values()) == {U.DONE} and U.UPGRADE_REQUIRED in seen:
            break
    assert set(states(c).values()) == {U.DONE}, states(c)
    visited = {e["message"].rsplit(" ", 1)[-1] for e in c.events if e["reason"] == U.EVENT_REASON}
    assert {U.UPGRADE_REQUIRED, U.CORDON_REQUIRED, U.WAIT_FOR_JOBS_REQUIRED, U.POD_DELETION_REQUIRED,
            U.POD_RESTART_REQUIRED, U.VALIDATION_REQUIRED, U.UNCORDON_REQUIRED, U.DONE} <= visited
    names = {o.name(p) for p in c.list("v1", "Pod", "default")}
    assert names == {"web"}                                       # GPU pods evicted, CPU pod kept
    assert not any((n.get("spec") or {}).get("unschedulable") for n in c.list("v1", "Node"))
    ds = c.get("apps/v1", "DaemonSet", C.DS_DRIVER, NS)
    rev = up.mgr.ds_revision_hash(ds)
    drv_pods = [p for p in c.list("v1", "Pod", NS, label_selector={"app": C.DS_DRIVER})]
    assert len(drv_pods) == 3 and all(o.get_labels(p)["controller-revision-hash"] == rev for p in drv_pods)


def test_max_unavailable_limits_parallelism():
    c, rec, sim, up = setup(n_nodes=4, maxParallelUpgrades=0, maxUnavailable="50%")
    up.reconcile(("", "cluster-policy"))
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(60):
        step(c, rec, sim, up, max_in_progress=2)
        if set(states(c).values()) == {U.DONE}:
            break
    assert set(states(c).values()) == {U.DONE}


def test_skip_label_and_precordoned_node_stays_cordoned():
    c, rec, sim, up = setup(n_nodes=2, maxParallelUpgrades=2)
    up.reconcile(("", "cluster-policy"))
    c.patch("v1", "Node", "n0", {"metadata": {"labels": {U.UPGRADE_SKIP_NODE_LABEL: "true"}}})
    c.patch("v1", "Node", "n1", {"spec": {"unschedulable": True}})
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(40):
        step(c, rec, sim, up)
    st = states(c)
    assert st["n0"] == U.UPGRADE_REQUIRED            # skipped
    assert st["n1"] == U.DONE
    assert c.get("v1", "Node", "n1")["spec"]["unschedulable"] is True


def test_unmanaged_gpu_pod_blocks_and_times_out_to_failed_without_drain():
    clock = [1000.0]
    c, rec, sim, up = setup(n_nodes=1, podDeletion={"timeoutSeconds": 30})
    up.mgr.clock = lambda: clock[0]
    up.reconcile(("", "cluster-policy"))
    c.create(gpu_workload("n0", "bare", owner=False))
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(10):
        step(c, rec, sim, up)
        clock[0] += 10
    assert states(c)["n0"] == U.FAILED
    assert any(e["reason"] == U.EVENT_REASON and e["type"] == "Warning" for e in c.events)


def test_failed_node_recovers_once_driver_pod_in_sync():
    c, rec, sim, up = setup(n_nodes=1, podDeletion={"force": True})
    up.reconcile(("", "cluster-policy"))
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    c.patch("v1", "Node", "n0", {"metadata": {"labels": {U.UPGRADE_STATE_LABEL: U.FAILED}}})
    for _ in range(20):
        step(c, rec, sim, up)
    # a failed node with an out-of-date pod stays failed until an admin restarts the pod
    assert states(c)["n0"] == U.FAILED
    for p in c.list("v1", "Pod", NS, label_selector={"app": C.DS_DRIVER}):
        c.delete("v1", "Pod", o.name(p), NS)
    for _ in range(10):
        step(c, rec, sim, up)
    assert states(c)["n0"] == U.DONE


def test_disabling_auto_upgrade_strips_state_labels():
    c, rec, sim, up = setup(n_nodes=2)
    up.reconcile(("", "cluster-policy"))
    assert all(v == U.DONE for v in states(c).values())
    cp = c.get("amd.com/v1", "ClusterPolicy", "cluster-policy")
    cp["spec"]["driver"]["upgradePolicy"]["autoUpgrade"] = False
    c.update(cp)
    up.reconcile(("", "cluster-policy"))
    assert all(v == "" for v in states(c).values())


def test_upgrade_state_survives_operator_restart():
    c, rec, sim, up = setup(n_nodes=2, maxParallelUpgrades=1)
    up.reconcile(("", "cluster-policy"))
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    step(c, rec, sim, up)
    step(c, rec, sim, up)
    mid = states(c)
    assert any(s in U.IN_PROGRESS for s in mid.values())
    up2 = UpgradeReconciler(c, NS, rec.sm.snapshot, rec.metrics, run_async=False)   # "restart"
    for _ in range(60):
        step(c, rec, sim, up2, max_in_progress=1)
        if set(states(c).values()) == {U.DONE}:
            break
    assert set(states(c).values()) == {U.DONE}


def test_gpu_pod_filter():
    assert U.gpu_pod_filter(gpu_workload("n", "p"))
    p = gpu_workload("n", "p")
    p["spec"]["containers"][0]["resources"] = {"requests": {"amd.com/partition-cpx": 1}}
    assert U.gpu_pod_filter(p)
    p["spec"]["containers"][0]["resources"] = {"limits": {"nvidia.com/gpu": 1}}
    assert not U.gpu_pod_filter(p)


def test_metrics_published():
    c, rec, sim, up = setup(n_nodes=2)
    up.reconcile(("", "cluster-policy"))
    up.reconcile(("", "cluster-policy"))
    assert rec.metrics.upgrades_done._value.get() == 2
    assert rec.metrics.driver_auto_upgrade_enabled._value.get() == 1
