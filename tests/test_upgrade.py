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


# -- eviction waits for deletion, PDB 429 retries (kubectl drain semantics) -------------------------

def _fake_time(up, hook=None):
    clock = [1000.0]
    up.mgr.clock = lambda: clock[0]

    def sleep(dt):
        clock[0] += dt
        if hook:
            hook(clock[0])
    up.mgr.sleep = sleep
    return clock


def _guard_driver_restart(c):
    """Fail the test if a driver pod is deleted while a GPU pod still exists on its node."""
    def hook(verb, av, kind, arg):
        if verb != "delete" or kind != "Pod" or not isinstance(arg, str) or not arg.startswith(C.DS_DRIVER):
            return
        drv = [p for p in c.list("v1", "Pod", NS) if o.name(p) == arg]
        if not drv:
            return
        node = drv[0]["spec"]["nodeName"]
        gpu = [o.name(p) for p in c.list("v1", "Pod", field_selector=f"spec.nodeName={node}") if U.gpu_pod_filter(p)]
        assert not gpu, f"driver pod {arg} deleted while GPU pods {gpu} remain on {node}"
    c.interceptors.append(hook)


def _start_upgrade(n_nodes=1, **policy):
    c, rec, sim, up = setup(n_nodes=n_nodes, **policy)
    up.reconcile(("", "cluster-policy"))
    return c, rec, sim, up


def test_pod_stuck_terminating_holds_pod_deletion_then_fails_at_timeout():
    c, rec, sim, up = _start_upgrade(podDeletion={"timeoutSeconds": 30})
    seen = []
    clock = _fake_time(up, lambda t: seen.append(states(c)["n0"]))
    stuck = gpu_workload("n0", "stuck")
    stuck["metadata"]["finalizers"] = ["example.com/hold"]
    c.create(stuck)
    _guard_driver_restart(c)
    drv_before = {o.name(p) for p in c.list("v1", "Pod", NS, label_selector={"app": C.DS_DRIVER})}
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(8):
        step(c, rec, sim, up)
        if states(c)["n0"] == U.FAILED:
            break
    assert states(c)["n0"] == U.FAILED
    assert seen and set(seen) == {U.POD_DELETION_REQUIRED}           # held there while waiting
    assert 30 <= clock[0] - 1000.0 <= 32                              # bounded by timeoutSeconds
    assert c.get("v1", "Pod", "stuck", "default")["metadata"].get("deletionTimestamp")
    assert U.POD_EVICTION_START_ANNOTATION not in o.get_annotations(c.get("v1", "Node", "n0"))
    assert any("global timeout 30s" in e["message"] for e in c.events if e["type"] == "Warning")
    drv_after = {o.name(p) for p in c.list("v1", "Pod", NS, label_selector={"app": C.DS_DRIVER})}
    assert drv_after == drv_before                                    # driver never restarted


def test_pod_stuck_terminating_falls_back_to_drain_then_fails():
    c, rec, sim, up = _start_upgrade(podDeletion={"timeoutSeconds": 20},
                                     drain={"enable": True, "force": True, "timeoutSeconds": 20})
    _fake_time(up)
    stuck = gpu_workload("n0", "stuck")
    stuck["metadata"]["finalizers"] = ["example.com/hold"]
    c.create(stuck)
    _guard_driver_restart(c)
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    visited = []
    for _ in range(10):
        step(c, rec, sim, up)
        visited.append(states(c)["n0"])
        if visited[-1] == U.FAILED:
            break
    assert U.DRAIN_REQUIRED in visited and visited[-1] == U.FAILED, visited


def test_terminating_pod_that_finishes_lets_the_upgrade_complete():
    c, rec, sim, up = _start_upgrade(podDeletion={"timeoutSeconds": 60})
    slow = gpu_workload("n0", "slow")
    slow["metadata"]["finalizers"] = ["example.com/hold"]
    c.create(slow)

    def release(t):
        if t >= 1010:          # the workload finishes its shutdown after ~10 s
            try:
                p = c.get("v1", "Pod", "slow", "default")
            except errors.NotFound:
                return
            p["metadata"]["finalizers"] = []
            c.update(p)
    _fake_time(up, release)
    _guard_driver_restart(c)
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(40):
        step(c, rec, sim, up)
        if states(c)["n0"] == U.DONE:
            break
    assert states(c)["n0"] == U.DONE
    assert not [p for p in c.list("v1", "Pod", "default") if o.name(p) == "slow"]


def test_pdb_refused_eviction_is_retried_until_allowed():
    c, rec, sim, up = _start_upgrade(podDeletion={"timeoutSeconds": 120})
    w = gpu_workload("n0", "guarded")
    w["metadata"]["labels"] = {"app": "trainer"}
    c.create(w)
    c.create({"apiVersion": "policy/v1", "kind": "PodDisruptionBudget",
              "metadata": {"name": "trainer-pdb", "namespace": "default"},
              "spec": {"selector": {"matchLabels": {"app": "trainer"}}, "minAvailable": 1},
              "status": {"disruptionsAllowed": 0}})
    evictions = []
    c.interceptors.append(lambda v, av, k, a: evictions.append(a) if v == "evict" else None)

    def allow(t):
        if t >= 1012:
            pdb = c.get("policy/v1", "PodDisruptionBudget", "trainer-pdb", "default")
            if pdb["status"]["disruptionsAllowed"] == 0:
                pdb["status"]["disruptionsAllowed"] = 1
                c.update_status(pdb)
    clock = _fake_time(up, allow)
    _guard_driver_restart(c)
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(40):
        step(c, rec, sim, up)
        if states(c)["n0"] == U.DONE:
            break
    assert states(c)["n0"] == U.DONE
    assert evictions.count("guarded") >= 3                # refused (429) at least twice, then allowed
    assert clock[0] - 1000.0 < 120


def test_pdb_that_never_allows_fails_the_node_at_timeout():
    c, rec, sim, up = _start_upgrade(podDeletion={"timeoutSeconds": 15})
    w = gpu_workload("n0", "guarded")
    w["metadata"]["labels"] = {"app": "trainer"}
    c.create(w)
    c.create({"apiVersion": "policy/v1", "kind": "PodDisruptionBudget",
              "metadata": {"name": "trainer-pdb", "namespace": "default"},
              "spec": {"selector": {"matchLabels": {"app": "trainer"}}}, "status": {"disruptionsAllowed": 0}})
    _fake_time(up)
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(8):
        step(c, rec, sim, up)
    assert states(c)["n0"] == U.FAILED
    assert c.get("v1", "Pod", "guarded", "default")                     # never deleted
    assert any("eviction refused" in e["message"] for e in c.events if e["type"] == "Warning")


def test_eviction_deadline_survives_operator_restart():
    """The wait's start time is a Node annotation: a restarted operator keeps the old deadline."""
    c, rec, sim, up = _start_upgrade(podDeletion={"timeoutSeconds": 50})
    stuck = gpu_workload("n0", "stuck")
    stuck["metadata"]["finalizers"] = ["example.com/hold"]
    c.create(stuck)
    clock = [1000.0]
    # the "previous operator" started waiting 40 s ago and died
    c.patch("v1", "Node", "n0", {"metadata": {"annotations": {U.POD_EVICTION_START_ANNOTATION: "960"}}})
    up.mgr.clock = lambda: clock[0]

    def sleep(dt):
        clock[0] += dt
    up.mgr.sleep = sleep
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(8):
        step(c, rec, sim, up)
        if states(c)["n0"] == U.FAILED:
            break
    assert states(c)["n0"] == U.FAILED
    assert clock[0] <= 1012          # ~10 s left of the 50 s budget, not a fresh 50 s


def test_gpu_pod_reappearing_before_driver_restart_is_evicted_first():
    c, rec, sim, up = _start_upgrade(podDeletion={"timeoutSeconds": 60})
    _fake_time(up)
    _guard_driver_restart(c)
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    for _ in range(10):
        step(c, rec, sim, up)
        if states(c)["n0"] == U.POD_RESTART_REQUIRED:
            break
    assert states(c)["n0"] == U.POD_RESTART_REQUIRED
    # a tolerating GPU pod lands on the cordoned node between eviction and the driver restart;
    # the worker pass below must evict it before the driver pod goes
    c.create(gpu_workload("n0", "late"))
    seen = []
    for _ in range(40):
        step(c, rec, sim, up)
        seen.append(states(c)["n0"])
        if seen[-1] == U.DONE:
            break
    assert states(c)["n0"] == U.DONE and seen[0] == U.POD_DELETION_REQUIRED, seen
    assert not [p for p in c.list("v1", "Pod", "default") if o.name(p) == "late"]


def _ds_gpu_pod(node, name="gpu-monitor"):
    pod = gpu_workload(node, name)
    pod["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "DaemonSet", "name": "mon",
                                           "uid": "ds-uid", "controller": True}]
    return pod


def test_daemonset_gpu_pod_without_drain_fails_the_node_instead_of_looping():
    """a DaemonSet-owned GPU pod comes straight back after eviction (it
    tolerates the cordon). Pod deletion must treat it as blocked -- upgrade-failed without drain
    -- not evict it and loop pod-deletion <-> pod-restart forever."""
    clock = [1000.0]
    c, rec, sim, up = setup(n_nodes=1, podDeletion={"timeoutSeconds": 30})
    sim._collect_orphans = lambda live: None          # the pod's DaemonSet lives outside this sim
    up.mgr.clock = lambda: clock[0]
    up.reconcile(("", "cluster-policy"))
    c.create(_ds_gpu_pod("n0"))
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    seen = []
    for _ in range(12):
        step(c, rec, sim, up)
        seen.append(states(c)["n0"])
        clock[0] += 10
    assert states(c)["n0"] == U.FAILED, seen
    assert seen.count(U.POD_DELETION_REQUIRED) <= 2, seen
    assert [p for p in c.list("v1", "Pod", "default") if o.name(p) == "gpu-monitor"]     # never evicted
    assert any("DaemonSet-managed" in e["message"] for e in c.events if e["reason"] == U.EVENT_REASON)


def test_daemonset_gpu_pod_with_drain_completes_the_upgrade():
    """With drain enabled the node goes to drain, which skips DaemonSet pods (kubectl drain
    --ignore-daemonsets), and the driver restart is not blocked by the DaemonSet pod again."""
    c, rec, sim, up = setup(n_nodes=1, podDeletion={"timeoutSeconds": 30},
                            drain={"enable": True, "force": True, "timeoutSeconds": 30})
    sim._collect_orphans = lambda live: None
    up.reconcile(("", "cluster-policy"))
    c.create(_ds_gpu_pod("n0"))
    bump_driver(c)
    rec.reconcile(("", "cluster-policy"))
    sim.sync()
    seen = []
    for _ in range(40):
        step(c, rec, sim, up)
        seen.append(states(c)["n0"])
        if seen[-1] == U.DONE:
            break
    assert states(c)["n0"] == U.DONE, seen
    assert U.DRAIN_REQUIRED in seen and seen.count(U.POD_DELETION_REQUIRED) <= 2, seen


def test_async_worker_publishes_its_state_after_leaving_inflight():
    """A worker's state label is the event that drives the next reconcile. Published while its node
    was still in _inflight, an async next step (pod deletion -> drain) was skipped by that reconcile
    and the node waited for the 2-minute requeue (the e2e upgrade timed out under load). The label
    is now written after the node has left _inflight."""
    import threading
    from gpu_operator_amd.k8s.fake import FakeClient

    node = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n0", "labels": {}}}
    c = FakeClient([node])
    mgr = U.UpgradeStateManager(c, NS, run_async=True, workers=2)
    seen = []
    orig_patch = c.patch

    def patch(av, kind, name, body, *a, **kw):
        labels = ((body.get("metadata") or {}).get("labels") or {})
        if U.UPGRADE_STATE_LABEL in labels:
            with mgr._lock:
                seen.append((labels[U.UPGRADE_STATE_LABEL], name in mgr._inflight))
        return orig_patch(av, kind, name, body, *a, **kw)
    c.patch = patch

    def work():
        mgr.set_state(c.get("v1", "Node", "n0"), U.DRAIN_REQUIRED)
        assert o.get_labels(c.get("v1", "Node", "n0")).get(U.UPGRADE_STATE_LABEL) is None   # not yet
    mgr._schedule("n0", work)
    for _ in range(200):
        if seen:
            break
        threading.Event().wait(0.01)
    assert seen == [(U.DRAIN_REQUIRED, False)]
    assert o.get_labels(c.get("v1", "Node", "n0"))[U.UPGRADE_STATE_LABEL] == U.DRAIN_REQUIRED
    # and the reconcile that label triggers can schedule the next async step at once
    ran = threading.Event()
    mgr._schedule("n0", ran.set)
    assert ran.wait(2)


def test_a_failed_deferred_publish_is_logged_and_the_others_still_land(caplog):
    """the deferred set_state calls ran in `finally` after the except that logs; a PATCH that
    raised there vanished into the pool's Future and skipped the states after it."""
    import logging
    import threading
    from gpu_operator_amd.k8s.fake import FakeClient

    nodes = [{"apiVersion": "v1", "kind": "Node", "metadata": {"name": n, "labels": {}}} for n in ("n0", "n1")]
    c = FakeClient(nodes)
    mgr = U.UpgradeStateManager(c, NS, run_async=True, workers=1)
    orig_patch = c.patch

    def patch(av, kind, name, body, *a, **kw):
        labels = ((body.get("metadata") or {}).get("labels") or {})
        if name == "n0" and U.UPGRADE_STATE_LABEL in labels:
            raise RuntimeError("apiserver went away")
        return orig_patch(av, kind, name, body, *a, **kw)
    c.patch = patch

    def work():
        mgr.set_state(c.get("v1", "Node", "n0"), U.DRAIN_REQUIRED)       # fails when published
        mgr.set_state(c.get("v1", "Node", "n1"), U.DRAIN_REQUIRED)       # must still land
    done = threading.Event()
    with caplog.at_level(logging.ERROR):
        mgr._schedule("n0", work)
        mgr._schedule("n9", done.set)           # same single worker: runs after the first job
        assert done.wait(5)
    assert o.get_labels(c.get("v1", "Node", "n1")).get(U.UPGRADE_STATE_LABEL) == U.DRAIN_REQUIRED
    assert any("publishing state" in r.getMessage() and "n0" in r.getMessage() for r in caplog.records)
    assert "n0" not in mgr._inflight
