"""Rolling amdgpu driver upgrade: a per-node, label-driven state machine.

Same states, policy knobs and safety rules as the library the reference vendors
(reference: vendor/github.com/NVIDIA/k8s-operator-libs/pkg/upgrade/consts.go:33-56,
upgrade_state.go:276-843, drain_manager.go:58-136, pod_manager.go:117-349,
validation_manager.go:30-165), re-implemented with ``amd.com/`` keys (the vendored library
hard-codes ``nvidia.com/``):

    ""  -> upgrade-required -> cordon-required -> wait-for-jobs-required
        -> pod-deletion-required -> drain-required -> pod-restart-required
        -> validation-required -> uncordon-required -> upgrade-done
    any -> upgrade-failed (drain/eviction failure, driver pod restartCount > 10)

All durable state is on the Node (state label, start-time annotations), so an operator
restart resumes every upgrade where it stopped. Drains and pod evictions run on background
workers guarded by a per-node in-flight set (the library's KeyedMutex + StringSet); like
kubectl's drain helper (vendor/k8s.io/kubectl/pkg/drain/drain.go:248-353,410) a worker retries
PDB-refused evictions and then waits until every evicted pod is gone, bounded by the policy's
timeout. The wait's start time is a Node annotation, so an operator restart resumes the same
deadline instead of starting a new one.
"""

from __future__ import annotations

import logging
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Set

from ..api.v1.upgrade import DriverUpgradePolicySpec
from ..k8s import errors
from ..k8s import objects as o
from . import consts as C

log = logging.getLogger("amd-gpu-operator.upgrade")

UPGRADE_STATE_LABEL = f"{C.PREFIX}/gpu-driver-upgrade-state"
UPGRADE_SKIP_NODE_LABEL = f"{C.PREFIX}/gpu-driver-upgrade.skip"
UPGRADE_SKIP_DRAIN_POD_LABEL = f"{C.PREFIX}/gpu-driver-upgrade-drain.skip"
UPGRADE_INITIAL_STATE_ANNOTATION = f"{C.PREFIX}/gpu-driver-upgrade.node-initial-state.unschedulable"
WAIT_FOR_POD_COMPLETION_START_ANNOTATION = f"{C.PREFIX}/gpu-driver-upgrade-wait-for-pod-completion-start-time"
POD_EVICTION_START_ANNOTATION = f"{C.PREFIX}/gpu-driver-upgrade-pod-eviction-start-time"
DRAIN_START_ANNOTATION = f"{C.PREFIX}/gpu-driver-upgrade-drain-start-time"
VALIDATION_START_ANNOTATION = f"{C.PREFIX}/gpu-driver-upgrade-validation-start-time"
EVENT_REASON = "AMDGPUDriverUpgrade"

UNKNOWN = ""
UPGRADE_REQUIRED = "upgrade-required"
CORDON_REQUIRED = "cordon-required"
WAIT_FOR_JOBS_REQUIRED = "wait-for-jobs-required"
POD_DELETION_REQUIRED = "pod-deletion-required"
DRAIN_REQUIRED = "drain-required"
POD_RESTART_REQUIRED = "pod-restart-required"
VALIDATION_REQUIRED = "validation-required"
UNCORDON_REQUIRED = "uncordon-required"
DONE = "upgrade-done"
FAILED = "upgrade-failed"

ALL_STATES = [UNKNOWN, UPGRADE_REQUIRED, CORDON_REQUIRED, WAIT_FOR_JOBS_REQUIRED, POD_DELETION_REQUIRED,
              DRAIN_REQUIRED, POD_RESTART_REQUIRED, VALIDATION_REQUIRED, UNCORDON_REQUIRED, DONE, FAILED]
IN_PROGRESS = {CORDON_REQUIRED, WAIT_FOR_JOBS_REQUIRED, POD_DELETION_REQUIRED, DRAIN_REQUIRED,
               POD_RESTART_REQUIRED, VALIDATION_REQUIRED, UNCORDON_REQUIRED, FAILED}

VALIDATION_TIMEOUT_S = 600
MAX_DRIVER_RESTARTS = 10
EVICTION_RETRY_S = 5.0      # kubectl drain: an eviction refused by a PDB (429) is retried after 5 s
DELETE_POLL_S = 1.0         # kubectl drain waitForDelete: poll interval


def gpu_pod_filter(pod: Dict[str, Any]) -> bool:
    """Pods that hold AMD GPUs and must go before the driver can be reloaded (the role of
    the reference's gpuPodSpecFilter, main.go:161-183: nvidia.com/gpu*, nvidia.com/mig-*)."""
    for c in (pod.get("spec") or {}).get("containers") or []:
        res = c.get("resources") or {}
        for section in ("limits", "requests"):
            for k in (res.get(section) or {}):
                if k.startswith("amd.com/gpu") or k.startswith("amd.com/partition-"):
                    return True
    return False


@dataclass
class NodeState:
    node: Dict[str, Any]
    driver_pod: Dict[str, Any]
    driver_ds: Dict[str, Any]


@dataclass
class ClusterUpgradeState:
    node_states: Dict[str, List[NodeState]] = field(default_factory=lambda: {s: [] for s in ALL_STATES})

    def count(self, states) -> int:
        return sum(len(self.node_states.get(s, [])) for s in states)

    def total(self) -> int:
        return sum(len(v) for v in self.node_states.values())


class UpgradeStateManager:
    def __init__(self, client, namespace: str, pod_filter: Callable[[Dict], bool] = gpu_pod_filter,
                 validation_selector: Optional[str] = "app=amd-operator-validator",
                 clock=time.time, run_async: bool = True, workers: int = 8, sleep=time.sleep):
        self.client = client
        self.sleep = sleep
        self.namespace = namespace
        self.pod_filter = pod_filter
        self.validation_selector = validation_selector
        self.clock = clock
        self.run_async = run_async
        self._pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="upgrade") if run_async else None
        self._inflight: Set[str] = set()
        self._lock = threading.Lock()
        self._worker = threading.local()     # .deferred: the state a running worker moves its node to

    # -- node label/annotation provider (durable state) ----------------------------------------
    def set_state(self, node: Dict, state: str) -> None:
        deferred = getattr(self._worker, "deferred", None)
        if deferred is not None:
            deferred.append((node, state))    # applied once the worker has left _inflight (_schedule)
            return
        name = o.name(node)
        self.client.patch("v1", "Node", name, {"metadata": {"labels": {UPGRADE_STATE_LABEL: state or None}}})
        o.labels(node)[UPGRADE_STATE_LABEL] = state
        self.client.create_event(node, EVENT_REASON, f"Successfully updated node state label to {state}")
        log.info("node %s: upgrade state -> %s", name, state or "<unknown>")

    def set_annotation(self, node: Dict, key: str, value: Optional[str]) -> None:
        self.client.patch("v1", "Node", o.name(node), {"metadata": {"annotations": {key: value}}})
        anns = o.annotations(node)
        if value is None:
            anns.pop(key, None)
        else:
            anns[key] = value

    # -- state building (reference: BuildState :160-212) -------------------------------------
    def build_state(self, driver_labels: Dict[str, str]) -> ClusterUpgradeState:
        dss = {d["metadata"]["uid"]: d for d in self.client.list("apps/v1", "DaemonSet", self.namespace,
                                                                 label_selector=driver_labels)}
        for d in dss.values():
            st = d.get("status") or {}
            if st.get("desiredNumberScheduled", 0) != st.get("currentNumberScheduled", 0):
                raise RuntimeError(f"driver DaemonSet {o.name(d)} has unscheduled pods; retry later")
        state = ClusterUpgradeState()
        pods = self.client.list("v1", "Pod", self.namespace, label_selector=driver_labels)
        for pod in pods:
            ref = o.controller_of(pod)
            if not ref or ref.get("uid") not in dss:
                continue
            node_name = (pod.get("spec") or {}).get("nodeName")
            if not node_name:
                continue
            try:
                node = self.client.get("v1", "Node", node_name)
            except errors.NotFound:
                continue
            s = o.get_labels(node).get(UPGRADE_STATE_LABEL, UNKNOWN)
            state.node_states.setdefault(s, []).append(NodeState(node, pod, dss[ref["uid"]]))
        return state

    # -- revision helpers ---------------------------------------------------------------------
    def ds_revision_hash(self, ds: Dict) -> str:
        name = o.name(ds)
        revs = [r for r in self.client.list("apps/v1", "ControllerRevision", self.namespace,
                                            label_selector=(ds["spec"].get("selector") or {}).get("matchLabels"))
                if o.name(r).startswith(name + "-") and o.owned_by(r, ds["metadata"]["uid"])]
        if not revs:
            raise RuntimeError(f"no ControllerRevision for DaemonSet {name}")
        revs.sort(key=lambda r: r.get("revision", 0))
        return o.name(revs[-1])[len(name) + 1:]

    @staticmethod
    def pod_revision_hash(pod: Dict) -> str:
        h = o.get_labels(pod).get("controller-revision-hash")
        if h is None:
            raise RuntimeError(f"pod {o.name(pod)} has no controller-revision-hash label")
        return h

    def pod_in_sync(self, ns: NodeState) -> bool:
        if self.pod_revision_hash(ns.driver_pod) != self.ds_revision_hash(ns.driver_ds):
            return False
        st = ns.driver_pod.get("status") or {}
        cs = st.get("containerStatuses") or []
        return st.get("phase") == "Running" and bool(cs) and all(c.get("ready") for c in cs)

    @staticmethod
    def pod_failing(pod: Dict) -> bool:
        st = pod.get("status") or {}
        return any(not c.get("ready") and c.get("restartCount", 0) > MAX_DRIVER_RESTARTS
                   for c in (st.get("initContainerStatuses") or []) + (st.get("containerStatuses") or []))

    # -- budget (reference: GetUpgradesAvailable :939-967) -----------------------------------
    def unavailable_nodes(self, state: ClusterUpgradeState) -> int:
        n = 0
        for s, lst in state.node_states.items():
            for ns in lst:
                unsched = bool((ns.node.get("spec") or {}).get("unschedulable"))
                ready = all(c.get("status") == "True" for c in (ns.node.get("status") or {}).get("conditions") or []
                            if c.get("type") == "Ready")
                if s in IN_PROGRESS or unsched or not ready:
                    n += 1
        return n

    def upgrades_available(self, state: ClusterUpgradeState, policy: DriverUpgradePolicySpec) -> int:
        total = state.total()
        in_progress = state.count(IN_PROGRESS)
        maxp = policy.max_parallel()
        avail = total if maxp == 0 else max(0, maxp - in_progress)
        max_unavail = policy.max_unavailable_nodes(total) if policy.maxUnavailable is not None else total
        cur_unavail = self.unavailable_nodes(state)
        avail = min(avail, max(0, max_unavail - cur_unavail))
        return avail

    # -- the FSM (reference: ApplyState :276-394) ---------------------------------------------
    def apply_state(self, state: ClusterUpgradeState, policy: Optional[DriverUpgradePolicySpec]) -> None:
        if policy is None or not policy.autoUpgrade:
            return
        avail = self.upgrades_available(state, policy)
        self._done_or_unknown(state, UNKNOWN)
        self._done_or_unknown(state, DONE)
        self._upgrade_required(state, avail)
        self._cordon(state)
        self._wait_for_jobs(state, policy)
        self._pod_deletion(state, policy)
        self._drain(state, policy)
        self._pod_restart(state)
        self._failed(state)
        self._validation(state)
        self._uncordon(state)

    def _done_or_unknown(self, state: ClusterUpgradeState, which: str) -> None:
        for ns in list(state.node_states.get(which, [])):
            if self.pod_revision_hash(ns.driver_pod) != self.ds_revision_hash(ns.driver_ds):
                if (ns.node.get("spec") or {}).get("unschedulable"):
                    self.set_annotation(ns.node, UPGRADE_INITIAL_STATE_ANNOTATION, "true")
                self.set_state(ns.node, UPGRADE_REQUIRED)
                self._move(state, ns, which, UPGRADE_REQUIRED)
            elif which == UNKNOWN:
                self.set_state(ns.node, DONE)
                self._move(state, ns, which, DONE)

    def _upgrade_required(self, state: ClusterUpgradeState, avail: int) -> None:
        for ns in list(state.node_states.get(UPGRADE_REQUIRED, [])):
            if o.get_labels(ns.node).get(UPGRADE_SKIP_NODE_LABEL) == "true":
                continue
            if avail <= 0 and not (ns.node.get("spec") or {}).get("unschedulable"):
                continue        # no slot; a manually cordoned node may still proceed
            self.set_state(ns.node, CORDON_REQUIRED)
            self._move(state, ns, UPGRADE_REQUIRED, CORDON_REQUIRED)
            avail -= 1

    def _cordon(self, state: ClusterUpgradeState) -> None:
        for ns in list(state.node_states.get(CORDON_REQUIRED, [])):
            self.client.patch("v1", "Node", o.name(ns.node), {"spec": {"unschedulable": True}})
            ns.node.setdefault("spec", {})["unschedulable"] = True
            self.set_state(ns.node, WAIT_FOR_JOBS_REQUIRED)
            self._move(state, ns, CORDON_REQUIRED, WAIT_FOR_JOBS_REQUIRED)

    def _next_after_jobs(self) -> str:
        return POD_DELETION_REQUIRED if self.pod_filter is not None else DRAIN_REQUIRED

    def _wait_for_jobs(self, state: ClusterUpgradeState, policy: DriverUpgradePolicySpec) -> None:
        wfc = policy.waitForCompletion
        for ns in list(state.node_states.get(WAIT_FOR_JOBS_REQUIRED, [])):
            if wfc is None or not wfc.podSelector:
                self.set_state(ns.node, self._next_after_jobs())
                self._move(state, ns, WAIT_FOR_JOBS_REQUIRED, self._next_after_jobs())
                continue
            running = [p for p in self.client.list("v1", "Pod", label_selector=wfc.podSelector,
                                                   field_selector=f"spec.nodeName={o.name(ns.node)}")
                       if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]
            if running and wfc.timeout() > 0:
                start = o.get_annotations(ns.node).get(WAIT_FOR_POD_COMPLETION_START_ANNOTATION)
                if start is None:
                    self.set_annotation(ns.node, WAIT_FOR_POD_COMPLETION_START_ANNOTATION, str(int(self.clock())))
                    continue
                if self.clock() - int(start) < wfc.timeout():
                    continue
                log.info("node %s: wait-for-completion timed out", o.name(ns.node))
            elif running:
                continue
            self.set_annotation(ns.node, WAIT_FOR_POD_COMPLETION_START_ANNOTATION, None)
            self.set_state(ns.node, self._next_after_jobs())
            self._move(state, ns, WAIT_FOR_JOBS_REQUIRED, self._next_after_jobs())

    def _pod_deletion(self, state: ClusterUpgradeState, policy: DriverUpgradePolicySpec) -> None:
        nodes = list(state.node_states.get(POD_DELETION_REQUIRED, []))
        if self.pod_filter is None:
            for ns in nodes:
                self.set_state(ns.node, DRAIN_REQUIRED)
                self._move(state, ns, POD_DELETION_REQUIRED, DRAIN_REQUIRED)
            return
        drain_enabled = policy.drain is not None and bool(policy.drain.enable)
        for ns in nodes:
            self._schedule(o.name(ns.node), lambda ns=ns: self._evict_gpu_pods(ns, policy, drain_enabled))

    def _gpu_pods_on(self, node: str) -> List[Dict]:
        return [p for p in self.client.list("v1", "Pod", field_selector=f"spec.nodeName={node}")
                if self.pod_filter(p) and (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]

    @staticmethod
    def _daemon_or_mirror(p: Dict) -> Optional[str]:
        """Why eviction cannot clear ``p`` from the node, or None: a DaemonSet pod comes straight
        back (it tolerates the cordon) and a mirror (static) pod is not the API server's to delete
        -- kubectl drain's IgnoreAllDaemonSets / mirror filters (reference pod_manager.go:147,186-197)."""
        owner = o.controller_of(p)
        if owner and owner.get("kind") == "DaemonSet":
            return "DaemonSet-managed"
        if "kubernetes.io/config.mirror" in o.get_annotations(p):
            return "mirror pod"
        return None

    def _drain_or_failed(self, ns: NodeState, drain_enabled: bool, why: str) -> None:
        """reference: pod_manager.go:369-377 (updateNodeToDrainOrFailed)."""
        self.client.create_event(ns.node, EVENT_REASON,
                                 f"Failed to delete workload pods on the node for the driver upgrade, {why}",
                                 "Warning")
        self.set_state(ns.node, DRAIN_REQUIRED if drain_enabled else FAILED)

    def _evict_gpu_pods(self, ns: NodeState, policy: DriverUpgradePolicySpec, drain_enabled: bool) -> None:
        """Delete the node's GPU pods and wait until they are gone (reference: pod_manager.go:117-223):
        nothing to delete -> pod-restart-required; a pod the policy may not delete (emptyDir
        without deleteEmptyDir, no controller without force) or an eviction error / timeout ->
        drain-required when drain is enabled, else upgrade-failed."""
        pd = policy.podDeletion
        timeout = pd.timeout() if pd else 300
        node = o.name(ns.node)
        pods = self._gpu_pods_on(node)
        if not pods:
            self.set_annotation(ns.node, POD_EVICTION_START_ANNOTATION, None)
            self.set_state(ns.node, POD_RESTART_REQUIRED)
            return
        blocked = []
        for p in pods:
            uses_emptydir = any("emptyDir" in v for v in (p.get("spec") or {}).get("volumes") or [])
            why = self._daemon_or_mirror(p)
            if why:
                blocked.append(f"{o.name(p)} ({why})")
            elif uses_emptydir and not (pd and pd.deleteEmptyDir):
                blocked.append(f"{o.name(p)} (emptyDir)")
            elif o.controller_of(p) is None and not (pd and pd.force):
                blocked.append(f"{o.name(p)} (unmanaged)")
        if blocked:
            log.info("node %s: cannot delete all required pods: %s", node, blocked)
            self.set_annotation(ns.node, POD_EVICTION_START_ANNOTATION, None)
            self._drain_or_failed(ns, drain_enabled, f"cannot delete {blocked}")
            return
        err = self._delete_or_evict(ns.node, pods, timeout, POD_EVICTION_START_ANNOTATION)
        if err:
            self._drain_or_failed(ns, drain_enabled, err)
            return
        self.client.create_event(ns.node, EVENT_REASON, "Deleted workload pods on the node for the driver upgrade")
        self.set_state(ns.node, POD_RESTART_REQUIRED)

    def _delete_or_evict(self, node: Dict, pods: List[Dict], timeout: int, start_key: str) -> Optional[str]:
        """Evict ``pods`` and wait until every one of them is gone (kubectl drain's DeleteOrEvictPods
        + waitForDelete, drain.go:248-353,410). A 429 (PodDisruptionBudget) is retried every
        EVICTION_RETRY_S; a pod counts as gone when GET returns 404 or a different UID. ``timeout``
        0 = no limit. The deadline runs from the ``start_key`` Node annotation, set on the first
        attempt and cleared when the wait ends. Returns None on success, else the reason."""
        start = o.get_annotations(node).get(start_key)
        if start is None:
            start = str(int(self.clock()))
            self.set_annotation(node, start_key, start)
        deadline = int(start) + timeout if timeout else None
        pending = {(o.namespace(p), o.name(p)): p for p in pods}
        evicted: Set[tuple] = set()
        next_evict = 0.0
        while True:
            now = self.clock()
            if now >= next_evict:
                refused = False
                for key, p in pending.items():
                    if key in evicted or (p.get("metadata") or {}).get("deletionTimestamp"):
                        evicted.add(key)
                        continue
                    try:
                        self.client.evict(key[1], key[0])
                        evicted.add(key)
                    except errors.NotFound:
                        evicted.add(key)
                    except errors.TooManyRequests:
                        refused = True          # PDB: retry after EVICTION_RETRY_S
                    except errors.ApiError as e:
                        self.set_annotation(node, start_key, None)
                        return f"error when evicting pods/{key[1]} -n {key[0]}: {e}"
                next_evict = now + EVICTION_RETRY_S if refused else float("inf")
            for key in list(pending):
                if key not in evicted:
                    continue
                try:
                    cur = self.client.get("v1", "Pod", key[1], key[0])
                except errors.NotFound:
                    cur = None
                if cur is None or cur["metadata"].get("uid") != pending[key]["metadata"].get("uid"):
                    del pending[key]
            if not pending:
                self.set_annotation(node, start_key, None)
                return None
            if deadline is not None and self.clock() >= deadline:
                self.set_annotation(node, start_key, None)
                left = sorted(f"{ns_}/{n}" for ns_, n in pending)
                what = "evicted but not yet deleted" if set(pending) <= evicted else "eviction refused"
                return f"global timeout {timeout}s reached; pods {what}: {left}"
            self.sleep(DELETE_POLL_S)

    def _drain(self, state: ClusterUpgradeState, policy: DriverUpgradePolicySpec) -> None:
        d = policy.drain
        for ns in list(state.node_states.get(DRAIN_REQUIRED, [])):
            if d is None or not d.enable:
                self.set_state(ns.node, POD_RESTART_REQUIRED)
                self._move(state, ns, DRAIN_REQUIRED, POD_RESTART_REQUIRED)
                continue
            self._schedule(o.name(ns.node), lambda ns=ns: self._drain_node(ns, d))

    def _drain_node(self, ns: NodeState, d) -> None:
        """Evict every pod on the node except DaemonSet pods, mirror pods and pods labelled
        to skip drain (the operator itself), with the kubectl-drain options of the policy, and
        wait for them to be gone (reference: drain_manager.go:58-136)."""
        node = o.name(ns.node)
        sel = f"{UPGRADE_SKIP_DRAIN_POD_LABEL}!=true"
        if d.podSelector:
            sel = f"{d.podSelector},{sel}"
        pods = self.client.list("v1", "Pod", label_selector=sel, field_selector=f"spec.nodeName={node}")
        errs, victims = [], []
        for p in pods:
            owner = o.controller_of(p)
            if owner and owner.get("kind") == "DaemonSet":
                continue
            if "kubernetes.io/config.mirror" in o.get_annotations(p):
                continue
            if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                continue
            uses_emptydir = any("emptyDir" in v for v in (p.get("spec") or {}).get("volumes") or [])
            if uses_emptydir and not d.deleteEmptyDir:
                errs.append(f"{o.name(p)}: uses emptyDir")
                continue
            if owner is None and not d.force:
                errs.append(f"{o.name(p)}: not managed by a controller")
                continue
            victims.append(p)
        if not errs and victims:
            err = self._delete_or_evict(ns.node, victims, d.timeout(), DRAIN_START_ANNOTATION)
            if err:
                errs.append(err)
        if errs:
            self.set_annotation(ns.node, DRAIN_START_ANNOTATION, None)
            self.client.create_event(ns.node, EVENT_REASON, f"Failed to drain the node, {errs}", "Warning")
            self.set_state(ns.node, FAILED)
        else:
            self.client.create_event(ns.node, EVENT_REASON, "Successfully drained the node")
            self.set_state(ns.node, POD_RESTART_REQUIRED)

    def _pod_restart(self, state: ClusterUpgradeState) -> None:
        for ns in list(state.node_states.get(POD_RESTART_REQUIRED, [])):
            if self.pod_revision_hash(ns.driver_pod) != self.ds_revision_hash(ns.driver_ds):
                if self.pod_filter is not None and [p for p in self._gpu_pods_on(o.name(ns.node))
                                                    if not self._daemon_or_mirror(p)]:
                    # never unload amdgpu under a pod that still holds /dev/kfd (one that started
                    # after the eviction, e.g. with a toleration for the cordon): evict again.
                    # DaemonSet / mirror GPU pods are not evictable: pod deletion routed them to
                    # drain (which skips them) or upgrade-failed, so they cannot loop the node here
                    log.info("node %s: GPU pods present again; back to pod deletion", o.name(ns.node))
                    self.set_state(ns.node, POD_DELETION_REQUIRED)
                    self._move(state, ns, POD_RESTART_REQUIRED, POD_DELETION_REQUIRED)
                    continue
                if not (ns.driver_pod.get("metadata") or {}).get("deletionTimestamp"):
                    try:
                        self.client.delete("v1", "Pod", o.name(ns.driver_pod), o.namespace(ns.driver_pod))
                        log.info("node %s: restarted driver pod %s", o.name(ns.node), o.name(ns.driver_pod))
                    except errors.NotFound:
                        pass
                continue
            if self.pod_in_sync(ns):
                nxt = VALIDATION_REQUIRED if self.validation_selector else self._uncordon_or_done(ns.node)
                if nxt == VALIDATION_REQUIRED:
                    self.set_state(ns.node, VALIDATION_REQUIRED)
                self._move(state, ns, POD_RESTART_REQUIRED, nxt)
            elif self.pod_failing(ns.driver_pod):
                self.set_state(ns.node, FAILED)
                self._move(state, ns, POD_RESTART_REQUIRED, FAILED)

    def _failed(self, state: ClusterUpgradeState) -> None:
        for ns in list(state.node_states.get(FAILED, [])):
            if self.pod_in_sync(ns):
                self._move(state, ns, FAILED, self._uncordon_or_done(ns.node))

    def _validation(self, state: ClusterUpgradeState) -> None:
        for ns in list(state.node_states.get(VALIDATION_REQUIRED, [])):
            if self._validated(ns.node):
                self._move(state, ns, VALIDATION_REQUIRED, self._uncordon_or_done(ns.node))

    def _validated(self, node: Dict) -> bool:
        """The validator pod on the node is Running and Ready (reference:
        validation_manager.go:71-111); FAILED after 600 s."""
        name = o.name(node)
        pods = self.client.list("v1", "Pod", label_selector=self.validation_selector,
                                field_selector=f"spec.nodeName={name}")
        ok = bool(pods) and all((p.get("status") or {}).get("phase") == "Running" and
                                all(c.get("ready") for c in (p.get("status") or {}).get("containerStatuses") or [{}])
                                for p in pods)
        if ok:
            self.set_annotation(node, VALIDATION_START_ANNOTATION, None)
            return True
        start = o.get_annotations(node).get(VALIDATION_START_ANNOTATION)
        if start is None:
            self.set_annotation(node, VALIDATION_START_ANNOTATION, str(int(self.clock())))
        elif self.clock() - int(start) > VALIDATION_TIMEOUT_S:
            self.set_annotation(node, VALIDATION_START_ANNOTATION, None)
            self.set_state(node, FAILED)
        return False

    def _uncordon_or_done(self, node: Dict) -> str:
        if UPGRADE_INITIAL_STATE_ANNOTATION in o.get_annotations(node):
            self.set_annotation(node, UPGRADE_INITIAL_STATE_ANNOTATION, None)
            self.set_state(node, DONE)      # node was cordoned by an admin before: keep it so
            return DONE
        self.set_state(node, UNCORDON_REQUIRED)
        return UNCORDON_REQUIRED

    def _uncordon(self, state: ClusterUpgradeState) -> None:
        for ns in list(state.node_states.get(UNCORDON_REQUIRED, [])):
            self.client.patch("v1", "Node", o.name(ns.node), {"spec": {"unschedulable": None}})
            self.set_state(ns.node, DONE)
            self._move(state, ns, UNCORDON_REQUIRED, DONE)

    # -- plumbing -----------------------------------------------------------------------------
    @staticmethod
    def _move(state: ClusterUpgradeState, ns: NodeState, src: str, dst: str) -> None:
        lst = state.node_states.get(src, [])
        if ns in lst:
            lst.remove(ns)
        state.node_states.setdefault(dst, []).append(ns)

    def _schedule(self, node: str, fn: Callable[[], None]) -> None:
        with self._lock:
            if node in self._inflight:
                return
            self._inflight.add(node)

        def run():
            # The worker's state change is the event that drives the next reconcile; published while
            # the node is still in _inflight, a next step that is async too (pod deletion -> drain)
            # would be skipped by that reconcile and wait for the 2-minute requeue. So the label is
            # written only after the node has left _inflight.
            self._worker.deferred = []
            try:
                fn()
            except Exception:  # noqa: BLE001
                log.exception("upgrade worker for node %s failed", node)
            finally:
                deferred, self._worker.deferred = self._worker.deferred, None
                with self._lock:
                    self._inflight.discard(node)
                # each deferred label on its own: a failed PATCH is logged (a Future nobody reads would
                # swallow it) and does not drop the states after it
                for n, st in deferred:
                    try:
                        self.set_state(n, st)
                    except Exception:  # noqa: BLE001
                        log.exception("upgrade worker for node %s: publishing state %s failed", node, st)
        if self._pool is None:
            run()
        else:
            self._pool.submit(run)

    def remove_upgrade_labels(self) -> None:
        for node in self.client.list("v1", "Node", label_selector=UPGRADE_STATE_LABEL):
            self.client.patch("v1", "Node", o.name(node), {"metadata": {"labels": {UPGRADE_STATE_LABEL: None}}})

    def stats(self, state: ClusterUpgradeState, policy: Optional[DriverUpgradePolicySpec]) -> Dict[str, int]:
        return {"in_progress": state.count(IN_PROGRESS - {FAILED}),
                "done": state.count([DONE]),
                "failed": state.count([FAILED]),
                "pending": state.count([UPGRADE_REQUIRED]),
                "available": self.upgrades_available(state, policy) if policy else 0}
