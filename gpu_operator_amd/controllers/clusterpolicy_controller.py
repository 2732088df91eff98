"""ClusterPolicy reconciler: the operator's core control loop.

Behaviour of the reference (reference: controllers/clusterpolicy_controller.go:84-218,
watches :220-344): one active ClusterPolicy (others are marked ``ignored``); every pass walks
*all* 17 states even when earlier ones are not ready (ordering between operands is enforced
on the node by barriers); requeue after 5 s while any state is not ready or on error, after
45 s when no node carries NFD labels; per-key back-off 100 ms -> 3 s.

Differences by design: the ``ignored`` status of a second CR is persisted (the reference
sets it in memory only); the CR status carries the list of states
not ready and a Ready condition; DaemonSet/Node events re-trigger a pass immediately, so
readiness is usually observed well before the 5 s requeue timer fires.
"""

from __future__ import annotations

import logging
import time
from typing import Any, Dict, List, Optional

from ..api.v1 import clusterpolicy as cp
from ..k8s import errors
from ..k8s import objects as o
from ..k8s.client import DELETED, MODIFIED, WatchEvent
from ..runtime.controller import Controller, Result
from . import consts as C
from . import object_controls as oc
from .operator_metrics import (RECONCILE_ERROR, RECONCILE_NO_CR, RECONCILE_NOT_READY, RECONCILE_OK,
                               OperatorMetrics)
from .state_manager import (SnapshotHolder, StateManager, has_common_gpu_label, has_gpu_labels,
                            has_operands_disabled, is_partition_capable, workload_config)

log = logging.getLogger("amd-gpu-operator.clusterpolicy")

REQUEUE_NOT_READY = 5.0
REQUEUE_NO_NFD = 45.0


class ClusterPolicyReconciler:
    def __init__(self, client, namespace: Optional[str] = None, metrics: Optional[OperatorMetrics] = None,
                 assets_base=None, snapshot: Optional[SnapshotHolder] = None):
        self.client = client
        self.metrics = metrics or OperatorMetrics()
        self.sm = StateManager(client, namespace, self.metrics, assets_base, snapshot)
        self.active: Optional[str] = None
        self.last_states: Dict[str, str] = {}

    @property
    def namespace(self) -> str:
        return self.sm.namespace

    # -- singleton ------------------------------------------------------------------------
    def _pick_active(self) -> Optional[str]:
        items = self.client.list(cp.API_VERSION, cp.KIND)
        if not items:
            return None
        names = {o.name(i) for i in items}
        if self.active in names:
            return self.active
        items.sort(key=lambda i: (i["metadata"].get("creationTimestamp", ""), o.name(i)))
        return o.name(items[0])

    def _set_state(self, name: str, state: str, not_ready: Optional[List[str]] = None,
                   message: str = "") -> None:
        for _ in range(3):
            try:
                obj = self.client.get(cp.API_VERSION, cp.KIND, name)
            except errors.NotFound:
                return
            st = obj.get("status") or {}
            new = {"state": state, "namespace": self.namespace}
            if not_ready:
                new["notReadyStates"] = list(not_ready)
            ready = "True" if state == cp.STATE_READY else "False"
            prev = next((c for c in st.get("conditions") or [] if c.get("type") == "Ready"), None)
            ltt = prev.get("lastTransitionTime") if prev and prev.get("status") == ready else \
                time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
            new["conditions"] = [{"type": "Ready", "status": ready, "lastTransitionTime": ltt,
                                  "reason": {cp.STATE_READY: "AllStatesReady", cp.STATE_IGNORED: "Ignored"}
                                  .get(state, "StatesNotReady"),
                                  "message": message or ("" if not not_ready else
                                                         "not ready: " + ", ".join(not_ready))}]
            if st == new:
                return
            obj["status"] = new
            try:
                self.client.update_status(obj)
                return
            except errors.Conflict:
                continue

    # -- reconcile ------------------------------------------------------------------------
    def reconcile(self, req) -> Result:
        name = req[1] if isinstance(req, tuple) else req
        t0 = time.monotonic()
        try:
            return self._reconcile(name)
        finally:
            self.metrics.reconcile_duration.set(time.monotonic() - t0)

    def _reconcile(self, name: str) -> Result:
        try:
            obj = self.client.get(cp.API_VERSION, cp.KIND, name)
        except errors.NotFound:
            self.metrics.reconciliation_status.set(RECONCILE_NO_CR)
            if self.active == name:
                self.active = None
            return Result()
        active = self._pick_active()
        if active != name:
            self._set_state(name, cp.STATE_IGNORED, message=f"ClusterPolicy {active} is active")
            return Result()
        self.active = name
        try:
            self.sm.init(obj)
        except Exception:
            self.metrics.reconciliation_status.set(RECONCILE_NO_CR)
            raise
        self.metrics.reconciliation_has_nfd_labels.set(1 if self.sm.has_nfd else 0)
        if not self.sm.has_nfd:
            log.warning("NFD labels missing in the cluster: GPU nodes cannot be discovered")
        self.metrics.reconciliation_total.inc()

        not_ready: List[str] = []
        for state in self.sm.states:
            try:
                st = self.sm.step(state)
            except Exception as e:
                log.error("state %s failed: %s", state.name, e)
                self.metrics.reconciliation_status.set(RECONCILE_ERROR)
                self.metrics.reconciliation_failed.inc()
                self._set_state(name, cp.STATE_NOT_READY, [state.name], message=f"{state.name}: {e}")
                raise
            self.last_states[state.name] = st
            if st == oc.NOT_READY:
                not_ready.append(state.name)
        self.metrics.states_not_ready.set(len(not_ready))
        if not_ready:
            self.metrics.reconciliation_status.set(RECONCILE_NOT_READY)
            self.metrics.reconciliation_failed.inc()
            self._set_state(name, cp.STATE_NOT_READY, not_ready)
            log.info("ClusterPolicy not ready: %s", not_ready)
            return Result(requeue_after=REQUEUE_NOT_READY)
        if not self.sm.has_nfd:
            self._set_state(name, cp.STATE_NOT_READY, message="no NFD-labelled node; waiting for nodes")
            self.metrics.reconciliation_status.set(RECONCILE_NOT_READY)
            return Result(requeue_after=REQUEUE_NO_NFD)
        self._set_state(name, cp.STATE_READY)
        self.metrics.reconciliation_status.set(RECONCILE_OK)
        self.metrics.reconciliation_last_success.set(time.time())
        log.info("ClusterPolicy %s ready (%d GPU nodes)", name, self.sm.gpu_node_count)
        return Result()

    # -- watches (reference: addWatchNewGPUNode :220-314) -----------------------------------
    def _all_policies(self, _ev: WatchEvent):
        return [("", o.name(i)) for i in self.client.list(cp.API_VERSION, cp.KIND)]

    @staticmethod
    def node_predicate(ev: WatchEvent) -> bool:
        new = o.get_labels(ev.obj)
        if ev.type == DELETED:
            return has_gpu_labels(new)
        if ev.type != MODIFIED or ev.old is None:
            return has_gpu_labels(new)
        old = o.get_labels(ev.old)
        return any((
            has_gpu_labels(new) and not has_common_gpu_label(new),
            not has_gpu_labels(new) and has_common_gpu_label(new),
            is_partition_capable(new) and C.PARTITION_MANAGER_DEPLOY_LABEL not in new
            and has_common_gpu_label(new) and not has_operands_disabled(new),
            has_operands_disabled(old) != has_operands_disabled(new),
            workload_config(old, True, "")[0] != workload_config(new, True, "")[0],
            old.get(C.NFD_OSTREE_LABEL) != new.get(C.NFD_OSTREE_LABEL),
            old.get(C.NFD_KERNEL_LABEL) != new.get(C.NFD_KERNEL_LABEL),
            old.get(C.PARTITION_CAPABLE_LABEL) != new.get(C.PARTITION_CAPABLE_LABEL),
            any(old.get(k) != new.get(k) for lm in C.GPU_STATE_LABELS.values() for k in lm),
        ))

    def _owner_policy(self, ev: WatchEvent):
        ref = o.controller_of(ev.obj)
        if ref and ref.get("kind") == cp.KIND:
            return [("", ref.get("name"))]
        return []

    @staticmethod
    def daemonset_predicate(ev: WatchEvent) -> bool:
        if ev.type != MODIFIED or ev.old is None:
            return True
        return (ev.obj.get("status") or {}) != (ev.old.get("status") or {}) or \
            ev.obj.get("spec") != ev.old.get("spec")

    def controller(self) -> Controller:
        c = Controller("clusterpolicy-controller", self.reconcile, workers=1)
        c.watch(cp.API_VERSION, cp.KIND, lambda ev: [("", o.name(ev.obj))])
        c.watch("v1", "Node", self._all_policies, self.node_predicate)
        c.watch("apps/v1", "DaemonSet", self._owner_policy, self.daemonset_predicate, namespace=self.namespace)
        return c
