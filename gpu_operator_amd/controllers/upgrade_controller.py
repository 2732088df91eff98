"""Upgrade reconciler: drives :class:`UpgradeStateManager` from the ClusterPolicy's driver
upgrade policy (reference: controllers/upgrade_controller.go:71-259).

Reads the shared :class:`ClusterSnapshot` (immutable) instead of the ClusterPolicy
reconciler's mutable state. Requeues every 2 minutes while enabled; node label changes and
driver DaemonSet/pod changes trigger it earlier.
"""

from __future__ import annotations

import logging
from typing import Optional

from ..api.v1 import clusterpolicy as cp
from ..k8s import errors
from ..k8s import objects as o
from ..k8s.client import MODIFIED, WatchEvent
from ..runtime.controller import Controller, Result
from . import consts as C
from .operator_metrics import OperatorMetrics
from .state_manager import SnapshotHolder
from .upgrade import UPGRADE_STATE_LABEL, UpgradeStateManager

log = logging.getLogger("amd-gpu-operator.upgrade-controller")

PLANNED_REQUEUE = 120.0


class UpgradeReconciler:
    def __init__(self, client, namespace: str, snapshot: SnapshotHolder,
                 metrics: Optional[OperatorMetrics] = None, run_async: bool = True):
        self.client = client
        self.namespace = namespace
        self.snapshot = snapshot
        self.metrics = metrics
        self.mgr = UpgradeStateManager(client, namespace, run_async=run_async)

    def reconcile(self, req) -> Result:
        name = req[1] if isinstance(req, tuple) else req
        try:
            obj = self.client.get(cp.API_VERSION, cp.KIND, name)
        except errors.NotFound:
            return Result()
        policy = cp.ClusterPolicy(obj).spec
        snap = self.snapshot.get()
        up = policy.driver.upgradePolicy
        if snap.sandbox_enabled or up is None or not up.autoUpgrade or not policy.driver.is_enabled():
            self.mgr.remove_upgrade_labels()
            if self.metrics:
                self.metrics.driver_auto_upgrade_enabled.set(0)
            return Result()
        if self.metrics:
            self.metrics.driver_auto_upgrade_enabled.set(1)
        labels = dict(snap.driver_app_labels)
        state = self.mgr.build_state(labels)
        st = self.mgr.stats(state, up)
        if self.metrics:
            self.metrics.upgrades_in_progress.set(st["in_progress"])
            self.metrics.upgrades_done.set(st["done"])
            self.metrics.upgrades_failed.set(st["failed"])
            self.metrics.upgrades_available.set(st["available"])
            self.metrics.upgrades_pending.set(st["pending"])
        self.mgr.apply_state(state, up)
        return Result(requeue_after=PLANNED_REQUEUE)

    def controller(self) -> Controller:
        c = Controller("upgrade-controller", self.reconcile, workers=1)
        all_cps = lambda ev: [("", o.name(i)) for i in self.client.list(cp.API_VERSION, cp.KIND)]  # noqa: E731
        c.watch(cp.API_VERSION, cp.KIND, lambda ev: [("", o.name(ev.obj))])

        def node_changed(ev: WatchEvent) -> bool:
            if ev.type != MODIFIED or ev.old is None:
                return False
            a, b = o.get_labels(ev.old), o.get_labels(ev.obj)
            return a.get(UPGRADE_STATE_LABEL) != b.get(UPGRADE_STATE_LABEL) or \
                (ev.old.get("spec") or {}).get("unschedulable") != (ev.obj.get("spec") or {}).get("unschedulable")
        c.watch("v1", "Node", all_cps, node_changed)
        c.watch("apps/v1", "DaemonSet", all_cps,
                lambda ev: o.get_labels(ev.obj).get("app") == C.DS_DRIVER, namespace=self.namespace)
        c.watch("v1", "Pod", all_cps, lambda ev: o.get_labels(ev.obj).get("app") == C.DS_DRIVER,
                namespace=self.namespace)
        return c
