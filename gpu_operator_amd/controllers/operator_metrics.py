"""Operator Prometheus metrics (reference: controllers/operator_metrics.go:13-185), same
families under the ``amd_gpu_operator_`` prefix, registered on the manager's registry."""

from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge

RECONCILE_OK = 1
RECONCILE_NOT_READY = 0
RECONCILE_NO_CR = -1
RECONCILE_ERROR = -2

DTK_DISABLED = 0
DTK_ENABLED = 1
DTK_NOT_POSSIBLE = -1


class OperatorMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        p = "amd_gpu_operator_"
        self.gpu_nodes_total = Gauge(p + "gpu_nodes_total", "Number of nodes with AMD GPUs", registry=r)
        self.reconciliation_last_success = Gauge(
            p + "reconciliation_last_success_ts_seconds",
            "Timestamp (in seconds) of the last ClusterPolicy reconciliation that ended ready", registry=r)
        self.reconciliation_status = Gauge(
            p + "reconciliation_status",
            "1 ready, 0 notReady, -1 no ClusterPolicy, -2 reconciliation error", registry=r)
        self.reconciliation_total = Counter(p + "reconciliation_total",
                                            "ClusterPolicy reconciliations", registry=r)
        self.reconciliation_failed = Counter(p + "reconciliation_failed_total",
                                             "ClusterPolicy reconciliations that errored", registry=r)
        self.reconciliation_has_nfd_labels = Gauge(
            p + "reconciliation_has_nfd_labels", "1 if at least one node carries NFD labels", registry=r)
        self.reconcile_duration = Gauge(p + "reconciliation_duration_seconds",
                                        "Wall time of the last reconciliation", registry=r)
        self.states_not_ready = Gauge(p + "states_not_ready", "Operand states not yet ready", registry=r)
        self.dtk_enabled = Gauge(p + "openshift_driver_toolkit_enabled",
                                 "1 enabled, 0 disabled, -1 requested but not possible", registry=r)
        self.dtk_nfd_too_old = Gauge(p + "openshift_driver_toolkit_nfd_too_old",
                                     "1 if NFD does not publish the RHCOS OSTree label", registry=r)
        self.dtk_imagestream_missing = Gauge(p + "openshift_driver_toolkit_imagestream_missing",
                                             "1 if the driver-toolkit ImageStream is missing", registry=r)
        self.dtk_rhcos_tags_missing = Gauge(p + "openshift_driver_toolkit_rhcos_tags_missing",
                                            "1 if an RHCOS version has no driver-toolkit tag", registry=r)
        self.dtk_imagestream_broken = Gauge(p + "openshift_driver_toolkit_imagestream_broken",
                                            "1 if a driver-toolkit tag points nowhere", registry=r)
        self.driver_auto_upgrade_enabled = Gauge(p + "driver_auto_upgrade_enabled",
                                                 "1 if amdgpu driver auto-upgrade is enabled", registry=r)
        self.upgrades_in_progress = Gauge(p + "nodes_upgrades_in_progress", "Nodes upgrading", registry=r)
        self.upgrades_done = Gauge(p + "nodes_upgrades_done", "Nodes upgraded", registry=r)
        self.upgrades_failed = Gauge(p + "nodes_upgrades_failed", "Nodes whose upgrade failed", registry=r)
        self.upgrades_available = Gauge(p + "nodes_upgrades_available",
                                        "Upgrade slots available under maxParallelUpgrades", registry=r)
        self.upgrades_pending = Gauge(p + "nodes_upgrades_pending", "Nodes waiting to upgrade", registry=r)

    def set_dtk(self, openshift: str, requested: bool, enabled: bool) -> None:
        if not openshift or not requested:
            self.dtk_enabled.set(DTK_DISABLED)
        else:
            self.dtk_enabled.set(DTK_ENABLED if enabled else DTK_NOT_POSSIBLE)
