"""``amd-gpu-operator``: the controller manager (reference: main.go:60-159).

Flags mirror the reference: ``--metrics-bind-address`` (:8080), ``--health-probe-bind-address``
(:8081), ``--leader-elect``, ``--leader-lease-renew-deadline``; plus ``--debug-bind-address``
(thread dump endpoint, the pprof role the reference leaves unset) and
``--zap-log-level`` / ``--zap-time-encoding`` accepted for Helm-values compatibility.
"""

from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import time


def parse_duration(s: str) -> float:
    s = s.strip()
    mult = {"ms": 1e-3, "s": 1, "m": 60, "h": 3600}
    for suf in ("ms", "s", "m", "h"):
        if s.endswith(suf):
            return float(s[: -len(suf)]) * mult[suf]
    return float(s)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="amd-gpu-operator")
    ap.add_argument("--metrics-bind-address", default=":8080")
    ap.add_argument("--health-probe-bind-address", default=":8081")
    ap.add_argument("--debug-bind-address", default="")
    ap.add_argument("--leader-elect", action="store_true")
    ap.add_argument("--leader-lease-renew-deadline", default="10s")
    ap.add_argument("--leader-lease-duration", default="15s")
    ap.add_argument("--zap-log-level", default="info")
    ap.add_argument("--zap-time-encoding", default="iso8601")
    ap.add_argument("--zap-devel", action="store_true")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--no-cache", action="store_true", help="read from the API server on every access (debugging)")
    a = ap.parse_args(argv)

    level = {"debug": logging.DEBUG, "info": logging.INFO, "error": logging.ERROR}.get(a.zap_log_level, logging.INFO)
    fmt = "%(created).3f %(levelname)s %(name)s %(message)s" if a.zap_time_encoding == "epoch" else \
        "%(asctime)s %(levelname)s %(name)s %(message)s"
    logging.basicConfig(level=level, format=fmt, stream=sys.stderr)
    log = logging.getLogger("amd-gpu-operator")

    namespace = os.environ.get("OPERATOR_NAMESPACE", "")
    if not namespace:
        log.error("OPERATOR_NAMESPACE environment variable not set, cannot proceed")
        return 1

    from ..controllers.clusterpolicy_controller import ClusterPolicyReconciler
    from ..controllers.operator_metrics import OperatorMetrics
    from ..controllers.state_manager import SnapshotHolder
    from ..controllers.upgrade_controller import UpgradeReconciler
    from ..k8s.rest import Config, RestClient
    from ..runtime.cache import CachedClient
    from ..runtime.manager import Manager

    cfg = Config.from_kubeconfig(a.kubeconfig) if a.kubeconfig else Config.auto()
    api = RestClient(cfg)
    # reconcilers read through informers (reference: main.go:104, the manager's cached client);
    # leader election keeps reading Leases from the API server itself
    client = api if a.no_cache else CachedClient(api)
    metrics = OperatorMetrics()
    # controllers watch through the same informers the reconcilers read from (controller-runtime's
    # event handlers sit on the cache's informers): with a separate watch stream an event could
    # trigger a reconcile that still reads the pre-event object from the cache, and the cache's
    # own copy of that event would then trigger nothing -- a lost update (found by the e2e flow:
    # a node's deploy.operands=true after a disable was never acted on)
    mgr = Manager(client, namespace, registry=metrics.registry, metrics_addr=a.metrics_bind_address,
                  probe_addr=a.health_probe_bind_address, leader_elect=a.leader_elect,
                  lease_duration=parse_duration(a.leader_lease_duration),
                  renew_deadline=parse_duration(a.leader_lease_renew_deadline),
                  debug_addr=a.debug_bind_address)
    snapshot = SnapshotHolder()
    cpr = ClusterPolicyReconciler(client, namespace, metrics, snapshot=snapshot)
    upr = UpgradeReconciler(client, namespace, snapshot, metrics)
    mgr.add(cpr.controller())
    mgr.add(upr.controller())
    signal.signal(signal.SIGTERM, lambda *_: mgr.stop())
    log.info("starting manager (namespace=%s, leader-elect=%s)", namespace, a.leader_elect)
    t0 = time.time()
    mgr.start(block=True)
    log.info("manager stopped after %.0fs", time.time() - t0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
