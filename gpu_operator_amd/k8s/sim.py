"""Minimal in-process simulation of the cluster-side controllers the operator depends on:
the DaemonSet controller (pods per matching node, ControllerRevisions, DaemonSet status) and
a kubelet that runs pods to Running/Ready (optionally gated by a readiness function).

Together with :class:`~gpu_operator_amd.k8s.fake.FakeClient` this gives the multi-node
"envtest" the reference never had ("There is no kind, KWOK or envtest
cluster test"): the reconciler can be driven to ``ready`` over N synthetic GPU nodes.
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional

from . import errors
from . import objects as o
from .fake import FakeClient

ReadyFn = Callable[[Dict, Dict], bool]   # (pod, node) -> ready?


def _node_matches(pod_spec: Dict, node: Dict) -> bool:
    sel = pod_spec.get("nodeSelector") or {}
    labels = o.get_labels(node)
    # DaemonSet pods tolerate node.kubernetes.io/unschedulable (added by the DS controller),
    # so a cordoned node keeps its operand pods.
    return not any(labels.get(k) != v for k, v in sel.items())


def pod_ready(pod: Dict) -> bool:
    """The Ready condition a kubelet reports."""
    for c in (pod.get("status") or {}).get("conditions") or []:
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return False


class ClusterSim:
    """``kubelet=False``: only the DaemonSet controller runs here; pod status belongs to an
    external kubelet (e2e/kubelet.py runs the pods as processes) and readiness is read from the
    pods' Ready condition."""

    def __init__(self, client: FakeClient, ready_fn: Optional[ReadyFn] = None, kubelet: bool = True):
        self.client = client
        self.ready_fn = ready_fn or (lambda pod, node: True)
        self.kubelet = kubelet

    def _revision(self, ds: Dict) -> str:
        return o.stable_hash(ds["spec"].get("template"))[:10]

    def sync(self) -> None:
        """One pass of DaemonSet controller + kubelet over every DaemonSet."""
        nodes = {o.name(n): n for n in self.client.list("v1", "Node")}
        dss = self.client.list("apps/v1", "DaemonSet")
        self._collect_orphans({d["metadata"]["uid"] for d in dss})
        for ds in dss:
            self._sync_ds(ds, nodes)

    def _collect_orphans(self, live_uids) -> None:
        """The garbage collector's half: a pod whose controlling DaemonSet is gone is deleted
        (a pass that raced the DaemonSet's deletion may have created it after the cascade)."""
        for p in self.client.list("v1", "Pod"):
            ref = o.controller_of(p)
            if ref and ref.get("kind") == "DaemonSet" and ref.get("uid") not in live_uids:
                try:
                    self.client.delete("v1", "Pod", o.name(p), o.namespace(p))
                except errors.NotFound:
                    pass

    def _sync_ds(self, ds: Dict, nodes: Dict[str, Dict]) -> None:
        ns, name = o.namespace(ds), o.name(ds)
        tmpl = ds["spec"]["template"]
        rev = self._revision(ds)
        rev_name = f"{name}-{rev}"
        revs = self.client.list("apps/v1", "ControllerRevision", ns)
        mine = [r for r in revs if o.owned_by(r, ds["metadata"]["uid"])]
        if not any(o.name(r) == rev_name for r in mine):
            nxt = max([r.get("revision", 0) for r in mine] or [0]) + 1
            cr = {"apiVersion": "apps/v1", "kind": "ControllerRevision",
                  "metadata": {"name": rev_name, "namespace": ns,
                               "labels": dict((ds["spec"].get("selector") or {}).get("matchLabels") or {})},
                  "revision": nxt, "data": {}}
            o.set_controller_reference(ds, cr)
            self.client.create(cr)
        on_delete = (ds["spec"].get("updateStrategy") or {}).get("type") == "OnDelete"
        want = {n for n, node in nodes.items() if _node_matches(tmpl.get("spec") or {}, node)}
        pods = [p for p in self.client.list("v1", "Pod", ns) if o.owned_by(p, ds["metadata"]["uid"])]
        by_node = {(p.get("spec") or {}).get("nodeName"): p for p in pods}
        for node_name, pod in list(by_node.items()):
            stale = o.get_labels(pod).get("controller-revision-hash") != rev
            if node_name not in want or (stale and not on_delete):
                try:
                    self.client.delete("v1", "Pod", o.name(pod), ns)
                except errors.NotFound:
                    pass
                by_node.pop(node_name)
        if want.difference(by_node):
            try:                                   # never create pods for a DaemonSet being deleted
                cur = self.client.get("apps/v1", "DaemonSet", name, ns)
            except errors.NotFound:
                return
            if cur["metadata"].get("uid") != ds["metadata"]["uid"] or cur["metadata"].get("deletionTimestamp"):
                return
        for node_name in sorted(want):
            if node_name in by_node:
                continue
            labels = dict((tmpl.get("metadata") or {}).get("labels") or {})
            labels["controller-revision-hash"] = rev
            pod = {"apiVersion": "v1", "kind": "Pod",
                   "metadata": {"name": f"{name}-{node_name}", "namespace": ns, "labels": labels},
                   "spec": dict(tmpl.get("spec") or {}, nodeName=node_name),
                   "status": {"phase": "Pending"}}
            o.set_controller_reference(ds, pod)
            by_node[node_name] = self.client.create(pod)
        available = 0
        for node_name, pod in by_node.items():
            if not self.kubelet:
                available += 1 if pod_ready(pod) else 0
                continue
            ready = self.ready_fn(pod, nodes[node_name])
            cstat = [{"name": c["name"], "ready": ready} for c in (pod["spec"].get("containers") or [])]
            st = {"phase": "Running" if ready else "Pending", "containerStatuses": cstat}
            if pod.get("status") != st:
                pod = self.client.get("v1", "Pod", o.name(pod), ns)
                pod["status"] = st
                self.client.update_status(pod)
            available += 1 if ready else 0
        desired = len(want)
        status = {"observedGeneration": ds["metadata"].get("generation", 1),
                  "desiredNumberScheduled": desired, "currentNumberScheduled": len(by_node),
                  "numberReady": available, "numberAvailable": available,
                  "numberUnavailable": desired - available,
                  "updatedNumberScheduled": sum(1 for p in by_node.values()
                                                if o.get_labels(p).get("controller-revision-hash") == rev)}
        if ds.get("status") != status:
            cur = self.client.get("apps/v1", "DaemonSet", name, ns)
            cur["status"] = status
            self.client.update_status(cur)

    def pods_on(self, node_name: str) -> List[Dict]:
        return [p for p in self.client.list("v1", "Pod", field_selector=f"spec.nodeName={node_name}")]
