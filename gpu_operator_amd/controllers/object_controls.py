"""Per-kind apply functions and readiness checks.

Every object of a state goes through ``apply_object``: fill the namespace placeholders,
delete it if the state is disabled, set the ClusterPolicy as controller (GC on CR delete),
then create or update. All kinds are change-detected with a spec hash annotation, not only
DaemonSets: the reference re-``Update``s Roles, ConfigMaps, Services, SCCs and
RuntimeClasses on every 5 s pass (SURVEY.md §3.2 "hot loop"); here an unchanged object costs
one GET.

Reference: controllers/object_controls.go (ServiceAccount :251, Role :286, RoleBinding :327,
ClusterRole :378, ClusterRoleBinding :419, ConfigMaps :464-552, Deployment :3241, DaemonSet
:3745-3888, SCC :3961, PSP :4021, Service :4069, ServiceMonitor :4131, RuntimeClasses :4430,
PrometheusRule :4467; readiness isDaemonSetReady :3107-3177).
"""

from __future__ import annotations

import copy
import logging
from typing import Any, Dict, List, Optional, Tuple

from ..k8s import errors
from ..k8s import objects as o
from . import consts as C
from . import transforms as T

log = logging.getLogger("amd-gpu-operator.controls")

READY = "ready"
NOT_READY = "notReady"
DISABLED = "disabled"

Obj = Dict[str, Any]


# ---------------------------------------------------------------------------------------------
# placeholders / ownership / hashing
# ---------------------------------------------------------------------------------------------
def fill_namespace(obj: Obj, ns: str) -> None:
    md = o.meta(obj)
    if o.kind(obj) not in o.CLUSTER_SCOPED:
        md["namespace"] = ns
    for s in obj.get("subjects") or []:
        if s.get("namespace") == C.PLACEHOLDER:
            s["namespace"] = ns
    if o.kind(obj) == "SecurityContextConstraints":
        obj["users"] = [u.replace(C.PLACEHOLDER, ns) for u in obj.get("users") or []]
    nss = ((obj.get("spec") or {}).get("namespaceSelector") or {}).get("matchNames")
    if nss:
        obj["spec"]["namespaceSelector"]["matchNames"] = [ns if x == C.PLACEHOLDER else x for x in nss]


def _hash_payload(obj: Obj) -> Any:
    body = {k: v for k, v in obj.items() if k not in ("metadata", "status")}
    md = obj.get("metadata") or {}
    anns = {k: v for k, v in (md.get("annotations") or {}).items() if k != C.LAST_APPLIED_HASH_ANNOTATION}
    return {"body": body, "labels": md.get("labels") or {}, "annotations": anns}


def spec_hash(obj: Obj) -> str:
    return o.stable_hash(_hash_payload(obj))


def _delete(n, obj: Obj) -> None:
    """Delete the object of a disabled state if it exists. The existence check is a cache read
    under the informer cache (runtime/cache.py), so a steady pass over disabled states writes
    nothing, where the reference issues a blind DELETE per object per pass."""
    try:
        n.client.get(obj["apiVersion"], obj["kind"], o.name(obj), o.namespace(obj))
        n.client.delete(obj["apiVersion"], obj["kind"], o.name(obj), o.namespace(obj))
        log.info("deleted %s/%s (state disabled)", obj["kind"], o.name(obj))
    except errors.NotFound:
        pass
    except errors.NoKindMatch:
        pass


def create_or_update(n, obj: Obj, create_only: bool = False,
                     preserve: Optional[List[Tuple[str, ...]]] = None) -> bool:
    """Create ``obj`` or update it when its spec hash changed. Returns True if written."""
    o.set_controller_reference(n.owner, obj)
    h = spec_hash(obj)
    o.annotations(obj)[C.LAST_APPLIED_HASH_ANNOTATION] = h
    try:
        found = n.client.get(obj["apiVersion"], obj["kind"], o.name(obj), o.namespace(obj))
    except errors.NotFound:
        n.client.create(obj)
        log.info("created %s/%s", obj["kind"], o.name(obj))
        return True
    if create_only:
        return False
    if o.get_annotations(found).get(C.LAST_APPLIED_HASH_ANNOTATION) == h:
        return False
    o.meta(obj)["resourceVersion"] = found["metadata"].get("resourceVersion")
    for path in preserve or []:
        src, dst = found, obj
        for p in path[:-1]:
            src = (src or {}).get(p) or {}
            dst = dst.setdefault(p, {})
        if path[-1] in (src or {}):
            dst[path[-1]] = copy.deepcopy(src[path[-1]])
    n.client.update(obj)
    log.info("updated %s/%s", obj["kind"], o.name(obj))
    return True


# ---------------------------------------------------------------------------------------------
# kind controls
# ---------------------------------------------------------------------------------------------
def control_generic(n, state, obj: Obj) -> str:
    if not n.is_state_enabled(state.name):
        _delete(n, obj)
        return DISABLED
    create_or_update(n, obj)
    return READY


def control_service_account(n, state, obj: Obj) -> str:
    if not n.is_state_enabled(state.name):
        _delete(n, obj)
        return DISABLED
    create_or_update(n, obj, create_only=True)   # token secrets are bound to the SA uid
    return READY


def control_configmap(n, state, obj: Obj) -> str:
    if not n.is_state_enabled(state.name):
        _delete(n, obj)
        return DISABLED
    if o.name(obj) == "amd-kata-manager-config":
        obj["data"] = T.render_kata_configmap_data(n.spec)
    create_or_update(n, obj)
    return READY


def control_service(n, state, obj: Obj) -> str:
    if not n.is_state_enabled(state.name):
        _delete(n, obj)
        return DISABLED
    create_or_update(n, obj, preserve=[("spec", "clusterIP"), ("spec", "clusterIPs")])
    return READY


def control_service_monitor(n, state, obj: Obj) -> str:
    if not n.client.has_kind(obj["apiVersion"], obj["kind"]):
        # prometheus-operator not installed: nothing to do (reference checks the CRD too)
        if state.name == "state-metrics-exporter" and n.spec.metricsExporter.serviceMonitor \
                and n.spec.metricsExporter.serviceMonitor.is_enabled():
            raise errors.NoKindMatch("metricsExporter.serviceMonitor.enabled but the ServiceMonitor CRD "
                                     "(monitoring.coreos.com/v1) is not installed")
        return READY
    enabled = n.is_state_enabled(state.name)
    if state.name == "state-metrics-exporter":
        sm = n.spec.metricsExporter.serviceMonitor
        enabled = enabled and sm is not None and sm.is_enabled()
        if enabled:
            ep = obj["spec"]["endpoints"][0]
            if sm.interval:
                ep["interval"] = sm.interval
            if sm.honorLabels is not None:
                ep["honorLabels"] = sm.honorLabels
            if sm.relabelings:
                ep["relabelings"] = copy.deepcopy(sm.relabelings)
            for k, v in (sm.additionalLabels or {}).items():
                o.labels(obj)[k] = v
    if not enabled:
        _delete(n, obj)
        return DISABLED
    create_or_update(n, obj)
    return READY


def control_prometheus_rule(n, state, obj: Obj) -> str:
    if not n.client.has_kind(obj["apiVersion"], obj["kind"]):
        return READY
    return control_generic(n, state, obj)


def control_psp(n, state, obj: Obj) -> str:
    if n.k8s_minor() >= 25:
        return READY          # policy/v1beta1 is no longer served (reference :168-172)
    if not n.spec.psp.is_enabled():
        _delete(n, obj)
        return DISABLED
    return control_generic(n, state, obj)


def control_scc(n, state, obj: Obj) -> str:
    if not n.openshift:
        return READY
    return control_generic(n, state, obj)


def control_runtime_class(n, state, obj: Obj) -> str:
    labels = o.get_labels(obj)
    if labels.get(C.KATA_RUNTIME_CLASS_LABEL) == "true":
        return _kata_runtime_classes(n, state, obj)
    if o.name(obj) == "amd-cdi":
        if not n.spec.cdi.is_enabled():
            _delete(n, obj)
            return READY
        return control_generic(n, state, obj)
    rc = n.spec.operator.runtime_class()
    obj["metadata"]["name"] = rc
    obj["handler"] = rc
    if n.k8s_minor() <= 20:
        obj["apiVersion"] = "node.k8s.io/v1beta1"
    return control_generic(n, state, obj)


def _kata_runtime_classes(n, state, template: Obj) -> str:
    want = {}
    if n.is_state_enabled(state.name):
        cfg = T.kata_config(n.spec)
        for rc in cfg.get("runtimeClasses") or []:
            obj = copy.deepcopy(template)
            obj["metadata"]["name"] = rc["name"]
            obj["handler"] = rc["name"]
            if rc.get("nodeSelector"):
                obj["scheduling"] = {"nodeSelector": dict(rc["nodeSelector"])}
            want[rc["name"]] = obj
    existing = n.client.list(template["apiVersion"], "RuntimeClass",
                             label_selector={C.KATA_RUNTIME_CLASS_LABEL: "true"})
    for ex in existing:
        if o.name(ex) not in want and o.owned_by(ex, n.owner["metadata"]["uid"]):
            _delete(n, ex)
    for obj in want.values():
        create_or_update(n, obj)
    return READY


def control_deployment(n, state, obj: Obj) -> str:
    if not n.is_state_enabled(state.name):
        _delete(n, obj)
        return DISABLED
    create_or_update(n, obj)
    return deployment_ready(n, o.name(obj))


def deployment_ready(n, name: str) -> str:
    try:
        d = n.client.get("apps/v1", "Deployment", name, n.namespace)
    except errors.NotFound:
        return NOT_READY
    st = d.get("status") or {}
    if st.get("observedGeneration", 0) < d["metadata"].get("generation", 1):
        return NOT_READY
    if st.get("unavailableReplicas", 0) != 0:
        return NOT_READY
    if st.get("availableReplicas", 0) < (d.get("spec") or {}).get("replicas", 1):
        return NOT_READY
    return READY


# ---------------------------------------------------------------------------------------------
# DaemonSets (reference: DaemonSet :3745-3888)
# ---------------------------------------------------------------------------------------------
def control_daemonset(n, state, obj: Obj) -> str:
    base = o.name(obj)
    if not n.is_state_enabled(state.name):
        for ds in n.daemonset_variants_existing(base):
            _delete(n, ds)
        _delete(n, obj)
        return DISABLED
    if not n.has_gpu_nodes:
        return READY
    variants = n.daemonset_variants(base)
    if variants is None:
        pending = n.cleanup_stale_variants(base, None) if base in n.FANOUT_BASES else False
        st = _apply_one_daemonset(n, obj)
        return NOT_READY if pending else st
    # fan-out: one DaemonSet per kernel (precompiled), RHCOS version (DTK) or node OS
    pending = n.cleanup_stale_variants(base, variants)
    overall = NOT_READY if pending else READY
    for v in variants:
        with n.variant(v):
            st = _apply_one_daemonset(n, copy.deepcopy(obj))
        if st != READY:
            overall = NOT_READY
    return overall


def _apply_one_daemonset(n, obj: Obj) -> str:
    T.preprocess_daemonset(obj, n.spec, n)
    for k, v in (n.spec.daemonsets.labels or {}).items():
        if k not in ("app", "app.kubernetes.io/part-of"):
            o.labels(obj)[k] = v
    for k, v in (n.spec.daemonsets.annotations or {}).items():
        o.annotations(obj)[k] = v
    create_or_update(n, obj)
    return daemonset_ready(n, o.name(obj))


def daemonset_ready(n, name: str) -> str:
    """All scheduled pods available on the current generation; for OnDelete DaemonSets also
    every pod on the latest ControllerRevision and all its containers Ready."""
    try:
        ds = n.client.get("apps/v1", "DaemonSet", name, n.namespace)
    except errors.NotFound:
        return NOT_READY
    st = ds.get("status") or {}
    if st.get("observedGeneration", 0) < ds["metadata"].get("generation", 1):
        return NOT_READY
    if st.get("numberUnavailable", 0) != 0:
        return NOT_READY
    if st.get("numberAvailable", 0) < st.get("desiredNumberScheduled", 0):
        return NOT_READY
    if ((ds.get("spec") or {}).get("updateStrategy") or {}).get("type") != "OnDelete":
        return READY
    if st.get("desiredNumberScheduled", 0) == 0:
        return READY
    pods = [p for p in n.client.list("v1", "Pod", n.namespace,
                                     label_selector=(ds["spec"].get("selector") or {}).get("matchLabels"))
            if o.owned_by(p, ds["metadata"]["uid"])]
    if not pods:
        return NOT_READY
    rev = latest_revision_hash(n, ds)
    if rev is None:
        return NOT_READY
    for p in pods:
        if o.get_labels(p).get("controller-revision-hash") != rev:
            return NOT_READY
        pst = p.get("status") or {}
        if pst.get("phase") != "Running":
            return NOT_READY
        if any(not cs.get("ready") for cs in pst.get("containerStatuses") or []):
            return NOT_READY
    return READY


def latest_revision_hash(n, ds: Obj) -> Optional[str]:
    name = o.name(ds)
    revs = [r for r in n.client.list("apps/v1", "ControllerRevision", n.namespace,
                                     label_selector=(ds["spec"].get("selector") or {}).get("matchLabels"))
            if o.name(r).startswith(name + "-") and o.owned_by(r, ds["metadata"]["uid"])]
    if not revs:
        return None
    revs.sort(key=lambda r: r.get("revision", 0))
    return o.name(revs[-1])[len(name) + 1:]


CONTROLS = {
    "ServiceAccount": control_service_account,
    "Role": control_generic,
    "RoleBinding": control_generic,
    "ClusterRole": control_generic,
    "ClusterRoleBinding": control_generic,
    "ConfigMap": control_configmap,
    "DaemonSet": control_daemonset,
    "Deployment": control_deployment,
    "Service": control_service,
    "ServiceMonitor": control_service_monitor,
    "PrometheusRule": control_prometheus_rule,
    "SecurityContextConstraints": control_scc,
    "PodSecurityPolicy": control_psp,
    "RuntimeClass": control_runtime_class,
}


def apply_object(n, state, template: Obj) -> str:
    obj = copy.deepcopy(template)
    fill_namespace(obj, n.namespace)
    fn = CONTROLS.get(obj["kind"])
    if fn is None:
        raise ValueError(f"no control function for kind {obj['kind']} ({state.name})")
    return fn(n, state, obj)
