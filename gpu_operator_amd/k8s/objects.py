"""Helpers over Kubernetes objects represented as plain dicts (the "unstructured" form).

The operator manipulates every Kubernetes kind through the same dict representation, so one
apply/readiness pipeline serves all kinds and any number of objects per kind (the reference
keeps a single typed slot per kind per state and silently drops the second Role of a state,
reference: controllers/resource_manager.go:35-53).
"""

from __future__ import annotations

import copy
import hashlib
import json
import re
from typing import Any, Dict, Iterable, List, Optional, Tuple

# apiVersion of every kind the operator manages (used when manifests omit nothing but
# callers look kinds up by name).
CORE_KINDS = {
    "Namespace": "v1", "Node": "v1", "Pod": "v1", "Service": "v1", "ServiceAccount": "v1",
    "ConfigMap": "v1", "Secret": "v1", "Event": "v1",
    "DaemonSet": "apps/v1", "Deployment": "apps/v1", "ControllerRevision": "apps/v1",
    "Role": "rbac.authorization.k8s.io/v1", "RoleBinding": "rbac.authorization.k8s.io/v1",
    "ClusterRole": "rbac.authorization.k8s.io/v1",
    "ClusterRoleBinding": "rbac.authorization.k8s.io/v1",
    "RuntimeClass": "node.k8s.io/v1", "PodSecurityPolicy": "policy/v1beta1",
    "Lease": "coordination.k8s.io/v1",
    "ServiceMonitor": "monitoring.coreos.com/v1", "PrometheusRule": "monitoring.coreos.com/v1",
    "SecurityContextConstraints": "security.openshift.io/v1",
    "CustomResourceDefinition": "apiextensions.k8s.io/v1",
    "Job": "batch/v1", "PodDisruptionBudget": "policy/v1",
}

CLUSTER_SCOPED = {"Namespace", "Node", "ClusterRole", "ClusterRoleBinding", "RuntimeClass",
                  "PodSecurityPolicy", "SecurityContextConstraints", "CustomResourceDefinition",
                  "ClusterPolicy", "ClusterVersion", "Proxy"}

ObjKey = Tuple[str, str, str, str]  # (apiVersion, kind, namespace, name)


def api_version_of(kind: str) -> str:
    return CORE_KINDS.get(kind, "v1")


def meta(obj: Dict[str, Any]) -> Dict[str, Any]:
    return obj.setdefault("metadata", {})


def name(obj: Dict[str, Any]) -> str:
    return (obj.get("metadata") or {}).get("name", "")


def namespace(obj: Dict[str, Any]) -> str:
    return (obj.get("metadata") or {}).get("namespace", "") or ""


def kind(obj: Dict[str, Any]) -> str:
    return obj.get("kind", "")


def key(obj: Dict[str, Any]) -> ObjKey:
    k = kind(obj)
    ns = "" if k in CLUSTER_SCOPED else namespace(obj)
    return (obj.get("apiVersion") or api_version_of(k), k, ns, name(obj))


def labels(obj: Dict[str, Any]) -> Dict[str, str]:
    return meta(obj).setdefault("labels", {}) if obj is not None else {}


def annotations(obj: Dict[str, Any]) -> Dict[str, str]:
    return meta(obj).setdefault("annotations", {})


def get_labels(obj: Dict[str, Any]) -> Dict[str, str]:
    return dict((obj.get("metadata") or {}).get("labels") or {})


def get_annotations(obj: Dict[str, Any]) -> Dict[str, str]:
    return dict((obj.get("metadata") or {}).get("annotations") or {})


def deepcopy(obj):
    return copy.deepcopy(obj)


def set_controller_reference(owner: Dict[str, Any], obj: Dict[str, Any]) -> None:
    """Make ``owner`` the controller of ``obj`` (garbage collection on owner delete)."""
    om = owner.get("metadata") or {}
    if not om.get("uid"):
        raise ValueError(f"owner {name(owner)} has no uid")
    ref = {"apiVersion": owner.get("apiVersion"), "kind": owner.get("kind"), "name": om.get("name"),
           "uid": om["uid"], "controller": True, "blockOwnerDeletion": True}
    existing = meta(obj).get("ownerReferences") or []
    for r in existing:
        if r.get("controller") and r.get("uid") != om["uid"]:
            raise ValueError(f"object {name(obj)} already controlled by {r.get('kind')}/{r.get('name')}")
    refs = [r for r in existing if r.get("uid") != om["uid"]]
    refs.append(ref)
    meta(obj)["ownerReferences"] = refs


def owned_by(obj: Dict[str, Any], owner_uid: str) -> bool:
    return any(r.get("uid") == owner_uid for r in (obj.get("metadata") or {}).get("ownerReferences") or [])


def controller_of(obj: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
        if r.get("controller"):
            return r
    return None


# ------------------------------------------------------------------------------------------
# label selectors
# ------------------------------------------------------------------------------------------
_SEL_TOKEN = re.compile(
    r"\s*(?:(?P<notexists>!\s*[\w./-]+)"
    r"|(?P<set>[\w./-]+\s+(?:in|notin)\s*\([^)]*\))"
    r"|(?P<cmp>[\w./-]+\s*(?:==|!=|=)\s*[\w./-]*)"
    r"|(?P<exists>[\w./-]+))\s*(?:,|$)")


def parse_label_selector(sel: Optional[str]) -> List[Tuple[str, str, Any]]:
    """Parse a Kubernetes label selector string into (key, op, value) requirements.

    Supported: ``k=v``, ``k==v``, ``k!=v``, ``k in (a,b)``, ``k notin (a,b)``, ``k``, ``!k``.
    """
    reqs: List[Tuple[str, str, Any]] = []
    if not sel or not sel.strip():
        return reqs
    pos = 0
    s = sel.strip()
    while pos < len(s):
        m = _SEL_TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise ValueError(f"invalid label selector {sel!r} at {pos}")
        if m.group("notexists"):
            reqs.append((m.group("notexists")[1:].strip(), "!", None))
        elif m.group("set"):
            k, rest = re.split(r"\s+", m.group("set").strip(), maxsplit=1)
            op, vals = re.match(r"(in|notin)\s*\(([^)]*)\)", rest).groups()
            reqs.append((k, op, {v.strip() for v in vals.split(",") if v.strip()}))
        elif m.group("cmp"):
            k, op, v = re.match(r"([\w./-]+)\s*(==|!=|=)\s*([\w./-]*)", m.group("cmp").strip()).groups()
            reqs.append((k, "!=" if op == "!=" else "=", v))
        else:
            reqs.append((m.group("exists").strip(), "exists", None))
        pos = m.end()
    return reqs


def selector_matches(selector: Any, lbls: Dict[str, str]) -> bool:
    """Match a selector given as a string, a ``{k: v}`` dict, or a LabelSelector object."""
    if selector is None or selector == "" or selector == {}:
        return True
    if isinstance(selector, str):
        return all(_req_ok(r, lbls) for r in parse_label_selector(selector))
    if isinstance(selector, dict) and ("matchLabels" in selector or "matchExpressions" in selector):
        for k, v in (selector.get("matchLabels") or {}).items():
            if lbls.get(k) != v:
                return False
        for e in selector.get("matchExpressions") or []:
            op = {"In": "in", "NotIn": "notin", "Exists": "exists", "DoesNotExist": "!"}[e["operator"]]
            if not _req_ok((e["key"], op, set(e.get("values") or [])), lbls):
                return False
        return True
    if isinstance(selector, dict):
        return all(lbls.get(k) == v for k, v in selector.items())
    raise TypeError(f"unsupported selector {selector!r}")


def _req_ok(req, lbls: Dict[str, str]) -> bool:
    k, op, v = req
    if op == "=":
        return lbls.get(k) == v
    if op == "!=":
        return lbls.get(k) != v
    if op == "in":
        return k in lbls and lbls[k] in v
    if op == "notin":
        return k not in lbls or lbls[k] not in v
    if op == "exists":
        return k in lbls
    if op == "!":
        return k not in lbls
    raise ValueError(op)


def field_value(obj: Dict[str, Any], path: str) -> Any:
    cur: Any = obj
    for part in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(part)
    return cur


def field_selector_matches(sel: Optional[str], obj: Dict[str, Any]) -> bool:
    if not sel:
        return True
    for term in sel.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            p, v = term.split("!=", 1)
            if str(field_value(obj, p.strip()) or "") == v.strip():
                return False
        else:
            p, v = term.replace("==", "=").split("=", 1)
            if str(field_value(obj, p.strip()) or "") != v.strip():
                return False
    return True


# ------------------------------------------------------------------------------------------
# hashing / containers
# ------------------------------------------------------------------------------------------
def stable_hash(obj: Any) -> str:
    """Deterministic hash of a JSON-compatible value (role of hashstructure in the reference,
    reference: controllers/object_controls.go:3890-3929)."""
    data = json.dumps(obj, sort_keys=True, separators=(",", ":"), default=str).encode()
    return hashlib.sha256(data).hexdigest()[:16]


def pod_spec(obj: Dict[str, Any]) -> Dict[str, Any]:
    """The pod spec of a Pod, or the pod template spec of a workload."""
    if obj.get("kind") == "Pod":
        return obj.setdefault("spec", {})
    return obj.setdefault("spec", {}).setdefault("template", {}).setdefault("spec", {})


def pod_template_meta(obj: Dict[str, Any]) -> Dict[str, Any]:
    return obj.setdefault("spec", {}).setdefault("template", {}).setdefault("metadata", {})


def containers(obj: Dict[str, Any], init: bool = False) -> List[Dict[str, Any]]:
    return pod_spec(obj).setdefault("initContainers" if init else "containers", [])


def find_container(obj: Dict[str, Any], cname: str, init: bool = False) -> Optional[Dict[str, Any]]:
    for c in containers(obj, init):
        if c.get("name") == cname:
            return c
    return None


def remove_container(obj: Dict[str, Any], cname: str, init: bool = False) -> bool:
    lst = containers(obj, init)
    kept = [c for c in lst if c.get("name") != cname]
    pod_spec(obj)["initContainers" if init else "containers"] = kept
    return len(kept) != len(lst)


def set_env(container: Dict[str, Any], ename: str, value: str) -> None:
    """Upsert an environment variable (reference: setContainerEnv, object_controls.go:2033)."""
    env = container.setdefault("env", [])
    for e in env:
        if e.get("name") == ename:
            e.pop("valueFrom", None)
            e["value"] = value
            return
    env.append({"name": ename, "value": value})


def get_env(container: Dict[str, Any], ename: str) -> Optional[str]:
    for e in container.get("env") or []:
        if e.get("name") == ename:
            return e.get("value")
    return None


def remove_env(container: Dict[str, Any], ename: str) -> None:
    container["env"] = [e for e in container.get("env") or [] if e.get("name") != ename]


def add_volume(obj: Dict[str, Any], volume: Dict[str, Any]) -> None:
    vols = pod_spec(obj).setdefault("volumes", [])
    for i, v in enumerate(vols):
        if v.get("name") == volume["name"]:
            vols[i] = volume
            return
    vols.append(volume)


def add_volume_mount(container: Dict[str, Any], mount: Dict[str, Any]) -> None:
    mounts = container.setdefault("volumeMounts", [])
    for i, m in enumerate(mounts):
        if m.get("name") == mount["name"] and m.get("mountPath") == mount.get("mountPath"):
            mounts[i] = mount
            return
    mounts.append(mount)


def host_path_volume(vname: str, path: str, type_: Optional[str] = None) -> Dict[str, Any]:
    hp: Dict[str, Any] = {"path": path}
    if type_:
        hp["type"] = type_
    return {"name": vname, "hostPath": hp}


def iter_all_containers(obj: Dict[str, Any]) -> Iterable[Dict[str, Any]]:
    yield from containers(obj, init=True)
    yield from containers(obj, init=False)
