"""In-memory Kubernetes API for tests: resourceVersion/uid/generation bookkeeping, optimistic
concurrency, status subresource, label/field selectors, owner-reference garbage collection,
watches and fault-injection interceptors.

The reference's unit tests use controller-runtime's fake client (reference:
controllers/object_controls_test.go:227); this one is also what the multi-node "envtest"
simulations (tests/test_e2e_sim.py) run against, together with :mod:`gpu_operator_amd.k8s.sim`.
"""

from __future__ import annotations

import copy
import itertools
import threading
import time
import uuid
from typing import Any, Callable, Dict, List, Optional, Set, Tuple

from . import errors
from . import objects as o
from .client import ADDED, DELETED, MODIFIED, Obj, WatchCallback, WatchEvent, merge_patch

STATUS_SUBRESOURCE = {"ClusterPolicy", "DaemonSet", "Deployment", "Pod", "Node", "Job"}

Interceptor = Callable[[str, str, str, Any], None]   # (verb, apiVersion, kind, obj|name) -> raise?


class FakeClient:
    def __init__(self, objs: Optional[List[Obj]] = None, server_version: str = "v1.29.2",
                 unserved_kinds: Optional[Set[str]] = None, collect_orphans: bool = False):
        self._lock = threading.RLock()
        # collect_orphans: the garbage collector's other half -- an object created with owner
        # references none of which exists (its owner was deleted while a controller was still
        # writing it) is removed right after its creation. Off by default: unit tests build
        # objects with synthetic owner uids.
        self.collect_orphans = collect_orphans
        self._store: Dict[Tuple[str, str, str, str], Obj] = {}
        self._rv = itertools.count(1)
        self._watchers: List[Tuple[str, str, str, WatchCallback, Optional[str]]] = []
        self.interceptors: List[Interceptor] = []
        self.unserved_kinds: Set[str] = set(unserved_kinds or ())
        self.version = server_version
        self.events: List[Obj] = []
        self.calls: List[Tuple[str, str, str]] = []   # (verb, kind, name) audit log
        for obj in objs or []:
            self.create(obj)

    # -- internals ------------------------------------------------------------------------
    @staticmethod
    def _k(api_version: str, kind: str, namespace: str, name: str):
        return (api_version, kind, "" if kind in o.CLUSTER_SCOPED else (namespace or ""), name)

    def _intercept(self, verb: str, api_version: str, kind: str, arg: Any) -> None:
        self.calls.append((verb, kind, arg if isinstance(arg, str) else o.name(arg)))
        for fn in list(self.interceptors):
            fn(verb, api_version, kind, arg)
        if kind in self.unserved_kinds:
            raise errors.NoKindMatch(f"no matches for kind {kind} in version {api_version}")

    def _notify(self, etype: str, obj: Obj, old: Optional[Obj] = None) -> None:
        for av, kind, ns, cb, fs in list(self._watchers):
            if av == obj.get("apiVersion") and kind == obj.get("kind") and (not ns or ns == o.namespace(obj)) \
                    and o.field_selector_matches(fs, obj):
                cb(WatchEvent(etype, copy.deepcopy(obj), copy.deepcopy(old) if old else None))

    def _bump(self, obj: Obj) -> None:
        o.meta(obj)["resourceVersion"] = str(next(self._rv))

    # -- reads ----------------------------------------------------------------------------
    def get(self, api_version: str, kind: str, name: str, namespace: str = "") -> Obj:
        with self._lock:
            self._intercept("get", api_version, kind, name)
            obj = self._store.get(self._k(api_version, kind, namespace, name))
            if obj is None:
                raise errors.NotFound(f'{kind} "{name}" not found')
            return copy.deepcopy(obj)

    def list(self, api_version: str, kind: str, namespace: str = "", label_selector: Any = None,
             field_selector: Optional[str] = None) -> List[Obj]:
        with self._lock:
            self._intercept("list", api_version, kind, "")
            out = []
            for (av, k, ns, _), obj in sorted(self._store.items()):
                if av != api_version or k != kind:
                    continue
                if namespace and ns != namespace:
                    continue
                if not o.selector_matches(label_selector, o.get_labels(obj)):
                    continue
                if not o.field_selector_matches(field_selector, obj):
                    continue
                out.append(copy.deepcopy(obj))
            return out

    # -- writes ---------------------------------------------------------------------------
    def create(self, obj: Obj) -> Obj:
        obj = copy.deepcopy(obj)
        if not obj.get("apiVersion"):
            obj["apiVersion"] = o.api_version_of(obj.get("kind", ""))
        with self._lock:
            self._intercept("create", obj["apiVersion"], obj.get("kind", ""), obj)
            md = o.meta(obj)
            if not md.get("name") and md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            if not md.get("name"):
                raise errors.Invalid("metadata.name required")
            k = o.key(obj)
            if k in self._store:
                raise errors.AlreadyExists(f'{obj["kind"]} "{md["name"]}" already exists')
            md["uid"] = md.get("uid") or str(uuid.uuid4())
            md["creationTimestamp"] = md.get("creationTimestamp") or time.strftime(
                "%Y-%m-%dT%H:%M:%SZ", time.gmtime())
            md["generation"] = 1
            self._bump(obj)
            self._store[k] = obj
            out = copy.deepcopy(obj)
            refs = [r.get("uid") for r in md.get("ownerReferences") or []]
            orphan = self.collect_orphans and bool(refs) and not any(
                (x.get("metadata") or {}).get("uid") in refs for x in self._store.values())
        self._notify(ADDED, out)
        if orphan:
            try:
                self.delete(out["apiVersion"], out["kind"], md["name"], o.namespace(out))
            except errors.NotFound:
                pass
        return out

    def update(self, obj: Obj, _status: bool = False) -> Obj:
        obj = copy.deepcopy(obj)
        if not obj.get("apiVersion"):
            obj["apiVersion"] = o.api_version_of(obj.get("kind", ""))
        with self._lock:
            self._intercept("update_status" if _status else "update", obj["apiVersion"], obj["kind"], obj)
            k = o.key(obj)
            cur = self._store.get(k)
            if cur is None:
                raise errors.NotFound(f'{obj["kind"]} "{o.name(obj)}" not found')
            rv = o.meta(obj).get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise errors.Conflict(f'the object {obj["kind"]} "{o.name(obj)}" has been modified; '
                                      "please apply your changes to the latest version")
            md = o.meta(obj)
            for keep in ("uid", "creationTimestamp"):
                md[keep] = cur["metadata"].get(keep)
            if _status:
                new = copy.deepcopy(cur)
                new["status"] = obj.get("status")
            else:
                new = obj
                if obj["kind"] in STATUS_SUBRESOURCE:
                    new["status"] = copy.deepcopy(cur.get("status"))
                gen = cur["metadata"].get("generation", 1)
                if cur.get("spec") != new.get("spec"):
                    gen += 1
                md["generation"] = gen
            if new.get("status") is None:
                new.pop("status", None)
            nmd = o.meta(new)
            if nmd.get("deletionTimestamp") is None and cur["metadata"].get("deletionTimestamp"):
                nmd["deletionTimestamp"] = cur["metadata"]["deletionTimestamp"]   # immutable once set
            self._bump(new)
            out = copy.deepcopy(new)
            if nmd.get("deletionTimestamp") and not nmd.get("finalizers"):
                # the last finalizer of a terminating object is gone: the API server removes it
                self._store.pop(k, None)
                removed = [out] + self._gc(nmd["uid"])
            else:
                self._store[k] = new
                removed = None
        if removed is not None:
            for r in removed:
                self._notify(DELETED, r)
            return out
        self._notify(MODIFIED, out, cur)
        return out

    def update_status(self, obj: Obj) -> Obj:
        return self.update(obj, _status=True)

    def patch(self, api_version: str, kind: str, name: str, patch: Obj, namespace: str = "",
              patch_type: str = "merge") -> Obj:
        with self._lock:
            cur = self.get(api_version, kind, name, namespace)
            new = merge_patch(cur, patch)
            o.meta(new)["resourceVersion"] = cur["metadata"]["resourceVersion"]
            status_only = set(patch.keys()) == {"status"}
            return self.update(new, _status=status_only)

    def delete(self, api_version: str, kind: str, name: str, namespace: str = "",
               propagation: Optional[str] = None, grace_period_seconds: Optional[int] = None) -> None:
        with self._lock:
            self._intercept("delete", api_version, kind, name)
            k = self._k(api_version, kind, namespace, name)
            obj = self._store.get(k)
            if obj is None:
                raise errors.NotFound(f'{kind} "{name}" not found')
            if obj["metadata"].get("finalizers"):
                # graceful: the object stays, terminating, until its finalizers are removed
                if obj["metadata"].get("deletionTimestamp"):
                    return
                obj["metadata"]["deletionTimestamp"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
                self._bump(obj)
                out = copy.deepcopy(obj)
                mod = True
            else:
                mod = False
                self._store.pop(k, None)
        if mod:
            self._notify(MODIFIED, out)
            return
        with self._lock:
            removed = [obj]
            if propagation != "Orphan":
                removed += self._gc(obj["metadata"]["uid"])
        for r in removed:
            self._notify(DELETED, r)

    def _gc(self, uid: str) -> List[Obj]:
        gone: List[Obj] = []
        for k, obj in list(self._store.items()):
            if o.owned_by(obj, uid):
                self._store.pop(k, None)
                gone.append(obj)
                gone += self._gc(obj["metadata"]["uid"])
        return gone

    def evict(self, name: str, namespace: str, grace_period_seconds: Optional[int] = None) -> None:
        """The pods/eviction subresource: 429 when a PodDisruptionBudget selecting the pod allows no
        disruption (status.disruptionsAllowed, kept up to date by the test), else a delete."""
        with self._lock:
            self._intercept("evict", "v1", "Pod", name)
            pod = self._store.get(self._k("v1", "Pod", namespace, name))
            if pod is None:
                raise errors.NotFound(f'pods "{name}" not found')
            if not pod["metadata"].get("deletionTimestamp"):
                for (av, k, ns, _), pdb in self._store.items():
                    if k != "PodDisruptionBudget" or ns != namespace:
                        continue
                    if not o.selector_matches((pdb.get("spec") or {}).get("selector"), o.get_labels(pod)):
                        continue
                    if int((pdb.get("status") or {}).get("disruptionsAllowed", 0)) <= 0:
                        raise errors.TooManyRequests(
                            "Cannot evict pod as it would violate the pod's disruption budget.")
        self.delete("v1", "Pod", name, namespace)

    # -- discovery / misc -----------------------------------------------------------------
    def has_kind(self, api_version: str, kind: str) -> bool:
        return kind not in self.unserved_kinds

    def server_version(self) -> str:
        return self.version

    def watch(self, api_version: str, kind: str, callback: WatchCallback,
              namespace: str = "", field_selector: Optional[str] = None) -> Callable[[], None]:
        entry = (api_version, kind, namespace, callback, field_selector)
        with self._lock:
            self._watchers.append(entry)
            existing = [copy.deepcopy(v) for (av, k, ns, _), v in sorted(self._store.items())
                        if av == api_version and k == kind and (not namespace or ns == namespace)
                        and o.field_selector_matches(field_selector, v)]
        for obj in existing:
            callback(WatchEvent(ADDED, obj))

        def stop():
            with self._lock:
                if entry in self._watchers:
                    self._watchers.remove(entry)
        return stop

    def create_event(self, involved: Obj, reason: str, message: str, type_: str = "Normal") -> None:
        self.events.append({"involvedObject": {"kind": involved.get("kind"), "name": o.name(involved),
                                               "namespace": o.namespace(involved)},
                            "reason": reason, "message": message, "type": type_})

    # -- test helpers ---------------------------------------------------------------------
    def objects(self, kind: Optional[str] = None) -> List[Obj]:
        with self._lock:
            return [copy.deepcopy(v) for (_, k, _, _), v in sorted(self._store.items())
                    if kind is None or k == kind]

    def set_status(self, api_version: str, kind: str, name: str, status: Dict[str, Any],
                   namespace: str = "") -> Obj:
        cur = self.get(api_version, kind, name, namespace)
        cur["status"] = status
        return self.update_status(cur)

    def fail_on(self, verb: str, kind: str, exc: Exception, times: int = 1,
                name: Optional[str] = None) -> None:
        """Inject ``exc`` on the next ``times`` matching calls (fault injection)."""
        state = {"left": times}

        def hook(v, av, k, arg):
            nm = arg if isinstance(arg, str) else o.name(arg)
            if v == verb and k == kind and (name is None or nm == name) and state["left"] > 0:
                state["left"] -= 1
                raise exc
        self.interceptors.append(hook)
