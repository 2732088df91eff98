"""Informer cache: reads served from watch-fed local stores, writes straight to the API server.

The reference reconciles through controller-runtime's cached client (main.go:104,
``ctrl.NewManager``): every Get/List of a kind is answered from a shared informer that keeps a
local copy of all objects of that kind, fed by one LIST + WATCH, so a steady-state pass over a
500-node cluster costs no API reads at all. :class:`CachedClient` is that layer for this
framework's :class:`~gpu_operator_amd.k8s.client.Client` protocol:

* the first ``get``/``list`` of a kind starts its informer (one LIST, then the client's WATCH,
  cluster-wide); every later read of that kind is a selector match over the local store and
  returns deep copies (callers mutate what they get, as with controller-runtime);
* writes (``create``/``update``/``update_status``/``patch``/``delete``/``evict``) go to the API;
  the object a write returns is folded into the store right away (never replacing a newer
  ``resourceVersion``), so a reconcile reads its own writes without waiting for the watch;
* kinds the server does not serve (``NoKindMatch``, e.g. OpenShift kinds on plain Kubernetes)
  and kinds listed in ``uncached`` (e.g. ``Lease``, whose freshness leader election depends
  on) pass straight through.

``stats()`` counts the API reads that reached the server, which is what the scale tests assert.
"""

from __future__ import annotations

import copy
import logging
import threading
from typing import Any, Callable, Dict, Iterable, List, Optional, Set, Tuple

from ..k8s import errors
from ..k8s import objects as o
from ..k8s.client import DELETED, Obj, WatchCallback, WatchEvent

log = logging.getLogger("amd-gpu-operator.cache")

Key = Tuple[str, str]          # (apiVersion, kind)


def _rv(obj: Obj) -> Optional[int]:
    try:
        return int((obj.get("metadata") or {}).get("resourceVersion", ""))
    except (TypeError, ValueError):
        return None


class _Informer:
    def __init__(self, client, api_version: str, kind: str):
        self.api_version, self.kind = api_version, kind
        self.store: Dict[Tuple[str, str], Obj] = {}
        self.lock = threading.RLock()
        self.handlers: List[WatchCallback] = []
        for obj in client.list(api_version, kind):          # initial sync (the only LIST)
            self._upsert(obj)
        self.stop = client.watch(api_version, kind, self._on_event)

    @staticmethod
    def _k(obj: Obj) -> Tuple[str, str]:
        return (o.namespace(obj), o.name(obj))

    def _upsert(self, obj: Obj) -> bool:
        obj.setdefault("apiVersion", self.api_version)
        obj.setdefault("kind", self.kind)
        k = self._k(obj)
        with self.lock:
            cur = self.store.get(k)
            if cur is not None:
                a, b = _rv(cur), _rv(obj)
                if a is not None and b is not None and b < a:
                    return False                               # an older event after our write
            self.store[k] = copy.deepcopy(obj)
            return True

    def _on_event(self, ev: WatchEvent) -> None:
        if ev.type == DELETED:
            with self.lock:
                cur = self.store.get(self._k(ev.obj))
                if cur is not None and cur["metadata"].get("uid") == (ev.obj.get("metadata") or {}).get("uid"):
                    self.store.pop(self._k(ev.obj), None)
        else:
            self._upsert(ev.obj)
        for h in list(self.handlers):
            h(ev)

    def get(self, name: str, namespace: str) -> Obj:
        ns = "" if self.kind in o.CLUSTER_SCOPED else (namespace or "")
        with self.lock:
            obj = self.store.get((ns, name))
            if obj is None:
                raise errors.NotFound(f'{self.kind} "{name}" not found')
            return copy.deepcopy(obj)

    def list(self, namespace: str, label_selector: Any, field_selector: Optional[str]) -> List[Obj]:
        with self.lock:
            items = sorted(self.store.items())
            out = []
            for (ns, _), obj in items:
                if namespace and ns != namespace:
                    continue
                if not o.selector_matches(label_selector, o.get_labels(obj)):
                    continue
                if not o.field_selector_matches(field_selector, obj):
                    continue
                out.append(copy.deepcopy(obj))
            return out


class CachedClient:
    """A :class:`Client` whose reads come from informers (see module doc)."""

    DEFAULT_UNCACHED = frozenset({"Lease", "Event", "Eviction"})

    def __init__(self, client, uncached: Iterable[str] = DEFAULT_UNCACHED):
        self.client = client
        self.uncached: Set[str] = set(uncached)
        self._informers: Dict[Key, _Informer] = {}
        self._unservable: Set[Key] = set()
        self._lock = threading.Lock()
        self._stats = {"get": 0, "list": 0}                   # reads that reached the API server

    # -- informers ---------------------------------------------------------------------------
    def _informer(self, api_version: str, kind: str) -> Optional[_Informer]:
        key = (api_version, kind)
        if kind in self.uncached or key in self._unservable:
            return None
        with self._lock:
            inf = self._informers.get(key)
            if inf is None:
                try:
                    self._stats["list"] += 1
                    inf = _Informer(self.client, api_version, kind)
                except errors.NoKindMatch:
                    self._unservable.add(key)
                    return None
                except errors.ApiError as e:
                    if e.status in (403, 404, 405):        # not listable/watchable: read through
                        self._unservable.add(key)
                        return None
                    raise
                self._informers[key] = inf
                log.info("informer started for %s %s (%d objects)", api_version, kind, len(inf.store))
            return inf

    def cached_kinds(self) -> List[Key]:
        return sorted(self._informers)

    def stats(self) -> Dict[str, int]:
        return dict(self._stats)

    def reset_stats(self) -> None:
        self._stats = {"get": 0, "list": 0}

    def stop(self) -> None:
        for inf in self._informers.values():
            inf.stop()

    # -- reads ------------------------------------------------------------------------------
    def get(self, api_version: str, kind: str, name: str, namespace: str = "") -> Obj:
        inf = self._informer(api_version, kind)
        if inf is None:
            self._stats["get"] += 1
            return self.client.get(api_version, kind, name, namespace)
        return inf.get(name, namespace)

    def list(self, api_version: str, kind: str, namespace: str = "", label_selector: Any = None,
             field_selector: Optional[str] = None) -> List[Obj]:
        inf = self._informer(api_version, kind)
        if inf is None:
            self._stats["list"] += 1
            return self.client.list(api_version, kind, namespace, label_selector=label_selector,
                                    field_selector=field_selector)
        return inf.list(namespace, label_selector, field_selector)

    # -- writes (write-through into the store) -------------------------------------------------
    def _fold(self, obj: Obj) -> Obj:
        inf = self._informers.get((obj.get("apiVersion", ""), obj.get("kind", "")))
        if inf is not None and obj.get("metadata"):
            inf._upsert(copy.deepcopy(obj))
        return obj

    def create(self, obj: Obj) -> Obj:
        return self._fold(self.client.create(obj))

    def update(self, obj: Obj) -> Obj:
        return self._fold(self.client.update(obj))

    def update_status(self, obj: Obj) -> Obj:
        return self._fold(self.client.update_status(obj))

    def patch(self, api_version: str, kind: str, name: str, patch: Obj, namespace: str = "",
              patch_type: str = "merge") -> Obj:
        return self._fold(self.client.patch(api_version, kind, name, patch, namespace, patch_type=patch_type))

    def delete(self, api_version: str, kind: str, name: str, namespace: str = "",
               propagation: Optional[str] = None, grace_period_seconds: Optional[int] = None) -> None:
        self.client.delete(api_version, kind, name, namespace, propagation=propagation,
                           grace_period_seconds=grace_period_seconds)

    def evict(self, name: str, namespace: str, grace_period_seconds: Optional[int] = None) -> None:
        self.client.evict(name, namespace, grace_period_seconds=grace_period_seconds)

    # -- pass-through ------------------------------------------------------------------------
    def has_kind(self, api_version: str, kind: str) -> bool:
        return self.client.has_kind(api_version, kind)

    def server_version(self) -> str:
        return self.client.server_version()

    def watch(self, api_version: str, kind: str, callback: WatchCallback, namespace: str = "",
              field_selector: Optional[str] = None) -> Callable[[], None]:
        """Controllers' event sources share the informer's stream (one WATCH per kind)."""
        inf = self._informer(api_version, kind)
        if inf is None:
            return self.client.watch(api_version, kind, callback, namespace, field_selector=field_selector)

        def filtered(ev: WatchEvent) -> None:
            if (not namespace or o.namespace(ev.obj) == namespace) and o.field_selector_matches(field_selector, ev.obj):
                callback(ev)
        for obj in inf.list(namespace, None, field_selector):
            callback(WatchEvent("ADDED", obj))
        inf.handlers.append(filtered)

        def stop():
            if filtered in inf.handlers:
                inf.handlers.remove(filtered)
        return stop

    def create_event(self, involved: Obj, reason: str, message: str, type_: str = "Normal") -> None:
        self.client.create_event(involved, reason, message, type_)

    def __getattr__(self, name: str):
        # test helpers of FakeClient (objects, set_status, fail_on, calls, events, ...)
        return getattr(self.client, name)
