"""Level-triggered controller: watches -> event handlers/predicates -> work queue -> reconcile.

The controller-runtime pattern the reference's two reconcilers are built on (reference:
controllers/clusterpolicy_controller.go:317-344, controllers/upgrade_controller.go:199-259),
with ``MaxConcurrentReconciles`` workers (default 1) and per-key exponential back-off.
"""

from __future__ import annotations

import logging
import threading
import time
from dataclasses import dataclass
from typing import Any, Callable, Hashable, Iterable, List, Optional, Tuple

from ..k8s.client import WatchEvent
from .workqueue import ExponentialBackoff, WorkQueue

log = logging.getLogger("amd-gpu-operator.runtime")


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0


Request = Hashable
Mapper = Callable[[WatchEvent], Iterable[Request]]
Predicate = Callable[[WatchEvent], bool]


@dataclass
class Watch:
    api_version: str
    kind: str
    mapper: Mapper
    predicate: Optional[Predicate] = None
    namespace: str = ""


class Controller:
    def __init__(self, name: str, reconcile: Callable[[Request], Result], workers: int = 1,
                 backoff: Optional[ExponentialBackoff] = None):
        self.name = name
        self.reconcile = reconcile
        self.workers = workers
        self.queue = WorkQueue(backoff or ExponentialBackoff(0.1, 3.0))
        self.watches: List[Watch] = []
        self._stops: List[Callable[[], None]] = []
        self._threads: List[threading.Thread] = []
        self._stop = threading.Event()
        self.reconciles = 0
        self.errors = 0

    def watch(self, api_version: str, kind: str, mapper: Mapper, predicate: Optional[Predicate] = None,
              namespace: str = "") -> "Controller":
        self.watches.append(Watch(api_version, kind, mapper, predicate, namespace))
        return self

    def _handler(self, w: Watch) -> Callable[[WatchEvent], None]:
        def on_event(ev: WatchEvent) -> None:
            try:
                if w.predicate is not None and not w.predicate(ev):
                    log.debug("%s: %s %s %s filtered", self.name, ev.type, w.kind, (ev.obj.get("metadata") or {}).get("name"))
                    return
                log.debug("%s: %s %s %s rv=%s", self.name, ev.type, w.kind, (ev.obj.get("metadata") or {}).get("name"),
                          (ev.obj.get("metadata") or {}).get("resourceVersion"))
                for req in w.mapper(ev):
                    self.queue.add(req)
            except Exception:  # noqa: BLE001 - a bad event must not kill the watch
                log.exception("%s: event handler failed for %s", self.name, w.kind)
        return on_event

    def start_watches(self, client) -> None:
        for w in self.watches:
            self._stops.append(client.watch(w.api_version, w.kind, self._handler(w), namespace=w.namespace))

    def process_one(self, timeout: Optional[float] = None) -> bool:
        key = self.queue.get(timeout=timeout)
        if key is None:
            return False
        try:
            self.reconciles += 1
            res = self.reconcile(key) or Result()
        except Exception as e:  # noqa: BLE001
            self.errors += 1
            delay = self.queue.add_rate_limited(key)
            log.warning("%s: reconcile %s failed (%s); retry in %.2fs", self.name, key, e, delay)
        else:
            if res.requeue_after > 0:
                self.queue.forget(key)
                self.queue.add_after(key, res.requeue_after)
            elif res.requeue:
                self.queue.add_rate_limited(key)
            else:
                self.queue.forget(key)
        finally:
            self.queue.done(key)
        return True

    def start(self, client) -> None:
        self.start_watches(client)

        def worker():
            while not self._stop.is_set():
                self.process_one(timeout=0.5)
        for i in range(self.workers):
            t = threading.Thread(target=worker, name=f"{self.name}-worker-{i}", daemon=True)
            t.start()
            self._threads.append(t)

    def stop(self) -> None:
        self._stop.set()
        for s in self._stops:
            s()
        self.queue.shutdown()
        for t in self._threads:
            t.join(timeout=2)

    def drain(self, max_items: int = 1000, include_delayed_within: float = 0.0) -> int:
        """Test helper: process queued keys synchronously until the queue is empty."""
        n = 0
        end = time.monotonic() + include_delayed_within
        while n < max_items:
            if not self.process_one(timeout=max(0.0, end - time.monotonic()) if include_delayed_within else 0.0):
                break
            n += 1
        return n


def enqueue_const(*keys: Request) -> Mapper:
    return lambda ev: keys


def enqueue_self(ev: WatchEvent) -> Tuple[Request, ...]:
    md = ev.obj.get("metadata") or {}
    return ((md.get("namespace", ""), md.get("name", "")),)
