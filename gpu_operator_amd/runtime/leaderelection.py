"""Lease-based leader election (coordination.k8s.io/v1), as used by the reference manager
(reference: main.go:88-102, ID ``53822513.nvidia.com``; ours ``53822513.amd.com``).

The holder renews every ``retry_period``; it gives up leadership if it could not renew
within ``renew_deadline``; a candidate takes over a lease not renewed for ``lease_duration``.
"""

from __future__ import annotations

import datetime as dt
import logging
import socket
import threading
import time
import uuid
from typing import Callable, Optional

from ..k8s import errors

log = logging.getLogger("amd-gpu-operator.leader")

LEASE_API = "coordination.k8s.io/v1"


def _now() -> dt.datetime:
    return dt.datetime.now(dt.timezone.utc)


def _fmt(t: dt.datetime) -> str:
    return t.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _parse(s: Optional[str]) -> Optional[dt.datetime]:
    if not s:
        return None
    for f in ("%Y-%m-%dT%H:%M:%S.%fZ", "%Y-%m-%dT%H:%M:%SZ"):
        try:
            return dt.datetime.strptime(s, f).replace(tzinfo=dt.timezone.utc)
        except ValueError:
            continue
    return None


class LeaderElector:
    def __init__(self, client, namespace: str, name: str = "53822513.amd.com",
                 identity: Optional[str] = None, lease_duration: float = 15.0,
                 renew_deadline: float = 10.0, retry_period: float = 2.0, clock=_now):
        self.client = client
        self.namespace = namespace
        self.name = name
        self.identity = identity or f"{socket.gethostname()}_{uuid.uuid4().hex[:8]}"
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.clock = clock
        self.is_leader = threading.Event()
        self._stop = threading.Event()

    def try_acquire_or_renew(self) -> bool:
        now = self.clock()
        try:
            lease = self.client.get(LEASE_API, "Lease", self.name, self.namespace)
        except errors.NotFound:
            lease = {"apiVersion": LEASE_API, "kind": "Lease",
                     "metadata": {"name": self.name, "namespace": self.namespace},
                     "spec": {"holderIdentity": self.identity,
                              "leaseDurationSeconds": int(self.lease_duration),
                              "acquireTime": _fmt(now), "renewTime": _fmt(now), "leaseTransitions": 0}}
            try:
                self.client.create(lease)
                return True
            except errors.AlreadyExists:
                return False
        spec = lease.setdefault("spec", {})
        holder = spec.get("holderIdentity")
        renew = _parse(spec.get("renewTime"))
        dur = spec.get("leaseDurationSeconds") or self.lease_duration
        expired = renew is None or (now - renew).total_seconds() > dur
        if holder and holder != self.identity and not expired:
            return False
        if holder != self.identity:
            spec["leaseTransitions"] = int(spec.get("leaseTransitions") or 0) + 1
            spec["acquireTime"] = _fmt(now)
        spec["holderIdentity"] = self.identity
        spec["renewTime"] = _fmt(now)
        spec["leaseDurationSeconds"] = int(self.lease_duration)
        try:
            self.client.update(lease)   # optimistic concurrency: resourceVersion guards races
            return True
        except errors.Conflict:
            return False

    def run(self, on_started: Callable[[], None], on_stopped: Callable[[], None]) -> None:
        """Block until leadership is acquired, then renew in the background."""
        while not self._stop.is_set():
            if self.try_acquire_or_renew():
                break
            self._stop.wait(self.retry_period)
        if self._stop.is_set():
            return
        log.info("acquired lease %s/%s as %s", self.namespace, self.name, self.identity)
        self.is_leader.set()
        on_started()

        def renew_loop():
            last_ok = time.monotonic()
            while not self._stop.is_set():
                self._stop.wait(self.retry_period)
                try:
                    ok = self.try_acquire_or_renew()
                except errors.ApiError as e:
                    log.warning("lease renew failed: %s", e)
                    ok = False
                if ok:
                    last_ok = time.monotonic()
                elif time.monotonic() - last_ok > self.renew_deadline:
                    log.error("lost leadership of %s", self.name)
                    self.is_leader.clear()
                    on_stopped()
                    return
        threading.Thread(target=renew_loop, name="lease-renew", daemon=True).start()

    def stop(self) -> None:
        self._stop.set()
