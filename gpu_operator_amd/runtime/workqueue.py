"""Rate-limited, de-duplicating work queue with delayed adds (client-go workqueue semantics).

* a key is queued at most once; a key re-added while it is being processed is re-queued when
  ``done`` is called (so one key is never reconciled by two workers at once);
* ``add_after`` schedules a delayed add (RequeueAfter);
* ``add_rate_limited`` backs off per key exponentially, like the reference's
  ``ItemExponentialFailureRateLimiter(100ms, 3s)`` (reference:
  controllers/clusterpolicy_controller.go:45-48,319); ``forget`` resets a key's back-off.
"""

from __future__ import annotations

import heapq
import itertools
import threading
import time
from collections import deque
from typing import Dict, Hashable, List, Optional, Set, Tuple


class ExponentialBackoff:
    def __init__(self, base: float = 0.1, cap: float = 3.0):
        self.base = base
        self.cap = cap
        self._failures: Dict[Hashable, int] = {}
        self._lock = threading.Lock()

    def when(self, key: Hashable) -> float:
        with self._lock:
            n = self._failures.get(key, 0)
            self._failures[key] = n + 1
        return min(self.cap, self.base * (2 ** n))

    def forget(self, key: Hashable) -> None:
        with self._lock:
            self._failures.pop(key, None)

    def failures(self, key: Hashable) -> int:
        with self._lock:
            return self._failures.get(key, 0)


class WorkQueue:
    def __init__(self, rate_limiter: Optional[ExponentialBackoff] = None, clock=time.monotonic):
        self._cond = threading.Condition()
        self._queue: deque = deque()
        self._dirty: Set[Hashable] = set()
        self._processing: Set[Hashable] = set()
        self._delayed: List[Tuple[float, int, Hashable]] = []
        self._seq = itertools.count()
        self._shutdown = False
        self.rate_limiter = rate_limiter or ExponentialBackoff()
        self.clock = clock

    # -- adds -----------------------------------------------------------------------------
    def add(self, key: Hashable) -> None:
        with self._cond:
            if self._shutdown or key in self._dirty:
                return
            self._dirty.add(key)
            if key in self._processing:
                return
            self._queue.append(key)
            self._cond.notify()

    def add_after(self, key: Hashable, delay: float) -> None:
        if delay <= 0:
            self.add(key)
            return
        with self._cond:
            if self._shutdown:
                return
            heapq.heappush(self._delayed, (self.clock() + delay, next(self._seq), key))
            self._cond.notify()

    def add_rate_limited(self, key: Hashable) -> float:
        d = self.rate_limiter.when(key)
        self.add_after(key, d)
        return d

    def forget(self, key: Hashable) -> None:
        self.rate_limiter.forget(key)

    # -- consumption ----------------------------------------------------------------------
    def _promote_due(self) -> Optional[float]:
        now = self.clock()
        while self._delayed and self._delayed[0][0] <= now:
            _, _, key = heapq.heappop(self._delayed)
            if key not in self._dirty:
                self._dirty.add(key)
                if key not in self._processing:
                    self._queue.append(key)
        return self._delayed[0][0] - now if self._delayed else None

    def get(self, timeout: Optional[float] = None) -> Optional[Hashable]:
        """Next key, or None on shutdown/timeout."""
        deadline = None if timeout is None else self.clock() + timeout
        with self._cond:
            while True:
                wait = self._promote_due()
                if self._queue:
                    key = self._queue.popleft()
                    self._processing.add(key)
                    self._dirty.discard(key)
                    return key
                if self._shutdown:
                    return None
                if deadline is not None:
                    remaining = deadline - self.clock()
                    if remaining <= 0:
                        return None
                    wait = remaining if wait is None else min(wait, remaining)
                self._cond.wait(wait)

    def done(self, key: Hashable) -> None:
        with self._cond:
            self._processing.discard(key)
            if key in self._dirty:
                self._queue.append(key)
                self._cond.notify()

    def shutdown(self) -> None:
        with self._cond:
            self._shutdown = True
            self._cond.notify_all()

    # -- introspection --------------------------------------------------------------------
    def __len__(self) -> int:
        with self._cond:
            return len(self._queue)

    def pending_delayed(self) -> List[Tuple[float, Hashable]]:
        with self._cond:
            return sorted((t - self.clock(), k) for t, _, k in self._delayed)
