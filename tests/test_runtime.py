"""Work queue, controller loop and leader election."""

import datetime as dt
import threading
import time

from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.runtime.controller import Controller, Result
from gpu_operator_amd.runtime.leaderelection import LeaderElector
from gpu_operator_amd.runtime.workqueue import ExponentialBackoff, WorkQueue


def test_queue_dedupes_and_defers_readd_while_processing():
    q = WorkQueue()
    q.add("a")
    q.add("a")
    q.add("b")
    assert len(q) == 2
    k = q.get(timeout=0)
    assert k == "a"
    q.add("a")                          # re-added while processing: not handed out twice
    assert q.get(timeout=0) == "b"
    assert q.get(timeout=0) is None
    q.done("a")
    assert q.get(timeout=0) == "a"


def test_add_after_and_ordering():
    t = [0.0]
    q = WorkQueue(clock=lambda: t[0])
    q.add_after("late", 5)
    q.add_after("early", 1)
    assert q.get(timeout=0) is None
    t[0] = 2
    assert q.get(timeout=0) == "early"
    t[0] = 6
    assert q.get(timeout=0) == "late"


def test_exponential_backoff_caps_and_forgets():
    b = ExponentialBackoff(0.1, 3.0)
    ds = [b.when("k") for _ in range(8)]
    assert ds[:4] == [0.1, 0.2, 0.4, 0.8] and ds[-1] == 3.0
    b.forget("k")
    assert b.when("k") == 0.1


def test_controller_requeue_after_error_and_success():
    calls = []

    def rec(key):
        calls.append(key)
        if len(calls) == 1:
            raise RuntimeError("transient")
        return Result(requeue_after=0)
    c = Controller("t", rec, backoff=ExponentialBackoff(0.01, 0.02))
    c.queue.add("x")
    c.process_one(timeout=0)
    assert c.errors == 1
    c.process_one(timeout=1.0)             # retried after back-off
    assert calls == ["x", "x"] and c.queue.rate_limiter.failures("x") == 0


def test_controller_threads_process_watch_events():
    client = FakeClient()
    seen = []
    ev = threading.Event()

    def rec(key):
        seen.append(key)
        ev.set()
        return Result()
    c = Controller("t", rec)
    c.watch("v1", "ConfigMap", lambda e: [e.obj["metadata"]["name"]])
    c.start(client)
    client.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm", "namespace": "n"}})
    assert ev.wait(5)
    c.stop()
    assert seen == ["cm"]


def test_leader_election_single_holder_and_takeover():
    now = [dt.datetime(2026, 1, 1, tzinfo=dt.timezone.utc)]
    clock = lambda: now[0]  # noqa: E731
    c = FakeClient()
    a = LeaderElector(c, "ns", identity="a", lease_duration=15, clock=clock)
    b = LeaderElector(c, "ns", identity="b", lease_duration=15, clock=clock)
    assert a.try_acquire_or_renew()
    assert not b.try_acquire_or_renew()
    now[0] += dt.timedelta(seconds=10)
    assert a.try_acquire_or_renew()          # renew
    now[0] += dt.timedelta(seconds=10)
    assert not b.try_acquire_or_renew()      # renewed 10 s ago: still valid
    now[0] += dt.timedelta(seconds=20)
    assert b.try_acquire_or_renew()          # a stopped renewing: b takes over
    lease = c.get("coordination.k8s.io/v1", "Lease", "53822513.amd.com", "ns")
    assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] == 1
    assert not a.try_acquire_or_renew()


def test_leader_election_run_invokes_callback():
    c = FakeClient()
    e = LeaderElector(c, "ns", identity="x", retry_period=0.01)
    started = threading.Event()
    e.run(on_started=started.set, on_stopped=lambda: None)
    assert started.is_set() and e.is_leader.is_set()
    e.stop()
    time.sleep(0.05)


def test_aborted_scrape_logs_no_traceback(capfd, caplog):
    """a client that resets the connection mid-response (an aborted
    Prometheus scrape) is logged at debug level; socketserver's default handle_error printed a
    traceback on stderr for every one."""
    import logging
    import socket
    import struct
    import time as _t
    from gpu_operator_amd.runtime.manager import _Server
    body = b"x" * (8 << 20)
    srv = _Server(("127.0.0.1", 0), {"/metrics": lambda: (200, "text/plain", body)})
    srv.start()
    try:
        with caplog.at_level(logging.DEBUG, logger="amd-gpu-operator.manager"):
            for _ in range(3):
                s = socket.create_connection(("127.0.0.1", srv.port))
                s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
                s.recv(1024)                                   # the response has started
                s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
                s.close()                                      # RST mid-body
            s = socket.create_connection(("127.0.0.1", srv.port))
            s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
            s.close()                                          # RST before the request line
            _t.sleep(0.5)
    finally:
        srv.stop()
    err = capfd.readouterr().err
    assert "Traceback" not in err and "ConnectionResetError" not in err and "BrokenPipeError" not in err, err
    assert any("went away" in r.getMessage() for r in caplog.records)
