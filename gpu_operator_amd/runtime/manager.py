"""Process manager: metrics endpoint, health/ready probes, optional pprof-style debug endpoint,
leader election and controller lifecycle (reference: main.go:60-159; metrics :8080,
healthz/readyz :8081)."""

from __future__ import annotations

import logging
import sys
import threading
import traceback
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Tuple

from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.exposition import CONTENT_TYPE_LATEST

from .controller import Controller
from .leaderelection import LeaderElector

log = logging.getLogger("amd-gpu-operator.manager")


def _parse_addr(addr: str, default_port: int) -> Tuple[str, int]:
    if not addr or addr == "0":
        return "", -1
    host, _, port = addr.rpartition(":")
    return host or "0.0.0.0", int(port or default_port)


_CLIENT_GONE = (ConnectionResetError, BrokenPipeError, ConnectionAbortedError, TimeoutError)


class QuietHTTPServer(ThreadingHTTPServer):
    """A ThreadingHTTPServer whose per-request errors go to logging: a client that disconnects
    mid-response (an aborted Prometheus scrape, a probe timing out) is routine and logged at
    debug level, anything else once with its traceback at error level -- socketserver's default
    prints every one as a traceback on stderr."""

    daemon_threads = True

    def handle_error(self, request, client_address):  # noqa: D401 - socketserver hook
        exc = sys.exc_info()[1]
        if isinstance(exc, _CLIENT_GONE):
            log.debug("client %s went away: %s", client_address, exc)
            return
        log.error("error serving %s", client_address, exc_info=True)


class _Server:
    def __init__(self, addr: Tuple[str, int], routes: Dict[str, Callable[[], Tuple[int, str, bytes]]]):
        class Handler(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                fn = routes.get(self.path.split("?")[0])
                if fn is None:
                    self.send_response(404)
                    self.end_headers()
                    return
                code, ctype, body = fn()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):  # quiet
                pass

        self.httpd = QuietHTTPServer(addr, Handler)
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    def start(self):
        self.thread.start()

    def stop(self):
        self.httpd.shutdown()


class Manager:
    def __init__(self, client, namespace: str, registry: Optional[CollectorRegistry] = None,
                 metrics_addr: str = ":8080", probe_addr: str = ":8081", leader_elect: bool = False,
                 lease_duration: float = 15.0, renew_deadline: float = 10.0, debug_addr: str = ""):
        self.client = client
        self.namespace = namespace
        self.registry = registry or CollectorRegistry()
        self.controllers: List[Controller] = []
        self.health_checks: Dict[str, Callable[[], bool]] = {"ping": lambda: True}
        self.ready_checks: Dict[str, Callable[[], bool]] = {"ping": lambda: True}
        self.metrics_addr = _parse_addr(metrics_addr, 8080)
        self.probe_addr = _parse_addr(probe_addr, 8081)
        self.debug_addr = _parse_addr(debug_addr, 6060) if debug_addr else ("", -1)
        self.leader_elect = leader_elect
        self.elector = LeaderElector(client, namespace, lease_duration=lease_duration,
                                     renew_deadline=renew_deadline) if leader_elect else None
        self.servers: List[_Server] = []
        self._stopped = threading.Event()

    def add(self, c: Controller) -> None:
        self.controllers.append(c)

    def _check(self, checks) -> Tuple[int, str, bytes]:
        failed = [k for k, f in checks.items() if not _safe(f)]
        if failed:
            return 500, "text/plain", ("failed: " + ",".join(failed)).encode()
        return 200, "text/plain", b"ok"

    def _start_servers(self) -> None:
        if self.metrics_addr[1] >= 0:
            s = _Server(self.metrics_addr, {"/metrics": lambda: (200, CONTENT_TYPE_LATEST,
                                                                 generate_latest(self.registry))})
            s.start()
            self.servers.append(s)
            self.metrics_addr = (self.metrics_addr[0], s.port)
        if self.probe_addr[1] >= 0:
            s = _Server(self.probe_addr, {"/healthz": lambda: self._check(self.health_checks),
                                          "/readyz": lambda: self._check(self.ready_checks)})
            s.start()
            self.servers.append(s)
            self.probe_addr = (self.probe_addr[0], s.port)
        if self.debug_addr[1] >= 0:
            s = _Server(self.debug_addr, {"/debug/threads": _thread_dump})
            s.start()
            self.servers.append(s)

    def start(self, block: bool = True) -> None:
        self._start_servers()

        def run_controllers():
            for c in self.controllers:
                c.start(self.client)
            log.info("started %d controllers", len(self.controllers))

        if self.elector is not None:
            self.elector.run(on_started=run_controllers, on_stopped=self._lost_leadership)
        else:
            run_controllers()
        if block:
            self._stopped.wait()

    def _lost_leadership(self) -> None:
        # like controller-runtime: exit and let the Deployment restart us as a candidate
        log.error("leader election lost; exiting")
        self.stop()
        sys.exit(1)

    def stop(self) -> None:
        for c in self.controllers:
            c.stop()
        for s in self.servers:
            s.stop()
        if self.elector:
            self.elector.stop()
        self._stopped.set()


def _safe(f) -> bool:
    try:
        return bool(f())
    except Exception:  # noqa: BLE001
        return False


def _thread_dump() -> Tuple[int, str, bytes]:
    frames = sys._current_frames()  # noqa: SLF001 - debug endpoint
    out = []
    for th in threading.enumerate():
        out.append(f"--- {th.name} ---")
        f = frames.get(th.ident)
        if f is not None:
            out.extend(traceback.format_stack(f))
    return 200, "text/plain", "\n".join(out).encode()
