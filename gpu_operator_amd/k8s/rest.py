"""Kubernetes API client over HTTPS, in-cluster or from a kubeconfig.

Implements the :class:`~gpu_operator_amd.k8s.client.Client` protocol: discovery-based
kind->resource mapping, CRUD, status subresource, merge patches, the pods/eviction
subresource, events and list+watch streams with resourceVersion resume.

The transport is the standard library's ``http.client`` with one keep-alive connection per
thread (a watch stream gets its own): every node agent and validator component builds this
client at start-up, and importing ``requests`` alone cost ~0.1 s of interpreter start per
process on the node bring-up's critical path.
"""

from __future__ import annotations

import base64
import http.client
import json
import logging
import os
import socket
import ssl
import tempfile
import threading
import time
import urllib.parse
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple


from . import errors
from . import objects as o
from .client import ADDED, DELETED, MODIFIED, Obj, WatchCallback, WatchEvent

log = logging.getLogger(__name__)

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class Config:
    def __init__(self, host: str, token: Optional[str] = None, ca_file: Optional[str] = None,
                 cert_file: Optional[str] = None, key_file: Optional[str] = None,
                 verify: bool = True, token_file: Optional[str] = None):
        self.host = host.rstrip("/")
        self.token = token
        self.token_file = token_file
        self.ca_file = ca_file
        self.cert_file = cert_file
        self.key_file = key_file
        self.verify = verify

    def bearer(self) -> Optional[str]:
        if self.token_file and os.path.exists(self.token_file):
            with open(self.token_file) as f:   # projected tokens rotate: re-read
                return f.read().strip()
        return self.token

    @classmethod
    def in_cluster(cls) -> "Config":
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        return cls(f"https://{host}:{port}", ca_file=f"{SA_DIR}/ca.crt", token_file=f"{SA_DIR}/token")

    @classmethod
    def from_kubeconfig(cls, path: Optional[str] = None, context: Optional[str] = None) -> "Config":
        import yaml            # in-cluster agents never parse a kubeconfig
        path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
        with open(path) as f:
            kc = yaml.safe_load(f)
        ctx_name = context or kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in kc.get("users", []) if u["name"] == ctx.get("user")), {})

        def materialise(data_key: str, file_key: str, src: Dict[str, Any]) -> Optional[str]:
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="kc-")
                with os.fdopen(fd, "wb") as fh:
                    fh.write(base64.b64decode(src[data_key]))
                return p
            return None

        return cls(cluster["server"], token=user.get("token"),
                   ca_file=materialise("certificate-authority-data", "certificate-authority", cluster),
                   cert_file=materialise("client-certificate-data", "client-certificate", user),
                   key_file=materialise("client-key-data", "client-key", user),
                   verify=not cluster.get("insecure-skip-tls-verify", False))

    @classmethod
    def auto(cls) -> "Config":
        if os.environ.get("KUBERNETES_SERVICE_HOST") and os.path.exists(f"{SA_DIR}/token"):
            return cls.in_cluster()
        return cls.from_kubeconfig()


class Response:
    """What the client reads back: status, body (or, streamed, the open response)."""

    def __init__(self, status: int, body: bytes = b"", stream: Optional[http.client.HTTPResponse] = None,
                 conn: Optional[http.client.HTTPConnection] = None):
        self.status_code = status
        self.content = body
        self._stream, self._conn = stream, conn

    @property
    def text(self) -> str:
        return self.content.decode("utf-8", errors="replace")

    def json(self) -> Any:
        return json.loads(self.content)

    def iter_lines(self) -> Iterator[bytes]:
        """Lines of a streamed (chunked) response as they arrive; closes the connection at the end."""
        try:
            while True:
                line = self._stream.readline()
                if not line:
                    return
                yield line.rstrip(b"\r\n")
        finally:
            self.close()

    def close(self) -> None:
        if self._conn is not None:
            self._conn.close()
            self._conn = None


_IDEMPOTENT = frozenset({"GET", "HEAD", "PUT", "DELETE", "OPTIONS"})
# merge patches set fields to values: applying one twice gives the same object (a JSON patch's "add" to a
# list does not), so a merge PATCH may be re-sent after a dropped kept-alive connection
_MERGE_PATCH_TYPES = frozenset({"application/merge-patch+json", "application/strategic-merge-patch+json",
                                "application/apply-patch+yaml"})
_KEEPALIVE_TRUST_S = 5.0    # a kept-alive connection idle longer than this is not reused for POST/PATCH


class _Transport:
    """HTTP(S) to one API server: a keep-alive connection per thread, TLS from the config (CA,
    client certificate, or no verification when the kubeconfig says insecure-skip-tls-verify)."""

    def __init__(self, cfg: "Config"):
        u = urllib.parse.urlsplit(cfg.host)
        self.https = u.scheme == "https"
        self.host, self.port = u.hostname or "localhost", u.port or (443 if self.https else 80)
        self.prefix = u.path.rstrip("/")
        self.ctx: Optional[ssl.SSLContext] = None
        if self.https:
            if cfg.verify:
                self.ctx = ssl.create_default_context(cafile=cfg.ca_file) if cfg.ca_file else \
                    ssl.create_default_context()
            else:
                self.ctx = ssl._create_unverified_context()   # noqa: S323 - the kubeconfig asked for it
            if cfg.cert_file:
                self.ctx.load_cert_chain(cfg.cert_file, cfg.key_file)
        self._local = threading.local()

    def _new(self, timeout: float) -> http.client.HTTPConnection:
        if self.https:
            return http.client.HTTPSConnection(self.host, self.port, timeout=timeout, context=self.ctx)
        return http.client.HTTPConnection(self.host, self.port, timeout=timeout)

    def request(self, method: str, path: str, body: Optional[bytes], headers: Dict[str, str], timeout: float,
                stream: bool = False) -> Response:
        path = self.prefix + path
        if stream:                                   # a watch: its own connection, closed after
            conn = self._new(timeout)
            conn.request(method, path, body=body, headers=headers)
            r = conn.getresponse()
            if r.status >= 400:
                data = r.read()
                conn.close()
                return Response(r.status, data)
            return Response(r.status, stream=r, conn=conn)
        ctype = next((v for k, v in headers.items() if k.lower() == "content-type"), "").split(";")[0].strip()
        idempotent = method in _IDEMPOTENT or (method == "PATCH" and ctype in _MERGE_PATCH_TYPES)
        for attempt in (0, 1):
            conn = getattr(self._local, "conn", None)
            if conn is not None and not idempotent and (
                    method == "POST" or time.monotonic() - getattr(self._local, "last", 0.0) > _KEEPALIVE_TRUST_S):
                # a POST (or a JSON patch) is never sent twice: rather than risk it on a kept-alive
                # connection the server -- or a proxy with a shorter idle timeout than ours -- may have
                # closed, a POST always goes out on a fresh connection, a JSON patch when idle
                conn.close()
                conn = self._local.conn = None
            fresh = conn is None
            if fresh:
                conn = self._local.conn = self._new(timeout)
            conn.timeout = timeout
            if conn.sock is not None:
                conn.sock.settimeout(timeout)
            try:
                conn.request(method, path, body=body, headers=headers)
                r = conn.getresponse()
                data = r.read()
                self._local.last = time.monotonic()
                if r.will_close:
                    conn.close()
                    self._local.conn = None
                return Response(r.status, data)
            except (http.client.HTTPException, OSError) as e:
                conn.close()
                self._local.conn = None
                # retry once, on a new connection, only what a server that closed an idle kept-alive
                # connection produces (no response byte ever came back) -- never a timeout (the request
                # may have been applied), never a non-idempotent request
                stale = isinstance(e, (http.client.RemoteDisconnected, ConnectionResetError, BrokenPipeError,
                                       ConnectionAbortedError)) and not isinstance(e, socket.timeout)
                if fresh or attempt == 1 or not stale or not idempotent:
                    raise
        raise RuntimeError("unreachable")


class RestClient:
    def __init__(self, config: Optional[Config] = None, timeout: float = 30.0):
        self.cfg = config or Config.auto()
        self.timeout = timeout
        self._http = _Transport(self.cfg)
        self._resources: Dict[str, Dict[str, Tuple[str, bool]]] = {}
        self._lock = threading.Lock()

    # -- plumbing -------------------------------------------------------------------------
    def _headers(self, content_type: str = "application/json") -> Dict[str, str]:
        h = {"Accept": "application/json", "Content-Type": content_type}
        tok = self.cfg.bearer()
        if tok:
            h["Authorization"] = f"Bearer {tok}"
        return h

    def _request(self, method: str, path: str, body: Any = None, params: Optional[Dict[str, Any]] = None,
                 content_type: str = "application/json", stream: bool = False, timeout=None) -> Response:
        if params:
            path += "?" + urllib.parse.urlencode(params)
        data = json.dumps(body).encode() if body is not None else None
        to = timeout if timeout is not None else self.timeout
        if isinstance(to, tuple):                     # (connect, read): one socket timeout, the read one
            to = to[-1]
        r = self._http.request(method, path, data, self._headers(content_type), to, stream=stream)
        if r.status_code >= 400:
            try:
                st = r.json()
                msg, reason = st.get("message", r.text), st.get("reason", "")
            except ValueError:
                msg, reason = r.text, ""
            raise errors.from_status(r.status_code, msg, reason)
        return r

    def _discover(self, api_version: str) -> Dict[str, Tuple[str, bool]]:
        with self._lock:
            if api_version in self._resources:
                return self._resources[api_version]
        path = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
        try:
            res = self._request("GET", path).json()
        except errors.NotFound:
            res = {"resources": []}
        m = {r["kind"]: (r["name"], r["namespaced"]) for r in res.get("resources", []) if "/" not in r["name"]}
        with self._lock:
            self._resources[api_version] = m
        return m

    def _path(self, api_version: str, kind: str, namespace: str = "", name: str = "",
              sub: str = "") -> str:
        res = self._discover(api_version).get(kind)
        if res is None:
            raise errors.NoKindMatch(f"no matches for kind {kind} in version {api_version}")
        plural, namespaced = res
        base = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
        p = base
        if namespaced and namespace:
            p += f"/namespaces/{namespace}"
        p += f"/{plural}"
        if name:
            p += f"/{name}"
        if sub:
            p += f"/{sub}"
        return p

    # -- Client protocol ------------------------------------------------------------------
    def get(self, api_version: str, kind: str, name: str, namespace: str = "") -> Obj:
        return self._request("GET", self._path(api_version, kind, namespace, name)).json()

    def list(self, api_version: str, kind: str, namespace: str = "", label_selector: Any = None,
             field_selector: Optional[str] = None) -> List[Obj]:
        params: Dict[str, Any] = {}
        if isinstance(label_selector, dict):
            label_selector = ",".join(f"{k}={v}" for k, v in label_selector.items())
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        items: List[Obj] = []
        while True:
            body = self._request("GET", self._path(api_version, kind, namespace), params=params).json()
            for it in body.get("items", []):
                it.setdefault("apiVersion", api_version)
                it.setdefault("kind", kind)
                items.append(it)
            cont = (body.get("metadata") or {}).get("continue")
            if not cont:
                return items
            params["continue"] = cont

    def create(self, obj: Obj) -> Obj:
        return self._request("POST", self._path(obj["apiVersion"], obj["kind"], o.namespace(obj)),
                             body=obj).json()

    def update(self, obj: Obj) -> Obj:
        return self._request("PUT", self._path(obj["apiVersion"], obj["kind"], o.namespace(obj), o.name(obj)),
                             body=obj).json()

    def update_status(self, obj: Obj) -> Obj:
        return self._request("PUT", self._path(obj["apiVersion"], obj["kind"], o.namespace(obj), o.name(obj),
                                               "status"), body=obj).json()

    def patch(self, api_version: str, kind: str, name: str, patch: Obj, namespace: str = "",
              patch_type: str = "merge") -> Obj:
        ct = {"merge": "application/merge-patch+json", "strategic": "application/strategic-merge-patch+json",
              "json": "application/json-patch+json"}[patch_type]
        sub = "status" if set(patch.keys()) == {"status"} else ""
        return self._request("PATCH", self._path(api_version, kind, namespace, name, sub), body=patch,
                             content_type=ct).json()

    def delete(self, api_version: str, kind: str, name: str, namespace: str = "",
               propagation: Optional[str] = None, grace_period_seconds: Optional[int] = None) -> None:
        body: Dict[str, Any] = {"kind": "DeleteOptions", "apiVersion": "v1"}
        if propagation:
            body["propagationPolicy"] = propagation
        if grace_period_seconds is not None:
            body["gracePeriodSeconds"] = grace_period_seconds
        self._request("DELETE", self._path(api_version, kind, namespace, name), body=body)

    def evict(self, name: str, namespace: str, grace_period_seconds: Optional[int] = None) -> None:
        body: Dict[str, Any] = {"apiVersion": "policy/v1", "kind": "Eviction",
                                "metadata": {"name": name, "namespace": namespace}}
        if grace_period_seconds is not None:
            body["deleteOptions"] = {"gracePeriodSeconds": grace_period_seconds}
        self._request("POST", self._path("v1", "Pod", namespace, name, "eviction"), body=body)

    def has_kind(self, api_version: str, kind: str) -> bool:
        return kind in self._discover(api_version)

    def server_version(self) -> str:
        return self._request("GET", "/version").json().get("gitVersion", "")

    def create_event(self, involved: Obj, reason: str, message: str, type_: str = "Normal") -> None:
        ns = o.namespace(involved) or "default"
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f"{o.name(involved)}.", "namespace": ns},
              "involvedObject": {"apiVersion": involved.get("apiVersion"), "kind": involved.get("kind"),
                                 "name": o.name(involved), "namespace": o.namespace(involved),
                                 "uid": (involved.get("metadata") or {}).get("uid")},
              "reason": reason, "message": message, "type": type_, "firstTimestamp": now,
              "lastTimestamp": now, "count": 1, "source": {"component": "amd-gpu-operator"}}
        try:
            self.create(ev)
        except errors.ApiError as e:   # events are best effort
            log.debug("event creation failed: %s", e)

    def watch(self, api_version: str, kind: str, callback: WatchCallback,
              namespace: str = "", field_selector: Optional[str] = None) -> Callable[[], None]:
        """List+watch ``kind``; ``field_selector`` (e.g. ``metadata.name=<node>``) is sent to the
        API server on both, so a node agent receives its own Node's events only instead of every
        Node update in the cluster."""
        stop = threading.Event()
        sel = {"fieldSelector": field_selector} if field_selector else {}

        def run():
            rv = ""
            known: Dict[Tuple[str, str], Obj] = {}
            while not stop.is_set():
                try:
                    if not rv:
                        body = self._request("GET", self._path(api_version, kind, namespace), params=sel or None).json()
                        rv = body["metadata"]["resourceVersion"]
                        log.debug("watch %s: list at rv=%s (%d items)", kind, rv, len(body.get("items", [])))
                        fresh = {}
                        for it in body.get("items", []):
                            it.setdefault("apiVersion", api_version)
                            it.setdefault("kind", kind)
                            fresh[(o.namespace(it), o.name(it))] = it
                            callback(WatchEvent(MODIFIED if (o.namespace(it), o.name(it)) in known else ADDED, it))
                        for k, gone in known.items():
                            if k not in fresh:
                                callback(WatchEvent(DELETED, gone))
                        known = fresh
                    r = self._request("GET", self._path(api_version, kind, namespace),
                                      params={"watch": "1", "resourceVersion": rv,
                                              "allowWatchBookmarks": "true", "timeoutSeconds": "300", **sel},
                                      stream=True, timeout=(10, 330))
                    # one JSON event per line, read as each arrives
                    for line in r.iter_lines():
                        if stop.is_set():
                            break
                        if not line:
                            continue
                        ev = json.loads(line)
                        t, obj = ev.get("type"), ev.get("object") or {}
                        if t == "ERROR":
                            rv = ""     # 410 Gone: relist
                            break
                        rv = (obj.get("metadata") or {}).get("resourceVersion", rv)
                        if t == "BOOKMARK":
                            continue
                        k = (o.namespace(obj), o.name(obj))
                        log.debug("watch %s: %s %s rv=%s", kind, t, o.name(obj), rv)
                        old = known.get(k)
                        if t == DELETED:
                            known.pop(k, None)
                        else:
                            known[k] = obj
                        callback(WatchEvent(t, obj, old))
                except Exception as e:  # noqa: BLE001 - a watch must survive API hiccups
                    log.warning("watch %s/%s failed: %s; retrying", api_version, kind, e)
                    rv = ""
                    stop.wait(2.0)

        th = threading.Thread(target=run, name=f"watch-{kind}", daemon=True)
        th.start()
        return stop.set
