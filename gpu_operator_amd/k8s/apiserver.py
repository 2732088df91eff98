"""An in-process Kubernetes API server over HTTP, backed by :class:`FakeClient`'s store.

The role envtest plays for controller-runtime projects ("add envtest for the
reconciler"): the production :class:`~gpu_operator_amd.k8s.rest.RestClient` — discovery,
paths, verbs, content types, label/field selectors, pagination-free lists, streaming watches
with resourceVersion, status and eviction subresources, Status error bodies — is exercised
against a real HTTP endpoint, and the operator can be run end to end over the wire.

Serves ``/version``, ``/api/v1``, ``/apis/<group>/<version>`` discovery and
``[/namespaces/<ns>]/<plural>[/<name>[/status|/eviction]]`` for every kind in
:data:`~gpu_operator_amd.k8s.objects.CORE_KINDS` plus the operator's CRD kinds.
"""

from __future__ import annotations

import json
import queue
import re
import threading
from http.server import BaseHTTPRequestHandler
from typing import Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlparse

from . import errors
from . import objects as o
from .client import ADDED, DELETED, MODIFIED, merge_patch
from .fake import FakeClient

EXTRA_KINDS = {"ClusterPolicy": "amd.com/v1", "NodeFeatureRule": "nfd.k8s-sigs.io/v1alpha1",
               "ClusterVersion": "config.openshift.io/v1", "Proxy": "config.openshift.io/v1",
               "ImageStream": "image.openshift.io/v1", "Eviction": "policy/v1"}


def plural(kind: str) -> str:
    k = kind.lower()
    if k.endswith("constraints") or k.endswith("endpoints"):
        return k
    if k.endswith("y") and not k.endswith("ey"):
        return k[:-1] + "ies"
    if k.endswith(("s", "x", "ch", "sh")):
        return k + "es"
    return k + "s"


class FakeAPIServer:
    def __init__(self, client: Optional[FakeClient] = None, version: str = "v1.29.2",
                 unserved: Tuple[str, ...] = ()):
        self.client = client or FakeClient()
        self.version = version
        kinds = dict(o.CORE_KINDS)
        kinds.update(EXTRA_KINDS)
        # kinds the backing store refuses (e.g. no prometheus-operator CRDs) are not discovered either
        unserved = tuple(unserved) + tuple(getattr(self.client, "unserved_kinds", ()) or ())
        self.kinds = {k: v for k, v in kinds.items() if k not in unserved}
        # api_version -> plural -> kind
        self.by_plural: Dict[str, Dict[str, str]] = {}
        for k, av in self.kinds.items():
            self.by_plural.setdefault(av, {})[plural(k)] = k
        from ..runtime.manager import QuietHTTPServer
        self.httpd = QuietHTTPServer(("127.0.0.1", 0), self._handler())
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self.url = f"http://127.0.0.1:{self.port}"
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.requests: List[Tuple[str, str]] = []
        self.connections = 0                       # TCP connections accepted (a client's churn shows here)
        self.authorization: List[str] = []        # the Authorization header of every request

    def start(self) -> "FakeAPIServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()

    # -- routing ---------------------------------------------------------------------------
    def _route(self, path: str):
        """-> (api_version, kind, namespace, name, sub) or discovery markers."""
        m = re.fullmatch(r"/api/v1(?P<rest>/.*)?", path) or re.fullmatch(r"/apis/(?P<g>[^/]+)/(?P<v>[^/]+)(?P<rest>/.*)?",
                                                                          path)
        if not m:
            return None
        av = "v1" if path.startswith("/api/") else f"{m.group('g')}/{m.group('v')}"
        rest = (m.group("rest") or "").strip("/")
        if not rest:
            return ("discovery", av)
        parts = rest.split("/")
        ns = ""
        if parts[0] == "namespaces" and len(parts) >= 3:
            ns, parts = parts[1], parts[2:]
        elif parts[0] == "namespaces" and len(parts) <= 2:
            return (av, "Namespace", "", parts[1] if len(parts) == 2 else "", "")
        kind = self.by_plural.get(av, {}).get(parts[0])
        if kind is None:
            raise errors.NotFound(f"the server could not find the requested resource ({path})")
        name = parts[1] if len(parts) > 1 else ""
        sub = parts[2] if len(parts) > 2 else ""
        if kind in o.CLUSTER_SCOPED:
            ns = ""
        return (av, kind, ns, name, sub)

    def _discovery(self, av: str) -> Dict:
        res = [{"name": plural(k), "kind": k, "namespaced": k not in o.CLUSTER_SCOPED,
                "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]}
               for k, v in sorted(self.kinds.items()) if v == av]
        if av == "v1":
            res.append({"name": "pods/eviction", "kind": "Eviction", "namespaced": True, "verbs": ["create"]})
        if not res:
            raise errors.NotFound(f"no resources for {av}")
        return {"kind": "APIResourceList", "groupVersion": av, "resources": res}

    # -- CRD schema admission (k8s/openapi.py) -------------------------------------------------
    def _crd_schema(self, av: str, kind: str):
        version = av.split("/")[-1]
        for crd in self.client.list("apiextensions.k8s.io/v1", "CustomResourceDefinition"):
            names = (crd.get("spec") or {}).get("names") or {}
            if names.get("kind") != kind:
                continue
            for v in (crd.get("spec") or {}).get("versions") or []:
                if v.get("name") == version:
                    return ((v.get("schema") or {}).get("openAPIV3Schema"))
        return None

    def _admit(self, av: str, kind: str, obj: Dict) -> None:
        """What kube-apiserver does before storing: a v1 CRD must be structural; a custom
        resource is pruned, defaulted and validated against its CRD's schema."""
        from . import openapi
        if kind == "CustomResourceDefinition":
            errs = []
            for v in (obj.get("spec") or {}).get("versions") or []:
                sch = (v.get("schema") or {}).get("openAPIV3Schema")
                if sch is None:
                    errs.append(f"spec.versions[{v.get('name')}].schema.openAPIV3Schema: Required value")
                else:
                    errs += [f"spec.versions[{v.get('name')}].schema.openAPIV3Schema.{e}"
                             for e in openapi.structural_errors(sch)]
            if errs:
                raise errors.Invalid(f'CustomResourceDefinition "{o.name(obj)}" is invalid: ' + "; ".join(errs[:20]))
            return
        sch = self._crd_schema(av, kind)
        if sch is None:
            return
        errs = openapi.admit(obj, sch)
        if errs:
            group = av.split("/")[0] if "/" in av else ""
            raise errors.Invalid(f'{kind}.{group} "{o.name(obj)}" is invalid: ' + "; ".join(errs[:20]))

    def _current_rv(self) -> int:
        rvs = [int((x.get("metadata") or {}).get("resourceVersion", 0) or 0) for x in self.client.objects()]
        return max(rvs, default=0)

    def _handler(self):
        srv = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"     # keep-alive; watches use chunked encoding like kube-apiserver

            def log_message(self, *a):
                pass

            def setup(self):
                srv.connections += 1
                super().setup()

            def _send(self, code: int, body) -> None:
                data = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def _error(self, e: errors.ApiError) -> None:
                self._send(e.status, {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                      "message": str(e), "reason": e.reason, "code": e.status})

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n) or b"null") if n else None

            def _dispatch(self, verb: str) -> None:
                u = urlparse(self.path)
                q = {k: v[-1] for k, v in parse_qs(u.query).items()}
                srv.requests.append((verb, u.path))
                srv.authorization.append(self.headers.get("Authorization", ""))
                try:
                    if u.path == "/version":
                        return self._send(200, {"gitVersion": srv.version, "major": "1",
                                                "minor": srv.version.split(".")[1]})
                    r = srv._route(u.path)
                    if r is None:
                        raise errors.NotFound(u.path)
                    if r[0] == "discovery":
                        return self._send(200, srv._discovery(r[1]))
                    av, kind, ns, name, sub = r
                    c = srv.client
                    if verb == "GET" and not name:
                        if q.get("watch") in ("1", "true"):
                            return self._watch(av, kind, ns, q)
                        items = c.list(av, kind, ns, label_selector=q.get("labelSelector"),
                                       field_selector=q.get("fieldSelector"))
                        return self._send(200, {"kind": kind + "List", "apiVersion": av, "items": items,
                                                "metadata": {"resourceVersion": str(srv._current_rv())}})
                    if verb == "GET":
                        return self._send(200, c.get(av, kind, name, ns))
                    body = self._body()
                    if verb == "POST" and sub == "eviction":
                        c.evict(name, ns)
                        return self._send(201, {"kind": "Status", "status": "Success"})
                    if verb == "POST":
                        body.setdefault("metadata", {})
                        if ns and kind not in o.CLUSTER_SCOPED:
                            body["metadata"]["namespace"] = ns
                        body.setdefault("apiVersion", av)
                        body.setdefault("kind", kind)
                        srv._admit(av, kind, body)
                        return self._send(201, c.create(body))
                    if verb == "PUT":
                        body.setdefault("apiVersion", av)
                        body.setdefault("kind", kind)
                        if sub != "status":
                            srv._admit(av, kind, body)
                        return self._send(200, c.update_status(body) if sub == "status" else c.update(body))
                    if verb == "PATCH":
                        ct = self.headers.get("Content-Type", "")
                        if "merge-patch" not in ct and "strategic" not in ct:
                            raise errors.ApiError(f"unsupported patch type {ct}", 415, "UnsupportedMediaType")
                        if sub != "status" and (kind == "CustomResourceDefinition" or srv._crd_schema(av, kind)):
                            cur = c.get(av, kind, name, ns)
                            new = merge_patch(cur, body)
                            srv._admit(av, kind, new)
                            return self._send(200, c.update(new))
                        return self._send(200, c.patch(av, kind, name, body, ns))
                    if verb == "DELETE":
                        c.delete(av, kind, name, ns, propagation=(body or {}).get("propagationPolicy"))
                        return self._send(200, {"kind": "Status", "status": "Success"})
                    raise errors.ApiError(f"method {verb} not allowed", 405, "MethodNotAllowed")
                except errors.ApiError as e:
                    return self._error(e)

            def _watch(self, av, kind, ns, q) -> None:
                since = int(q.get("resourceVersion") or 0)
                timeout = float(q.get("timeoutSeconds") or 300)
                events: "queue.Queue" = queue.Queue()
                registering = [True]

                def cb(ev):
                    rv = int((ev.obj.get("metadata") or {}).get("resourceVersion", 0) or 0)
                    if registering[0] and ev.type == ADDED and rv <= since:
                        return            # the initial list replay: the client already has it
                    if ev.type in (ADDED, MODIFIED) and rv <= since:
                        return
                    events.put(ev)
                stop = srv.client.watch(av, kind, cb, ns, field_selector=q.get("fieldSelector"))
                registering[0] = False
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                deadline = threading.Event()
                timer = threading.Timer(timeout, deadline.set)
                timer.start()
                try:
                    while not deadline.is_set():
                        try:
                            ev = events.get(timeout=0.2)
                        except queue.Empty:
                            continue
                        line = (json.dumps({"type": ev.type, "object": ev.obj}) + "\n").encode()
                        self.wfile.write(b"%x\r\n%s\r\n" % (len(line), line))
                        self.wfile.flush()
                    self.wfile.write(b"0\r\n\r\n")
                except (BrokenPipeError, ConnectionResetError):
                    pass
                finally:
                    timer.cancel()
                    stop()

            def do_GET(self):  # noqa: N802
                self._dispatch("GET")

            def do_POST(self):  # noqa: N802
                self._dispatch("POST")

            def do_PUT(self):  # noqa: N802
                self._dispatch("PUT")

            def do_PATCH(self):  # noqa: N802
                self._dispatch("PATCH")

            def do_DELETE(self):  # noqa: N802
                self._dispatch("DELETE")

        return H
