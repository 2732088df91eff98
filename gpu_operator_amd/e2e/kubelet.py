"""A kubelet that runs a node's pods as OS processes (the e2e harness's node).

Every pod bound to the node (or schedulable onto it) runs here: init containers in order, then
the main containers, each one an OS process started from the pod spec's ``command``/``args``
with its env, its volume mounts and its restart policy. The node's filesystem is a directory
tree (``<base>/host``); ``/sys`` and ``/dev`` are the machine's (or a fake sysfs on CPU).

What a container sees, and how
  * volumes: ``hostPath`` -> the node tree, ``configMap`` -> files written from the API object,
    ``emptyDir`` -> a per-pod directory; ``subPath`` honoured. The mount table goes to the process
    in ``AMD_MOUNTS`` (utils/mounts.py) and is applied to its argv, its env values and the
    ConfigMap scripts it runs, so ``/bin/entrypoint.sh`` and ``/run/amd/validations`` resolve as
    they would inside the container;
  * env: ``value``, ``fieldRef`` (metadata.name/namespace/uid, spec.nodeName,
    spec.serviceAccountName, status.hostIP/podIP), ``configMapKeyRef``, plus the harness's
    cluster access (``KUBECONFIG`` instead of an in-cluster service account token);
  * extended resources (``amd.com/gpu``): real device-plugin gRPC. Plugins register on the
    node's ``kubelet.sock``; ListAndWatch feeds the Node's capacity/allocatable; a container's
    limits are served by ``Allocate`` and its env reaches the process. The pod-resources API
    (``List``) reports the assignments to the metrics exporter;
  * ``runtimeClassName``: sandbox creation waits until the runtime handler is configured in
    the node's containerd config (what the toolkit's ``amd-ctk install`` writes), retried every
    ``SYNC_S`` as kubelet does;
  * restart policy ``Always`` with kubelet's crash-loop back-off; ``OnFailure``/``Never`` pods
    end ``Succeeded``/``Failed``; a failing init container fails a ``Never`` pod and is restarted
    with back-off otherwise (the pod stays ``Pending``, the previous exit in ``lastState``);
    termination messages from ``terminationMessagePath`` (``FallbackToLogsOnError`` honoured);
  * exec readiness / startup probes; the Ready condition and containerStatuses are written back
    through the API, so DaemonSet status and the operator see real readiness;
  * pods deleted from the API have their process groups terminated (SIGTERM, then SIGKILL
    after the grace period).

Not emulated: image pulls (every image is this repository), cgroups/namespaces (a container's
device visibility is the runtime hook's job, not the kubelet's), liveness probes.
"""

from __future__ import annotations

import json
import logging
import os
import re
import shutil
import signal
import subprocess
import threading
import time
from concurrent import futures
from typing import Callable, Any, Dict, List, Optional, Tuple

from ..k8s import errors
from ..k8s import objects as o
from ..utils import mounts

log = logging.getLogger("amd-e2e.kubelet")

SYNC_S = 0.2                                                      # pod sync / sandbox retry period
CRASHLOOP_BACKOFF_S = [1.0, 2.0, 4.0, 8.0, 16.0, 30.0]            # scaled-down kubelet back-off
GRACE_S = 5.0


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


class DevicePlugins:
    """kubelet's device-manager side: registration server, ListAndWatch clients, Allocate."""

    def __init__(self, plugin_dir: str, on_capacity):
        import grpc
        from ..operands import kubeletapi as K
        self.K, self.grpc = K, grpc
        self.plugin_dir = plugin_dir
        self.on_capacity = on_capacity
        self.devices: Dict[str, Dict[str, str]] = {}        # resource -> {device id: health}
        self.endpoints: Dict[str, str] = {}
        self.assigned: Dict[Tuple[str, str, str], List[str]] = {}   # (pod uid, container, resource) -> ids
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        self.server.add_generic_rpc_handlers((K.registration_handler(self._on_register),))
        os.makedirs(plugin_dir, exist_ok=True)
        self.server.add_insecure_port("unix://" + os.path.join(plugin_dir, "kubelet.sock"))

    def start(self) -> None:
        self.server.start()

    def stop(self) -> None:
        self._stop.set()
        self.server.stop(0)

    def _on_register(self, req) -> None:
        log.info("device plugin registered: %s at %s", req.resource_name, req.endpoint)
        with self._lock:
            self.endpoints[req.resource_name] = req.endpoint
        threading.Thread(target=self._watch, args=(req.resource_name, req.endpoint), daemon=True).start()

    def _watch(self, resource: str, endpoint: str) -> None:
        K = self.K
        try:
            with self.grpc.insecure_channel("unix://" + os.path.join(self.plugin_dir, endpoint)) as ch:
                for resp in K.device_plugin_stub(ch)["ListAndWatch"](K.DP["Empty"]()):
                    with self._lock:
                        if self.endpoints.get(resource) != endpoint:
                            return                                 # re-registered elsewhere
                        self.devices[resource] = {d.ID: d.health for d in resp.devices}
                    self.on_capacity(resource, sum(1 for h in self.devices[resource].values() if h == K.HEALTHY))
                    if self._stop.is_set():
                        return
        except Exception as e:  # noqa: BLE001 - plugin restarted or went away
            if not self._stop.is_set():
                log.info("ListAndWatch %s ended: %s", resource, e)
        with self._lock:
            if self.endpoints.get(resource) == endpoint:
                self.devices[resource] = {}
        if not self._stop.is_set():
            self.on_capacity(resource, 0)

    def allocate(self, uid: str, container: str, resource: str, n: int) -> Dict[str, Any]:
        """Pick n free healthy devices and call the plugin's Allocate. Raises when short."""
        K = self.K
        with self._lock:
            endpoint = self.endpoints.get(resource)
            healthy = [d for d, h in sorted(self.devices.get(resource, {}).items()) if h == K.HEALTHY]
            used = {d for (u, _, r), ids in self.assigned.items() if r == resource and u != uid for d in ids}
            free = [d for d in healthy if d not in used]
        if endpoint is None or len(free) < n:
            raise RuntimeError(f"UnexpectedAdmissionError: {resource}: requested {n}, available {len(free)}")
        ids = free[:n]
        with self.grpc.insecure_channel("unix://" + os.path.join(self.plugin_dir, endpoint)) as ch:
            req = K.DP["AllocateRequest"]()
            req.container_requests.add().devicesIDs.extend(ids)
            resp = K.device_plugin_stub(ch)["Allocate"](req, timeout=10)
        car = resp.container_responses[0]
        with self._lock:
            self.assigned[(uid, container, resource)] = ids
        return {"ids": ids, "envs": dict(car.envs),
                "mounts": [(m.container_path, m.host_path) for m in car.mounts],
                "devices": [(d.container_path, d.host_path) for d in car.devices],
                "annotations": dict(car.annotations), "cdi": [c.name for c in car.cdi_devices]}

    def release(self, uid: str) -> None:
        with self._lock:
            for k in [k for k in self.assigned if k[0] == uid]:
                del self.assigned[k]

    def list_pod_resources(self, pods: Dict[str, Dict]):
        """PodResourcesLister.List: what the metrics exporter attributes GPUs with."""
        K = self.K
        resp = K.PR["ListPodResourcesResponse"]()
        by_pod: Dict[str, Dict[str, List[Tuple[str, List[str]]]]] = {}
        with self._lock:
            for (uid, ctr, res), ids in self.assigned.items():
                by_pod.setdefault(uid, {}).setdefault(ctr, []).append((res, ids))
        for uid, ctrs in by_pod.items():
            pod = pods.get(uid)
            if pod is None:
                continue
            pr = resp.pod_resources.add(name=o.name(pod), namespace=o.namespace(pod))
            for ctr, items in ctrs.items():
                cr = pr.containers.add(name=ctr)
                for res, ids in items:
                    cr.devices.add(resource_name=res, device_ids=ids)
        return resp


class PodRun:
    """One pod's lifecycle on this node."""

    def __init__(self, kl: "ProcessKubelet", pod: Dict):
        self.kl = kl
        self.pod = pod
        self.uid = pod["metadata"]["uid"]
        self.name, self.ns = o.name(pod), o.namespace(pod)
        self.dir = os.path.join(kl.base, "pods", f"{self.ns}_{self.name}_{self.uid[:8]}")
        self.procs: Dict[str, subprocess.Popen] = {}
        self.restarts: Dict[str, int] = {}
        self.terminated: Dict[str, Dict] = {}
        self.alloc: Dict[str, Dict[str, Any]] = {}
        self.stop_evt = threading.Event()
        self.ready = False
        self.phase = "Pending"
        self.reason = self.message = ""          # status.reason / message (admission failures)
        self.started_at: Dict[str, float] = {}
        self.thread = threading.Thread(target=self._main, name=f"pod-{self.name}", daemon=True)

    # -- status ------------------------------------------------------------------------------
    def _ctr_status(self, c: Dict, init: bool) -> Dict:
        name = c["name"]
        p = self.procs.get(name)
        st: Dict[str, Any] = {"name": name, "image": c.get("image", ""), "restartCount": self.restarts.get(name, 0),
                              "ready": bool(not init and p is not None and p.poll() is None and self.ready)}
        if p is not None and p.poll() is None:
            st["state"] = {"running": {"startedAt": _now()}}
            st["started"] = True
            if name in self.terminated:
                # a restarted container: the previous run's exit, as kubelet reports it
                st["lastState"] = {"terminated": {k: v for k, v in self.terminated[name].items() if not k.startswith("_")}}
        elif name in self.terminated:
            st["state"] = {"terminated": {k: v for k, v in self.terminated[name].items() if not k.startswith("_")}}
        else:
            st["state"] = {"waiting": {"reason": "PodInitializing" if not init else "Waiting"}}
        return st

    def publish(self) -> None:
        if self.phase in ("Succeeded", "Failed"):
            self.kl.plugins.release(self.uid)      # a terminated pod's devices are free again
        spec = self.pod.get("spec") or {}
        status = {"phase": self.phase, "hostIP": "127.0.0.1", "podIP": "127.0.0.1",
                  "conditions": [{"type": "Ready", "status": "True" if self.ready else "False"},
                                 {"type": "ContainersReady", "status": "True" if self.ready else "False"},
                                 {"type": "PodScheduled", "status": "True"}],
                  "initContainerStatuses": [self._ctr_status(c, True) for c in spec.get("initContainers") or []],
                  "containerStatuses": [self._ctr_status(c, False) for c in spec.get("containers") or []]}
        if self.reason:
            status.update(reason=self.reason, message=self.message)
        self.kl.set_status(self.ns, self.name, self.uid, status)

    # -- container plumbing ------------------------------------------------------------------
    def _volumes(self) -> Dict[str, Tuple[str, Dict]]:
        """volume name -> (host path, volume spec); materialises ConfigMaps and emptyDirs."""
        out = {}
        for v in (self.pod.get("spec") or {}).get("volumes") or []:
            name = v["name"]
            if "hostPath" in v:
                hp = self.kl.host_path(v["hostPath"]["path"])
                t = v["hostPath"].get("type", "")
                # directories are created in the node tree only; /sys and /dev are the machine's
                if t in ("DirectoryOrCreate", "Directory", "") and not os.path.splitext(hp)[1] and \
                        hp.startswith(self.kl.host):
                    os.makedirs(hp, exist_ok=True)
                out[name] = (hp, v)
            elif "configMap" in v:
                d = os.path.join(self.dir, "configmaps", name)
                os.makedirs(d, exist_ok=True)
                cm = self.kl.get_configmap(self.ns, v["configMap"]["name"])
                items = v["configMap"].get("items")
                data = (cm or {}).get("data") or {}
                keys = [(i["key"], i.get("path", i["key"])) for i in items] if items else [(k, k) for k in data]
                for key, rel in keys:
                    if key in data:
                        fp = os.path.join(d, rel)
                        os.makedirs(os.path.dirname(fp), exist_ok=True)
                        with open(fp, "w") as f:
                            f.write(data[key])
                        mode = v["configMap"].get("defaultMode", 0o644)
                        os.chmod(fp, mode | 0o400)
                out[name] = (d, v)
            else:                                         # emptyDir, secret, projected, downwardAPI
                d = os.path.join(self.dir, "volumes", name)
                os.makedirs(d, exist_ok=True)
                out[name] = (d, v)
        return out

    def _mount_pairs(self, c: Dict, vols: Dict[str, Tuple[str, Dict]]) -> List[Tuple[str, str]]:
        pairs = []
        for m in c.get("volumeMounts") or []:
            if m["name"] not in vols:
                continue
            src, _ = vols[m["name"]]
            if m.get("subPath"):
                src = os.path.join(src, m["subPath"])
            pairs.append((m["mountPath"].rstrip("/") or "/", src))
        term = os.path.join(self.dir, "termination", c["name"])
        os.makedirs(os.path.dirname(term), exist_ok=True)
        pairs.append((c.get("terminationMessagePath") or "/dev/termination-log", term))
        for r, a in self.alloc.items():
            if r.startswith(c["name"] + "/"):
                pairs += [(cp, hp) for cp, hp in a["mounts"]]
        pairs.sort(key=lambda p: len(p[0]), reverse=True)
        return pairs

    def _env(self, c: Dict, pairs: List[Tuple[str, str]]) -> Dict[str, str]:
        env = dict(self.kl.base_env)
        env.update(self.kl.image_env(c.get("image", "")))          # the image's own ENV
        env["AMD_MOUNTS"] = json.dumps(pairs)
        env["HOSTNAME"] = self.name
        md, spec = self.pod["metadata"], self.pod.get("spec") or {}
        fields = {"metadata.name": self.name, "metadata.namespace": self.ns, "metadata.uid": self.uid,
                  "spec.nodeName": self.kl.node, "spec.serviceAccountName": spec.get("serviceAccountName", "default"),
                  "status.hostIP": "127.0.0.1", "status.podIP": "127.0.0.1"}
        for e in c.get("env") or []:
            if "value" in e:
                env[e["name"]] = mounts.rewrite_text(str(e["value"]), pairs)
            elif "valueFrom" in e:
                vf = e["valueFrom"]
                if "fieldRef" in vf:
                    fp = vf["fieldRef"].get("fieldPath", "")
                    m = re.match(r"metadata\.(labels|annotations)\['(.+)'\]", fp)
                    if m:
                        env[e["name"]] = str((md.get(m.group(1)) or {}).get(m.group(2), ""))
                    else:
                        env[e["name"]] = fields.get(fp, "")
                elif "configMapKeyRef" in vf:
                    ref = vf["configMapKeyRef"]
                    cm = self.kl.get_configmap(self.ns, ref["name"]) or {}
                    if ref["key"] in (cm.get("data") or {}):
                        env[e["name"]] = cm["data"][ref["key"]]
            else:
                env[e["name"]] = ""
        for r, a in self.alloc.items():
            if r.startswith(c["name"] + "/"):
                env.update(a["envs"])
        return env

    def _argv(self, c: Dict, pairs: List[Tuple[str, str]]) -> List[str]:
        argv = list(c.get("command") or []) + list(c.get("args") or [])
        if not argv:
            raise RuntimeError(f"container {c['name']}: no command (image entrypoints are not emulated)")
        out = []
        for a in argv:
            a = mounts.rewrite_text(a, pairs)
            out.append(a)
        # scripts coming from ConfigMap mounts see the same container paths: rewrite a private copy
        for i, a in enumerate(out):
            for cpath, hpath in pairs:
                if a == hpath and os.path.isfile(hpath) and hpath.startswith(self.dir):
                    out[i] = self._rewritten_script(c["name"], hpath, pairs)
        if len(out) >= 3 and out[0] in ("/bin/sh", "sh", "/bin/bash", "bash") and out[1] == "-c":
            # `sh -c /bin/entrypoint.sh` : the script path is inside the -c string
            for cpath, hpath in pairs:
                if os.path.isfile(hpath) and hpath.startswith(self.dir) and hpath in out[2]:
                    out[2] = out[2].replace(hpath, self._rewritten_script(c["name"], hpath, pairs))
        return out

    def _rewritten_script(self, ctr: str, src: str, pairs) -> str:
        dst = os.path.join(self.dir, "scripts", ctr, os.path.basename(src))
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(src) as f:
            text = f.read()
        with open(dst, "w") as f:
            f.write(mounts.rewrite_text(text, pairs))
        os.chmod(dst, 0o755)
        return dst

    def _spawn(self, c: Dict, vols) -> subprocess.Popen:
        pairs = self._mount_pairs(c, vols)
        argv = self._argv(c, pairs)
        env = self._env(c, pairs)
        os.makedirs(os.path.join(self.dir, "logs"), exist_ok=True)
        logp = os.path.join(self.dir, "logs", f"{c['name']}.log")
        logf = open(logp, "ab")
        term = dict(pairs).get(c.get("terminationMessagePath") or "/dev/termination-log")
        if term and os.path.exists(term):
            os.remove(term)
        p = subprocess.Popen(argv, env=env, stdout=logf, stderr=subprocess.STDOUT, cwd=self.dir,
                             start_new_session=True)
        logf.close()
        self.procs[c["name"]] = p
        self.started_at[c["name"]] = time.monotonic()
        self.kl.event(f"{self.name}:{c['name']}:started", pid=p.pid)
        return p

    def _record_exit(self, c: Dict, p: subprocess.Popen, vols) -> None:
        pairs = self._mount_pairs(c, vols)
        term = dict(pairs).get(c.get("terminationMessagePath") or "/dev/termination-log")
        msg = ""
        if term and os.path.exists(term):
            with open(term, errors="replace") as f:
                msg = f.read()[:4096]
        if not msg and p.returncode != 0 and c.get("terminationMessagePolicy") == "FallbackToLogsOnError":
            logp = os.path.join(self.dir, "logs", f"{c['name']}.log")
            try:
                with open(logp, errors="replace") as f:
                    msg = "\n".join(f.read().splitlines()[-80:])[-2048:]
            except OSError:
                pass
        self.terminated[c["name"]] = {"exitCode": p.returncode, "reason": "Completed" if p.returncode == 0 else "Error",
                                      "message": msg, "finishedAt": _now()}

    def _probe(self, c: Dict, key: str, vols) -> bool:
        probe = c.get(key) or {}
        cmd = (probe.get("exec") or {}).get("command")
        if not cmd:
            return True
        pairs = self._mount_pairs(c, vols)
        try:
            return subprocess.run([mounts.rewrite_text(a, pairs) for a in cmd], env=self._env(c, pairs),
                                  capture_output=True, timeout=probe.get("timeoutSeconds", 10)).returncode == 0
        except (subprocess.TimeoutExpired, OSError):
            return False

    def _sleep(self, s: float) -> bool:
        return not self.stop_evt.wait(s)

    # -- lifecycle ---------------------------------------------------------------------------
    def _main(self) -> None:
        try:
            self._lifecycle()
        except Exception as e:  # noqa: BLE001 - report as a failed pod, keep the kubelet alive
            log.exception("pod %s/%s: %s", self.ns, self.name, e)
            self.kl.event(f"{self.name}:error", error=str(e))
            self.phase = "Failed"
            if str(e).startswith("UnexpectedAdmissionError"):
                # a nodeName-bound pod whose device request the node cannot serve: the kubelet
                # rejects it at admission (it is never Pending)
                self.reason, self.message = "UnexpectedAdmissionError", str(e)
            self.publish()

    def _lifecycle(self) -> None:
        spec = self.pod.get("spec") or {}
        policy = spec.get("restartPolicy", "Always")
        rc = spec.get("runtimeClassName")
        while rc and not self.kl.runtime_handler_ready(rc):
            if not self._sleep(SYNC_S):
                return
        self.kl.event(f"{self.name}:sandbox")
        vols = self._volumes()
        for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
            for r, q in ((c.get("resources") or {}).get("limits") or {}).items():
                if "/" in r and not r.startswith(("hugepages-", "requests.")):
                    self.alloc[f"{c['name']}/{r}"] = self.kl.plugins.allocate(self.uid, c["name"], r, int(q))
        self.publish()
        for c in spec.get("initContainers") or []:
            attempt = 0
            while True:
                p = self._spawn(c, vols)
                self.publish()
                while p.poll() is None:
                    if self.stop_evt.wait(0.05):
                        return
                self._record_exit(c, p, vols)
                if p.returncode == 0:
                    break
                if policy == "Never":
                    self.phase = "Failed"
                    self.publish()
                    return
                # Always / OnFailure: the init container restarts with crash-loop back-off and the pod
                # stays Pending (kubelet never fails a pod whose policy restarts it)
                self.restarts[c["name"]] = self.restarts.get(c["name"], 0) + 1
                self.publish()
                if not self._sleep(CRASHLOOP_BACKOFF_S[min(attempt, len(CRASHLOOP_BACKOFF_S) - 1)]):
                    return
                attempt += 1
            self.kl.event(f"{self.name}:{c['name']}:done")
        mains = spec.get("containers") or []
        for c in mains:
            self._spawn(c, vols)
        self.phase = "Running"
        self.publish()
        started = {c["name"]: False for c in mains}
        backoff = {c["name"]: 0 for c in mains}
        next_probe = 0.0
        while not self.stop_evt.is_set():
            changed = False
            for c in mains:
                p = self.procs[c["name"]]
                if p.poll() is None:
                    continue
                if c["name"] not in self.terminated or self.terminated[c["name"]].get("_pid") != p.pid:
                    self._record_exit(c, p, vols)
                    self.terminated[c["name"]]["_pid"] = p.pid
                    changed = True
                    if policy == "Always" or (policy == "OnFailure" and p.returncode != 0):
                        self.restarts[c["name"]] = self.restarts.get(c["name"], 0) + 1
                        self.ready = False
                        self.publish()
                        wait = CRASHLOOP_BACKOFF_S[min(backoff[c["name"]], len(CRASHLOOP_BACKOFF_S) - 1)]
                        backoff[c["name"]] += 1
                        if not self._sleep(wait):
                            return
                        self._spawn(c, vols)
                        changed = True
            if policy != "Always" and all(self.procs[c["name"]].poll() is not None for c in mains) and \
                    not any(policy == "OnFailure" and self.procs[c["name"]].returncode != 0 for c in mains):
                self.ready = False
                self.phase = "Succeeded" if all(self.procs[c["name"]].returncode == 0 for c in mains) else "Failed"
                self.publish()
                self.kl.event(f"{self.name}:{self.phase.lower()}")
                return
            now = time.monotonic()
            if now >= next_probe:
                next_probe = now + 0.5
                running = all(self.procs[c["name"]].poll() is None for c in mains)
                ok = running
                for c in mains:
                    if not ok:
                        break
                    if not started[c["name"]]:
                        started[c["name"]] = self._probe(c, "startupProbe", vols)
                    ok = started[c["name"]] and self._probe(c, "readinessProbe", vols)
                if ok != self.ready:
                    self.ready = ok
                    changed = True
                    if ok:
                        self.kl.event(f"{self.name}:ready")
            if changed:
                self.publish()
            self.stop_evt.wait(0.05)

    def start(self) -> None:
        self.thread.start()

    def _pre_stop(self) -> None:
        """lifecycle.preStop exec hooks of the running main containers, before the SIGTERM."""
        vols = None
        for c in (self.pod.get("spec") or {}).get("containers") or []:
            cmd = (((c.get("lifecycle") or {}).get("preStop") or {}).get("exec") or {}).get("command")
            p = self.procs.get(c["name"])
            if not cmd or p is None or p.poll() is not None:
                continue
            try:
                vols = vols or self._volumes()
                pairs = self._mount_pairs(c, vols)
                subprocess.run([mounts.rewrite_text(a, pairs) for a in cmd], env=self._env(c, pairs),
                               capture_output=True, timeout=GRACE_S)
            except (OSError, subprocess.TimeoutExpired) as e:
                log.info("preStop of %s/%s: %s", self.name, c["name"], e)

    def kill(self, grace: float = GRACE_S) -> None:
        self.stop_evt.set()
        self._pre_stop()
        for p in self.procs.values():
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except (ProcessLookupError, PermissionError):
                    pass
        deadline = time.monotonic() + grace
        for p in self.procs.values():
            try:
                p.wait(timeout=max(0.05, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                p.wait()
        self.thread.join(timeout=2)
        self.kl.plugins.release(self.uid)

    def pids(self) -> List[int]:
        return [p.pid for p in self.procs.values() if p.poll() is None]


class ProcessKubelet:
    def __init__(self, client, node: str, base: str, base_env: Dict[str, str], sys_root: str = "/",
                 dev_root: str = "/", events=None, host_links: Optional[Dict[str, str]] = None,
                 image_env=None):
        self.client, self.node, self.base = client, node, base
        self.host = os.path.join(base, "host")
        # the node tree is synthetic (every hostPath a pod writes lands in it); what the host has
        # installed is linked in read-mostly: by default its ROCm (the host driver's userspace,
        # which the driver validation looks for under /host)
        if host_links is None:
            host_links = {"/opt/rocm": "/opt/rocm"} if os.path.isdir("/opt/rocm") else {}
        for cpath, real in host_links.items():
            dst = os.path.join(self.host, cpath.lstrip("/"))
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            if not os.path.lexists(dst):
                os.symlink(real, dst)
        self.sys_root, self.dev_root = sys_root, dev_root
        self.base_env = dict(base_env)
        self.base_env.setdefault("AMD_SYSFS_ROOT", sys_root)
        self.base_env.setdefault("AMD_DEV_ROOT", dev_root)
        self._events = events or (lambda name, **kw: None)
        # an image's ENV (images are not pulled: the harness says what a tag's config carries)
        self.image_env = image_env or (lambda image: {})
        self.pods: Dict[str, PodRun] = {}
        # harness hook: pods (not yet running here) for which this returns True are not admitted yet
        self.hold_admission: Optional[Callable[[Dict], bool]] = None
        self._terminating: set = set()                 # deleted pods whose processes are being killed
        self._lock = threading.Lock()
        self._stop = threading.Event()
        os.makedirs(self.host, exist_ok=True)
        self.plugins = DevicePlugins(self.host_path("/var/lib/kubelet/device-plugins"), self._capacity)
        self._pr_server = None
        self.thread = threading.Thread(target=self._loop, name="kubelet", daemon=True)

    # -- node filesystem -------------------------------------------------------------------------
    def host_path(self, p: str) -> str:
        p = "/" + p.strip("/")
        if p == "/sys" or p.startswith("/sys/"):
            return os.path.join(self.sys_root, p.lstrip("/"))
        if p == "/dev" or p.startswith("/dev/"):
            return os.path.join(self.dev_root, p.lstrip("/"))
        return self.host if p == "/" else os.path.join(self.host, p.lstrip("/"))

    def runtime_handler_ready(self, handler: str) -> bool:
        """containerd has a runtime for ``handler`` (what the RuntimeClass names) in its config."""
        cfg = self.host_path("/etc/containerd/config.toml")
        try:
            with open(cfg) as f:
                text = f.read()
        except OSError:
            return False
        return re.search(r"runtimes\.[\"']?" + re.escape(handler) + r"[\"']?\]", text) is not None

    # -- API plumbing ----------------------------------------------------------------------------
    def event(self, name: str, **kw) -> None:
        self._events(name, **kw)

    def get_configmap(self, ns: str, name: str) -> Optional[Dict]:
        try:
            return self.client.get("v1", "ConfigMap", name, ns)
        except errors.NotFound:
            return None

    def set_status(self, ns: str, name: str, uid: str, status: Dict) -> None:
        for _ in range(10):
            try:
                cur = self.client.get("v1", "Pod", name, ns)
            except errors.NotFound:
                return
            if cur["metadata"].get("uid") != uid:
                return
            cur["status"] = status
            try:
                self.client.update_status(cur)
                return
            except errors.Conflict:
                continue
            except errors.NotFound:
                return

    def _capacity(self, resource: str, n: int) -> None:
        self.client.patch("v1", "Node", self.node, {"status": {"capacity": {resource: str(n)},
                                                               "allocatable": {resource: str(n)}}})
        self.event(f"kubelet:capacity:{resource}={n}")

    # -- pods ------------------------------------------------------------------------------------
    def _schedulable(self, pod: Dict, node: Dict) -> bool:
        spec = pod.get("spec") or {}
        labels = o.get_labels(node)
        return all(labels.get(k) == v for k, v in (spec.get("nodeSelector") or {}).items())

    def _sync(self) -> None:
        node = self.client.get("v1", "Node", self.node)
        pods = self.client.list("v1", "Pod")
        live = {}
        hold = self.hold_admission
        for p in pods:
            if hold is not None and p["metadata"]["uid"] not in self.pods and hold(p):
                continue                     # the harness orders admissions (race rehearsals)
            spec = p.get("spec") or {}
            if not spec.get("nodeName"):
                if (p.get("status") or {}).get("phase", "Pending") == "Pending" and self._schedulable(p, node):
                    p["spec"]["nodeName"] = self.node              # the scheduler's binding
                    try:
                        p = self.client.update(p)
                    except (errors.Conflict, errors.NotFound):
                        continue
                else:
                    continue
            if p["spec"].get("nodeName") != self.node:
                continue
            if (p["metadata"].get("deletionTimestamp")):
                continue
            live[p["metadata"]["uid"]] = p
        with self._lock:
            gone = [uid for uid in self.pods if uid not in live]
            for uid in gone:
                run = self.pods.pop(uid)
                self._terminating.add(run)          # still holds processes until the reap finishes
                threading.Thread(target=self._reap, args=(run,), daemon=True).start()
            for uid, p in live.items():
                if uid not in self.pods and (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed"):
                    run = PodRun(self, p)
                    self.pods[uid] = run
                    run.start()

    def _reap(self, run: PodRun) -> None:
        try:
            run.kill()
        finally:
            with self._lock:
                self._terminating.discard(run)
        self.event(f"{run.name}:killed")

    def _loop(self) -> None:
        while not self._stop.is_set():
            try:
                self._sync()
            except Exception as e:  # noqa: BLE001 - keep the node alive through API hiccups
                log.warning("kubelet sync: %s", e)
            self._stop.wait(SYNC_S)

    def _serve_pod_resources(self) -> None:
        import grpc
        from ..operands import kubeletapi as K
        sock = self.host_path("/var/lib/kubelet/pod-resources/kubelet.sock")
        os.makedirs(os.path.dirname(sock), exist_ok=True)

        def list_fn(req, ctx):
            with self._lock:
                pods = {uid: r.pod for uid, r in self.pods.items()}
            return self.plugins.list_pod_resources(pods)
        self._pr_server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self._pr_server.add_generic_rpc_handlers((K.pod_resources_handler(list_fn),))
        self._pr_server.add_insecure_port("unix://" + sock)
        self._pr_server.start()

    def start(self) -> "ProcessKubelet":
        self.plugins.start()
        self._serve_pod_resources()
        self.thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self.thread.join(timeout=5)
        with self._lock:
            runs = list(self.pods.values())
            self.pods.clear()
        for r in runs:
            r.kill(grace=2.0)
        self.plugins.stop()
        if self._pr_server is not None:
            self._pr_server.stop(0)

    # -- inspection (tests, the harness) ---------------------------------------------------------
    def running(self) -> Dict[str, PodRun]:
        with self._lock:
            return {r.name: r for r in self.pods.values()}

    def all_pids(self) -> List[int]:
        with self._lock:
            runs = list(self.pods.values()) + list(self._terminating)
        return [pid for r in runs for pid in r.pids()]

    def cleanup(self) -> None:
        shutil.rmtree(self.base, ignore_errors=True)
