"""Spawned validation pods (reference: validator/main.go:931-1081, 1217-1293).

The validator creates a pod pinned to its node (``nodeName``), owned by the validator
DaemonSet's owners (so it is garbage-collected with the ClusterPolicy), tolerating what the
validator tolerates, with the validator's own image / pull policy / secrets / runtime class
(passed in by the operator through ``VALIDATOR_*`` env). It then waits for the pod to finish:
event-driven on a pod watch with a bounded timeout, where the reference polls 60 x 5 s.

The workload writes its JSON results to the termination message, which the validator reads
back from the pod status and stores in the barrier file -- also when the workload failed: the pods
run with ``restartPolicy: Never`` (a failing init container of an ``OnFailure`` pod is restarted with
crash-loop back-off and the pod stays ``Pending``; the reference's ``OnFailure``,
validator/cuda-workload-validation.yaml:13, turns a sick GPU into a 300 s timeout), and
``wait_for_pod`` returns at the first non-zero container exit whatever the policy.
"""

from __future__ import annotations

import copy
import json
import logging
import os
import threading
import time
from typing import Any, Callable, Dict, List, Optional


from ..k8s import errors
from ..k8s import objects as o

log = logging.getLogger("amd-validator.workload")

MANIFEST_DIRS = ["/var/amd/manifests", os.path.join(os.path.dirname(__file__), "manifests")]


def load_pod_spec(name: str) -> Dict[str, Any]:
    for d in MANIFEST_DIRS:
        p = os.path.join(d, name)
        if os.path.exists(p):
            import yaml        # only here: the validator's other components never parse YAML
            with open(p) as f:
                return yaml.safe_load(f)
    raise FileNotFoundError(f"validation pod manifest {name} not found in {MANIFEST_DIRS}")


def _validator_ds(client, namespace: str, app: str) -> Optional[Dict[str, Any]]:
    try:
        return client.get("apps/v1", "DaemonSet", app, namespace)
    except errors.NotFound:
        return None


def prepare_pod(client, template: Dict[str, Any], namespace: str, node: str, env: Dict[str, str],
                validator_app: str = "amd-operator-validator") -> Dict[str, Any]:
    pod = copy.deepcopy(template)
    md = o.meta(pod)
    md["namespace"] = namespace
    md["name"] = f"{md['name']}-{node}"[:63].rstrip("-")
    spec = pod.setdefault("spec", {})
    image = env.get("VALIDATOR_IMAGE", "")
    if not image:
        raise ValueError("VALIDATOR_IMAGE env not set")
    policy = env.get("VALIDATOR_IMAGE_PULL_POLICY", "IfNotPresent")
    for c in spec.get("initContainers", []) + spec.get("containers", []):
        c["image"] = image
        c["imagePullPolicy"] = policy
        # termination message carries the workload's JSON result
        c.setdefault("terminationMessagePolicy", "FallbackToLogsOnError")
    for c in spec.get("initContainers", []):
        # workload knobs (RCCL_RANKS, RCCL_MIN_BUSBW_GBPS, NCCL_*, ...) reach the workload process
        for k, v in sorted(env.items()):
            if not k.startswith("VALIDATOR_"):
                o.set_env(c, k, v)
    secrets = [s for s in env.get("VALIDATOR_IMAGE_PULL_SECRETS", "").split(",") if s]
    if secrets:
        spec["imagePullSecrets"] = [{"name": s} for s in secrets]
    if env.get("VALIDATOR_RUNTIME_CLASS"):
        spec["runtimeClassName"] = env["VALIDATOR_RUNTIME_CLASS"]
    spec["nodeName"] = node
    ds = _validator_ds(client, namespace, validator_app)
    if ds is not None:
        # owned like the validator DaemonSet (by the ClusterPolicy): GC'd with it
        owners = copy.deepcopy((ds.get("metadata") or {}).get("ownerReferences") or [])
        if owners:
            md["ownerReferences"] = owners
        tol = ((ds.get("spec") or {}).get("template") or {}).get("spec", {}).get("tolerations")
        if tol:
            spec["tolerations"] = copy.deepcopy(tol)
    return pod


class PodFailed(RuntimeError):
    """The validation pod failed: it ended ``Failed`` (``restartPolicy: Never``), or one of its
    containers exited non-zero while the pod had not (``OnFailure``: the kubelet would restart it with
    crash-loop back-off and the pod would stay ``Pending``, never ``Failed`` -- reason
    ``ContainerFailed``). ``reason`` is the pod's status.reason (the kubelet's admission rejection,
    e.g. ``UnexpectedAdmissionError`` / ``OutOfamd.com/gpu``) or ``ContainerFailed``; ``results``
    the JSON lines of the termination message (what the workload measured before it failed);
    ``exit_code`` the failing container's."""

    def __init__(self, msg: str, reason: str = "", results: Optional[List[Dict[str, Any]]] = None,
                 exit_code: Optional[int] = None, container: str = ""):
        super().__init__(msg)
        self.reason = reason
        self.results = results or []
        self.exit_code = exit_code
        self.container = container

    @property
    def admission(self) -> bool:
        return self.reason == "UnexpectedAdmissionError" or self.reason.startswith("OutOf")


class WorkloadAborted(RuntimeError):
    """The caller's abort check fired while the pod was waiting or running; the pod was deleted."""


def delete_stale(client, namespace: str, app: str, node: str) -> None:
    for p in client.list("v1", "Pod", namespace, label_selector={"app": app},
                         field_selector=f"spec.nodeName={node}"):
        try:
            client.delete("v1", "Pod", o.name(p), namespace, grace_period_seconds=0)
        except errors.NotFound:
            pass


def failed_container(pod: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """The first container (init containers first) that terminated with a non-zero exit code, now
    (``state``) or before a restart (``lastState``): ``{"name", "exitCode", "message", "restarts"}``."""
    st = pod.get("status") or {}
    for cs in (st.get("initContainerStatuses") or []) + (st.get("containerStatuses") or []):
        for key in ("state", "lastState"):
            term = (cs.get(key) or {}).get("terminated") or {}
            code = term.get("exitCode")
            if isinstance(code, int) and code != 0:
                return {"name": cs.get("name", ""), "exitCode": code, "message": term.get("message", ""),
                        "restarts": cs.get("restartCount", 0)}
    return None


def wait_for_pod(client, namespace: str, name: str, timeout: float = 300.0,
                 abort_check: Optional[Callable[[Dict[str, Any]], Optional[str]]] = None) -> Dict[str, Any]:
    """Block until the pod Succeeds (returns it), or raise: PodFailed as soon as the pod is
    ``Failed`` or any of its containers has exited non-zero (the validator never waits out a
    crash-loop back-off: reference validator/main.go:1042-1059 polls the phase only, and a failing
    init container of an ``OnFailure`` pod never gives it one), TimeoutError after ``timeout``.
    ``abort_check`` sees the current pod at least every 2 s; a non-empty reason raises
    WorkloadAborted."""
    done = threading.Event()
    state: Dict[str, Any] = {}

    def finished(pod: Dict[str, Any]) -> bool:
        return (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed") or failed_container(pod) is not None

    def on_event(ev):
        if o.name(ev.obj) != name or o.namespace(ev.obj) != namespace:
            return
        if ev.type == "DELETED":
            state["error"] = "pod deleted"
            done.set()
        elif finished(ev.obj):
            state["pod"] = ev.obj
            done.set()
    stop = client.watch("v1", "Pod", on_event, namespace=namespace)
    try:
        # the watch delivers the current object first; also re-check directly (fake clients)
        deadline = time.monotonic() + timeout
        while not done.is_set():
            try:
                cur = client.get("v1", "Pod", name, namespace)
                if finished(cur):
                    state["pod"] = cur
                    break
                why = abort_check(cur) if abort_check else None
                if why:
                    raise WorkloadAborted(why)
            except errors.NotFound:
                pass
            remaining = deadline - time.monotonic()
            if remaining <= 0:
                raise TimeoutError(f"pod {namespace}/{name} did not complete within {timeout:.0f}s")
            done.wait(min(remaining, 2.0))
    finally:
        stop()
    if "error" in state and "pod" not in state:
        raise RuntimeError(state["error"])
    pod = state["pod"]
    st = pod.get("status") or {}
    if st.get("phase") == "Succeeded":
        return pod
    bad = failed_container(pod)
    msg = termination_message(pod)
    why = ": ".join(x for x in (st.get("reason", ""), st.get("message", "")) if x)
    if bad is not None:
        why = why or f"container {bad['name']} exited {bad['exitCode']}"
    raise PodFailed(f"pod {name} failed{' (' + why + ')' if why else ''}: {msg}"[:2000],
                    reason=st.get("reason", "") or ("ContainerFailed" if st.get("phase") != "Failed" else ""),
                    results=parse_results(msg), exit_code=bad["exitCode"] if bad else None,
                    container=bad["name"] if bad else "")


def termination_message(pod: Dict[str, Any]) -> str:
    st = pod.get("status") or {}
    msgs = []
    for cs in (st.get("initContainerStatuses") or []) + (st.get("containerStatuses") or []):
        term = ((cs.get("state") or {}).get("terminated") or (cs.get("lastState") or {}).get("terminated") or {})
        if term.get("message"):
            msgs.append(term["message"])
    return "\n".join(msgs)


def parse_results(msg: str) -> List[Dict[str, Any]]:
    out = []
    for line in msg.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                out.append(json.loads(line))
            except ValueError:
                continue
    return out


def run_workload_pod(client, manifest: str, namespace: str, node: str, env: Dict[str, str],
                     timeout: float = 300.0, gpu_limit: Optional[Dict[str, int]] = None,
                     privileged: bool = False,
                     abort_check: Optional[Callable[[Dict[str, Any]], Optional[str]]] = None) -> Dict[str, Any]:
    """``gpu_limit``: GPU resources the workload container requests through the scheduler;
    ``privileged``: the container sees every device instead (AMD_VISIBLE_DEVICES=all in ``env``);
    ``abort_check``: see wait_for_pod -- on an abort the pod is deleted before WorkloadAborted
    propagates."""
    template = load_pod_spec(manifest)
    pod = prepare_pod(client, template, namespace, node, env)
    for c in pod["spec"].get("initContainers", []):
        if gpu_limit:
            c.setdefault("resources", {})["limits"] = dict(gpu_limit)
        if privileged:
            c.setdefault("securityContext", {})["privileged"] = True
    app = o.get_labels(pod).get("app", "")
    delete_stale(client, namespace, app, node)
    client.create(pod)
    log.info("created validation pod %s/%s", namespace, o.name(pod))
    try:
        done = wait_for_pod(client, namespace, o.name(pod), timeout, abort_check=abort_check)
    except (WorkloadAborted, PodFailed, TimeoutError) as e:
        # withdrawn, failed (a pod the kubelet would restart must not re-run the workload behind
        # the validator's back) or timed out: the pod goes
        if not isinstance(e, PodFailed) or e.reason == "ContainerFailed" or \
                (template.get("spec") or {}).get("restartPolicy", "Always") != "Never":
            try:
                client.delete("v1", "Pod", o.name(pod), namespace, grace_period_seconds=0)
            except errors.NotFound:
                pass
        raise
    return {"pod": o.name(pod), "results": parse_results(termination_message(done))}
