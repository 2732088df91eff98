"""Node time-to-ready: the bring-up chain of one GPU node, measured end to end.

BASELINE.json's metric is "node time-to-ready (driver -> validator)". This harness runs the
REAL node-side components of this framework concurrently, the way their DaemonSet pods start
together on a fresh node, and wires them only through what they use in production — the
barrier directory (inotify waits), a Kubernetes API (in-process fake), the kubelet device-plugin
gRPC API (an in-process fake kubelet that registers plugins and mirrors ListAndWatch into the
Node's capacity) and the GPUs themselves:

    validator      driver check -> toolkit check -> HIP smoke + MFMA GEMM (real GPU) -> plugin
                   (event-driven wait for amd.com/gpu capacity) -> rccl (>=2 GPUs) -> ready
    toolkit        waits driver-ready -> amd-ctk install (runtime shim + config edit)
    device plugin  waits toolkit-ready -> discovers KFD agents -> registers -> ListAndWatch
    labeller       waits toolkit-ready -> labels the Node
    exporter       waits toolkit-ready -> first scrape

The host's amdgpu driver is used (the reference's host-driver mode); the
driver container's own load time is not part of this measurement.

The same measured step durations are then fed to a model of the reference's chain with its
fixed constants: 5 s barrier polling in init containers, the 5 s
toolkit sleep, toolkit validation by crash-loop back-off (10 s, 20 s, ...), 5 s polls for the
CUDA workload pod and for GPU capacity, the device plugin's 5 s poll for toolkit-ready.
"""

from __future__ import annotations

import json
import logging
import math
import os
import tempfile
import threading
import time
from concurrent import futures
from typing import Dict, List, Optional

from .. import devices
from ..k8s.fake import FakeClient
from . import components as Cm
from . import status as S

log = logging.getLogger("amd-ttr")


class FakeKubelet:
    """Registration server + a ListAndWatch client per registered plugin that mirrors the
    healthy device count into the Node's capacity/allocatable (what kubelet does)."""

    def __init__(self, plugin_dir: str, client, node: str):
        import grpc
        from ..operands import kubeletapi as K
        self.K = K
        self.grpc = grpc
        self.plugin_dir = plugin_dir
        self.client = client
        self.node = node
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        self.server.add_generic_rpc_handlers((K.registration_handler(self._on_register),))
        self.server.add_insecure_port("unix://" + os.path.join(plugin_dir, "kubelet.sock"))
        self.threads: List[threading.Thread] = []
        self._stop = threading.Event()

    def start(self):
        self.server.start()

    def _on_register(self, req):
        t = threading.Thread(target=self._watch, args=(req.endpoint, req.resource_name), daemon=True)
        t.start()
        self.threads.append(t)

    def _watch(self, endpoint: str, resource: str):
        K = self.K
        with self.grpc.insecure_channel("unix://" + os.path.join(self.plugin_dir, endpoint)) as ch:
            stream = K.device_plugin_stub(ch)["ListAndWatch"](K.DP["Empty"]())
            for resp in stream:
                n = sum(1 for d in resp.devices if d.health == K.HEALTHY)
                self.client.patch("v1", "Node", self.node, {"status": {"capacity": {resource: str(n)},
                                                                       "allocatable": {resource: str(n)}}})
                if self._stop.is_set():
                    stream.cancel()
                    break

    def stop(self):
        self._stop.set()
        self.server.stop(0)


def _node(name: str) -> Dict:
    return {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": name, "labels": {"feature.node.kubernetes.io/pci-1002.present": "true",
                                                   "amd.com/gpu.present": "true"}},
            "status": {"capacity": {}, "allocatable": {}}}


def run_chain(workdir: Optional[str] = None, gemm_shapes: str = "8192", sys_root: str = "/",
              dev_root: str = "/", hip_mode: str = "local", timeout: float = 300.0) -> Dict:
    """Run the node chain once; returns timestamps relative to t0 and the step durations."""
    from ..operands.device_plugin import Config as DPConfig, DevicePlugin
    from ..operands.metrics_exporter import build_registry, load_fields
    from ..operands.node_labeller import apply_node, compute_labels
    from ..toolkit.ctk import Installer

    wd = workdir or tempfile.mkdtemp(prefix="amd-ttr-")
    vdir = os.path.join(wd, "validations")
    pdir = os.path.join(wd, "device-plugins")
    os.makedirs(pdir, exist_ok=True)
    sd = S.StatusDir(vdir)
    sd.ensure()
    node = "ttr-node"
    client = FakeClient([_node(node)])
    kubelet = FakeKubelet(pdir, client, node)
    kubelet.start()
    marks: Dict[str, float] = {}
    steps: Dict[str, float] = {}
    errors: List[str] = []
    lock = threading.Lock()

    def mark(name: str, t: float):
        with lock:
            marks[name] = t

    env = dict(os.environ, HIP_VALIDATION_MODE=hip_mode, GEMM_SHAPES=gemm_shapes, DRIVER_ROOT_MODE="host",
               DRIVER_VALIDATION_STRICT="false")
    ctx = Cm.Context(status=sd, node_name=node, namespace="amd-gpu-operator", client=client, host_root="/",
                     sys_root=sys_root, dev_root=dev_root, with_wait=True, wait_timeout=timeout,
                     resource_timeout=timeout, env=env)
    plugin: Dict[str, DevicePlugin] = {}
    t0 = time.monotonic()

    def timed(name, fn):
        s = time.monotonic()
        r = fn()
        steps[name] = time.monotonic() - s
        mark(name, time.monotonic() - t0)
        return r

    def validator():
        try:
            timed("driver", lambda: Cm.validate_driver(ctx))
            timed("toolkit_validation", lambda: (sd.wait([".toolkit-installed"], timeout=timeout),
                                                 Cm.validate_toolkit(ctx)))
            if hip_mode == "skip":      # CPU tests: no GPU work
                timed("hip", lambda: sd.create(S.HIP_READY, {"skipped": True}))
            else:
                timed("hip", lambda: Cm.validate_hip(ctx))
            timed("plugin_validation", lambda: Cm.validate_plugin(ctx))
            ngpu = len({g["pci_bdf"] for g in devices.enumerate_gpus(sys_root)})   # KFD-visible GPUs
            if ngpu >= 2 and hip_mode == "local":
                from .workload_main import run_rccl
                timed("rccl", lambda: run_rccl(64 << 20, "bf16"))
            sd.create("validator-ready", {"ok": True})
            mark("ready", time.monotonic() - t0)
        except Exception as e:  # noqa: BLE001
            errors.append(f"validator: {e}")
            sd.create(".abort")

    def toolkit():
        try:
            got = sd.wait([S.DRIVER_READY, S.HOST_DRIVER_READY, ".abort"], any_of=True, timeout=timeout)
            if ".abort" in got or not got:
                return
            cfgf = os.path.join(wd, "containerd", "config.toml")
            inst = Installer(root=os.path.join(wd, "usr-local-amd"), runtime="containerd", runtime_config=cfgf,
                             runtime_socket=os.path.join(wd, "containerd.sock"), restart_mode="none",
                             sys_root=sys_root, dev_root=dev_root)
            timed("toolkit_install", inst.install)
            sd.create(".toolkit-installed")
        except Exception as e:  # noqa: BLE001
            errors.append(f"toolkit: {e}")

    def device_plugin():
        try:
            got = sd.wait([S.TOOLKIT_READY, ".abort"], any_of=True, timeout=timeout)
            if S.TOOLKIT_READY not in got:
                return

            def start():
                p = DevicePlugin(DPConfig.load(None, {}), root=sys_root, plugin_dir=pdir)
                p.start(register=True)
                plugin["p"] = p
            timed("device_plugin_start", start)
        except Exception as e:  # noqa: BLE001
            errors.append(f"device-plugin: {e}")

    def labeller():
        try:
            got = sd.wait([S.TOOLKIT_READY, ".abort"], any_of=True, timeout=timeout)
            if S.TOOLKIT_READY not in got:
                return
            timed("labeller", lambda: apply_node(client, node, compute_labels(sys_root)))
        except Exception as e:  # noqa: BLE001
            errors.append(f"labeller: {e}")

    def exporter():
        try:
            got = sd.wait([S.TOOLKIT_READY, ".abort"], any_of=True, timeout=timeout)
            if S.TOOLKIT_READY not in got:
                return
            from prometheus_client import generate_latest
            timed("exporter_first_scrape", lambda: generate_latest(build_registry(load_fields(None), sys_root)))
        except Exception as e:  # noqa: BLE001
            errors.append(f"exporter: {e}")

    threads = [threading.Thread(target=f, daemon=True) for f in (validator, toolkit, device_plugin, labeller, exporter)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout + 10)
    if "p" in plugin:
        plugin["p"].stop()
    kubelet.stop()
    barriers = {}
    for b in (S.HOST_DRIVER_READY, S.DRIVER_READY, S.TOOLKIT_READY, S.HIP_READY, S.PLUGIN_READY, "validator-ready"):
        p = sd.read(b)
        if p and "ts" in p:
            barriers[b] = p["ts"]
    hip = sd.read(S.HIP_READY) or {}
    return {"time_to_ready_s": marks.get("ready"), "marks_s": {k: round(v, 4) for k, v in sorted(marks.items(),
                                                                                             key=lambda kv: kv[1])},
            "steps_s": {k: round(v, 4) for k, v in steps.items()}, "errors": errors,
            "gemm_tflops_per_gpu": hip.get("gemm_tflops_per_gpu"), "gpus": hip.get("gpus"),
            "capacity": (client.get("v1", "Node", node).get("status") or {}).get("capacity")}


# ---------------------------------------------------------------------------------------------
# the reference's chain, same step durations, its fixed delays and polling periods
# ---------------------------------------------------------------------------------------------
POLL = 5.0                 # init containers / --with-wait / capacity / workload pod (validator/main.go:127,159,163)
TOOLKIT_SLEEP = 5.0        # assets/state-container-toolkit/0400_configmap.yaml:34
BACKOFF = [10.0, 20.0, 40.0, 80.0, 160.0, 300.0]   # kubelet crash-loop back-off (toolkit validation)
POD_START = 1.0            # container start of a spawned workload pod (image cached)


def _next_poll(t_ready: float, t_start: float, period: float = POLL) -> float:
    """First poll tick (start + k*period, k>=0) at or after t_ready."""
    if t_ready <= t_start:
        return t_start
    return t_start + math.ceil((t_ready - t_start) / period) * period


def reference_model(steps: Dict[str, float]) -> Dict[str, float]:
    d = steps.get("driver", 0.5)
    tk_install = steps.get("toolkit_install", 0.5)
    tk_check = max(steps.get("toolkit_validation", 0.1) - 0.0, 0.05)
    hip = steps.get("hip", 2.0)
    dp_start = steps.get("device_plugin_start", 0.2)
    # toolkit DaemonSet: driver-validation (first check immediate) -> sleep 5 -> install
    toolkit_ready_at = d + TOOLKIT_SLEEP + tk_install
    # validator: driver (d) -> toolkit validation without wait: crash-loops until the hook works
    t = d
    attempt = 0
    while t + tk_check < toolkit_ready_at:
        t = t + tk_check + BACKOFF[min(attempt, len(BACKOFF) - 1)] + d   # restart reruns driver-validation
        attempt += 1
    t_toolkit_ok = t + tk_check
    # device plugin: init container polls toolkit-ready every 5 s from pod start (t=0)
    dp_registered = _next_poll(t_toolkit_ok, 0.0) + dp_start
    # cuda validation: spawn pod, poll its phase every 5 s
    t_cuda_start = t_toolkit_ok
    t_cuda_done = _next_poll(t_cuda_start + POD_START + hip, t_cuda_start)
    # plugin validation: poll node capacity every 5 s (first check immediately)
    t_plugin = _next_poll(max(dp_registered, t_cuda_done), t_cuda_done)
    return {"time_to_ready_s": round(t_plugin, 3), "toolkit_crashloops": attempt,
            "toolkit_ready_s": round(toolkit_ready_at, 3), "device_plugin_registered_s": round(dp_registered, 3),
            "cuda_validation_done_s": round(t_cuda_done, 3)}


def main(argv=None) -> int:
    import argparse
    logging.basicConfig(level=logging.WARNING)
    ap = argparse.ArgumentParser(prog="amd-ttr")
    ap.add_argument("--gemm-shapes", default="8192")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=120.0)
    a = ap.parse_args(argv)
    for i in range(a.runs):
        r = run_chain(gemm_shapes=a.gemm_shapes, timeout=a.timeout)
        r["reference_model"] = reference_model(r["steps_s"])
        r["run"] = i
        print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(main())
