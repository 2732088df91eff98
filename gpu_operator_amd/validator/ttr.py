"""Node time-to-ready, measured on real processes: the bring-up of one GPU node from "operand
pods scheduled" to "validator Ready", run twice in the same harness -- once with this
framework's protocol and once with the reference's protocol constants executed.

BASELINE.json's metric is "node time-to-ready (driver -> validator)"; the reference's timing
envelope is the sum of its fixed sleeps, 5 s polls and crash-loop back-offs.

What is real
  * every container is its own OS process started through its console-script name
    (``amd-validator``, ``amd-ctk``, ``amd-device-plugin``, ``amd-node-labeller``,
    ``amd-metrics-exporter``: one-line wrappers on PATH around cmd/entry.py), init containers
    run in order, main containers concurrently;
  * the entrypoint scripts are the ConfigMap scripts of this repo's assets, run by ``sh`` with
    their hostPath volumes mapped to the harness's directories; init gates are the native
    ``amd-barrier-wait`` binary (inotify);
  * the agents talk to a Kubernetes API over HTTP (the in-process API server of k8s/apiserver.py,
    through RestClient and a kubeconfig) and to a kubelet device-plugin gRPC endpoint (a fake
    kubelet that registers plugins and mirrors ListAndWatch into the Node's capacity, as kubelet
    does); the device plugin, labeller and exporter read the GPUs through libamdnode, and the
    validator's HIP check runs the MFMA GEMM probe on the GPU (``HIP_VALIDATION_MODE=local``;
    ``skip`` on CPU-only rehearsals).

What is simulated (identically for both protocols) -- and reported apart from the measurement
  * the container runtime: pods with ``runtimeClassName`` (validator, device plugin, labeller,
    exporter) cannot start until ``amd-ctk install`` has put the runtime handler into the
    (harness-local) containerd config -- the kubelet retries sandbox creation every
    KUBELET_SYNC_S; a failing init container restarts with kubelet's crash-loop back-off;
  * every run reports ``time_to_ready_modelled_s``: the time the validator pod's critical path spent
    in those simulated waits -- its sandbox retries after the runtime handler was already
    configured (the KUBELET_SYNC_S tick) and any crash-loop back-off of its init containers -- and
    ``time_to_ready_measured_s``, the rest: processes, API calls, barriers and the GPU work;
  * the host driver is already live (the box's preinstalled amdgpu: the reference's host-driver
    mode), so the driver DaemonSet's module load is not part of the measurement; its startup
    probe ``amdgpu-driver probe`` still gates ``.driver-ctr-ready`` in the ``driver-container``
    scenario.

The reference protocol (host driver), from its assets and validator: init gates poll every 5 s
(assets/state-device-plugin/0500_daemonset.yaml:31), the toolkit entrypoint sleeps 5 s
(assets/state-container-toolkit/0400_configmap.yaml:34), the device-plugin entrypoint polls for
the driver barrier every 5 s (assets/state-device-plugin/0400_configmap.yaml:9-36), the validator
retries with 5 s sleeps and polls workload pods and node capacity every 5 s
(validator/main.go:127,556-572,1042-1059,1102-1122), toolkit validation runs without wait
(crash-loop back-off), and plugin validation runs a second workload (WITH_WORKLOAD=true). The
driver container's startup probe starts after 60 s and repeats every 10 s
(assets/state-driver/0500_daemonset.yaml:132-140). Here those constants are executed by our own
agents in the reference's wait mode (``VALIDATOR_WAIT_MODE=poll``), not modelled.
"""

from __future__ import annotations

import json
import logging
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time
from concurrent import futures
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import yaml

from . import status as S

log = logging.getLogger("amd-ttr")

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ASSETS = os.path.join(REPO, "gpu_operator_amd", "assets")
NATIVE_BIN = os.path.join(REPO, "gpu_operator_amd", "_native", "bin")

KUBELET_SYNC_S = 1.0                              # harness kubelet: sandbox-creation retry period
CONTAINER_POLL_S = 0.005                          # harness kubelet: container-exit detection granularity
CRASHLOOP_BACKOFF_S = [10.0, 20.0, 40.0, 80.0, 160.0, 300.0]   # kubelet container restart back-off
NODE = "ttr-node"
NAMESPACE = "amd-gpu-operator"


@dataclass
class Ctr:
    name: str
    argv: List[str]
    env: Dict[str, str] = field(default_factory=dict)


@dataclass
class Probe:
    argv: List[str]
    initial_delay: float
    period: float


@dataclass
class Pod:
    name: str
    inits: List[Ctr]
    mains: List[Ctr]
    runtime_class: bool = False
    startup_probe: Optional[Probe] = None


# ---------------------------------------------------------------------------------------------
# kubelet-side fakes
# ---------------------------------------------------------------------------------------------
class FakeKubelet:
    """Device-plugin registration server + a ListAndWatch client per registered plugin that
    mirrors the healthy device count into the Node's capacity/allocatable (what kubelet does)."""

    def __init__(self, plugin_dir: str, client, node: str, on_event=None):
        import grpc
        from ..operands import kubeletapi as K
        self.K = K
        self.grpc = grpc
        self.plugin_dir = plugin_dir
        self.client = client
        self.node = node
        self.on_event = on_event or (lambda name: None)
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        self.server.add_generic_rpc_handlers((K.registration_handler(self._on_register),))
        self.server.add_insecure_port("unix://" + os.path.join(plugin_dir, "kubelet.sock"))
        self._stop = threading.Event()

    def start(self):
        self.server.start()

    def _on_register(self, req):
        self.on_event(f"kubelet:registered:{req.resource_name}")
        threading.Thread(target=self._watch, args=(req.endpoint, req.resource_name), daemon=True).start()

    def _watch(self, endpoint: str, resource: str):
        K = self.K
        try:
            with self.grpc.insecure_channel("unix://" + os.path.join(self.plugin_dir, endpoint)) as ch:
                stream = K.device_plugin_stub(ch)["ListAndWatch"](K.DP["Empty"]())
                for resp in stream:
                    n = sum(1 for d in resp.devices if d.health == K.HEALTHY)
                    # marked as the PATCH goes out: a validator polling the Node can see the new
                    # capacity before this thread gets the response back
                    self.on_event(f"kubelet:capacity:{resource}={n}")
                    self.client.patch("v1", "Node", self.node, {"status": {"capacity": {resource: str(n)},
                                                                           "allocatable": {resource: str(n)}}})
                    if self._stop.is_set():
                        stream.cancel()
                        break
        except Exception as e:  # noqa: BLE001 - the plugin went away at teardown
            if not self._stop.is_set():
                log.warning("ListAndWatch %s ended: %s", resource, e)

    def stop(self):
        self._stop.set()
        self.server.stop(0)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _asset_script(state: str, fname: str) -> str:
    with open(os.path.join(ASSETS, state, fname)) as f:
        return yaml.safe_load(f)["data"]["entrypoint.sh"]


# ---------------------------------------------------------------------------------------------
# the harness
# ---------------------------------------------------------------------------------------------
class Harness:
    def __init__(self, workdir: Optional[str] = None, sys_root: str = "/", dev_root: str = "/",
                 hip_mode: str = "local", gemm_shapes: str = "8192", timeout: float = 240.0,
                 scenario: str = "host-driver", hip_full: bool = False):
        """``hip_full``: our validator's HIP check runs what the production pod runs (bf16 and fp8,
        the 1/2/4/8 sweep, one rocprofv3 counter pass per dtype) instead of one bf16 shape."""
        if scenario not in ("host-driver", "driver-container"):
            raise ValueError(f"unknown scenario {scenario!r}")
        self.hip_env = ({"GEMM_DTYPE": "both", "GEMM_SCALING": "1,2,4,8", "GEMM_COUNTERS": "1"} if hip_full
                        else {})
        self.wd = workdir or tempfile.mkdtemp(prefix="amd-ttr-")
        self.sys_root, self.dev_root = sys_root, dev_root
        self.hip_mode, self.gemm_shapes, self.timeout, self.scenario = hip_mode, gemm_shapes, timeout, scenario
        self.marks: Dict[str, float] = {}
        self.restarts: Dict[str, int] = {}
        self.errors: List[str] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._procs: List[subprocess.Popen] = []
        self.modelled: Dict[str, Dict[str, float]] = {}     # pod -> simulated waits on its path (s)

    # -- bookkeeping -----------------------------------------------------------------------------
    def mark(self, name: str) -> None:
        with self._lock:
            self.marks.setdefault(name, round(time.monotonic() - self.t0, 4))

    def _setup(self, tag: str) -> None:
        base = os.path.join(self.wd, tag)
        shutil.rmtree(base, ignore_errors=True)
        self.base = base
        self.vdir = os.path.join(base, "validations")
        self.pdir = os.path.join(base, "device-plugins")
        self.amd_root = os.path.join(base, "usr-local-amd")
        self.cfg = os.path.join(base, "containerd", "config.toml")
        self.bin = os.path.join(base, "bin")
        self.logs = os.path.join(base, "logs")
        for d in (self.vdir, self.pdir, self.amd_root, os.path.dirname(self.cfg), self.bin, self.logs,
                  os.path.join(base, "cdi")):
            os.makedirs(d, exist_ok=True)
        from ..cmd.entry import install_wrappers
        install_wrappers(self.bin)
        # the API server (HTTP) with this node, and a kubeconfig for the agents
        from ..k8s.apiserver import FakeAPIServer
        from ..k8s.fake import FakeClient
        node = {"apiVersion": "v1", "kind": "Node",
                "metadata": {"name": NODE, "labels": {"feature.node.kubernetes.io/pci-1002.present": "true",
                                                      "amd.com/gpu.present": "true"}},
                "status": {"capacity": {}, "allocatable": {}}}
        ns = {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NAMESPACE}}
        self.backing = FakeClient([ns, node])
        self.api = FakeAPIServer(self.backing).start()
        self.kubeconfig = os.path.join(base, "kubeconfig")
        with open(self.kubeconfig, "w") as f:
            yaml.safe_dump({"apiVersion": "v1", "kind": "Config", "current-context": "ttr",
                            "clusters": [{"name": "ttr", "cluster": {"server": self.api.url}}],
                            "contexts": [{"name": "ttr", "context": {"cluster": "ttr", "user": "ttr"}}],
                            "users": [{"name": "ttr", "user": {}}]}, f)
        from ..k8s.rest import Config, RestClient
        self.client = RestClient(Config.from_kubeconfig(self.kubeconfig))
        self.kubelet = FakeKubelet(self.pdir, self.client, NODE, on_event=self.mark)
        self.kubelet.start()

        from ..k8s import objects as o

        def on_node(ev):
            if o.get_labels(ev.obj).get("amd.com/gpu.gfx"):
                self.mark("node:labelled")
        self.backing.watch("v1", "Node", on_node)
        self.env = dict(os.environ)
        self.env.update({
            "PATH": f"{self.bin}:{os.environ.get('PATH', '/usr/bin:/bin')}",
            "PYTHONPATH": REPO + (os.pathsep + os.environ["PYTHONPATH"] if os.environ.get("PYTHONPATH") else ""),
            "KUBECONFIG": self.kubeconfig, "NODE_NAME": NODE, "OPERATOR_NAMESPACE": NAMESPACE,
            "OUTPUT_DIR": self.vdir, "AMD_SYSFS_ROOT": self.sys_root, "AMD_DEV_ROOT": self.dev_root,
            "HIP_VALIDATION_MODE": self.hip_mode, "GEMM_SHAPES": self.gemm_shapes,
            "DRIVER_ROOT_MODE": "host" if self.scenario == "host-driver" else "container",
            "DRIVER_VALIDATION_STRICT": "false", "WAIT_TIMEOUT_SECONDS": str(int(self.timeout)),
            "ROOT": self.amd_root, "RUNTIME": "containerd", "RUNTIME_CONFIG": self.cfg,
            "RUNTIME_SOCKET": os.path.join(base, "containerd.sock"), "RESTART_MODE": "none",
            "CDI_SPEC_DIR": os.path.join(base, "cdi"), "NO_CLEANUP": "true", "PYTHONUNBUFFERED": "1",
            "HSA_ENABLE_IPC_MODE_LEGACY": "0", "LABELLER_OUTPUT": "node",
        })

    def _teardown(self) -> None:
        self._stop.set()
        for p in self._procs:          # every container is its own process group (its session)
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
        deadline = time.monotonic() + 5
        for p in self._procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                p.wait()
        self.kubelet.stop()
        self.api.stop()

    # -- pod runtime ------------------------------------------------------------------------------
    def _map(self, text: str) -> str:
        """hostPath volumes -> harness directories."""
        return (text.replace("/run/amd/validations", self.vdir).replace("/run/amd/driver", os.path.join(self.base, "driver"))
                .replace("/var/lib/kubelet/device-plugins", self.pdir))

    def runtime_ready(self) -> bool:
        shim = os.path.join(self.amd_root, "toolkit", "amd-container-runtime")
        try:
            with open(self.cfg) as f:
                cfg = f.read()
        except OSError:
            return False
        return os.path.exists(shim) and "amd-container-runtime" in cfg

    def _spawn(self, pod: Pod, c: Ctr) -> subprocess.Popen:
        env = dict(self.env)
        env.update(c.env)
        logf = open(os.path.join(self.logs, f"{pod.name}.{c.name}.log"), "ab")
        p = subprocess.Popen([self._map(a) for a in c.argv], env=env, stdout=logf, stderr=subprocess.STDOUT,
                             start_new_session=True)
        logf.close()
        with self._lock:
            self._procs.append(p)
        return p

    def _sleep(self, s: float) -> bool:
        return not self._stop.wait(s)

    def _model(self, pod: str, what: str, seconds: float) -> None:
        with self._lock:
            d = self.modelled.setdefault(pod, {})
            d[what] = round(d.get(what, 0.0) + max(0.0, seconds), 4)

    def _watch_runtime(self) -> None:
        """When the runtime handler became usable (fine-grained): the start of each runtime-class
        pod's modelled sandbox-retry wait."""
        while not self._stop.is_set():
            if self.runtime_ready():
                self.mark("runtime:ready")
                return
            self._stop.wait(CONTAINER_POLL_S)

    def _run_pod(self, pod: Pod) -> None:
        try:
            if pod.runtime_class:
                t_wait = time.monotonic()
                while not self.runtime_ready():
                    if not self._sleep(KUBELET_SYNC_S):
                        return
                # the part of the wait after the handler existed is the harness kubelet's retry tick
                ready_at = self.marks.get("runtime:ready")
                if ready_at is not None:
                    self._model(pod.name, "sandbox_retry_s", time.monotonic() - max(t_wait, self.t0 + ready_at))
            self.mark(f"{pod.name}:started")
            for c in pod.inits:
                attempt = 0
                while True:
                    p = self._spawn(pod, c)
                    # the exit of an init container is seen within CONTAINER_POLL_S (measurement
                    # granularity, the same for both protocols)
                    while p.poll() is None:
                        if self._stop.wait(CONTAINER_POLL_S):
                            return
                    if p.returncode == 0:
                        break
                    key = f"{pod.name}:{c.name}"
                    self.restarts[key] = self.restarts.get(key, 0) + 1
                    backoff = CRASHLOOP_BACKOFF_S[min(attempt, len(CRASHLOOP_BACKOFF_S) - 1)]
                    self._model(pod.name, "crashloop_backoff_s", backoff)
                    if not self._sleep(backoff):
                        return
                    attempt += 1
                self.mark(f"{pod.name}:{c.name}:done")
            for c in pod.mains:
                self._spawn(pod, c)
                self.mark(f"{pod.name}:{c.name}:started")
            if pod.startup_probe is not None:
                pr = pod.startup_probe
                if not self._sleep(pr.initial_delay):
                    return
                while True:
                    env = dict(self.env)
                    if subprocess.run([self._map(a) for a in pr.argv], env=env, capture_output=True,
                                      timeout=60).returncode == 0:
                        self.mark(f"{pod.name}:startup-probe:ok")
                        break
                    if not self._sleep(pr.period):
                        return
        except Exception as e:  # noqa: BLE001
            self.errors.append(f"{pod.name}: {e}")

    def _scrape_exporter(self, port: int) -> None:
        import urllib.request
        while not self._stop.is_set():
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2) as r:
                    if r.status == 200 and b"amd_gpu_" in r.read():
                        self.mark("exporter:first-scrape")
                        return
            except OSError:
                pass
            self._stop.wait(0.05)

    # -- protocols --------------------------------------------------------------------------------
    def pods_ours(self, port: int) -> List[Pod]:
        """This framework's operand pods (gpu_operator_amd/assets, container workload)."""
        gate = ["amd-barrier-wait", "--dir", "/run/amd/validations", "--all", "toolkit-ready", "--timeout", "3600"]
        v = lambda comp, **e: Ctr(f"{comp}-validation", ["amd-validator"], dict({"COMPONENT": comp}, **e))  # noqa: E731
        # as in the assets: the API-free checks are the static amd-node-validate, the rccl init
        # container falls through to amd-validator when there is a fabric to prove
        nv = lambda comp, **e: Ctr(f"{comp}-validation", ["amd-node-validate", comp], dict({"COMPONENT": comp}, **e))  # noqa: E731
        fast = lambda comp, **e: Ctr(f"{comp}-validation", ["sh", "-c", f'amd-node-validate {comp}; rc=$?; '  # noqa: E731
                                                             '[ "$rc" -eq 3 ] && exec amd-validator; exit "$rc"'],
                                     dict({"COMPONENT": comp}, **e))
        pods = [
            Pod("toolkit", [nv("driver", WITH_WAIT="true")],
                [Ctr("amd-container-toolkit-ctr",
                     ["sh", "-c", self._map(_asset_script("state-container-toolkit", "0400_configmap.yaml"))])]),
            Pod("validator", [nv("driver", WITH_WAIT="true"), nv("toolkit", WITH_WAIT="true"), v("hip", **self.hip_env),
                              fast("plugin", WITH_WORKLOAD="false"), fast("rccl")],
                [Ctr("amd-operator-validator", ["amd-validator", "--component", "ready"])], runtime_class=True),
            Pod("device-plugin", [Ctr("toolkit-validation", gate)],
                [Ctr("amd-device-plugin", ["sh", "-c", self._map(_asset_script("state-device-plugin",
                                                                                "0400_configmap.yaml")),
                                           "entrypoint", "--plugin-dir", self.pdir])], runtime_class=True),
            Pod("node-labeller", [Ctr("toolkit-validation", gate)],
                [Ctr("amd-node-labeller", ["amd-node-labeller", "--output", "node", "--barrier-dir", self.vdir])],
                runtime_class=True),
            Pod("metrics-exporter", [Ctr("toolkit-validation", gate)],
                [Ctr("amd-metrics-exporter", ["amd-metrics-exporter", "--listen", f"127.0.0.1:{port}"])],
                runtime_class=True),
        ]
        if self.scenario == "driver-container":
            pods.insert(0, Pod("driver", [], [Ctr("amdgpu-driver-ctr", ["sleep", "infinity"])],
                               startup_probe=Probe(["sh", "-c", "amdgpu-driver probe && touch "
                                                    "/run/amd/validations/.driver-ctr-ready"], 0.0, 2.0)))
        return pods

    def pods_reference(self, port: int) -> List[Pod]:
        """The reference's operand protocol executed with our agents (see module doc)."""
        poll = lambda f: f"until [ -f /run/amd/validations/{f} ]; do sleep 5; done"  # noqa: E731
        gate = ["sh", "-c", poll("toolkit-ready")]
        ref = {"VALIDATOR_WAIT_MODE": "poll", "SLEEP_INTERVAL_SECONDS": "5"}
        v = lambda comp, **e: Ctr(f"{comp}-validation", ["amd-validator"], dict(ref, COMPONENT=comp, **e))  # noqa: E731
        toolkit = ("driver_root=/run/amd/driver; if [ -f /run/amd/validations/host-driver-ready ]; then "
                   "driver_root=/; fi; export AMD_DRIVER_ROOT=$driver_root; sleep 5; exec amd-ctk install --daemon")
        plugin = ("while true; do if [ -f /run/amd/validations/host-driver-ready ] || "
                  "[ -f /run/amd/validations/driver-ready ]; then break; fi; sleep 5; done; "
                  "exec amd-device-plugin \"$@\"")
        pods = [
            Pod("toolkit", [v("driver", WITH_WAIT="true")], [Ctr("toolkit-ctr", ["sh", "-c", self._map(toolkit)])]),
            Pod("validator", [v("driver", WITH_WAIT="true"), v("toolkit", WITH_WAIT="false"), v("hip"),
                              v("plugin", WITH_WORKLOAD="true")],
                [Ctr("validator", ["amd-validator", "--component", "ready"])], runtime_class=True),
            Pod("device-plugin", [Ctr("toolkit-validation", gate)],
                [Ctr("device-plugin", ["sh", "-c", self._map(plugin), "entrypoint", "--plugin-dir", self.pdir])],
                runtime_class=True),
            Pod("node-labeller", [Ctr("toolkit-validation", gate)],
                [Ctr("gfd", ["amd-node-labeller", "--output", "node", "--barrier-dir", self.vdir])], runtime_class=True),
            Pod("metrics-exporter", [Ctr("toolkit-validation", gate)],
                [Ctr("dcgm-exporter", ["amd-metrics-exporter", "--listen", f"127.0.0.1:{port}"])], runtime_class=True),
        ]
        if self.scenario == "driver-container":
            pods.insert(0, Pod("driver", [], [Ctr("driver-ctr", ["sleep", "infinity"])],
                               startup_probe=Probe(["sh", "-c", "amdgpu-driver probe && touch "
                                                    "/run/amd/validations/.driver-ctr-ready"], 60.0, 10.0)))
        return pods

    def run(self, protocol: str = "ours") -> Dict:
        self._stop.clear()
        self._procs = []
        self.marks, self.restarts, self.errors, self.modelled = {}, {}, [], {}
        self._setup(protocol)
        port = _free_port()
        pods = self.pods_ours(port) if protocol == "ours" else self.pods_reference(port)
        self.t0 = time.monotonic()
        self.t0_wall = time.time()
        threads = [threading.Thread(target=self._run_pod, args=(p,), daemon=True) for p in pods]
        threads.append(threading.Thread(target=self._scrape_exporter, args=(port,), daemon=True))
        threads.append(threading.Thread(target=self._watch_runtime, daemon=True))
        for t in threads:
            t.start()
        ready_key = "validator:amd-operator-validator:started" if protocol == "ours" else "validator:validator:started"
        deadline = self.t0 + self.timeout
        while time.monotonic() < deadline and ready_key not in self.marks and not self.errors:
            if any(self.restarts.get(f"validator:{c}", 0) > 5 for c in ("hip-validation", "plugin-validation")):
                break
            time.sleep(0.02)
        # let the concurrent operands finish their first action (bounded) for the breakdown
        settle = time.monotonic() + 15
        while time.monotonic() < settle and not {"node:labelled", "exporter:first-scrape"} <= set(self.marks):
            time.sleep(0.05)
        self._teardown()
        barriers = {}
        sd = S.StatusDir(self.vdir)
        for b in (S.DRIVER_CTR_READY, S.HOST_DRIVER_READY, S.DRIVER_READY, S.TOOLKIT_READY, S.HIP_READY,
                  S.PLUGIN_READY, S.RCCL_READY):
            d = sd.read(b)
            if d is not None:
                ts = d.get("ts") if isinstance(d, dict) else None
                barriers[b] = round((ts if ts else os.path.getmtime(sd.file(b))) - self.t0_wall, 4)
        hip = sd.read(S.HIP_READY) or {}
        ttr = self.marks.get(ready_key)
        if ttr is None and not self.errors:
            self.errors.append(f"validator not ready within {self.timeout:.0f}s; logs in {self.logs}")
        # the validator pod is the critical path: its simulated waits are the modelled part
        modelled = round(sum(self.modelled.get("validator", {}).values()), 4)
        return {"protocol": protocol, "scenario": self.scenario, "time_to_ready_s": ttr,
                "time_to_ready_modelled_s": modelled if ttr is not None else None,
                "time_to_ready_measured_s": round(ttr - modelled, 4) if ttr is not None else None,
                "modelled_waits_s": self.modelled,
                "barriers_s": dict(sorted(barriers.items(), key=lambda kv: kv[1])),
                "marks_s": dict(sorted(self.marks.items(), key=lambda kv: kv[1])),
                "restarts": self.restarts, "errors": self.errors,
                "gemm_tflops_per_gpu": hip.get("gemm_tflops_per_gpu"), "processes": len(self._procs)}


def run_both(hip_mode: str = "local", gemm_shapes: str = "8192", sys_root: str = "/", dev_root: str = "/",
             scenario: str = "host-driver", timeout: float = 240.0, keep: bool = False, full: bool = False) -> Dict:
    """Our chain and the reference protocol in the same harness; ``full`` adds our chain once more
    with the production HIP workload (bf16 + fp8, the scaling sweep, counters)."""
    h = Harness(sys_root=sys_root, dev_root=dev_root, hip_mode=hip_mode, gemm_shapes=gemm_shapes,
                timeout=timeout, scenario=scenario)
    try:
        ours = h.run("ours")
        ref = h.run("reference")
        hf = None
        if full:
            hf = Harness(workdir=os.path.join(h.wd, "full"), sys_root=sys_root, dev_root=dev_root, hip_mode=hip_mode,
                         gemm_shapes=gemm_shapes, timeout=timeout, scenario=scenario, hip_full=True).run("ours")
    finally:
        if not keep:
            shutil.rmtree(h.wd, ignore_errors=True)
    out = {"agent_chain_time_to_ready_s": ours["time_to_ready_s"],
           "reference_protocol_time_to_ready_s": ref["time_to_ready_s"], "ours": ours, "reference": ref,
           "agent_chain_time_to_ready_measured_s": ours["time_to_ready_measured_s"],
           "agent_chain_time_to_ready_modelled_s": ours["time_to_ready_modelled_s"],
           "reference_protocol_time_to_ready_measured_s": ref["time_to_ready_measured_s"],
           "reference_protocol_time_to_ready_modelled_s": ref["time_to_ready_modelled_s"]}
    if hf is not None:
        out.update(agent_chain_full_time_to_ready_s=hf["time_to_ready_s"], ours_full=hf)
    return out


def main(argv=None) -> int:
    import argparse
    logging.basicConfig(level=logging.WARNING)
    ap = argparse.ArgumentParser(prog="amd-ttr", description=__doc__.split("\n\n")[0])
    ap.add_argument("--protocol", choices=["ours", "reference", "both"], default="both")
    ap.add_argument("--scenario", choices=["host-driver", "driver-container"], default="host-driver")
    ap.add_argument("--hip-mode", choices=["local", "skip"], default="local")
    ap.add_argument("--gemm-shapes", default="8192")
    ap.add_argument("--sys-root", default=os.environ.get("AMD_SYSFS_ROOT", "/"))
    ap.add_argument("--dev-root", default=os.environ.get("AMD_DEV_ROOT", "/"))
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--keep", action="store_true", help="keep the work dir (logs of every container)")
    a = ap.parse_args(argv)
    h = Harness(sys_root=a.sys_root, dev_root=a.dev_root, hip_mode=a.hip_mode, gemm_shapes=a.gemm_shapes,
                timeout=a.timeout, scenario=a.scenario)
    protos = ["ours", "reference"] if a.protocol == "both" else [a.protocol]
    ok = True
    for p in protos:
        r = h.run(p)
        ok = ok and r["time_to_ready_s"] is not None
        print(json.dumps(r), flush=True)
    if not a.keep:
        shutil.rmtree(h.wd, ignore_errors=True)
    else:
        print(json.dumps({"workdir": h.wd}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
