"""The reference's end-to-end test, executed on one node of real processes.

Reference: ``tests/scripts/end-to-end.sh`` with ``checks.sh`` (install the operator, every
operand pod Ready, no operand restarts, a GPU workload pod, ClusterPolicy updates reaching the
DaemonSets, operator restart, disabling and re-enabling operands, uninstall). There it needs an
AWS GPU instance and a kind/kubeadm cluster; here the cluster is:

  * the API server: k8s/apiserver.py over HTTP, serving this repo's CRDs with their schemas
    (prune/default/validate on admission);
  * the operator: ``amd-gpu-operator`` as its own OS process, talking to that API server
    through a kubeconfig (informer cache, watches, leader-election-free);
  * the DaemonSet controller: k8s/sim.py (pods per matching node, revisions, DaemonSet
    status from the pods' real Ready conditions);
  * the node: e2e/kubelet.py, which runs every pod bound to it as OS processes, including
    the validator's HIP workload pod and the test's GPU workload pod, with device-plugin
    gRPC Allocate for ``amd.com/gpu``.

On an MI355X box (``sys_root="/"``, ``dev_root="/"``) the operands read the real GPU: the
device plugin advertises it, the validator's HIP workload pod runs the MFMA GEMM probe on it,
and the test workload pod runs ``amd-hip-smoke`` through a device-plugin allocation. On CPU
(fake sysfs, ``hip_mode="skip"``) the same flow runs without GPU work.

Timings reported: ``time_to_ready_s`` (ClusterPolicy created -> ClusterPolicy ``ready`` with
every operand pod Ready: the node's whole bring-up including the operator's reconcile),
per-operand ready times, the re-enable time after ``deploy.operands=false``, and the operator
restart recovery time (checks.sh:97-113 bounds it at 100 s).
"""

from __future__ import annotations

import glob
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
import urllib.request
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml

from ..k8s import errors
from ..k8s import objects as o

log = logging.getLogger("amd-e2e")

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NS = "amd-gpu-operator"
CP_NAME = "cluster-policy"
GPU = "amd.com/gpu"
OPERANDS_LABEL = "amd.com/gpu.deploy.operands"
RESTART_BOUND_S = 100.0               # checks.sh:97-113: 10 x 10 s


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class StepFailed(AssertionError):
    pass


class E2E:
    def __init__(self, workdir: Optional[str] = None, sys_root: str = "/", dev_root: str = "/",
                 hip_mode: str = "pod", timeout: float = 240.0, node: str = "e2e-node",
                 workload_cmd: Optional[List[str]] = None, keep: bool = False, driver: str = "host"):
        """``driver="container"``: the driver DaemonSet installs amdgpu (CPU rehearsal only: a fake
        sysfs without the module and the simulated kernel of devices/fakekernel.py on PATH)."""
        if driver not in ("host", "container"):
            raise ValueError(driver)
        if driver == "container" and os.path.realpath(sys_root) == "/":
            raise ValueError("the driver-container flow needs a fake sysfs (it loads a simulated amdgpu)")
        self.driver = driver
        # unix socket paths (kubelet.sock, plugin endpoints) must stay under 108 bytes: short base
        self.wd = workdir or tempfile.mkdtemp(prefix="amd-e2e-", dir="/tmp" if os.path.isdir("/tmp") else None)
        self.sys_root, self.dev_root = sys_root, dev_root
        self.hip_mode, self.timeout, self.node, self.keep = hip_mode, timeout, node, keep
        # the GPU workload: a HIP kernel on the allocated GPU; on CPU, proof of the allocation
        self.workload_cmd = workload_cmd or (
            ["amd-hip-smoke"] if hip_mode != "skip" else
            ["sh", "-c", 'test -n "$AMD_VISIBLE_DEVICES" && echo "allocated: $AMD_VISIBLE_DEVICES"'])
        self.marks: Dict[str, float] = {}
        self.errors: List[str] = []
        self.steps: List[Dict[str, Any]] = []
        self.result: Dict[str, Any] = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.operator: Optional[subprocess.Popen] = None
        self.t0 = time.monotonic()
        self.installed_at = 0.0
        self.expected_operands: List[str] = []

    # -- bookkeeping ---------------------------------------------------------------------------
    def mark(self, name: str, **kw) -> None:
        with self._lock:
            self.marks.setdefault(name, round(time.monotonic() - self.t0, 3))
            if kw.get("error"):
                self.errors.append(f"{name}: {kw['error']}"[:500])

    def _wait(self, what: str, fn: Callable[[], Any], timeout: Optional[float] = None, period: float = 0.1):
        deadline = time.monotonic() + (timeout or self.timeout)
        last = None
        while time.monotonic() < deadline:
            try:
                last = fn()
                if last:
                    return last
            except errors.ApiError as e:
                last = e
            time.sleep(period)
        raise StepFailed(f"timed out after {timeout or self.timeout:.0f}s waiting for {what} (last: {last!r})")

    def step(self, name: str, fn: Callable[[], Any]) -> Any:
        t = time.monotonic()
        rec: Dict[str, Any] = {"name": name}
        try:
            out = fn()
            rec.update(ok=True, detail=out)
            return out
        except Exception as e:
            rec.update(ok=False, error=f"{type(e).__name__}: {e}")
            raise
        finally:
            rec["seconds"] = round(time.monotonic() - t, 3)
            self.steps.append(rec)
            log.info("step %s: %s (%.2fs)", name, "ok" if rec.get("ok") else rec.get("error"), rec["seconds"])

    # -- cluster -------------------------------------------------------------------------------
    def node_specs(self) -> List[Tuple[str, str, str]]:
        """(node name, sysfs root, dev root) of every node this harness runs a kubelet for."""
        return [(self.node, self.sys_root, self.dev_root)]

    def _node_obj(self, name: str) -> Dict:
        labels = {"feature.node.kubernetes.io/pci-1002.present": "true",
                  "feature.node.kubernetes.io/kernel-version.full": os.uname().release,
                  "feature.node.kubernetes.io/system-os_release.ID": "ubuntu",
                  "feature.node.kubernetes.io/system-os_release.VERSION_ID": "22.04",
                  "kubernetes.io/hostname": name}
        return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": labels},
                "status": {"capacity": {}, "allocatable": {},
                           "nodeInfo": {"containerRuntimeVersion": "containerd://1.7.13",
                                        "kernelVersion": os.uname().release}}}

    def _crds(self) -> List[Dict]:
        out = []
        for p in sorted(glob.glob(os.path.join(REPO, "config", "crd", "bases", "*.yaml"))):
            with open(p) as f:
                out += [d for d in yaml.safe_load_all(f) if d]
        return out

    def cluster_policy(self, sandbox: bool = False) -> Dict:
        with open(os.path.join(REPO, "config", "samples", "amd_v1_clusterpolicy.yaml")) as f:
            cp = yaml.safe_load(f)
        spec = cp["spec"]
        if self.driver == "container":
            spec.setdefault("driver", {})["enabled"] = True
        if sandbox:
            # end-to-end.sh's second install: sandboxWorkloads.enabled=true, defaultWorkload=container
            spec["sandboxWorkloads"] = {"enabled": True, "defaultWorkload": "container"}
        if self.driver == "host":
            spec.setdefault("driver", {})["enabled"] = False      # the host's preinstalled amdgpu
        v = spec.setdefault("validator", {})
        env = [{"name": "HIP_VALIDATION_MODE", "value": self.hip_mode}]
        # on CPU the GEMM pod is planned (free / tenant-held GPUs), scheduled and run, without GEMMs
        v.setdefault("hip", {})["env"] = list(env) + (
            [{"name": "GEMM_VALIDATION_MODE", "value": "dry-run"}] if self.hip_mode == "skip" else [])
        # on CPU the fabric pod is still planned, scheduled and run (topology check on the fake
        # sysfs), without the collective
        v.setdefault("rccl", {})["env"] = list(env) + (
            [{"name": "RCCL_VALIDATION_MODE", "value": "dry-run"}] if self.hip_mode == "skip" else [])
        # a job box exposes its own GPUs' KFD agents only, while PCI sysfs lists every GPU of the
        # host: the driver check counts what it can open (what an unprivileged validator sees)
        v.setdefault("driver", {})["env"] = [{"name": "DRIVER_VALIDATION_STRICT", "value": "false"}]
        me = spec.setdefault("metricsExporter", {})
        me["env"] = [e for e in me.get("env") or [] if e.get("name") != "METRICS_EXPORTER_LISTEN"] + \
            [{"name": "METRICS_EXPORTER_LISTEN", "value": f"127.0.0.1:{self.exporter_port}"}]
        return cp

    def setup(self) -> None:
        from ..cmd.entry import install_wrappers
        from ..k8s.apiserver import FakeAPIServer
        from ..k8s.fake import FakeClient
        from ..k8s.sim import ClusterSim
        from .kubelet import ProcessKubelet

        self.base = os.path.join(self.wd, "e2e")
        shutil.rmtree(self.base, ignore_errors=True)
        os.makedirs(self.base)
        self.bin = install_wrappers(os.path.join(self.base, "bin"))
        if self.driver == "container":
            from ..devices import fakekernel
            fakekernel.install_tools(self.bin)
        ns = {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NS}}
        nodes = [self._node_obj(n) for n, _, _ in self.node_specs()]
        self.backing = FakeClient([ns] + nodes + self._crds(),
                                  unserved_kinds={"ServiceMonitor", "PrometheusRule"}, collect_orphans=True)
        self.api = FakeAPIServer(self.backing).start()
        self.kubeconfig = os.path.join(self.base, "kubeconfig")
        with open(self.kubeconfig, "w") as f:
            yaml.safe_dump({"apiVersion": "v1", "kind": "Config", "current-context": "e2e",
                            "clusters": [{"name": "e2e", "cluster": {"server": self.api.url}}],
                            "contexts": [{"name": "e2e", "context": {"cluster": "e2e", "user": "e2e"}}],
                            "users": [{"name": "e2e", "user": {}}]}, f)
        self.exporter_port = _free_port()
        self.env = {k: v for k, v in os.environ.items() if not k.startswith(("AMD_MOUNTS", "KUBECONFIG"))}
        self.env.update({
            "PATH": f"{self.bin}:{os.environ.get('PATH', '/usr/bin:/bin')}",
            "PYTHONPATH": REPO + (os.pathsep + os.environ["PYTHONPATH"] if os.environ.get("PYTHONPATH") else ""),
            "KUBECONFIG": self.kubeconfig, "PYTHONUNBUFFERED": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0",
            "AMD_SYSFS_ROOT": self.sys_root, "AMD_DEV_ROOT": self.dev_root,
            # no containerd runs on this node: the toolkit edits its config (which the kubelet's
            # runtime-handler gate reads) but has no daemon to restart
            "RESTART_MODE": "none",
            # a job box exposes its own GPUs' KFD agents only while PCI sysfs lists all of the host's:
            # every driver-validation init container (validator and operand DaemonSets) counts
            # what it can open, as an unprivileged container on such a node would
            "DRIVER_VALIDATION_STRICT": "false",
        })
        specs = self.node_specs()
        self.kubelets = []
        for name, sys_root, dev_root in specs:
            env = dict(self.env, AMD_SYSFS_ROOT=sys_root, AMD_DEV_ROOT=dev_root)
            base = self.base if len(specs) == 1 else os.path.join(self.base, name)
            self.kubelets.append(ProcessKubelet(self.backing, name, base, env, sys_root, dev_root,
                                                events=self.mark, image_env=self.image_env,
                                                host_links={} if self.driver == "container" else None).start())
        self.kubelet = self.kubelets[0]
        self.dsc = ClusterSim(self.backing, kubelet=False)

        def ds_controller():
            while not self._stop.is_set():
                try:
                    self.dsc.sync()
                except Exception as e:  # noqa: BLE001 - objects racing with deletion
                    log.debug("ds controller: %s", e)
                self._stop.wait(0.1)
        self._dsc_thread = threading.Thread(target=ds_controller, name="ds-controller", daemon=True)
        self._dsc_thread.start()
        self.metrics_port, self.health_port = _free_port(), _free_port()

    @staticmethod
    def image_env(image: str) -> Dict[str, str]:
        """The ENV an image's config carries (docker/Dockerfile.driver: DRIVER_VERSION)."""
        repo, _, tag = image.rpartition(":")
        if repo.endswith("amdgpu-driver") and tag:
            return {"DRIVER_VERSION": tag.split("-")[0]}
        return {}

    def start_operator(self) -> subprocess.Popen:
        env = dict(self.env, OPERATOR_NAMESPACE=NS)
        logf = open(os.path.join(self.base, f"operator.{len(glob.glob(os.path.join(self.base, 'operator.*')))}.log"),
                    "ab")
        self.operator = subprocess.Popen(
            [os.path.join(self.bin, "amd-gpu-operator"), "--kubeconfig", self.kubeconfig,
             "--metrics-bind-address", f"127.0.0.1:{self.metrics_port}",
             "--health-probe-bind-address", f"127.0.0.1:{self.health_port}",
             "--zap-log-level", os.environ.get("AMD_E2E_OPERATOR_LOG_LEVEL", "info")],
            env=env, stdout=logf, stderr=subprocess.STDOUT, start_new_session=True)
        logf.close()
        return self.operator

    def stop_operator(self, sig=signal.SIGTERM) -> None:
        p, self.operator = self.operator, None
        if p is None or p.poll() is not None:
            return
        os.killpg(p.pid, sig)
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()

    def teardown(self) -> None:
        self._stop.set()
        self.stop_operator()
        for k in self.kubelets:
            k.stop()
        self.api.stop()
        if not self.keep:
            shutil.rmtree(self.base, ignore_errors=True)

    # -- observations --------------------------------------------------------------------------
    def cp_state(self) -> Optional[str]:
        try:
            return (self.backing.get("amd.com/v1", "ClusterPolicy", CP_NAME).get("status") or {}).get("state")
        except errors.NotFound:
            return None

    def operand_daemonsets(self) -> List[Dict]:
        return [d for d in self.backing.list("apps/v1", "DaemonSet", NS)
                if ((d.get("status") or {}).get("desiredNumberScheduled") or 0) > 0]

    def operand_pods(self) -> List[Dict]:
        return [p for p in self.backing.list("v1", "Pod", NS)
                if any(r.get("kind") == "DaemonSet" for r in p["metadata"].get("ownerReferences") or [])]

    def all_ready(self) -> Optional[Dict[str, int]]:
        """ClusterPolicy ready and every scheduled operand DaemonSet rolled out and Ready; once the
        first install has established the operand set, every one of those must be scheduled too
        (a DaemonSet whose node label is not set yet has 0 desired pods and counts as ready for
        the operator)."""
        if self.cp_state() != "ready":
            return None
        dss = self.operand_daemonsets()
        if not dss:
            return None
        out = {}
        for d in dss:
            st = d.get("status") or {}
            if st.get("numberReady") != st.get("desiredNumberScheduled") or st.get("numberUnavailable"):
                return None
            # rolled out: the controller has seen this generation and every pod runs its template
            if st.get("observedGeneration", 0) < d["metadata"].get("generation", 1) or \
                    st.get("updatedNumberScheduled") != st.get("desiredNumberScheduled"):
                return None
            out[o.name(d)] = st["numberReady"]
        if self.expected_operands and not set(self.expected_operands) <= set(out):
            return None
        return out

    def validations(self) -> List[str]:
        d = self.kubelet.host_path("/run/amd/validations")
        return sorted(os.listdir(d)) if os.path.isdir(d) else []

    # -- the reference's steps -----------------------------------------------------------------
    def install_operator(self, sandbox: bool = False) -> Dict:
        if not sandbox:
            self.t0 = time.monotonic()
        self.installed_at = time.time()
        self.backing.create(self.cluster_policy(sandbox))
        self.mark("clusterpolicy:created" + (":sandbox" if sandbox else ""))
        self.start_operator()
        return {"operator_pid": self.operator.pid}

    def verify_operator(self, tag: str) -> Dict:
        t = time.monotonic()
        ready = self._wait("ClusterPolicy ready and every operand pod Ready", self.all_ready)
        dt = time.monotonic() - t
        self.mark(f"{tag}:ready")
        files = self.validations()
        for f in ("toolkit-ready", "hip-ready", "plugin-ready"):
            if f not in files:
                raise StepFailed(f"validation barrier {f} missing: {files}")
        cap = (self.backing.get("v1", "Node", self.node).get("status") or {}).get("allocatable") or {}
        if int(cap.get(GPU, 0) or 0) < 1:
            raise StepFailed(f"node advertises no {GPU}: {cap}")
        out = {"daemonsets": ready, "seconds": round(dt, 3), "validations": files, GPU: cap.get(GPU)}
        for f in ("hip-ready", "host-driver-ready", "rccl-ready"):
            try:
                with open(os.path.join(self.kubelet.host_path("/run/amd/validations"), f)) as fh:
                    out[f] = json.load(fh)
            except (OSError, ValueError):
                pass
        # barriers survive in /run across installs (as on a node): this install must have rewritten them
        for f in ("driver-ready",):
            try:
                with open(os.path.join(self.kubelet.host_path("/run/amd/validations"), f)) as fh:
                    out[f] = json.load(fh)
            except (OSError, ValueError):
                pass
        drv = "driver-ready" if self.driver == "container" else "host-driver-ready"
        if drv not in out:
            raise StepFailed(f"{drv} missing: {files}")
        stale = [f for f in ("hip-ready", drv) if (out.get(f) or {}).get("ts", 0) < self.installed_at]
        if stale:
            pods = {o.name(p): [p["metadata"].get("uid", "")[:8], (p.get("status") or {}).get("phase"),
                                [c.get("type") + "=" + c.get("status") for c in (p.get("status") or {}).get("conditions") or []]]
                    for p in self.operand_pods() if "validator" in o.name(p)}
            dss = {o.name(d): d.get("status") for d in self.backing.list("apps/v1", "DaemonSet", NS)
                   if "validator" in o.name(d)}
            raise StepFailed(f"validation barriers not rewritten by this install: {stale}; pods {pods}; ds {dss}; "
                             f"installed_at {self.installed_at:.3f} ts {[(f, (out.get(f) or {}).get('ts')) for f in stale]}")
        labels = o.get_labels(self.backing.get("v1", "Node", self.node))
        out["gpu_labels"] = {k: v for k, v in labels.items()
                             if k.startswith("amd.com/gpu.") and not k.startswith("amd.com/gpu.deploy.")}
        return out

    def verify_operand_restarts(self) -> Dict:
        out = {}
        for p in self.operand_pods():
            n = sum(cs.get("restartCount", 0) for cs in (p.get("status") or {}).get("containerStatuses") or [])
            out[o.name(p)] = n
        bad = {k: v for k, v in out.items() if v}
        if bad:
            raise StepFailed(f"operand containers restarted: {bad}")
        return out

    def workload_pod(self) -> Dict:
        return {"apiVersion": "v1", "kind": "Pod",
                "metadata": {"name": "gpu-operator-test", "namespace": "default", "labels": {"app": "gpu-operator-test"}},
                "spec": {"restartPolicy": "OnFailure",
                         "containers": [{"name": "hip-smoke", "image": "amd-gpu-operator-node",
                                         "command": list(self.workload_cmd),
                                         "resources": {"limits": {GPU: 1}}}]}}

    def install_and_verify_workload(self) -> Dict:
        if not any(o.name(n) == "default" for n in self.backing.list("v1", "Namespace")):
            self.backing.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "default"}})
        self.backing.create(self.workload_pod())

        def done():
            p = self.backing.get("v1", "Pod", "gpu-operator-test", "default")
            ph = (p.get("status") or {}).get("phase")
            if ph == "Failed":
                raise StepFailed(f"workload pod failed: {p.get('status')}")
            return p if ph == "Succeeded" else None
        p = self._wait("the GPU workload pod to succeed", done)
        run_dir = [d for d in glob.glob(os.path.join(self.base, "pods", "default_gpu-operator-test_*"))]
        log_text = ""
        for d in run_dir:
            lp = os.path.join(d, "logs", "hip-smoke.log")
            if os.path.exists(lp):
                with open(lp, errors="replace") as f:
                    log_text = f.read()[-2000:]
        return {"phase": p["status"]["phase"], "node": p["spec"].get("nodeName"), "log_tail": log_text.strip()[-400:]}

    def exporter_attribution(self) -> Dict:
        """The metrics exporter's per-pod GPU attribution (the dcgm-exporter role): a running pod
        holding an ``amd.com/gpu`` shows up as the ``pod`` label of that GPU's series, through
        the kubelet's pod-resources API."""
        pod = self.workload_pod()
        pod["metadata"]["name"] = "gpu-attribution"
        pod["spec"]["restartPolicy"] = "Never"
        pod["spec"]["containers"][0]["command"] = ["sleep", "600"]
        self.backing.create(pod)
        self._wait("the attributed pod to run", lambda: (self.backing.get(
            "v1", "Pod", "gpu-attribution", "default").get("status") or {}).get("phase") == "Running")

        def scrape():
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{self.exporter_port}/metrics", timeout=2) as r:
                    text = r.read().decode()
            except OSError:
                return None
            hits = [ln for ln in text.splitlines() if ln.startswith("amd_gpu_") and 'pod="gpu-attribution"' in ln]
            return (text, hits) if hits else None
        text, hits = self._wait("a GPU series labelled with the pod", scrape)
        series = [ln for ln in text.splitlines() if ln.startswith("amd_gpu_")]
        self.backing.delete("v1", "Pod", "gpu-attribution", "default")
        self._wait("the attributed pod gone", lambda: not any(
            r.name == "gpu-attribution" for k in self.kubelets for r in k.running().values()))
        names = sorted({h.split("{", 1)[0] for h in hits})
        return {"series": len(series), "attributed_metrics": names[:12], "sample": hits[0][:300]}

    def _ds(self, name: str) -> Dict:
        return self.backing.get("apps/v1", "DaemonSet", name, NS)

    def _plugin_ds_name(self) -> str:
        return next(o.name(d) for d in self.backing.list("apps/v1", "DaemonSet", NS) if "device-plugin" in o.name(d)
                    and "sandbox" not in o.name(d))

    def update_clusterpolicy(self) -> Dict:
        """update-clusterpolicy.sh: an env and an image-version change reach the DaemonSet and the
        restarted pod."""
        name = self._plugin_ds_name()
        cp = self.backing.get("amd.com/v1", "ClusterPolicy", CP_NAME)
        dp = cp["spec"].setdefault("devicePlugin", {})
        dp["env"] = list(dp.get("env") or []) + [{"name": "MY_TEST_ENV_NAME", "value": "test"}]
        self.backing.update(cp)

        def env_in_ds():
            c = self._ds(name)["spec"]["template"]["spec"]["containers"][0]
            return any(e.get("name") == "MY_TEST_ENV_NAME" and e.get("value") == "test" for e in c.get("env") or [])
        self._wait("the device-plugin DaemonSet to carry the new env", env_in_ds)

        def env_in_process():
            runs = [r for r in self.kubelet.running().values() if r.name.startswith(name)]
            for r in runs:
                c0 = r.pod["spec"]["containers"][0]["name"]
                p = r.procs.get(c0)
                if p is None or p.poll() is not None or not r.ready:
                    continue
                with open(f"/proc/{p.pid}/environ", "rb") as f:
                    if b"MY_TEST_ENV_NAME=test\0" in f.read():
                        return p.pid
            return None
        pid = self._wait("a device-plugin process started with the new env", env_in_process)
        cp = self.backing.get("amd.com/v1", "ClusterPolicy", CP_NAME)
        cp["spec"]["devicePlugin"]["version"] = "v0.1.1"
        self.backing.update(cp)
        self._wait("the device-plugin image update",
                   lambda: self._ds(name)["spec"]["template"]["spec"]["containers"][0]["image"].endswith(":v0.1.1"))
        self._wait("the updated device plugin Ready", self.all_ready)
        return {"daemonset": name, "env_pid": pid}

    def _alloc(self) -> int:
        st = self.backing.get("v1", "Node", self.node).get("status") or {}
        return int((st.get("allocatable") or {}).get(GPU, 0) or 0)

    def _cp_update(self, fn) -> None:
        cp = self.backing.get("amd.com/v1", "ClusterPolicy", CP_NAME)
        fn(cp["spec"])
        self.backing.update(cp)

    def time_slicing(self, replicas: int = 10, pods: int = 5) -> Dict:
        """update-clusterpolicy.sh's time-slicing test: a sharing config in a ConfigMap, named by
        devicePlugin.config, multiplies the advertised amd.com/gpu; the labeller reports the
        replicas and a -SHARED product; more GPU pods than physical GPUs all run; removing the config
        restores the physical count."""
        # the plugin re-registers after each rollout: its count is 0 until the kubelet has it again
        phys = self._wait(f"{GPU} advertised", lambda: self._alloc() or None)
        cfg = {"version": "v1", "sharing": {"timeSlicing": {"resources": [{"name": GPU, "replicas": replicas}]}}}
        self.backing.create({"apiVersion": "v1", "kind": "ConfigMap",
                             "metadata": {"name": "time-slicing-config", "namespace": NS},
                             "data": {"any": yaml.safe_dump(cfg)}})
        self._cp_update(lambda sp: sp.setdefault("devicePlugin", {}).update(
            config={"name": "time-slicing-config", "default": "any"}))
        self._wait(f"{GPU} x{replicas} advertised", lambda: self._alloc() == phys * replicas)

        def shared_labels():
            lb = o.get_labels(self.backing.get("v1", "Node", self.node))
            return lb if lb.get("amd.com/gpu.replicas") == str(replicas) and \
                lb.get("amd.com/gpu.product", "").endswith("-SHARED") else None
        lb = self._wait("the labeller's replicas / -SHARED labels", shared_labels)
        self._wait("the device plugin rollout", self.all_ready)
        names = [f"time-slicing-{i}" for i in range(pods)]
        for n in names:
            pod = self.workload_pod()
            pod["metadata"]["name"] = n
            self.backing.create(pod)

        def all_done():
            ph = [(self.backing.get("v1", "Pod", n, "default").get("status") or {}).get("phase") for n in names]
            if "Failed" in ph:
                raise StepFailed(f"time-sliced pod failed: {ph}")
            return ph if all(p == "Succeeded" for p in ph) else None
        self._wait(f"{pods} time-sliced GPU pods to succeed", all_done)
        for n in names:
            self.backing.delete("v1", "Pod", n, "default")
        self._cp_update(lambda sp: sp.get("devicePlugin", {}).pop("config", None))
        self._wait(f"{GPU} back to the physical count", lambda: self._alloc() == phys)
        self._wait("replicas label back to 1", lambda: o.get_labels(self.backing.get("v1", "Node", self.node))
                   .get("amd.com/gpu.replicas") == "1")
        self._wait("the device plugin rollout", self.all_ready)
        return {"physical": phys, "advertised": phys * replicas, "pods": pods,
                "labels": {k: lb[k] for k in ("amd.com/gpu.replicas", "amd.com/gpu.sharing-strategy",
                                              "amd.com/gpu.product")}}

    def _module_version(self) -> Optional[str]:
        try:
            with open(os.path.join(self.sys_root, "sys/module/amdgpu/version")) as f:
                return f.read().strip()
        except OSError:
            return None

    def driver_upgrade(self, new_version: str = "6.12.13") -> Dict:
        """driver.version bump with autoUpgrade: the upgrade controller's state machine drives the
        node (cordon, evict the GPU pod, delete the driver pod, the new driver container unloads
        and loads amdgpu, validation, uncordon) -- the reference's test_image_updates, where the
        driver pod is deleted by hand, done by the operator itself."""
        from ..controllers.upgrade import DONE, UPGRADE_STATE_LABEL
        # a controller-managed GPU pod (kubectl-drain semantics: bare pods need podDeletion.force)
        job = self.backing.create({"apiVersion": "batch/v1", "kind": "Job",
                                   "metadata": {"name": "gpu-long-running", "namespace": "default"},
                                   "spec": {"template": {"spec": {"containers": []}}}})
        pod = self.workload_pod()
        pod["metadata"]["name"] = "gpu-long-running"
        pod["metadata"]["ownerReferences"] = [{"apiVersion": "batch/v1", "kind": "Job", "name": "gpu-long-running",
                                               "uid": job["metadata"]["uid"], "controller": True}]
        pod["spec"]["restartPolicy"] = "Never"
        pod["spec"]["containers"][0]["command"] = ["sleep", "600"]
        self.backing.create(pod)
        self._wait("the long-running GPU pod to run", lambda: (self.backing.get(
            "v1", "Pod", "gpu-long-running", "default").get("status") or {}).get("phase") == "Running")
        before = self._module_version()
        self._cp_update(lambda sp: sp.setdefault("driver", {}).update(version=new_version))
        t = time.monotonic()
        states: List[str] = []

        def done():
            node = self.backing.get("v1", "Node", self.node)
            st = o.get_labels(node).get(UPGRADE_STATE_LABEL, "")
            if st and (not states or states[-1] != st):
                states.append(st)
            if st == "upgrade-failed":
                raise StepFailed(f"upgrade failed: {states}")
            return st == DONE and self._module_version() == new_version and \
                not (node.get("spec") or {}).get("unschedulable") and self.all_ready()
        self._wait("the driver upgrade to complete", done, period=0.05)
        try:
            self.backing.get("v1", "Pod", "gpu-long-running", "default")
            raise StepFailed("the GPU pod was not evicted before the driver pod restarted")
        except errors.NotFound:
            pass
        return {"from": before, "to": self._module_version(), "states": states,
                "seconds": round(time.monotonic() - t, 3)}

    def restart_operator(self) -> Dict:
        """checks.sh test_restart_operator: the operator pod is killed; its replacement must get
        the ClusterPolicy back to ready without churning the operands."""
        before = {o.name(p): p["metadata"]["uid"] for p in self.operand_pods()}
        self.stop_operator(signal.SIGKILL)
        t = time.monotonic()
        self.start_operator()

        def healthy():
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{self.health_port}/readyz", timeout=1) as r:
                    return r.status == 200 and self.all_ready()
            except OSError:
                return None
        self._wait("the restarted operator healthy and the ClusterPolicy ready", healthy, timeout=RESTART_BOUND_S)
        dt = time.monotonic() - t
        time.sleep(1.0)                                  # a reconcile pass after the restart
        after = {o.name(p): p["metadata"]["uid"] for p in self.operand_pods()}
        churned = sorted(k for k in before if after.get(k) != before[k])
        if churned:
            raise StepFailed(f"operand pods recreated by the restarted operator: {churned}")
        return {"recovery_s": round(dt, 3), "bound_s": RESTART_BOUND_S}

    def disable_operands(self) -> Dict:
        pids = self.kubelet.all_pids()
        self.backing.patch("v1", "Node", self.node, {"metadata": {"labels": {OPERANDS_LABEL: "false"}}})
        self._wait("every operand pod deleted", lambda: not self.operand_pods())

        def gone():
            alive = []
            for pid in pids:
                try:
                    os.kill(pid, 0)
                    alive.append(pid)
                except ProcessLookupError:
                    pass
                except PermissionError:
                    alive.append(pid)
            return not alive or None
        self._wait("operand processes to exit", gone, timeout=30)
        return {"terminated_processes": len(pids)}

    def enable_operands(self) -> Dict:
        t = time.monotonic()
        self.backing.patch("v1", "Node", self.node, {"metadata": {"labels": {OPERANDS_LABEL: "true"}}})
        out = self.verify_operator("reenable")
        out["reenable_time_to_ready_s"] = round(time.monotonic() - t, 3)
        return out

    def uninstall(self) -> Dict:
        try:
            self.backing.delete("v1", "Pod", "gpu-operator-test", "default")
        except errors.NotFound:
            pass
        self.backing.delete("amd.com/v1", "ClusterPolicy", CP_NAME)
        self._wait("operand DaemonSets garbage-collected", lambda: not self.backing.list("apps/v1", "DaemonSet", NS))
        self._wait("operand pods gone", lambda: not self.operand_pods())
        self._wait("every node process gone", lambda: not self.kubelet.all_pids(), timeout=30)
        self.stop_operator()
        return {"ok": True}

    # -- fabric validation on real node shapes ----------------------------------------------------
    def _barrier(self, name: str) -> Optional[Dict]:
        try:
            with open(os.path.join(self.kubelet.host_path("/run/amd/validations"), name)) as fh:
                return json.load(fh)
        except (OSError, ValueError):
            return None

    def _rccl_pod_shape(self) -> Dict:
        pods = [p for p in self.backing.list("v1", "Pod", NS) if o.get_labels(p).get("app") == "amd-rccl-validator"]
        if not pods:
            return {"pod": None}
        c0 = pods[-1]["spec"]["initContainers"][0]
        env = {e["name"]: e.get("value") for e in c0.get("env") or []}
        return {"pod": o.name(pods[-1]), "limits": (c0.get("resources") or {}).get("limits"),
                "privileged": bool((c0.get("securityContext") or {}).get("privileged")),
                "env": {k: env[k] for k in ("RCCL_RANKS", "AMD_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES") if k in env}}

    def _validation_pod_env(self, app: str) -> Dict[str, str]:
        pods = [p for p in self.backing.list("v1", "Pod", NS) if o.get_labels(p).get("app") == app]
        if not pods:
            return {}
        c0 = pods[-1]["spec"]["initContainers"][0]
        return {e["name"]: e.get("value") for e in c0.get("env") or []}

    def restart_validator(self) -> Dict:
        """Delete the validator pod (a restart, as after an upgrade or a node reboot) and wait for
        the DaemonSet's replacement to re-run the chain and write a fresh rccl-ready."""
        before = (self._barrier("rccl-ready") or {}).get("ts", 0.0)
        t = time.monotonic()
        for p in self.operand_pods():
            if o.name(p).startswith("amd-operator-validator"):
                self.backing.delete("v1", "Pod", o.name(p), NS)
        self._wait("a fresh rccl-ready from the restarted validator",
                   lambda: (self._barrier("rccl-ready") or {}).get("ts", 0.0) > before)
        self._wait("the validator Ready again", self.all_ready)
        env = self._validation_pod_env("amd-hip-validator")
        return {"rccl-ready": self._barrier("rccl-ready"), "rccl_pod": self._rccl_pod_shape(),
                "hip-ready": self._barrier("hip-ready"), "ready_s": round(time.monotonic() - t, 3),
                "hip_pod_env": {k: env[k] for k in ("GEMM_DEVICES", "GEMM_PROBE_DEVICES", "GEMM_DRY_RUN") if k in env}}

    def _gpu_job(self, name: str, gpus: int = 1) -> None:
        pod = self.workload_pod()
        pod["metadata"]["name"] = name
        pod["metadata"]["labels"] = {"app": name}
        pod["spec"]["restartPolicy"] = "Never"
        pod["spec"]["containers"][0]["command"] = ["sleep", "600"]
        pod["spec"]["containers"][0]["resources"] = {"limits": {GPU: gpus}}
        if not any(o.name(n) == "default" for n in self.backing.list("v1", "Namespace")):
            self.backing.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "default"}})
        self.backing.create(pod)
        self._wait(f"the GPU pod {name} to run", lambda: (self.backing.get(
            "v1", "Pod", name, "default").get("status") or {}).get("phase") == "Running")

    def run_fabric_shapes(self, replicas: int = 10) -> Dict[str, Any]:
        """The fabric validator on the node shapes where allocatable is not the GPU count
        (VERDICT r2 item 3): whole GPUs (the pod requests every physical GPU through the
        scheduler), time-slicing xN (the pod asks for no replica and sees every GPU), a GPU pod
        holding a device while the validator restarts (topology-only, never blocks). On a CPX
        sysfs the install itself covers partitions (one agent per physical GPU pinned)."""
        self.setup()
        out: Dict[str, Any] = {}
        try:
            self.step("install-operator", self.install_operator)
            self.step("verify-operator", lambda: self.verify_operator("install"))
            out["install"] = {"rccl-ready": self._barrier("rccl-ready"), "rccl_pod": self._rccl_pod_shape()}
            phys = self._wait(f"{GPU} advertised", lambda: self._alloc() or None)
            cfg = {"version": "v1", "sharing": {"timeSlicing": {"resources": [{"name": GPU, "replicas": replicas}]}}}
            self.backing.create({"apiVersion": "v1", "kind": "ConfigMap",
                                 "metadata": {"name": "time-slicing-config", "namespace": NS},
                                 "data": {"any": yaml.safe_dump(cfg)}})
            self._cp_update(lambda sp: sp.setdefault("devicePlugin", {}).update(
                config={"name": "time-slicing-config", "default": "any"}))
            self._wait(f"{GPU} x{replicas} advertised", lambda: self._alloc() == phys * replicas)
            self._wait("the device plugin rollout", self.all_ready)
            out["time-slicing"] = self.step("validator-restart[time-slicing]", self.restart_validator)
            out["time-slicing"]["allocatable"] = self._alloc()
            self._gpu_job("gpu-busy")
            out["busy"] = self.step("validator-restart[busy]", self.restart_validator)
            self.backing.delete("v1", "Pod", "gpu-busy", "default")
        except Exception as e:  # noqa: BLE001 - reported in the result
            self.result["error"] = f"{type(e).__name__}: {e}"
            self.result["logs_dir"] = self.base
            self.keep = True
        finally:
            self.teardown()
        self.result.update(out)
        self.result.update(ok=all(s.get("ok") for s in self.steps) and "error" not in self.result, steps=self.steps)
        return self.result

    def _tenant_race(self) -> Dict:
        """A tenant scheduled between the validator's busy check and its fabric pod: the kubelet
        holds the fabric pod's admission until a 1-GPU tenant runs, then admits it -- the
        validator must fall back to topology-only in seconds, not wait out the pod timeout."""
        released = threading.Event()
        seen = threading.Event()
        errs: List[str] = []
        old = {p["metadata"]["uid"] for p in self.backing.list("v1", "Pod", NS)
               if o.get_labels(p).get("app") == "amd-rccl-validator"}

        def hold(p):
            return o.get_labels(p).get("app") == "amd-rccl-validator" and not released.is_set()

        def start_tenant():
            try:
                self._gpu_job("tenant-race", gpus=1)
            except Exception as e:  # noqa: BLE001 - reported in the step's result
                errs.append(f"{type(e).__name__}: {e}")
            finally:
                released.set()

        def on_event(ev):
            if ev.type == "ADDED" and o.get_labels(ev.obj).get("app") == "amd-rccl-validator" and \
                    ev.obj["metadata"]["uid"] not in old and not seen.is_set():
                seen.set()
                threading.Thread(target=start_tenant, daemon=True).start()
        self.kubelet.hold_admission = hold
        stop = self.backing.watch("v1", "Pod", on_event, namespace=NS)
        try:
            out = self.restart_validator()
        finally:
            stop()
            self.kubelet.hold_admission = None
            released.set()
        out["tenant_started_after_busy_check"] = seen.is_set()
        if errs:
            raise StepFailed(f"the racing tenant did not start: {errs}")
        return out

    def _standin_gemm(self, **env) -> Dict[str, str]:
        """The scripted amd-gemm-validate (e2e/gemm_standin.py) on the node's PATH for the pods the
        kubelet starts from now on: the validator's real HIP pod and workload entry run, the GEMM lines
        are scripted. Returns the env it put in place."""
        d = os.path.join(self.base, "standin")
        os.makedirs(d, exist_ok=True)
        for name, body in (("amd-gemm-validate", f'exec "{sys.executable}" -m gpu_operator_amd.e2e.gemm_standin "$@"\n'),
                           ("rocprofv3", "exit 1\n")):            # no profiler on a CPU node
            p = os.path.join(d, name)
            with open(p, "w") as f:
                f.write("#!/bin/sh\n" + body)
            os.chmod(p, 0o755)
        add = {"PATH": f"{d}:{self.kubelet.base_env.get('PATH', '')}", "AMDGO_BIN_DIR": d,
               "GEMM_STANDIN_STATE": os.path.join(d, "runs"), **env}
        self.kubelet.base_env.update(add)
        return add

    def _tenant_during_hip_sweep(self) -> Dict:
        """Case (iv): a 1-GPU tenant is scheduled while the HIP pod's sweep runs (the pod is privileged
        and requests no GPU, so the device plugin keeps advertising every GPU). The tenant's GPU then
        measures slow -- the sharing -- and the validator must report it ``disturbed``, keep its numbers
        out of the gates and open hip-ready: no floor failure, no re-measure."""
        d = os.path.join(self.base, "standin")
        slow_file = os.path.join(d, "tenant-gpu")
        env = self._standin_gemm(GEMM_STANDIN_SCRIPT="fast", GEMM_STANDIN_RUNTIME_S="0.5",
                                 GEMM_STANDIN_SLOW_FILE=slow_file)
        running = env["GEMM_STANDIN_STATE"] + ".running"
        errs: List[str] = []

        def tenant():
            try:
                end = time.monotonic() + 120
                while not os.path.exists(running) and time.monotonic() < end:
                    time.sleep(0.02)
                self._gpu_job("tenant-sweep", gpus=1)
                pod = self.backing.get("v1", "Pod", "tenant-sweep", "default")
                ids = [i for (uid, _, _), v in self.kubelet.plugins.assigned.items()
                       if uid == pod["metadata"]["uid"] for i in v]
                from ..devices import enumerate_gpus
                from ..validator.components import _agent_of
                gpus = enumerate_gpus(self.sys_root)
                idx = sorted({_agent_of(i, gpus)["index"] for i in ids})
                with open(slow_file + ".tmp", "w") as f:
                    f.write(",".join(map(str, idx)))
                os.rename(slow_file + ".tmp", slow_file)
            except Exception as e:  # noqa: BLE001 - reported in the step's result
                errs.append(f"{type(e).__name__}: {e}")
                open(slow_file, "w").close()
        th = threading.Thread(target=tenant, daemon=True)
        th.start()
        # the validator runs its HIP pod for real (no dry run) with the scripted GEMM
        self._cp_update(lambda sp: sp["validator"]["hip"].update(env=[{"name": "HIP_VALIDATION_MODE", "value": "pod"}]))
        out = self.restart_validator()
        th.join(timeout=5)
        if errs:
            raise StepFailed(f"the tenant did not start during the sweep: {errs}")
        with open(slow_file) as f:
            out["tenant_gpus"] = [int(x) for x in f.read().split(",") if x]
        return out

    def run_tenant_cases(self) -> Dict[str, Any]:
        """The validator beside tenants, on real processes: (i) a pod holds 2 GPUs
        -- the HIP pod's full sweep gets the 6 free GPUs, the 2 held ones a probe; (ii) pods hold all
        8 -- the probe only; (iii) a tenant lands between the fabric busy check and the fabric pod --
        topology-only; (iv) a tenant is given a GPU while the HIP sweep runs -- that GPU is reported
        disturbed, out of the throughput gates. The validator reaches Ready in each."""
        self.setup()
        out: Dict[str, Any] = {}
        try:
            self.step("install-operator", self.install_operator)
            self.step("verify-operator", lambda: self.verify_operator("install"))
            env = self._validation_pod_env("amd-hip-validator")
            out["idle"] = {"hip-ready": self._barrier("hip-ready"), "rccl-ready": self._barrier("rccl-ready"),
                           "hip_pod_env": {k: env[k] for k in ("GEMM_DEVICES", "GEMM_PROBE_DEVICES") if k in env}}
            self._gpu_job("tenant-a", gpus=2)
            out["two-held"] = self.step("validator-restart[2 GPUs held]", self.restart_validator)
            self._gpu_job("tenant-b", gpus=6)
            out["all-held"] = self.step("validator-restart[8 GPUs held]", self.restart_validator)
            for name in ("tenant-a", "tenant-b"):
                self.backing.delete("v1", "Pod", name, "default")
            self._wait("the tenants gone", lambda: not [p for p in self.backing.list("v1", "Pod", "default")
                                                        if o.name(p).startswith("tenant-")])
            out["race"] = self.step("validator-restart[tenant before the fabric pod]", self._tenant_race)
            self.backing.delete("v1", "Pod", "tenant-race", "default")
            self._wait("the race tenant gone", lambda: not [p for p in self.backing.list("v1", "Pod", "default")
                                                            if o.name(p) == "tenant-race"])
            out["during-sweep"] = self.step("validator-restart[tenant during the HIP sweep]",
                                            self._tenant_during_hip_sweep)
            self.backing.delete("v1", "Pod", "tenant-sweep", "default")
        except Exception as e:  # noqa: BLE001 - reported in the result
            self.result["error"] = f"{type(e).__name__}: {e}"
            self.result["logs_dir"] = self.base
            self.keep = True
        finally:
            self.teardown()
        self.result.update(out)
        self.result.update(ok=all(s.get("ok") for s in self.steps) and "error" not in self.result, steps=self.steps)
        return self.result

    # -- the flow -------------------------------------------------------------------------------
    def run(self) -> Dict[str, Any]:
        if self.driver == "container":
            return self.run_driver_container()
        self.setup()
        try:
            self.step("install-operator", self.install_operator)
            first = self.step("verify-operator", lambda: self.verify_operator("install"))
            self.result["time_to_ready_s"] = self.marks.get("install:ready")
            self.result["operands_ready"] = first["daemonsets"]
            self.expected_operands = sorted(first["daemonsets"])
            self.step("verify-operand-restarts", self.verify_operand_restarts)
            self.step("install+verify-workload", self.install_and_verify_workload)
            self.step("exporter-attribution", self.exporter_attribution)
            self.step("update-clusterpolicy", self.update_clusterpolicy)
            self.step("time-slicing", self.time_slicing)
            rs = self.step("restart-operator", self.restart_operator)
            self.result["operator_restart_recovery_s"] = rs["recovery_s"]
            self.step("disable-operands", self.disable_operands)
            en = self.step("enable-operands", self.enable_operands)
            self.result["reenable_time_to_ready_s"] = en["reenable_time_to_ready_s"]
            self.step("uninstall", self.uninstall)
            # end-to-end.sh, second half: the operator with sandbox workloads enabled still serves
            # container workloads (defaultWorkload=container)
            self.step("install-operator[sandbox]", lambda: self.install_operator(sandbox=True))
            sb = self.step("verify-operator[sandbox]", lambda: self.verify_operator("sandbox"))
            self.result["sandbox_operands_ready"] = sb["daemonsets"]
            self.step("install+verify-workload[sandbox]", self.install_and_verify_workload)
            self.step("uninstall[sandbox]", self.uninstall)
        except Exception as e:  # noqa: BLE001 - reported in the result
            self.result["error"] = f"{type(e).__name__}: {e}"
            self.result["pods"] = {o.name(p): (p.get("status") or {}).get("phase")
                                   for p in self.backing.list("v1", "Pod")}
            node = self.backing.get("v1", "Node", self.node)
            self.result["node_labels"] = {k: v for k, v in o.get_labels(node).items() if k.startswith("amd.com/")}
            self.result["clusterpolicy_state"] = self.cp_state()
            self.result["logs_dir"] = self.base
            self.keep = True
        finally:
            self.teardown()
        if self.errors:
            self.result["kubelet_errors"] = self.errors[:20]
        self.result.update(ok=all(s.get("ok") for s in self.steps) and "error" not in self.result,
                           steps=self.steps, marks_s=dict(sorted(self.marks.items(), key=lambda kv: kv[1])),
                           hip_mode=self.hip_mode, sys_root=self.sys_root)
        return self.result


    def run_driver_container(self) -> Dict[str, Any]:
        """The flow with the driver DaemonSet installing amdgpu (driver.enabled=true)."""
        self.setup()
        try:
            self.step("install-operator", self.install_operator)
            first = self.step("verify-operator", lambda: self.verify_operator("install"))
            self.result["time_to_ready_s"] = self.marks.get("install:ready")
            self.result["operands_ready"] = first["daemonsets"]
            self.expected_operands = sorted(first["daemonsets"])
            self.step("verify-operand-restarts", self.verify_operand_restarts)
            self.step("install+verify-workload", self.install_and_verify_workload)
            up = self.step("driver-upgrade", self.driver_upgrade)
            self.result["driver_upgrade_s"] = up["seconds"]
            self.step("uninstall", self.uninstall)
        except Exception as e:  # noqa: BLE001 - reported in the result
            self.result["error"] = f"{type(e).__name__}: {e}"
            self.result["logs_dir"] = self.base
            self.keep = True
        finally:
            self.teardown()
        self.result.update(ok=all(s.get("ok") for s in self.steps) and "error" not in self.result,
                           steps=self.steps, driver="container",
                           marks_s=dict(sorted(self.marks.items(), key=lambda kv: kv[1])))
        return self.result


class MultiNodeE2E(E2E):
    """The same stack over N nodes on one machine (CPU rehearsal): one process kubelet per node,
    each on its own fake sysfs with ``gpus`` GPUs. What the single-node flow cannot show: the
    operator fanning its DaemonSets out over nodes, per-node scheduling of GPU pods, and a
    per-node operands switch (``deploy.operands=false`` on one node) leaving the other nodes'
    pods untouched. The reference has no multi-node test at all."""

    def __init__(self, nodes: int = 3, gpus: int = 8, **kw):
        kw.setdefault("hip_mode", "skip")
        super().__init__(**kw)
        self.n_nodes, self.gpus = nodes, gpus
        self.names = [f"{self.node}-{i}" for i in range(nodes)]

    def node_specs(self) -> List[Tuple[str, str, str]]:
        from ..devices import fakesys
        out = []
        for n in self.names:
            root = str(fakesys.make_node(os.path.join(self.wd, "sys", n), n_gpus=self.gpus))
            out.append((n, root, root))
        return out

    def cluster_policy(self, sandbox: bool = False) -> Dict:
        cp = super().cluster_policy(sandbox)
        # one host, many nodes: every exporter binds an ephemeral port (no pod network namespaces)
        for e in cp["spec"]["metricsExporter"]["env"]:
            if e["name"] == "METRICS_EXPORTER_LISTEN":
                e["value"] = "127.0.0.1:0"
        return cp

    def _pods_by_node(self) -> Dict[str, Dict[str, str]]:
        out: Dict[str, Dict[str, str]] = {n: {} for n in self.names}
        for p in self.operand_pods():
            out.setdefault(p["spec"].get("nodeName", ""), {})[o.name(p)] = p["metadata"]["uid"]
        return out

    def verify_nodes(self) -> Dict:
        ready = self._wait("every operand pod Ready on every node", self.all_ready)
        per = {}
        for k in self.kubelets:
            files = os.listdir(k.host_path("/run/amd/validations"))
            alloc = ((self.backing.get("v1", "Node", k.node).get("status") or {}).get("allocatable") or {}).get(GPU)
            if not {"toolkit-ready", "hip-ready", "plugin-ready"} <= set(files) or alloc != str(self.gpus):
                raise StepFailed(f"node {k.node}: validations {sorted(files)}, {GPU}={alloc}")
            per[k.node] = {GPU: alloc, "validations": len(files)}
        if any(v != self.n_nodes for v in ready.values()):
            raise StepFailed(f"operand DaemonSets not on every node: {ready}")
        return {"daemonsets": ready, "nodes": per}

    def workload_per_node(self) -> Dict:
        names = []
        for n in self.names:
            pod = self.workload_pod()
            pod["metadata"]["name"] = f"gpu-test-{n}"
            pod["spec"]["nodeSelector"] = {"kubernetes.io/hostname": n}
            self.backing.create(pod)
            names.append(pod["metadata"]["name"])

        def done():
            ps = [self.backing.get("v1", "Pod", x, "default") for x in names]
            if any((p.get("status") or {}).get("phase") == "Failed" for p in ps):
                raise StepFailed("a workload pod failed")
            return ps if all((p.get("status") or {}).get("phase") == "Succeeded" for p in ps) else None
        ps = self._wait("one GPU pod per node to succeed", done)
        placed = {o.name(p): p["spec"]["nodeName"] for p in ps}
        if sorted(placed.values()) != sorted(self.names):
            raise StepFailed(f"pods not spread one per node: {placed}")
        for x in names:
            self.backing.delete("v1", "Pod", x, "default")
        return placed

    def disable_one_node(self) -> Dict:
        target, others = self.names[0], self.names[1:]
        before = self._pods_by_node()
        self.backing.patch("v1", "Node", target, {"metadata": {"labels": {OPERANDS_LABEL: "false"}}})
        self._wait(f"operand pods gone from {target}", lambda: not self._pods_by_node().get(target))
        time.sleep(1.0)
        after = self._pods_by_node()
        touched = [n for n in others if after.get(n) != before.get(n)]
        if touched:
            raise StepFailed(f"disabling {target} touched the pods of {touched}")
        self.backing.patch("v1", "Node", target, {"metadata": {"labels": {OPERANDS_LABEL: "true"}}})
        t = time.monotonic()
        self._wait(f"{target} back", lambda: self.all_ready() and len(self._pods_by_node().get(target, {})) ==
                   len(before[target]))
        return {"node": target, "untouched": others, "reenable_s": round(time.monotonic() - t, 3)}

    def uninstall_all(self) -> Dict:
        self.backing.delete("amd.com/v1", "ClusterPolicy", CP_NAME)
        self._wait("operand pods gone", lambda: not self.operand_pods())
        self._wait("every node process gone", lambda: not any(k.all_pids() for k in self.kubelets), timeout=30)
        self.stop_operator()
        return {"ok": True}

    def run(self) -> Dict[str, Any]:
        if self.driver == "container":
            return self.run_driver_container()
        self.setup()
        try:
            self.step("install-operator", self.install_operator)
            first = self.step("verify-operator", self.verify_nodes)
            self.mark("install:ready")
            self.result["time_to_ready_s"] = self.marks.get("install:ready")
            self.result["operands_ready"] = first["daemonsets"]
            self.expected_operands = sorted(first["daemonsets"])
            self.step("verify-operand-restarts", self.verify_operand_restarts)
            self.step("workload-per-node", self.workload_per_node)
            rs = self.step("restart-operator", self.restart_operator)
            self.result["operator_restart_recovery_s"] = rs["recovery_s"]
            self.step("disable-one-node", self.disable_one_node)
            self.step("uninstall", self.uninstall_all)
        except Exception as e:  # noqa: BLE001 - reported in the result
            self.result["error"] = f"{type(e).__name__}: {e}"
            self.result["logs_dir"] = self.base
            self.keep = True
        finally:
            self.teardown()
        self.result.update(ok=all(s.get("ok") for s in self.steps) and "error" not in self.result,
                           steps=self.steps, nodes=self.n_nodes, gpus_per_node=self.gpus,
                           marks_s=dict(sorted(self.marks.items(), key=lambda kv: kv[1])))
        return self.result


def main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="python -m gpu_operator_amd.e2e")
    ap.add_argument("--sys-root", default="/")
    ap.add_argument("--dev-root", default="/")
    ap.add_argument("--hip-mode", default="pod", choices=["pod", "local", "skip"])
    ap.add_argument("--fake-gpus", type=int, default=0, help="run on a fake sysfs with N GPUs (CPU rehearsal)")
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--nodes", type=int, default=1, help="N > 1: that many nodes on fake sysfs (CPU rehearsal)")
    ap.add_argument("--driver-container", action="store_true",
                    help="the driver DaemonSet installs a simulated amdgpu on a fake sysfs (CPU rehearsal)")
    ap.add_argument("--flow", choices=["reference", "fabric", "tenants"], default="reference",
                    help="reference: end-to-end.sh; fabric: the fabric pod on node shapes; tenants: the "
                         "validator beside GPU pods (fake sysfs, no GPU work)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    if a.nodes > 1:
        r = MultiNodeE2E(nodes=a.nodes, gpus=a.fake_gpus or 8, timeout=a.timeout, keep=a.keep).run()
        print(json.dumps(r, default=str))
        return 0 if r["ok"] else 1
    sys_root, dev_root = a.sys_root, a.dev_root
    if a.driver_container:
        from ..devices import fakesys
        root = str(fakesys.make_node(os.path.join(tempfile.mkdtemp(prefix="amd-e2e-sys-"), "root"),
                                     n_gpus=a.fake_gpus or 8, live=False, kfd=False))
        r = E2E(sys_root=root, dev_root=root, hip_mode="skip", timeout=a.timeout, keep=a.keep,
                driver="container").run()
        print(json.dumps(r, default=str))
        return 0 if r["ok"] else 1
    if a.fake_gpus or a.flow != "reference":
        from ..devices import fakesys
        sys_root = dev_root = str(fakesys.make_node(os.path.join(tempfile.mkdtemp(prefix="amd-e2e-sys-"), "root"),
                                                    n_gpus=a.fake_gpus or 8))
    if a.flow != "reference":
        e = E2E(sys_root=sys_root, dev_root=dev_root, hip_mode="skip", timeout=a.timeout, keep=a.keep)
        r = e.run_tenant_cases() if a.flow == "tenants" else e.run_fabric_shapes()
        print(json.dumps(r, default=str))
        return 0 if r["ok"] else 1
    r = E2E(sys_root=sys_root, dev_root=dev_root, hip_mode=a.hip_mode, timeout=a.timeout, keep=a.keep).run()
    print(json.dumps(r, default=str))
    return 0 if r["ok"] else 1
