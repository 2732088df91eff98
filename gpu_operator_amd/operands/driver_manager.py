"""``amd-driver-manager``: safe amdgpu unload before a (new) driver container starts.

Counterpart of the reference's external ``k8s-driver-manager uninstall_driver`` init container
(SURVEY.md §2.3, §3.2 step 3): the driver DaemonSet's first init container. Steps:

1. fast path — nothing to unload: amdgpu not loaded, or loaded by the host (no driver-container
   marker in ``/run/amd/driver``; the host's driver is never touched). This is the common case
   on a fresh node and costs one sysfs read (time-to-ready);
2. pause the GPU operands on this node (deploy labels -> ``paused-for-driver-upgrade``) and
   wait for their pods to leave, so no KFD client holds the device;
3. evict pods holding ``amd.com/gpu*`` / ``amd.com/partition-*`` (``ENABLE_GPU_POD_EVICTION``);
   on failure, drain the node if ``ENABLE_AUTO_DRAIN`` (kubectl-drain options from env);
4. unload amdgpu (and its companion modules) once its refcount is 0; remove the driver
   container's barrier files;
5. always: restore the operand labels and uncordon if this run cordoned.
"""

from __future__ import annotations

import argparse
import logging
import os
import re
import subprocess
import sys
import time
from typing import Callable, Dict, List, Optional

from .. import devices
from ..utils import mounts
from ..controllers.upgrade import gpu_pod_filter
from ..k8s import errors
from ..k8s import objects as o

log = logging.getLogger("amd-driver-manager")

PAUSED = "paused-for-driver-upgrade"
OPERAND_LABELS = {  # deploy label -> app label of its pods
    "amd.com/gpu.deploy.container-toolkit": "amd-container-toolkit-daemonset",
    "amd.com/gpu.deploy.device-plugin": "amd-device-plugin-daemonset",
    "amd.com/gpu.deploy.rdc": "amd-rdc",
    "amd.com/gpu.deploy.metrics-exporter": "amd-metrics-exporter",
    "amd.com/gpu.deploy.node-labeller": "amd-node-labeller",
    "amd.com/gpu.deploy.operator-validator": "amd-operator-validator",
    "amd.com/gpu.deploy.partition-manager": "amd-partition-manager",
    "amd.com/gpu.deploy.node-status-exporter": "amd-node-status-exporter",
}
MODULES = ["amdgpu", "amdxcp", "amddrm_ttm_helper", "amdttm", "amdkcl"]   # DKMS stack, unload order
DRIVER_CTR_MARKER = ".driver-ctr"                                            # in /run/amd/driver
BARRIERS = [".driver-ctr-ready", "driver-ready"]


class DriverManagerError(Exception):
    pass


def _dur(s: str) -> float:
    m = re.fullmatch(r"\s*(\d+(?:\.\d+)?)\s*(ms|s|m|h)?\s*", s or "0")
    if not m:
        raise ValueError(s)
    return float(m.group(1)) * {"ms": 1e-3, "s": 1, "m": 60, "h": 3600, None: 1}[m.group(2)]


class DriverManager:
    def __init__(self, client, node: str, namespace: str, sys_root: str = "/", run_dir: str = "/run/amd",
                 evict_gpu_pods: bool = True, auto_drain: bool = False, drain_force: bool = False,
                 drain_selector: str = "", drain_timeout: float = 0.0, drain_empty_dir: bool = False,
                 pods_timeout: float = 300.0, poll: float = 1.0, run: Callable = subprocess.run,
                 host_root: str = "/host"):
        self.client = client
        self.node = node
        self.namespace = namespace
        self.sys_root = sys_root
        self.run_dir = run_dir
        self.evict_gpu_pods = evict_gpu_pods
        self.auto_drain = auto_drain
        self.drain_force = drain_force
        self.drain_selector = drain_selector
        self.drain_timeout = drain_timeout
        self.drain_empty_dir = drain_empty_dir
        self.pods_timeout = pods_timeout
        self.poll = poll
        self.run = run
        self.host_root = host_root
        self.cordoned = False

    @classmethod
    def from_env(cls, client, **kw) -> "DriverManager":
        e = os.environ
        t = lambda k, d: e.get(k, d).lower() == "true"  # noqa: E731
        return cls(client, e.get("NODE_NAME", ""), e.get("OPERATOR_NAMESPACE", ""),
                   sys_root=e.get("AMD_SYSFS_ROOT", "/"), run_dir=mounts.path("/run/amd"),
                   host_root=mounts.path("/host"),
                   evict_gpu_pods=t("ENABLE_GPU_POD_EVICTION", "true"), auto_drain=t("ENABLE_AUTO_DRAIN", "false"),
                   drain_force=t("DRAIN_USE_FORCE", "false"), drain_selector=e.get("DRAIN_POD_SELECTOR_LABEL", ""),
                   drain_timeout=_dur(e.get("DRAIN_TIMEOUT_SECONDS", "0s")),
                   drain_empty_dir=t("DRAIN_DELETE_EMPTYDIR_DATA", "false"), **kw)

    # -- driver state -------------------------------------------------------------------------
    def module_loaded(self) -> bool:
        return devices.driver_state(self.sys_root)["module_loaded"]

    def loaded_by_container(self) -> bool:
        return os.path.exists(os.path.join(self.run_dir, "driver", DRIVER_CTR_MARKER))

    def refcount(self, module: str = "amdgpu") -> int:
        try:
            with open(os.path.join(self.sys_root, "sys/module", module, "refcnt")) as f:
                return int(f.read().strip() or 0)
        except (OSError, ValueError):
            return 0

    # -- main ---------------------------------------------------------------------------------
    def uninstall_driver(self) -> str:
        t0 = time.monotonic()
        if not self.module_loaded():
            self._clear_barriers()
            log.info("amdgpu not loaded: nothing to unload (%.3fs)", time.monotonic() - t0)
            return "not-loaded"
        if not self.loaded_by_container():
            log.info("amdgpu was loaded by the host: leaving it in place")
            return "host-driver"
        paused: Dict[str, str] = {}
        try:
            paused = self.pause_operands()
            self.wait_operands_gone()
            if self.evict_gpu_pods:
                ok = self.evict()
                if not ok:
                    if not self.auto_drain:
                        raise DriverManagerError("GPU pods could not be evicted and auto drain is disabled")
                    self.drain()
            elif self.auto_drain:
                self.drain()
            self.unload()
        finally:
            self.resume_operands(paused)
            if self.cordoned:
                self.client.patch("v1", "Node", self.node, {"spec": {"unschedulable": None}})
                self.cordoned = False
        self._clear_barriers()
        log.info("driver unloaded in %.3fs", time.monotonic() - t0)
        return "unloaded"

    # -- operands -----------------------------------------------------------------------------
    def pause_operands(self) -> Dict[str, str]:
        labels = o.get_labels(self.client.get("v1", "Node", self.node))
        paused = {k: v for k, v in labels.items() if k in OPERAND_LABELS and v == "true"}
        if paused:
            self.client.patch("v1", "Node", self.node, {"metadata": {"labels": {k: PAUSED for k in paused}}})
            log.info("paused operands: %s", sorted(paused))
        return paused

    def resume_operands(self, paused: Dict[str, str]) -> None:
        if not paused:
            return
        labels = o.get_labels(self.client.get("v1", "Node", self.node))
        patch = {k: v for k, v in paused.items() if labels.get(k) == PAUSED}
        if patch:
            self.client.patch("v1", "Node", self.node, {"metadata": {"labels": patch}})

    def _node_pods(self, label_selector=None) -> List[Dict]:
        return [p for p in self.client.list("v1", "Pod", label_selector=label_selector,
                                            field_selector=f"spec.nodeName={self.node}")
                if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]

    def wait_operands_gone(self) -> None:
        apps = set(OPERAND_LABELS.values())
        deadline = time.monotonic() + self.pods_timeout
        while True:
            left = [o.name(p) for p in self._node_pods() if o.get_labels(p).get("app") in apps]
            if not left:
                return
            if time.monotonic() > deadline:
                raise DriverManagerError(f"operand pods still running: {left}")
            time.sleep(self.poll)

    # -- eviction / drain ---------------------------------------------------------------------
    def _evict_all(self, pods: List[Dict], force: bool, empty_dir: bool, deadline: Optional[float]) -> List[str]:
        errs = []
        for p in pods:
            owner = o.controller_of(p)
            if owner and owner.get("kind") == "DaemonSet":
                continue
            if "kubernetes.io/config.mirror" in o.get_annotations(p):
                continue
            if any("emptyDir" in v for v in (p.get("spec") or {}).get("volumes") or []) and not empty_dir:
                errs.append(f"{o.name(p)}: uses emptyDir")
                continue
            if owner is None and not force:
                errs.append(f"{o.name(p)}: not managed by a controller")
                continue
            try:
                self.client.evict(o.name(p), o.namespace(p))
            except errors.NotFound:
                pass
            except errors.ApiError as e:
                errs.append(f"{o.name(p)}: {e}")
        if errs:
            return errs
        # wait for them to be gone
        names = {(o.namespace(p), o.name(p)) for p in pods}
        while True:
            left = [p for p in self._node_pods() if (o.namespace(p), o.name(p)) in names]
            if not left:
                return []
            if deadline is not None and time.monotonic() > deadline:
                return [f"{o.name(p)}: still terminating" for p in left]
            time.sleep(self.poll)

    def evict(self) -> bool:
        pods = [p for p in self._node_pods() if gpu_pod_filter(p)]
        if not pods:
            return True
        log.info("evicting %d GPU pod(s)", len(pods))
        # conservative (no force, no emptyDir loss); the drain fallback applies the drain options
        errs = self._evict_all(pods, force=False, empty_dir=False, deadline=time.monotonic() + self.pods_timeout)
        if errs:
            log.warning("GPU pod eviction incomplete: %s", errs)
        return not errs

    def drain(self) -> None:
        self.client.patch("v1", "Node", self.node, {"spec": {"unschedulable": True}})
        self.cordoned = True
        sel = "amd.com/gpu-driver-upgrade-drain.skip!=true"
        if self.drain_selector:
            sel = f"{self.drain_selector},{sel}"
        deadline = time.monotonic() + self.drain_timeout if self.drain_timeout else None
        errs = self._evict_all(self._node_pods(sel), force=self.drain_force, empty_dir=self.drain_empty_dir,
                               deadline=deadline)
        if errs:
            raise DriverManagerError(f"drain failed: {errs}")

    # -- module unload ------------------------------------------------------------------------
    def unload(self) -> None:
        users = self.refcount("amdgpu")
        if users > 0:
            raise DriverManagerError(f"amdgpu still in use (refcnt {users})")
        loaded = [m for m in MODULES if os.path.isdir(os.path.join(self.sys_root, "sys/module", m))]
        if not loaded:
            return
        p = self.run(["chroot", self.host_root, "modprobe", "-r"] + loaded, capture_output=True, text=True,
                     timeout=120)
        if p.returncode != 0:
            raise DriverManagerError(f"modprobe -r {' '.join(loaded)} failed: {(p.stderr or '').strip()}")
        log.info("unloaded %s", loaded)

    def _clear_barriers(self) -> None:
        for b in BARRIERS:
            try:
                os.unlink(os.path.join(self.run_dir, "validations", b))
            except FileNotFoundError:
                pass


def main(argv=None, client=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-driver-manager")
    ap.add_argument("command", choices=["uninstall_driver", "preflight"])
    a = ap.parse_args(argv)
    if client is None:
        from ..k8s.rest import RestClient
        client = RestClient()
    dm = DriverManager.from_env(client)
    if a.command == "preflight":
        print({"loaded": dm.module_loaded(), "container": dm.loaded_by_container(), "refcnt": dm.refcount()})
        return 0
    try:
        print(dm.uninstall_driver())
        return 0
    except DriverManagerError as e:
        log.error("%s", e)
        client.create_event(client.get("v1", "Node", dm.node), "DriverUnloadFailed", str(e), "Warning")
        return 1


if __name__ == "__main__":
    sys.exit(main())
