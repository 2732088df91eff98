"""Compute / memory partition manager (``amd-partition-manager``): the MIG-manager role.

The reference deploys NVIDIA's mig-manager driven by the ``nvidia.com/mig.config`` label
(reference: assets/state-mig-manager/*). MI355X partitions differently:
a physical GPU (8 XCDs, 256 CUs, 288 GB) is split into 1/2/4/8 compute partitions
(SPX/DPX/QPX/CPX) and its memory into NPS1/NPS2 domains, through
``current_{compute,memory}_partition`` in sysfs; the driver then re-enumerates the KFD
agents and render nodes. This agent:

1. reads the desired layout (node label ``amd.com/gpu.partition.config`` -> a named entry of
   the partition ConfigMap, or DEFAULT_PARTITION_CONFIG);
2. if the node differs: state ``pending``; pauses the GPU clients by flipping their deploy
   labels to ``paused-for-partition-change`` (their DaemonSet pods leave the node) and waits
   for those pods to be gone; stops listed host services;
3. applies the memory (NPS) modes; an NPS change only takes effect once amdgpu reloads, so the
   node goes ``reload-required`` -> ``reloading``: ``modprobe -r amdgpu && modprobe amdgpu`` on
   the host, a request to the driver container when it owns the module (DRIVER_RELOAD_VIA=
   driver-container), or DRIVER_RELOAD_CMD; then a bounded wait for
   ``initstate=live``; then the compute modes (validated against ``available_*_partition``);
4. waits (bounded) until the KFD agent count matches the new layout — the re-enumeration;
5. restores the deploy labels (the device plugin comes back and re-registers the new
   devices), writes the ``partition-applied`` barrier (relabels the node), records
   ``state=success`` and the applied config on the node. Any failure -> ``state=failed``
   with the reason in an event; labels are always restored (also labels a crashed agent left
   paused: the next reconcile restores them).

All state lives on the Node, so a restarted agent resumes or re-verifies.
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import shlex
import subprocess
import sys
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

import yaml

from .. import devices
from ..utils import mounts
from ..k8s import errors
from ..k8s import objects as o

log = logging.getLogger("amd-partition-manager")

CONFIG_LABEL = "amd.com/gpu.partition.config"
STATE_LABEL = "amd.com/gpu.partition.state"
APPLIED_ANNOTATION = "amd.com/gpu.partition.applied"
PAUSED = "paused-for-partition-change"
PARTS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
CLIENT_DEPLOY_LABELS = ["amd.com/gpu.deploy.device-plugin", "amd.com/gpu.deploy.metrics-exporter",
                        "amd.com/gpu.deploy.rdc", "amd.com/gpu.deploy.operator-validator",
                        "amd.com/gpu.deploy.node-status-exporter"]
CLIENT_APPS = ["amd-device-plugin-daemonset", "amd-metrics-exporter", "amd-rdc", "amd-operator-validator",
               "amd-node-status-exporter"]


class PartitionError(Exception):
    pass


def load_config(path: str) -> Dict[str, List[Dict]]:
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    if doc.get("version") != "v1":
        raise PartitionError(f"unsupported partition config version {doc.get('version')!r}")
    return doc.get("partition-configs") or {}


def desired_layout(entries: List[Dict], n_gpus: int) -> Dict[int, Tuple[str, str]]:
    out: Dict[int, Tuple[str, str]] = {}
    for e in entries:
        devs = list(range(n_gpus)) if e.get("devices") == "all" else [int(x) for x in e.get("devices", [])]
        compute = str(e.get("compute", "SPX")).upper()
        memory = str(e.get("memory", "NPS1")).upper()
        if compute not in PARTS:
            raise PartitionError(f"invalid compute partition {compute}")
        for d in devs:
            if d >= n_gpus:
                raise PartitionError(f"device {d} out of range (node has {n_gpus} GPUs)")
            out[d] = (compute, memory)
    return out


def physical_gpus(root: Optional[str]) -> List[Dict]:
    seen: Dict[str, Dict] = {}
    for g in devices.enumerate_gpus(root):
        seen.setdefault(g["pci_bdf"], g)
    return [seen[k] for k in sorted(seen)]


class PartitionManager:
    def __init__(self, client, node: str, config_file: str, root: Optional[str] = None,
                 default_config: str = "", barrier_dir: str = "/run/amd/validations",
                 reenumerate: Optional[Callable[[], None]] = None, enum_timeout: float = 120.0,
                 pods_timeout: float = 300.0, host_services: Optional[List[str]] = None,
                 run: Callable = subprocess.run, namespace: str = "",
                 reload_driver: Optional[Callable[[], None]] = None, reload_cmd: str = "",
                 reload_timeout: float = 600.0, reload_via: str = "", driver_dir: str = "/run/amd/driver"):
        self.client = client
        self.node = node
        self.config_file = config_file
        self.root = root
        self.default_config = default_config
        self.barrier_dir = barrier_dir
        self.reenumerate = reenumerate        # tests: simulate the driver's re-enumeration
        self.enum_timeout = enum_timeout
        self.pods_timeout = pods_timeout
        self.host_services = host_services or []
        self.run = run
        self.namespace = namespace
        self.reload_driver = reload_driver or self._reload_driver   # tests inject the driver's reload
        self.reload_cmd = reload_cmd
        self.reload_timeout = reload_timeout
        self.reload_via = reload_via          # "driver-container": ask the driver pod (request file)
        self.driver_dir = driver_dir

    # -- node state -----------------------------------------------------------------------------
    def _node(self) -> Dict:
        return self.client.get("v1", "Node", self.node)

    def _label(self, key: str, value: Optional[str]) -> None:
        self.client.patch("v1", "Node", self.node, {"metadata": {"labels": {key: value}}})

    def set_state(self, state: str, applied: Optional[str] = None) -> None:
        patch: Dict = {"metadata": {"labels": {STATE_LABEL: state}}}
        if applied is not None:
            patch["metadata"]["annotations"] = {APPLIED_ANNOTATION: applied}
        self.client.patch("v1", "Node", self.node, patch)

    # -- main entry -------------------------------------------------------------------------------
    def reconcile(self) -> str:
        node = self._node()
        labels = o.get_labels(node)
        selected = labels.get(CONFIG_LABEL) or self.default_config
        if not selected:
            return "no-config"
        gpus = physical_gpus(self.root)
        try:
            configs = load_config(self.config_file)
            if selected not in configs:
                raise PartitionError(f"partition config {selected!r} not found in {sorted(configs)}")
            want = desired_layout(configs[selected], len(gpus))
        except PartitionError as e:
            self._fail(str(e))
            return "failed"
        todo = [(i, g, want[i]) for i, g in enumerate(gpus) if i in want and
                (g["compute_partition"], g["memory_partition"]) != want[i]]
        if not todo:
            self.resume_clients(self._left_paused(labels))      # a crashed agent's pause
            if labels.get(STATE_LABEL) != "success" or o.get_annotations(node).get(APPLIED_ANNOTATION) != selected:
                self.set_state("success", selected)
                self._barrier(selected)
            return "in-sync"
        log.info("applying partition config %s to %d GPU(s)", selected, len(todo))
        self.set_state("pending")
        paused: List[str] = []
        try:
            # the relabel is recorded before the wait, so the finally below always restores it
            paused = self.pause_clients(labels)
            self.wait_clients_gone()
            self.stop_host_services()
            mem = [(g, m) for _, g, (_, m) in todo if g["memory_partition"] and g["memory_partition"] != m]
            for g, memory in mem:
                self._set(g, "memory", memory)
            if mem:
                self.set_state("reload-required")
                self.set_state("reloading")
                self.reload_driver()
                self.wait_driver_live()
                gpus = physical_gpus(self.root)                 # re-read: the reload re-enumerated
            for i, g in enumerate(gpus):
                if i in want and g["compute_partition"] != want[i][0]:
                    self._set(g, "compute", want[i][0])
            if self.reenumerate:
                self.reenumerate()
            self.wait_reenumerated(want, len(gpus))
        except PartitionError as e:
            self._fail(str(e))
            return "failed"
        finally:
            self.resume_clients(paused)
            self.start_host_services()
        self.set_state("success", selected)
        self._barrier(selected)
        return "applied"

    # -- driver reload (memory partition) ----------------------------------------------------------
    def _reload_driver(self) -> None:
        """Unload and reload amdgpu so a new NPS mode takes effect. The GPU clients
        are paused and the host services stopped by now; a failing step is a PartitionError.

        With the driver container owning the module (``reload_via="driver-container"``) the
        reload is its job -- only it has the module tree that loaded amdgpu: a request file in the
        shared driver dir, answered by ``amdgpu-driver`` with a result carrying the same id."""
        if self.reload_via == "driver-container":
            self._reload_via_driver_container()
            return
        cmds = [shlex.split(c) for c in self.reload_cmd.split(";") if c.strip()] if self.reload_cmd else \
            [["chroot", "/host", "modprobe", "-r", "amdgpu"], ["chroot", "/host", "modprobe", "amdgpu"]]
        for cmd in cmds:
            try:
                p = self.run(cmd, capture_output=True, text=True, timeout=self.reload_timeout)
            except (OSError, subprocess.TimeoutExpired) as e:
                raise PartitionError(f"driver reload: {' '.join(cmd)}: {e}") from e
            if getattr(p, "returncode", 0) != 0:
                err = (getattr(p, "stderr", "") or "").strip()[-300:]
                raise PartitionError(f"driver reload: {' '.join(cmd)} exited {p.returncode}: {err}")

    def _reload_via_driver_container(self) -> None:
        import uuid
        from .driver_container import RELOAD_REQUEST, RELOAD_RESULT
        rid = uuid.uuid4().hex
        os.makedirs(self.driver_dir, exist_ok=True)
        req = os.path.join(self.driver_dir, RELOAD_REQUEST)
        now = time.time()
        # the deadline travels with the request: the driver container fits its unload / load /
        # readiness wait into it, and ignores the request once it has passed
        with open(req + ".tmp", "w") as f:
            json.dump({"id": rid, "node": self.node, "ts": now, "deadline": now + self.reload_timeout}, f)
        os.replace(req + ".tmp", req)
        try:
            self._await_reload(rid)
        except PartitionError:
            self._withdraw_request(req, rid)
            raise

    @staticmethod
    def _withdraw_request(req: str, rid: str) -> None:
        """Remove our request if it is still unanswered: a driver container that (re)starts later
        must not unload amdgpu for a request nobody waits for any more."""
        try:
            with open(req) as f:
                if (json.load(f) or {}).get("id") != rid:
                    return
            os.unlink(req)
        except (OSError, ValueError):
            pass

    def _await_reload(self, rid: str) -> None:
        from .driver_container import RELOAD_RESULT
        res_path = os.path.join(self.driver_dir, RELOAD_RESULT)
        deadline = time.monotonic() + self.reload_timeout
        while True:
            try:
                with open(res_path) as f:
                    res = json.load(f)
                if res.get("id") == rid:
                    break
            except (OSError, ValueError):
                pass
            left = deadline - time.monotonic()
            if left <= 0:
                raise PartitionError(f"driver container did not answer reload request {rid} within "
                                     f"{self.reload_timeout:.0f}s (is the driver pod running?)")
            if os.path.exists(res_path):            # an older request's answer: poll for ours
                time.sleep(min(0.1, left))
                continue
            try:
                devices.wait_files(self.driver_dir, [RELOAD_RESULT], timeout=min(1.0, left))
            except Exception:  # noqa: BLE001 - no inotify: poll
                time.sleep(min(0.2, left))
        if not res.get("ok"):
            raise PartitionError(f"driver container reload failed: {res.get('error')}")
        log.info("driver container reloaded amdgpu: %s", res.get("info"))

    def wait_driver_live(self) -> None:
        deadline = time.monotonic() + self.reload_timeout
        while not devices.driver_state(self.root)["live"]:
            if time.monotonic() > deadline:
                raise PartitionError("amdgpu did not come back live after the reload")
            time.sleep(0.5)

    def _set(self, g: Dict, kind: str, mode: str) -> None:
        avail = g[f"available_{kind}_partitions"]
        if avail and mode not in avail:
            raise PartitionError(f"GPU {g['pci_bdf']}: {kind} partition {mode} not in {avail}")
        try:
            devices.set_partition(g["pci_bdf"], kind, mode, root=self.root)
        except ValueError as e:
            raise PartitionError(f"GPU {g['pci_bdf']}: {e}") from e

    def wait_reenumerated(self, want: Dict[int, Tuple[str, str]], n_gpus: int) -> None:
        expected = sum(PARTS[want.get(i, (None,))[0]] if i in want else 0 for i in range(n_gpus))
        untouched = [g for i, g in enumerate(physical_gpus(self.root)) if i not in want]
        expected += sum(PARTS.get(g["compute_partition"] or "SPX", 1) for g in untouched)
        deadline = time.monotonic() + self.enum_timeout
        while True:
            agents = devices.enumerate_gpus(self.root)
            modes_ok = all((g["compute_partition"], g["memory_partition"]) == want[i]
                           for i, g in enumerate(physical_gpus(self.root)) if i in want)
            if len(agents) == expected and modes_ok:
                return
            if time.monotonic() > deadline:
                raise PartitionError(f"KFD re-enumeration incomplete: {len(agents)} agents, expected {expected}")
            time.sleep(0.5)

    # -- GPU clients -----------------------------------------------------------------------------
    @staticmethod
    def _left_paused(labels: Dict[str, str]) -> List[str]:
        return [k for k in CLIENT_DEPLOY_LABELS if labels.get(k) == PAUSED]

    def pause_clients(self, labels: Optional[Dict[str, str]] = None) -> List[str]:
        """Flip the enabled GPU clients' deploy labels to PAUSED (their DaemonSet pods leave the node);
        returns what it paused (including labels an earlier, crashed run left paused)."""
        labels = labels if labels is not None else o.get_labels(self._node())
        paused = [k for k in CLIENT_DEPLOY_LABELS if labels.get(k) in ("true", PAUSED)]
        if paused:
            self.client.patch("v1", "Node", self.node, {"metadata": {"labels": {k: PAUSED for k in paused}}})
        return paused

    def wait_clients_gone(self) -> None:
        deadline = time.monotonic() + self.pods_timeout
        while True:
            left = [p for p in self.client.list("v1", "Pod", self.namespace,
                                                field_selector=f"spec.nodeName={self.node}")
                    if o.get_labels(p).get("app") in CLIENT_APPS]
            if not left:
                return
            if time.monotonic() > deadline:
                raise PartitionError(f"GPU clients still running: {[o.name(p) for p in left]}")
            time.sleep(1.0)

    def resume_clients(self, paused: List[str]) -> None:
        if paused:
            self.client.patch("v1", "Node", self.node, {"metadata": {"labels": {k: "true" for k in paused}}})

    def _systemctl(self, verb: str, svc: str) -> None:
        try:
            self.run(["chroot", "/host", "systemctl", verb, svc], capture_output=True, timeout=60)
        except (OSError, subprocess.TimeoutExpired) as e:
            log.warning("systemctl %s %s: %s", verb, svc, e)

    def stop_host_services(self) -> None:
        for s in self.host_services:
            self._systemctl("stop", s)

    def start_host_services(self) -> None:
        for s in self.host_services:
            self._systemctl("start", s)

    def _barrier(self, config: str) -> None:
        try:
            os.makedirs(self.barrier_dir, exist_ok=True)
            with open(os.path.join(self.barrier_dir, "partition-applied"), "w") as f:
                f.write(f'{{"config": "{config}", "ts": {time.time()}}}')
        except OSError as e:
            log.warning("cannot write partition barrier: %s", e)

    def _fail(self, msg: str) -> None:
        log.error("partitioning failed: %s", msg)
        self.set_state("failed")
        node = self._node()
        self.client.create_event(node, "PartitionFailed", msg, "Warning")


def load_clients(path: Optional[str]) -> List[str]:
    if not path or not os.path.exists(path):
        return []
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    return list(doc.get("systemd-services") or [])


def main(argv=None, client=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-partition-manager")
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--config-file", default=os.environ.get("CONFIG_FILE", mounts.path("/partition-config/config.yaml")))
    ap.add_argument("--gpu-clients-file", default=os.environ.get("GPU_CLIENTS_FILE", mounts.path("/gpu-clients/clients.yaml")))
    ap.add_argument("--default", default=os.environ.get("DEFAULT_PARTITION_CONFIG", ""))
    ap.add_argument("--namespace", default=os.environ.get("OPERATOR_NAMESPACE", ""))
    ap.add_argument("--resync", type=float, default=300.0)
    ap.add_argument("--reload-cmd", default=os.environ.get("DRIVER_RELOAD_CMD", ""),
                    help="';'-separated commands that reload amdgpu (default: modprobe -r/modprobe via /host)")
    ap.add_argument("--reload-via", default=os.environ.get("DRIVER_RELOAD_VIA", ""), choices=["", "driver-container"],
                    help="driver-container: ask the amdgpu driver pod to reload (it owns the module tree)")
    a = ap.parse_args(argv)
    if client is None:
        from ..k8s.rest import RestClient
        client = RestClient()
    pm = PartitionManager(client, a.node_name, a.config_file, default_config=a.default, namespace=a.namespace,
                          barrier_dir=mounts.path("/run/amd/validations"),
                          host_services=load_clients(a.gpu_clients_file), reload_cmd=a.reload_cmd,
                          reload_via=a.reload_via, driver_dir=mounts.path("/run/amd/driver"))
    kick = threading.Event()

    def on_node(ev):
        if o.name(ev.obj) != a.node_name:
            return
        old = o.get_labels(ev.old) if ev.old else {}
        if old.get(CONFIG_LABEL) != o.get_labels(ev.obj).get(CONFIG_LABEL):
            kick.set()
    client.watch("v1", "Node", on_node, field_selector=f"metadata.name={a.node_name}")
    while True:
        try:
            log.info("reconcile: %s", pm.reconcile())
        except errors.ApiError as e:
            log.error("API error: %s", e)
        kick.wait(a.resync)
        kick.clear()


if __name__ == "__main__":
    sys.exit(main())
