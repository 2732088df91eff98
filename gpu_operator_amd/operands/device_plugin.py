"""ROCm device plugin: advertises AMD GPUs to the kubelet (``amd-device-plugin``).

The reference deploys NVIDIA's external k8s-device-plugin image; this is
the MI355X-native counterpart the north star asks for:

* one schedulable device per KFD GPU agent, i.e. per whole GPU in SPX mode and per compute
  partition otherwise (a CPX-mode MI355X node exposes 64 devices of 32 CUs);
* resource naming by ``PARTITION_STRATEGY``: ``single``/``none`` -> every agent is
  ``amd.com/gpu``; ``mixed`` -> SPX GPUs are ``amd.com/gpu``, partitions are
  ``amd.com/partition-<mode>`` (mirrors the reference's MIG strategies, reference:
  api/v1/clusterpolicy_types.go:1483-1493);
* Allocate injects ``/dev/kfd`` + the agent's ``/dev/dri/renderD<minor>`` (device-specs) or
  CDI device names, and ``AMD_VISIBLE_DEVICES`` with the allocated unique ids;
* GetPreferredAllocation packs partitions of one physical GPU together and otherwise keeps
  allocations inside one NUMA domain / xGMI hive;
* time-slicing (``sharing.timeSlicing.resources[].replicas``) advertises N replicas per
  device, as the reference's e2e exercises with NVIDIA's plugin (tests/scripts/update-
  clusterpolicy.sh);
* re-registers when kubelet restarts (inotify on kubelet.sock) and reloads its config on
  SIGHUP (sent by the config-manager sidecar);
* health (``check_health``, every ``DP_HEALTH_PERIOD_S``): a device is Unhealthy -- the kubelet stops
  allocating it -- when the driver is not live, its KFD agent vanished, it reports uncorrectable RAS
  errors in any block (HBM/umc, gfx, sdma, xgmi, ... above ``DP_HEALTH_UE_MAX``, default 0) or its
  retired HBM pages reach ``DP_HEALTH_RETIRED_PAGES_MAX`` (default 128). The RAS counters are the
  libamdnode telemetry the metrics exporter publishes. The reference ships NVIDIA's plugin, which
  withdraws devices on critical XID events; in-repo it re-validates the driver every 60 s
  (reference: validator/metrics.go:237-250). Each device's state and reason go to the node status
  directory (``device-health``) for the node metrics exporter (``node_device_unhealthy``).
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import sys
import threading
import time
from concurrent import futures
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional

import yaml

from .. import devices
from ..utils import mounts
from . import kubeletapi as K

log = logging.getLogger("amd-device-plugin")

GPU_RESOURCE = "amd.com/gpu"
DEVICE_HEALTH_FILE = "device-health"     # in the node status directory (validator/status.py)
PARTITION_PREFIX = "amd.com/partition-"
REPLICA_SEP = "::"


def _unlink(path: str) -> None:
    """Remove a unix socket path that grpc's ``server.stop()`` may be unlinking concurrently."""
    try:
        os.remove(path)
    except FileNotFoundError:
        pass


@dataclass
class Device:
    id: str
    resource: str
    render_minor: int
    card: int
    numa: int
    bdf: str
    unique_id: int
    partition: str
    hive: int
    healthy: bool = True
    reason: str = ""             # why it is unhealthy ("" when healthy)
    replica_of: Optional[str] = None
    vram_bytes: int = 0          # this device's HBM share from sysfs (a partition's under CPX/NPSx)


@dataclass
class Config:
    partition_strategy: str = "single"
    device_id_strategy: str = "uuid"          # uuid | index
    device_list_strategy: str = "device-specs"  # device-specs | envvar | cdi-annotations | cdi-cri
    pass_device_specs: bool = True
    fail_on_init_error: bool = True
    replicas: Dict[str, int] = field(default_factory=dict)
    rename_by_default: bool = False
    cdi_annotation_prefix: str = "amd.cdi.k8s.io/"

    @classmethod
    def load(cls, path: Optional[str], env: Dict[str, str]) -> "Config":
        c = cls(partition_strategy=env.get("PARTITION_STRATEGY", "single"),
                device_id_strategy=env.get("DEVICE_ID_STRATEGY", "uuid"),
                device_list_strategy=env.get("DEVICE_LIST_STRATEGY", "device-specs"),
                pass_device_specs=env.get("PASS_DEVICE_SPECS", "true") == "true",
                fail_on_init_error=env.get("FAIL_ON_INIT_ERROR", "true") == "true",
                cdi_annotation_prefix=env.get("CDI_ANNOTATION_PREFIX", "amd.cdi.k8s.io/"))
        if path and os.path.exists(path):
            with open(path) as f:
                doc = yaml.safe_load(f) or {}
            flags = doc.get("flags") or {}
            c.partition_strategy = flags.get("partitionStrategy", flags.get("migStrategy", c.partition_strategy))
            c.device_id_strategy = flags.get("deviceIDStrategy", c.device_id_strategy)
            c.device_list_strategy = flags.get("deviceListStrategy", c.device_list_strategy)
            ts = ((doc.get("sharing") or {}).get("timeSlicing") or {})
            c.rename_by_default = bool(ts.get("renameByDefault", False))
            for r in ts.get("resources") or []:
                c.replicas[r["name"]] = int(r.get("replicas", 1))
        return c


@dataclass
class HealthPolicy:
    """When a device stops being allocatable (module docstring). ``ue_max``: uncorrectable RAS errors
    tolerated over all blocks (-1: not checked); ``retired_pages_max``: retired HBM pages at which the
    device is withdrawn (-1: not checked)."""
    ue_max: int = 0
    retired_pages_max: int = 128

    @classmethod
    def from_env(cls, env: Dict[str, str]) -> "HealthPolicy":
        return cls(ue_max=int(env.get("DP_HEALTH_UE_MAX", "0") or 0),
                   retired_pages_max=int(env.get("DP_HEALTH_RETIRED_PAGES_MAX", "128") or 128))

    def verdict(self, tele: Optional[Dict]) -> str:
        """"" when the telemetry is healthy, else the reason."""
        if not tele:
            return ""
        ue = tele.get("ras_ue_total", -1)
        if ue is None or ue < 0:
            ue = tele.get("ecc_uncorrectable", -1)
        if self.ue_max >= 0 and ue is not None and ue > self.ue_max:
            blocks = tele.get("ras_ue_blocks") or "umc"
            return f"uncorrectable RAS errors: {ue} ({blocks})"
        retired = tele.get("bad_pages_retired", -1)
        if self.retired_pages_max >= 0 and retired is not None and retired >= self.retired_pages_max:
            return f"retired HBM pages: {retired} (limit {self.retired_pages_max})"
        return ""


def discover(cfg: Config, root: Optional[str] = None) -> List[Device]:
    gpus = devices.enumerate_gpus(root)
    out: List[Device] = []
    for g in gpus:
        part = (g["compute_partition"] or "SPX").upper()
        if cfg.partition_strategy == "mixed" and part != "SPX":
            res = PARTITION_PREFIX + part.lower()
        else:
            res = GPU_RESOURCE
        did = f"amdgpu-{g['unique_id']:016x}" if cfg.device_id_strategy == "uuid" and g["unique_id"] \
            else str(g["index"])
        out.append(Device(did, res, g["drm_render_minor"], g["drm_card"], g["numa_node"], g["pci_bdf"],
                          g["unique_id"], part, g["xgmi_hive_id"], vram_bytes=int(g.get("vram_total") or 0)))
    if cfg.partition_strategy == "single":
        modes = {d.partition for d in out}
        if len(modes) > 1:
            raise ValueError(f"partition strategy 'single' needs uniformly partitioned GPUs, found {sorted(modes)}")
    # time-slicing replicas
    if cfg.replicas:
        rep: List[Device] = []
        for d in out:
            n = cfg.replicas.get(d.resource, 1)
            if n <= 1:
                rep.append(d)
                continue
            for k in range(n):
                r = Device(**{**d.__dict__, "id": f"{d.id}{REPLICA_SEP}{k}", "replica_of": d.id})
                if cfg.rename_by_default:
                    r.resource = d.resource + ".shared"
                rep.append(r)
        out = rep
    return out


def prefer(available: List[Device], must: List[Device], size: int) -> List[str]:
    """Pick ``size`` devices: must-includes first; then prefer the same physical GPU (packs
    partitions), the same NUMA node and xGMI hive as what is already chosen."""
    chosen = list(must)
    pool = [d for d in available if d.id not in {c.id for c in chosen}]
    while len(chosen) < size and pool:
        def score(d: Device):
            s = 0
            for c in chosen:
                s += 100 if d.bdf == c.bdf else 0
                s += 10 if d.numa == c.numa else 0
                s += 5 if d.hive and d.hive == c.hive else 0
            # stable: lowest render minor first on ties
            return (-s, d.numa, d.render_minor, d.id)
        pool.sort(key=score)
        chosen.append(pool.pop(0))
    return [c.id for c in chosen[:size]]


class ResourceServer:
    """One gRPC DevicePlugin server per resource name."""

    def __init__(self, resource: str, plugin: "DevicePlugin"):
        self.resource = resource
        self.plugin = plugin
        self.socket = os.path.join(plugin.plugin_dir,
                                   "amd-" + resource.split("/", 1)[1].replace(".", "-") + ".sock")
        self.server = None
        self._changed = threading.Condition()
        self._version = 0
        self._stop = threading.Event()

    def devices(self) -> List[Device]:
        return [d for d in self.plugin.devices if d.resource == self.resource]

    def notify(self) -> None:
        with self._changed:
            self._version += 1
            self._changed.notify_all()

    # -- DevicePlugin service -------------------------------------------------------------------
    def GetDevicePluginOptions(self, req, ctx):  # noqa: N802
        return K.DP["DevicePluginOptions"](pre_start_required=False, get_preferred_allocation_available=True)

    def _list(self):
        resp = K.DP["ListAndWatchResponse"]()
        for d in self.devices():
            dev = resp.devices.add(ID=d.id, health=K.HEALTHY if d.healthy else K.UNHEALTHY)
            if d.numa >= 0:
                dev.topology.nodes.add(ID=d.numa)
        return resp

    def ListAndWatch(self, req, ctx):  # noqa: N802
        seen = -1
        while not self._stop.is_set() and (ctx is None or ctx.is_active()):
            with self._changed:
                if seen == self._version:
                    self._changed.wait(timeout=1.0)
                    if seen == self._version:
                        continue
                seen = self._version
            yield self._list()

    def GetPreferredAllocation(self, req, ctx):  # noqa: N802
        resp = K.DP["PreferredAllocationResponse"]()
        by_id = {d.id: d for d in self.devices()}
        for cr in req.container_requests:
            avail = [by_id[i] for i in cr.available_deviceIDs if i in by_id]
            must = [by_id[i] for i in cr.must_include_deviceIDs if i in by_id]
            resp.container_responses.add(deviceIDs=prefer(avail, must, cr.allocation_size))
        return resp

    def Allocate(self, req, ctx):  # noqa: N802
        resp = K.DP["AllocateResponse"]()
        by_id = {d.id: d for d in self.devices()}
        cfg = self.plugin.cfg
        for cr in req.container_requests:
            car = resp.container_responses.add()
            ids = list(cr.devicesIDs)
            unknown = [i for i in ids if i not in by_id]
            if unknown:
                msg = f"unknown device ids {unknown} for {self.resource}"
                if ctx is not None:
                    import grpc
                    ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, msg)
                raise ValueError(msg)
            devs = [by_id[i] for i in ids]
            physical = sorted({d.replica_of or d.id for d in devs})
            car.envs["AMD_VISIBLE_DEVICES"] = ",".join(physical)
            if cfg.device_list_strategy.startswith("cdi"):
                names = [f"amd.com/gpu={d.replica_of or d.id}" for d in devs]
                if cfg.device_list_strategy == "cdi-annotations":
                    car.annotations[cfg.cdi_annotation_prefix + "amd-device-plugin"] = ",".join(sorted(set(names)))
                else:
                    for n in sorted(set(names)):
                        car.cdi_devices.add(name=n)
                continue
            if cfg.pass_device_specs or cfg.device_list_strategy == "device-specs":
                car.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
                seen = set()
                for d in devs:
                    if d.render_minor < 0 or d.render_minor in seen:
                        continue
                    seen.add(d.render_minor)
                    p = f"/dev/dri/renderD{d.render_minor}"
                    car.devices.add(container_path=p, host_path=p, permissions="rw")
        return resp

    def PreStartContainer(self, req, ctx):  # noqa: N802
        return K.DP["PreStartContainerResponse"]()

    # -- lifecycle ----------------------------------------------------------------------------
    def serve(self) -> None:
        import grpc
        _unlink(self.socket)
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        self.server.add_generic_rpc_handlers((K.device_plugin_handler(self),))
        self.server.add_insecure_port("unix://" + self.socket)
        self.server.start()

    def register(self, kubelet_socket: str) -> None:
        import grpc
        with grpc.insecure_channel("unix://" + kubelet_socket) as ch:
            K.registration_stub(ch)(K.DP["RegisterRequest"](
                version=K.API_VERSION, endpoint=os.path.basename(self.socket), resource_name=self.resource,
                options=K.DP["DevicePluginOptions"](get_preferred_allocation_available=True)), timeout=10)
        log.info("registered %s (%d devices) with kubelet", self.resource, len(self.devices()))

    def stop(self) -> None:
        self._stop.set()
        self.notify()
        if self.server is not None:
            self.server.stop(grace=1)
        _unlink(self.socket)


class DevicePlugin:
    def __init__(self, cfg: Config, root: Optional[str] = None, plugin_dir: str = K.DEVICE_PLUGIN_PATH,
                 health_period: float = 5.0, policy: Optional[HealthPolicy] = None,
                 status_dir: Optional[str] = None):
        self.cfg = cfg
        self.root = root
        self.plugin_dir = plugin_dir
        self.health_period = health_period
        self.policy = policy or HealthPolicy()
        self.status_dir = status_dir
        self.devices: List[Device] = []
        self.servers: Dict[str, ResourceServer] = {}
        self._stop = threading.Event()

    def start(self, register: bool = True) -> None:
        self.devices = discover(self.cfg, self.root)
        for res in sorted({d.resource for d in self.devices}):
            s = ResourceServer(res, self)
            s.serve()
            self.servers[res] = s
        if register:
            for s in self.servers.values():
                s.register(os.path.join(self.plugin_dir, "kubelet.sock"))
        log.info("serving %s", {r: len(s.devices()) for r, s in self.servers.items()})
        self.check_health()              # a device that is already sick is never advertised Healthy

    def check_health(self) -> bool:
        """Re-evaluate every device (module docstring): driver live, KFD agent present, RAS within the
        policy. Streams a ListAndWatch update when any device changed; returns whether one did."""
        live_driver = False
        agents: Dict[int, Dict] = {}
        tele: Dict[int, Dict] = {}
        try:
            live_driver = bool(devices.driver_state(self.root)["live"])
            if live_driver:
                gpus = devices.enumerate_gpus(self.root)
                agents = {g["drm_render_minor"]: g for g in gpus}
                by_index = {t["index"]: t for t in devices.read_telemetry(self.root)}
                tele = {g["drm_render_minor"]: by_index.get(g["index"]) for g in gpus}
        except Exception as e:  # noqa: BLE001 -- a failed read withdraws nothing but is logged
            log.warning("health read failed: %s", e)
            if not agents:
                live_driver, agents = False, {}
        changed = False
        for d in self.devices:
            if not live_driver:
                why = "amdgpu driver not live"
            elif d.render_minor not in agents:
                why = "KFD agent lost"
            else:
                why = self.policy.verdict(tele.get(d.render_minor))
            ok = not why
            if ok != d.healthy or why != d.reason:
                if ok != d.healthy:
                    changed = True
                    log.warning("device %s is now %s%s", d.id, "healthy" if ok else "unhealthy",
                                "" if ok else f": {why}")
                d.healthy, d.reason = ok, why
        self._publish_health()           # before the stream update: whoever sees it finds the reason
        if changed:
            for s in self.servers.values():
                s.notify()
        return changed

    def _publish_health(self) -> None:
        """``device-health`` in the node status directory: every device's state and reason, read by the
        node metrics exporter. Best effort (the directory may not be mounted)."""
        if not self.status_dir:
            return
        from ..validator import status as S
        try:
            S.StatusDir(self.status_dir).write_raw(DEVICE_HEALTH_FILE, json.dumps({
                "ts": time.time(),
                "devices": {d.id: {"healthy": d.healthy, "reason": d.reason, "resource": d.resource, "bdf": d.bdf}
                            for d in self.devices}}))
        except OSError as e:
            log.debug("device-health not written: %s", e)

    def stop(self) -> None:
        self._stop.set()
        for s in self.servers.values():
            s.stop()
        self.servers.clear()

    def run_forever(self) -> None:
        """Serve until stopped; re-register when kubelet.sock is recreated (kubelet restart)."""
        kubelet_sock = os.path.join(self.plugin_dir, "kubelet.sock")
        last_ino = os.stat(kubelet_sock).st_ino if os.path.exists(kubelet_sock) else None
        while not self._stop.is_set():
            self._stop.wait(self.health_period)
            self.check_health()
            ino = os.stat(kubelet_sock).st_ino if os.path.exists(kubelet_sock) else None
            if ino is not None and ino != last_ino:
                log.info("kubelet restarted; re-registering")
                for s in self.servers.values():
                    try:
                        s.register(kubelet_sock)
                    except Exception as e:  # noqa: BLE001
                        log.error("re-register %s failed: %s", s.resource, e)
                last_ino = ino


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-device-plugin")
    ap.add_argument("--config-file", default=os.environ.get("CONFIG_FILE"))
    ap.add_argument("--plugin-dir", default=mounts.path(K.DEVICE_PLUGIN_PATH))
    ap.add_argument("--status-dir", default=os.environ.get("VALIDATIONS_DIR", mounts.path("/run/amd/validations")))
    ap.add_argument("--health-period", type=float, default=float(os.environ.get("DP_HEALTH_PERIOD_S", "5")))
    a = ap.parse_args(argv)
    stop = threading.Event()
    reload_ = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGHUP, lambda *_: reload_.set())
    while not stop.is_set():
        cfg = Config.load(a.config_file, dict(os.environ))
        p = DevicePlugin(cfg, plugin_dir=a.plugin_dir, health_period=a.health_period,
                         policy=HealthPolicy.from_env(dict(os.environ)), status_dir=a.status_dir)
        try:
            p.start()
        except Exception as e:  # noqa: BLE001
            log.error("device plugin failed to start: %s", e)
            if cfg.fail_on_init_error:
                return 1
            stop.wait(30)
            continue
        t = threading.Thread(target=p.run_forever, daemon=True)
        t.start()
        while not stop.is_set() and not reload_.is_set():
            stop.wait(1)
        p.stop()
        if reload_.is_set():
            log.info("SIGHUP: reloading configuration")
            reload_.clear()
    return 0


if __name__ == "__main__":
    sys.exit(main())
