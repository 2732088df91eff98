"""``amd-sandbox-device-plugin``: AMD GPUs for KubeVirt VMs (passthrough PFs and MxGPU VFs).

Counterpart of the reference's external kubevirt-gpu-device-plugin (SURVEY.md §2.2 row 16,
§2.3). Advertises every AMD GPU PCI function bound to ``vfio-pci``:

* whole GPUs (vm-passthrough) as ``amd.com/<PRODUCT>`` (e.g. ``amd.com/MI355X``),
* SR-IOV virtual functions (vm-mxgpu) as ``amd.com/<PRODUCT>_VF``,

one resource per product so mixed nodes stay schedulable. Allocate hands KubeVirt's
virt-launcher the VFIO container node plus each function's IOMMU group node, and the
``PCI_RESOURCE_AMD_COM_<NAME>`` env KubeVirt reads the BDFs from. A device turns unhealthy
when its IOMMU group node disappears or it is rebound away from vfio-pci.
"""

from __future__ import annotations

import argparse
import logging
import os
import re
import sys
import threading
from concurrent import futures
from dataclasses import dataclass
from typing import Dict, List, Optional

from .. import devices, models
from ..utils import mounts
from . import kubeletapi as K

log = logging.getLogger("amd-sandbox-device-plugin")


def _unlink(path: str) -> None:
    """Remove a unix socket path that grpc's ``server.stop()`` may be unlinking concurrently."""
    try:
        os.remove(path)
    except FileNotFoundError:
        pass


def resource_name(device_id: int, is_vf: bool) -> str:
    hit = models.by_device_id(device_id)
    name = hit[0].name if hit else f"DEVICE_{device_id:04X}"
    if is_vf or (hit and hit[1]):
        name += "_VF"
    return "amd.com/" + name


def env_name(resource: str) -> str:
    return "PCI_RESOURCE_" + re.sub(r"[^A-Za-z0-9]", "_", resource).upper()


@dataclass
class VfioDevice:
    bdf: str
    resource: str
    iommu_group: int
    healthy: bool = True


def discover(root: Optional[str] = None) -> List[VfioDevice]:
    out = []
    for f in devices.scan_pci(root):
        if f["driver"] != "vfio-pci" or f["iommu_group"] < 0:
            continue
        out.append(VfioDevice(f["bdf"], resource_name(f["device_id"], f["is_virtfn"]), f["iommu_group"]))
    return sorted(out, key=lambda d: (d.resource, d.bdf))


class VfioResourceServer:
    def __init__(self, resource: str, plugin: "SandboxDevicePlugin"):
        self.resource = resource
        self.plugin = plugin
        self.socket = os.path.join(plugin.plugin_dir, "amd-vfio-" + resource.split("/", 1)[1].lower() + ".sock")
        self.server = None
        self._cv = threading.Condition()
        self._version = 0
        self._stop = threading.Event()

    def devices(self) -> List[VfioDevice]:
        return [d for d in self.plugin.devices if d.resource == self.resource]

    def notify(self) -> None:
        with self._cv:
            self._version += 1
            self._cv.notify_all()

    def GetDevicePluginOptions(self, req, ctx):  # noqa: N802
        return K.DP["DevicePluginOptions"]()

    def _list(self):
        resp = K.DP["ListAndWatchResponse"]()
        for d in self.devices():
            resp.devices.add(ID=d.bdf, health=K.HEALTHY if d.healthy else K.UNHEALTHY)
        return resp

    def ListAndWatch(self, req, ctx):  # noqa: N802
        seen = -1
        while not self._stop.is_set() and (ctx is None or ctx.is_active()):
            with self._cv:
                if seen == self._version:
                    self._cv.wait(timeout=1.0)
                    if seen == self._version:
                        continue
                seen = self._version
            yield self._list()

    def GetPreferredAllocation(self, req, ctx):  # noqa: N802
        return K.DP["PreferredAllocationResponse"]()

    def Allocate(self, req, ctx):  # noqa: N802
        resp = K.DP["AllocateResponse"]()
        by_id = {d.bdf: d for d in self.devices()}
        for cr in req.container_requests:
            car = resp.container_responses.add()
            unknown = [i for i in cr.devicesIDs if i not in by_id]
            if unknown:
                msg = f"unknown devices {unknown} for {self.resource}"
                if ctx is not None:
                    import grpc
                    ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, msg)
                raise ValueError(msg)
            car.devices.add(container_path="/dev/vfio/vfio", host_path="/dev/vfio/vfio", permissions="mrw")
            groups = []
            for i in cr.devicesIDs:
                g = by_id[i].iommu_group
                if g not in groups:
                    groups.append(g)
                    p = f"/dev/vfio/{g}"
                    car.devices.add(container_path=p, host_path=p, permissions="mrw")
            car.envs[env_name(self.resource)] = ",".join(cr.devicesIDs)
        return resp

    def PreStartContainer(self, req, ctx):  # noqa: N802
        return K.DP["PreStartContainerResponse"]()

    def serve(self) -> None:
        import grpc
        _unlink(self.socket)
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        self.server.add_generic_rpc_handlers((K.device_plugin_handler(self),))
        self.server.add_insecure_port("unix://" + self.socket)
        self.server.start()

    def register(self, kubelet_socket: str) -> None:
        import grpc
        with grpc.insecure_channel("unix://" + kubelet_socket) as ch:
            K.registration_stub(ch)(K.DP["RegisterRequest"](
                version=K.API_VERSION, endpoint=os.path.basename(self.socket), resource_name=self.resource,
                options=K.DP["DevicePluginOptions"]()), timeout=10)

    def stop(self) -> None:
        self._stop.set()
        self.notify()
        if self.server is not None:
            self.server.stop(grace=1)
        _unlink(self.socket)


class SandboxDevicePlugin:
    def __init__(self, root: Optional[str] = None, dev_root: str = "/", plugin_dir: str = K.DEVICE_PLUGIN_PATH,
                 period: float = 5.0):
        self.root = root
        self.dev_root = dev_root
        self.plugin_dir = plugin_dir
        self.period = period
        self.devices: List[VfioDevice] = []
        self.servers: Dict[str, VfioResourceServer] = {}
        self._stop = threading.Event()

    def start(self, register: bool = True) -> None:
        self.devices = discover(self.root)
        for res in sorted({d.resource for d in self.devices}):
            s = VfioResourceServer(res, self)
            s.serve()
            self.servers[res] = s
            if register:
                s.register(os.path.join(self.plugin_dir, "kubelet.sock"))
        log.info("serving %s", {r: len(s.devices()) for r, s in self.servers.items()})

    def check_health(self) -> bool:
        bound = {f["bdf"] for f in devices.scan_pci(self.root) if f["driver"] == "vfio-pci"}
        changed = set()
        for d in self.devices:
            ok = d.bdf in bound and os.path.exists(os.path.join(self.dev_root, "dev/vfio", str(d.iommu_group)))
            if ok != d.healthy:
                d.healthy = ok
                changed.add(d.resource)
                log.warning("%s %s is now %s", d.resource, d.bdf, "healthy" if ok else "unhealthy")
        for r in changed:
            self.servers[r].notify()
        return bool(changed)

    def stop(self) -> None:
        self._stop.set()
        for s in self.servers.values():
            s.stop()
        self.servers.clear()

    def run_forever(self) -> None:
        while not self._stop.wait(self.period):
            self.check_health()


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-sandbox-device-plugin")
    ap.add_argument("--plugin-dir", default=mounts.path(K.DEVICE_PLUGIN_PATH))
    a = ap.parse_args(argv)
    p = SandboxDevicePlugin(os.environ.get("AMD_SYSFS_ROOT"), plugin_dir=a.plugin_dir)
    p.start()
    try:
        p.run_forever()
    finally:
        p.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
