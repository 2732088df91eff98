"""``amd-mxgpu-device-manager``: SR-IOV virtual-function layout for MxGPU (vm-mxgpu nodes).

Counterpart of the reference's vGPU device manager (``nvidia.com/vgpu.config`` label,
DEFAULT_VGPU_CONFIG). On AMD the host driver (GIM) splits a GPU into
SR-IOV VFs; the count per PF is the knob. The manager:

1. reads the named layout selected by the node label ``amd.com/mxgpu.config`` (or
   ``DEFAULT_MXGPU_CONFIG``) from the config file (``version: v1``, ``mxgpu-configs:
   {name: [{devices: all|[i..], vfs: N}]}``);
2. for each PF whose ``sriov_numvfs`` differs: writes 0 then N (the kernel rejects N->M
   directly), waits for the ``virtfn*`` links to appear;
3. binds every VF to ``vfio-pci`` (``driver_override`` + ``drivers_probe``) so the sandbox
   device plugin advertises it, and reports ``amd.com/mxgpu.config.state`` on the Node.
"""

from __future__ import annotations

import argparse
import logging
import os
import sys
import threading
import time
from typing import Dict, List, Optional

import yaml

from .. import devices
from ..k8s import objects as o

log = logging.getLogger("amd-mxgpu-device-manager")

CONFIG_LABEL = "amd.com/mxgpu.config"
STATE_LABEL = "amd.com/mxgpu.config.state"


class MxGPUError(Exception):
    pass


class SysfsKernel:
    """The two kernel interactions, isolated so tests can simulate the kernel's reaction."""

    def __init__(self, root: str = "/"):
        self.root = root

    def _p(self, *parts: str) -> str:
        return os.path.join(self.root, "sys/bus/pci", *parts)

    def set_numvfs(self, pf: str, n: int) -> None:
        with open(self._p("devices", pf, "sriov_numvfs"), "w") as f:
            f.write(str(n))

    def bind(self, bdf: str, driver: str) -> None:
        dev = self._p("devices", bdf)
        if os.path.islink(os.path.join(dev, "driver")):
            cur = os.path.basename(os.readlink(os.path.join(dev, "driver")))
            if cur == driver:
                return
            with open(os.path.join(dev, "driver", "unbind"), "w") as f:
                f.write(bdf)
        with open(os.path.join(dev, "driver_override"), "w") as f:
            f.write(driver)
        with open(self._p("drivers_probe"), "w") as f:
            f.write(bdf)


def load_configs(path: str) -> Dict[str, List[Dict]]:
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    if doc.get("version") != "v1":
        raise MxGPUError(f"unsupported config version {doc.get('version')!r}")
    return doc.get("mxgpu-configs") or {}


class MxGPUDeviceManager:
    def __init__(self, client, node: str, config_file: str, root: Optional[str] = None,
                 default_config: str = "", kernel=None, vf_timeout: float = 60.0, poll: float = 0.1):
        self.client = client
        self.node = node
        self.config_file = config_file
        self.root = root or devices.sys_root()
        self.default_config = default_config
        self.kernel = kernel or SysfsKernel(self.root)
        self.vf_timeout = vf_timeout
        self.poll = poll

    def _state(self, s: str) -> None:
        self.client.patch("v1", "Node", self.node, {"metadata": {"labels": {STATE_LABEL: s}}})

    def pfs(self) -> List[Dict]:
        return [f for f in devices.scan_pci(self.root) if not f["is_virtfn"] and f["sriov_totalvfs"] > 0]

    def vfs_of(self, pf: str) -> List[Dict]:
        return [f for f in devices.scan_pci(self.root) if f["is_virtfn"] and f["physfn"] == pf]

    def desired(self, entries: List[Dict], pfs: List[Dict]) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for e in entries:
            idx = range(len(pfs)) if e.get("devices", "all") == "all" else [int(i) for i in e["devices"]]
            n = int(e.get("vfs", 1))
            for i in idx:
                if i >= len(pfs):
                    raise MxGPUError(f"device {i} out of range ({len(pfs)} SR-IOV capable GPUs)")
                if n > pfs[i]["sriov_totalvfs"]:
                    raise MxGPUError(f"{pfs[i]['bdf']}: {n} VFs requested, {pfs[i]['sriov_totalvfs']} supported")
                out[pfs[i]["bdf"]] = n
        return out

    def reconcile(self) -> str:
        labels = o.get_labels(self.client.get("v1", "Node", self.node))
        selected = labels.get(CONFIG_LABEL) or self.default_config
        if not selected:
            return "no-config"
        try:
            configs = load_configs(self.config_file)
            if selected not in configs:
                raise MxGPUError(f"config {selected!r} not in {sorted(configs)}")
            pfs = self.pfs()
            if not pfs:
                raise MxGPUError("no SR-IOV capable AMD GPU found")
            want = self.desired(configs[selected], pfs)
            changed = False
            for pf in pfs:
                n = want.get(pf["bdf"])
                if n is None:
                    continue
                if pf["sriov_numvfs"] != n:
                    if not changed:
                        self._state("pending")
                    changed = True
                    if pf["sriov_numvfs"]:
                        self.kernel.set_numvfs(pf["bdf"], 0)
                    self.kernel.set_numvfs(pf["bdf"], n)
                    self._wait_vfs(pf["bdf"], n)
                for vf in self.vfs_of(pf["bdf"]):
                    if vf["driver"] != "vfio-pci":
                        self.kernel.bind(vf["bdf"], "vfio-pci")
                        changed = True
            self._wait_bound(want)
        except (MxGPUError, OSError) as e:
            log.error("mxgpu layout failed: %s", e)
            self._state("failed")
            self.client.create_event(self.client.get("v1", "Node", self.node), "MxGPUConfigFailed", str(e), "Warning")
            return "failed"
        if labels.get(STATE_LABEL) != "success" or changed:
            self._state("success")
        return "applied" if changed else "in-sync"

    def _wait_vfs(self, pf: str, n: int) -> None:
        deadline = time.monotonic() + self.vf_timeout
        while len(self.vfs_of(pf)) != n:
            if time.monotonic() > deadline:
                raise MxGPUError(f"{pf}: {len(self.vfs_of(pf))} VFs appeared, expected {n}")
            time.sleep(self.poll)

    def _wait_bound(self, want: Dict[str, int]) -> None:
        deadline = time.monotonic() + self.vf_timeout
        while True:
            unbound = [vf["bdf"] for pf in want for vf in self.vfs_of(pf) if vf["driver"] != "vfio-pci"]
            if not unbound:
                return
            if time.monotonic() > deadline:
                raise MxGPUError(f"VFs not bound to vfio-pci: {unbound}")
            time.sleep(self.poll)


def main(argv=None, client=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-mxgpu-device-manager")
    ap.add_argument("--config-file", default=os.environ.get("CONFIG_FILE", "/mxgpu-config/config.yaml"))
    ap.add_argument("--default", default=os.environ.get("DEFAULT_MXGPU_CONFIG", "default"))
    ap.add_argument("--resync", type=float, default=300.0)
    a = ap.parse_args(argv)
    if client is None:
        from ..k8s.rest import RestClient
        client = RestClient()
    node = os.environ.get("NODE_NAME", "")
    m = MxGPUDeviceManager(client, node, a.config_file, default_config=a.default)
    kick = threading.Event()

    def on_node(ev):
        if o.name(ev.obj) == node and (ev.old is None or o.get_labels(ev.old).get(CONFIG_LABEL) !=
                                       o.get_labels(ev.obj).get(CONFIG_LABEL)):
            kick.set()
    client.watch("v1", "Node", on_node, field_selector=f"metadata.name={node}")
    while True:
        log.info("reconcile: %s", m.reconcile())
        kick.wait(a.resync)
        kick.clear()


if __name__ == "__main__":
    sys.exit(main())
