"""Node barrier files in ``/run/amd/validations`` (hostPath, tmpfs: cleared on reboot).

Same protocol as the reference (reference: validator/main.go:123-157):
a file's existence is the barrier. Ours are written atomically (tmp + rename, so an
inotify waiter never reads a half-written file) and carry a JSON payload with the time
they were produced and the validation's results, which is what the node metrics exporter
turns into the time-to-ready and GEMM/all-reduce gauges.
"""

from __future__ import annotations

import glob
import json
import os
import time
from typing import Any, Dict, Iterable, List, Optional

DEFAULT_DIR = "/run/amd/validations"

DRIVER_CTR_READY = ".driver-ctr-ready"
DRIVER_READY = "driver-ready"
HOST_DRIVER_READY = "host-driver-ready"
TOOLKIT_READY = "toolkit-ready"
HIP_READY = "hip-ready"
PLUGIN_READY = "plugin-ready"
RCCL_READY = "rccl-ready"
RDMA_READY = "rdma-ready"
VFIO_PCI_READY = "vfio-pci-ready"
MXGPU_MANAGER_READY = "mxgpu-manager-ready"
HOST_MXGPU_MANAGER_READY = "host-mxgpu-manager-ready"
MXGPU_DEVICES_READY = "mxgpu-devices-ready"
WORKLOAD_TYPE = "workload-type"
# the last full RCCL fabric result (no "-ready" suffix: it outlives validator restarts, whose preStop
# removes *-ready; tmpfs, so a reboot -- after which the fabric is measured again -- clears it)
FABRIC_LAST_FULL = "fabric-last-full"
# the last failed HIP validation with the location of every wrong result it found (tile, XCD, CU): kept
# across validator restarts (no "-ready" suffix), removed by the next passing validation
HIP_LAST_FAILURE = "hip-last-failure"

CONTAINER_CHAIN = [DRIVER_READY, TOOLKIT_READY, HIP_READY, PLUGIN_READY, RCCL_READY]


class StatusDir:
    def __init__(self, path: str = DEFAULT_DIR):
        self.path = path

    def ensure(self) -> None:
        os.makedirs(self.path, exist_ok=True)

    def file(self, name: str) -> str:
        return os.path.join(self.path, name)

    def create(self, name: str, payload: Optional[Dict[str, Any]] = None) -> None:
        """Write barrier ``name`` atomically. A barrier that already exists keeps its first ``ts`` (the
        moment the gate first opened, as the native writer in node_validate.cpp does) and records the
        re-validation as ``revalidated_ts``."""
        self.ensure()
        body = dict(payload or {})
        now = time.time()
        if "ts" not in body:
            old = self.read(name)
            first = old.get("ts") if isinstance(old, dict) else None
            if isinstance(first, (int, float)):
                body["ts"], body["revalidated_ts"] = first, now
            else:
                body["ts"] = now
        tmp = self.file(f".{name}.tmp.{os.getpid()}")
        with open(tmp, "w") as f:
            json.dump(body, f)
        os.replace(tmp, self.file(name))

    def write_raw(self, name: str, content: str) -> None:
        self.ensure()
        tmp = self.file(f".{name}.tmp.{os.getpid()}")
        with open(tmp, "w") as f:
            f.write(content)
        os.replace(tmp, self.file(name))

    def delete(self, name: str) -> None:
        try:
            os.remove(self.file(name))
        except FileNotFoundError:
            pass

    def exists(self, name: str) -> bool:
        return os.path.exists(self.file(name))

    def read(self, name: str) -> Optional[Dict[str, Any]]:
        try:
            with open(self.file(name)) as f:
                txt = f.read()
        except FileNotFoundError:
            return None
        try:
            d = json.loads(txt) if txt.strip() else {}
        except ValueError:
            d = {"raw": txt.strip()}
        if "ts" not in d:
            d["ts"] = os.path.getmtime(self.file(name))
        return d

    def cleanup_ready(self) -> None:
        for p in glob.glob(os.path.join(self.path, "*-ready")):
            os.remove(p)

    def cleanup_all(self) -> None:
        for p in glob.glob(os.path.join(self.path, "*")) + glob.glob(os.path.join(self.path, ".*")):
            if os.path.isfile(p):
                os.remove(p)

    def wait(self, names: Iterable[str], any_of: bool = False, timeout: Optional[float] = None) -> List[str]:
        """Event-driven (inotify, native) wait for barrier files."""
        from .. import devices
        self.ensure()
        return devices.wait_files(self.path, list(names), any_of=any_of, timeout=timeout)


def time_to_ready(sd: StatusDir, chain: Optional[List[str]] = None) -> Optional[float]:
    """Seconds from the driver becoming ready (driver container barrier, or host driver) to the
    last barrier of the validation chain present. None until the chain has an end."""
    chain = chain or CONTAINER_CHAIN
    start = None
    for n in (DRIVER_CTR_READY, HOST_DRIVER_READY, DRIVER_READY):
        d = sd.read(n)
        if d is not None:
            start = d["ts"] if start is None else min(start, d["ts"])
    if start is None:
        return None
    ends = [sd.read(n) for n in chain[1:]]
    ends = [e["ts"] for e in ends if e is not None]
    if not ends:
        return None
    return max(ends) - start
