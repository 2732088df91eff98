"""Node-feature labeller (``amd-node-labeller``): the GPU-feature-discovery role.

The reference deploys NVIDIA's GFD (NVML-based). Here labels come from the
kernel interfaces via libamdnode (no ROCm runtime in the loop):

    amd.com/gpu.product, .family (cdna4), .gfx (gfx950), .device-id, .count (physical GPUs),
    .cu-count, .simd-count, .lds-kib, .vram (GiB per GPU), .compute-partition,
    .memory-partition, .partition.capable, .partition.count (schedulable agents),
    .numa-nodes, .xgmi.hive-id, .xgmi.links, .xgmi.fully-connected, .driver-version

Output to the Node directly (``LABELLER_OUTPUT=node``, needs RBAC) or as an NFD local feature
file (``LABELLER_OUTPUT=nfd``). Event-driven: relabels immediately when a barrier changes
(e.g. the partition manager finished), with a periodic resync (LABELLER_SLEEP_INTERVAL).
"""

from __future__ import annotations

import argparse
import logging
import os
import re
import sys
import threading
from typing import Dict, List, Optional

from .. import devices, models
from ..utils import mounts
from ..k8s import objects as o

log = logging.getLogger("amd-node-labeller")

PREFIX = "amd.com/gpu."
OWNED = re.compile(r"^amd\.com/gpu\.(product|family|gfx|device-id|count|cu-count|simd-count|lds-kib|vram|"
                   r"compute-partition|memory-partition|partition\.capable|partition\.count|numa-nodes|"
                   r"xgmi\.hive-id|xgmi\.links|xgmi\.fully-connected|driver-version|replicas|"
                   r"sharing-strategy)$")
NFD_FEATURE_FILE = "/etc/kubernetes/node-feature-discovery/features.d/amd-gpu"

FAMILIES = models.GFX_FAMILY


def sanitize(v: str) -> str:
    """Label values: [A-Za-z0-9._-], max 63, alphanumeric at both ends."""
    s = re.sub(r"[^A-Za-z0-9._-]+", "-", v).strip("-_.")
    return s[:63].rstrip("-_.")


def compute_labels(root: Optional[str] = None) -> Dict[str, str]:
    gpus = devices.enumerate_gpus(root)
    if not gpus:
        return {}
    drv = devices.driver_state(root)
    physical: Dict[str, Dict] = {}
    for g in gpus:
        physical.setdefault(g["pci_bdf"], g)
    first = gpus[0]
    cus_per_physical = {}
    for g in gpus:
        cus_per_physical[g["pci_bdf"]] = cus_per_physical.get(g["pci_bdf"], 0) + g["cu_count"]
    gfx = first["gfx_target"]
    labels = {
        PREFIX + "product": sanitize(first["product_name"] or f"device-{first['device_id']:04x}"),
        PREFIX + "family": FAMILIES.get(gfx, "unknown"),
        PREFIX + "gfx": gfx,
        PREFIX + "device-id": f"{first['device_id']:04x}",
        PREFIX + "count": str(len(physical)),
        PREFIX + "cu-count": str(max(cus_per_physical.values())),
        PREFIX + "simd-count": str(sum(g["simd_count"] for g in gpus if g["pci_bdf"] == first["pci_bdf"])),
        PREFIX + "lds-kib": str(first["lds_size_kib"]),
        PREFIX + "vram": f"{round(first['vram_total'] / (1 << 30))}G",   # nearest GiB (firmware reserves a few MiB)
        PREFIX + "partition.capable": "true" if first["partition_capable"] else "false",
        PREFIX + "partition.count": str(len(gpus)),
        PREFIX + "numa-nodes": str(len({g["numa_node"] for g in gpus if g["numa_node"] >= 0}) or 1),
    }
    if first["compute_partition"]:
        labels[PREFIX + "compute-partition"] = first["compute_partition"]
        modes = {g["compute_partition"] for g in gpus}
        if len(modes) > 1:
            labels[PREFIX + "compute-partition"] = "mixed"
    if first["memory_partition"]:
        labels[PREFIX + "memory-partition"] = first["memory_partition"]
    if first["xgmi_hive_id"]:
        labels[PREFIX + "xgmi.hive-id"] = f"{first['xgmi_hive_id']:x}"
    phys_links = max((g["xgmi_links"] for g in gpus), default=0)
    # links are counted between agents; express them per physical GPU
    per_phys = len(gpus) // max(1, len(physical))
    labels[PREFIX + "xgmi.links"] = str(phys_links // max(1, per_phys))
    topo = devices.xgmi_topology(gpus)
    by_bdf: Dict[str, set] = {}
    idx_bdf = {g["index"]: g["pci_bdf"] for g in gpus}
    for i, peers in topo.items():
        by_bdf.setdefault(idx_bdf[i], set()).update(idx_bdf[p] for p in peers)
    full = len(physical) > 1 and all(len(v) == len(physical) - 1 for v in by_bdf.values()) and devices.single_hive(gpus)
    labels[PREFIX + "xgmi.fully-connected"] = "true" if full else "false"
    if drv["version"]:
        labels[PREFIX + "driver-version"] = sanitize(drv["version"])
    return labels


def sharing_labels(node: Dict, want: Dict[str, str]) -> Dict[str, str]:
    """Time-slicing as GFD reports it (``gpu.replicas``, ``gpu.sharing-strategy``, product
    ``-SHARED``): read from what the device plugin actually advertises -- the Node's allocatable
    ``amd.com/gpu`` over the GPU (partition) count -- rather than from a second copy of its config.
    Nothing until the plugin has registered (allocatable absent or 0)."""
    alloc = ((node.get("status") or {}).get("allocatable") or {}).get("amd.com/gpu")
    try:
        n, parts = int(alloc or 0), int(want.get(PREFIX + "partition.count", "0"))
    except ValueError:
        return {}
    if n <= 0 or parts <= 0:
        return {}
    if n > parts and n % parts == 0:
        out = {PREFIX + "replicas": str(n // parts), PREFIX + "sharing-strategy": "time-slicing"}
        if want.get(PREFIX + "product"):
            out[PREFIX + "product"] = sanitize(want[PREFIX + "product"][:56] + "-SHARED")
        return out
    return {PREFIX + "replicas": "1", PREFIX + "sharing-strategy": "none"}


def label_patch(current: Dict[str, str], want: Dict[str, str]) -> Dict[str, Optional[str]]:
    patch: Dict[str, Optional[str]] = {k: v for k, v in want.items() if current.get(k) != v}
    for k in current:
        if OWNED.match(k) and k not in want:
            patch[k] = None
    return patch


def apply_node(client, node: str, want: Dict[str, str]) -> Dict[str, Optional[str]]:
    obj = client.get("v1", "Node", node)
    cur = o.get_labels(obj)
    want = dict(want, **sharing_labels(obj, want))
    patch = label_patch(cur, want)
    if patch:
        client.patch("v1", "Node", node, {"metadata": {"labels": patch}})
        log.info("node %s labels updated: %s", node, sorted(patch))
    return patch


def write_nfd(path: str, want: Dict[str, str]) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        for k, v in sorted(want.items()):
            f.write(f"{k}={v}\n")
    os.replace(tmp, path)


def parse_duration(s: str) -> float:
    m = re.fullmatch(r"(\d+(?:\.\d+)?)(ms|s|m|h)?", s.strip())
    if not m:
        raise ValueError(s)
    return float(m.group(1)) * {"ms": 1e-3, "s": 1, "m": 60, "h": 3600, None: 1}[m.group(2)]


def main(argv=None, client=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-node-labeller")
    ap.add_argument("--oneshot", action="store_true")
    ap.add_argument("--output", default=os.environ.get("LABELLER_OUTPUT", "node"))
    ap.add_argument("--sleep-interval", default=os.environ.get("LABELLER_SLEEP_INTERVAL", "60s"))
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--nfd-file", default=mounts.path(NFD_FEATURE_FILE))
    ap.add_argument("--barrier-dir", default=mounts.path("/run/amd/validations"))
    a = ap.parse_args(argv)
    if a.output == "node" and client is None:
        from ..k8s.rest import RestClient
        client = RestClient()
    period = parse_duration(a.sleep_interval)
    stop = threading.Event()
    kick = threading.Event()
    if a.output == "node":
        # re-label as soon as the advertised amd.com/gpu count changes (time-slicing replicas)
        seen: Dict[str, Optional[str]] = {}

        def on_node(ev):
            if o.name(ev.obj) != a.node_name:
                return
            v = ((ev.obj.get("status") or {}).get("allocatable") or {}).get("amd.com/gpu")
            if seen.get("v", "unset") != v:
                seen["v"] = v
                kick.set()
        client.watch("v1", "Node", on_node, field_selector=f"metadata.name={a.node_name}")
    while not stop.is_set():
        try:
            want = compute_labels()
            if a.output == "node":
                apply_node(client, a.node_name, want)
            else:
                write_nfd(a.nfd_file, want)
        except Exception as e:  # noqa: BLE001
            log.error("labelling failed: %s", e)
        if a.oneshot:
            return 0
        # wake early when the partition manager (re)writes its barrier, else resync periodically
        wait_for_change(os.path.join(a.barrier_dir, "partition-applied"), period, stop, kick)
    return 0


def wait_for_change(path: str, period: float, stop: threading.Event,
                    kick: Optional[threading.Event] = None) -> bool:
    """Return True as soon as ``path`` is created or rewritten or ``kick`` is set, False after
    ``period``."""
    def mtime():
        try:
            return os.stat(path).st_mtime_ns
        except FileNotFoundError:
            return None
    start = mtime()
    deadline = period
    step = 1.0
    waited = 0.0
    while waited < deadline and not stop.is_set():
        if kick is not None and kick.is_set():
            kick.clear()
            return True
        slice_ = min(step, deadline - waited)
        if start is None and os.path.isdir(os.path.dirname(path)):
            # absent: block on inotify for its creation, a slice at a time so a kick is seen
            if devices.wait_files(os.path.dirname(path), [os.path.basename(path)], timeout=slice_):
                return True
        else:
            (kick or stop).wait(slice_)
        waited += slice_
        if mtime() != start:
            return True
    return False


if __name__ == "__main__":
    sys.exit(main())
