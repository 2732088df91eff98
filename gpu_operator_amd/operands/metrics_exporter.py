"""GPU telemetry exporter (``amd-metrics-exporter``): the DCGM-exporter role.

Per-GPU gauges from the kernel's telemetry interfaces (hwmon power/temperatures, busy %,
VRAM, DPM clocks, RAS ECC counters, PCIe bandwidth, xGMI links) plus the PMFW metrics table
(sysfs ``gpu_metrics``: energy, socket power, per-link xGMI bytes read/written with derived
throughput, link status/width/speed), all read natively by libamdnode,
published on ``:9400/metrics`` (reference default port, assets/state-dcgm-exporter). Which
fields are exported comes from a CSV field list (``METRICS_EXPORTER_FIELDS``, overridable
through ``spec.metricsExporter.config.name`` like the reference's DCGM counter CSV).

With ``METRICS_EXPORTER_KUBERNETES=true`` every sample carries the pod/namespace/container
that was allocated the GPU, resolved through the kubelet pod-resources API (device ids ->
``amdgpu-<unique id>`` as advertised by the device plugin).
"""

from __future__ import annotations

import argparse
import logging
import os
import socket
import sys
import threading
from typing import Dict, Iterable, List, Optional, Tuple

from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily
from prometheus_client.registry import Collector, CollectorRegistry

from .. import devices
from ..utils import mounts
from . import kubeletapi as K

log = logging.getLogger("amd-metrics-exporter")

# field -> (telemetry key or callable, kind, help)
FIELDS = {
    "gpu_power_watts": ("power_w", "gauge", "Average package power (W)"),
    "gpu_temperature_edge_celsius": ("temp_edge_c", "gauge", "Edge temperature (C)"),
    "gpu_temperature_junction_celsius": ("temp_junction_c", "gauge", "Junction temperature (C)"),
    "gpu_temperature_memory_celsius": ("temp_mem_c", "gauge", "HBM temperature (C)"),
    "gpu_utilization_percent": ("gpu_busy_pct", "gauge", "GFX engine busy (%)"),
    "gpu_memory_utilization_percent": ("mem_busy_pct", "gauge", "Memory controller busy (%)"),
    "gpu_vram_used_bytes": ("vram_used", "gauge", "HBM in use (bytes)"),
    "gpu_vram_total_bytes": ("vram_total", "gauge", "HBM capacity (bytes)"),
    "gpu_sclk_mhz": ("sclk_mhz", "gauge", "Current shader clock (MHz)"),
    "gpu_mclk_mhz": ("mclk_mhz", "gauge", "Current memory clock (MHz)"),
    "gpu_ecc_correctable_total": ("ecc_correctable", "counter", "Correctable ECC errors"),
    "gpu_ecc_uncorrectable_total": ("ecc_uncorrectable", "counter", "Uncorrectable ECC errors"),
    "gpu_pcie_bandwidth_bytes": ("pcie_bw_bytes", "gauge", "PCIe bandwidth estimate (bytes/s)"),
    "gpu_ras_uncorrectable_total": ("ras_ue_total", "counter", "Uncorrectable RAS errors over every block"),
    "gpu_ras_correctable_total": ("ras_ce_total", "counter", "Correctable RAS errors over every block"),
    "gpu_retired_pages": ("bad_pages_retired", "gauge", "HBM pages the driver retired"),
    "gpu_pending_retired_pages": ("bad_pages_pending", "gauge", "HBM pages pending retirement"),
    "gpu_xgmi_link_count": ("xgmi_links", "gauge", "xGMI links to other GPUs (KFD io_links)"),
}

# From the decoded PMFW metrics table (sysfs gpu_metrics, devices.read_gpu_metrics): per GPU ...
GM_FIELDS = {
    "gpu_socket_power_watts": ("socket_power_w", "gauge", "Current socket power from the PMFW table (W)"),
    "gpu_energy_joules_total": ("energy_j", "counter", "Accumulated energy (J)"),
    "gpu_xgmi_link_speed_gbps": ("xgmi_link_speed", "gauge", "xGMI per-lane bit rate (Gbps)"),
    "gpu_xgmi_link_width": ("xgmi_link_width", "gauge", "xGMI link width (lanes)"),
    "gpu_pcie_bandwidth_inst_gbps": ("pcie_bandwidth_inst", "gauge", "PCIe instantaneous bandwidth (GB/s)"),
}
# ... and per xGMI link (label ``link``); throughputs are derived between two scrapes from the
# accumulators and the table's own sample clock.
LINK_FIELDS = {
    "gpu_xgmi_read_bytes_total": ("counter", "Bytes read over the xGMI link (accumulated)"),
    "gpu_xgmi_write_bytes_total": ("counter", "Bytes written over the xGMI link (accumulated)"),
    "gpu_xgmi_read_throughput_bytes_per_second": ("gauge", "xGMI read throughput since the previous scrape"),
    "gpu_xgmi_write_throughput_bytes_per_second": ("gauge", "xGMI write throughput since the previous scrape"),
    "gpu_xgmi_link_up": ("gauge", "xGMI link status (1 up, 0 down)"),
}
ALL_FIELDS = list(FIELDS) + list(GM_FIELDS) + list(LINK_FIELDS)
# hwmon / RAS / PCIe readings of the physical device (one PCI function): under CPX/DPX every
# partition agent would report the same value again
DEVICE_LEVEL_FIELDS = frozenset({"gpu_power_watts", "gpu_temperature_edge_celsius", "gpu_temperature_junction_celsius",
                                 "gpu_temperature_memory_celsius", "gpu_ecc_correctable_total",
                                 "gpu_ecc_uncorrectable_total", "gpu_pcie_bandwidth_bytes", "gpu_ras_uncorrectable_total",
                                 "gpu_ras_correctable_total", "gpu_retired_pages", "gpu_pending_retired_pages"})


def load_fields(path: Optional[str]) -> List[str]:
    if not path or not os.path.exists(path):
        return list(ALL_FIELDS)
    out = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            name = line.split(",")[0].strip()
            if name in ALL_FIELDS:
                out.append(name)
            else:
                log.warning("unknown field %s ignored", name)
    return out


def pod_attribution(socket_path: str = K.POD_RESOURCES_SOCKET, timeout: float = 5.0) -> Dict[str, Tuple[str, str, str]]:
    """device id -> (namespace, pod, container) from the kubelet pod-resources API."""
    import grpc
    out: Dict[str, Tuple[str, str, str]] = {}
    if not os.path.exists(socket_path):
        return out
    with grpc.insecure_channel("unix://" + socket_path) as ch:
        resp = K.pod_resources_stub(ch)(K.PR["ListPodResourcesRequest"](), timeout=timeout)
    for pr in resp.pod_resources:
        for c in pr.containers:
            for d in c.devices:
                if not d.resource_name.startswith("amd.com/"):
                    continue
                for did in d.device_ids:
                    out[did.split("::")[0]] = (pr.namespace, pr.name, c.name)
    return out


class GPUCollector(Collector):
    def __init__(self, fields: List[str], root: Optional[str] = None, hostname: str = "",
                 kubernetes: bool = False, pod_socket: str = K.POD_RESOURCES_SOCKET):
        self.fields = fields
        self.root = root
        self.hostname = hostname or socket.gethostname()
        self.kubernetes = kubernetes
        self.pod_socket = pod_socket
        self._prev: Dict[Tuple[str, int], Tuple[int, int, int]] = {}   # (bdf, link) -> (clock ns, rd KiB, wr KiB)
        self._rate: Dict[Tuple[str, int], Tuple[float, float]] = {}    # (bdf, link) -> last (rd, wr) B/s
        self._lock = threading.Lock()

    def _metrics_tables(self) -> Dict[int, Dict]:
        try:
            return {m["index"]: m for m in devices.read_gpu_metrics(self.root) if m["valid"]}
        except Exception as e:  # noqa: BLE001 - a telemetry source must not break the scrape
            log.warning("gpu_metrics read failed: %s", e)
            return {}

    def collect(self) -> Iterable:
        gpus = devices.enumerate_gpus(self.root)
        tele = {t["index"]: t for t in devices.read_telemetry(self.root)}
        gm = self._metrics_tables() if any(f in GM_FIELDS or f in LINK_FIELDS for f in self.fields) else {}
        pods = {}
        if self.kubernetes:
            try:
                pods = pod_attribution(self.pod_socket)
            except Exception as e:  # noqa: BLE001
                log.warning("pod-resources query failed: %s", e)
        labels = ["gpu", "gpu_uid", "bdf", "partition", "product", "hostname", "namespace", "pod", "container"]
        fams = {}
        for f in self.fields:
            if f in LINK_FIELDS:
                kind, help_ = LINK_FIELDS[f]
                lbl = labels + ["link"]
            else:
                key, kind, help_ = FIELDS[f] if f in FIELDS else GM_FIELDS[f]
                lbl = labels
            cls = CounterMetricFamily if kind == "counter" else GaugeMetricFamily
            fams[f] = cls("amd_" + f.replace("_total", "") if kind == "counter" else "amd_" + f, help_, labels=lbl)
        # the PMFW gpu_metrics table (energy, socket power, per-link xGMI bytes) belongs to the
        # physical device, which CPX/DPX enumerate once per partition: its series come from the
        # lowest-index agent of each PCI function only, so sums over `gpu` do not multiply them
        owner = {}
        for g in sorted(gpus, key=lambda g: g["index"]):
            owner.setdefault(g["pci_bdf"], g["index"])
        for g in gpus:
            t = tele.get(g["index"], {})
            did = f"amdgpu-{g['unique_id']:016x}"
            ns, pod, ctr = pods.get(did, ("", "", ""))
            lv = [str(g["index"]), did, g["pci_bdf"], g["compute_partition"] or "SPX", g["product_name"],
                  self.hostname, ns, pod, ctr]
            first = owner.get(g["pci_bdf"]) == g["index"]
            m = gm.get(g["index"]) if first else None
            for f in self.fields:
                if f in LINK_FIELDS or (f in DEVICE_LEVEL_FIELDS and not first):
                    continue
                if f in GM_FIELDS:
                    if m is None:
                        continue
                    key = GM_FIELDS[f][0]
                    v = m["energy_acc"] * devices.ENERGY_UNIT_J if key == "energy_j" else m.get(key)
                else:
                    key = FIELDS[f][0]
                    v = t.get(key) if key in t else g.get(key)
                if v is None or (isinstance(v, (int, float)) and v < 0):
                    continue
                fams[f].add_metric(lv, float(v))
            if m is not None:
                self._link_metrics(fams, lv, g["pci_bdf"], m)
        yield from fams.values()

    def _link_metrics(self, fams, lv, bdf: str, m: Dict) -> None:
        clock = m["system_clock_ns"]
        for link, (rd, wr, st) in enumerate(zip(m["xgmi_read_kb"], m["xgmi_write_kb"], m["xgmi_link_status"])):
            if st < 0:
                continue                         # no link in this slot (N/A in the table)
            ll = lv + [str(link)]
            if "gpu_xgmi_link_up" in fams:
                fams["gpu_xgmi_link_up"].add_metric(ll, float(st))
            if "gpu_xgmi_read_bytes_total" in fams:
                fams["gpu_xgmi_read_bytes_total"].add_metric(ll, float(rd) * 1024)
            if "gpu_xgmi_write_bytes_total" in fams:
                fams["gpu_xgmi_write_bytes_total"].add_metric(ll, float(wr) * 1024)
            key = (bdf, link)
            with self._lock:
                prev = self._prev.get(key)
                if prev is None or clock > prev[0]:
                    self._prev[key] = (clock, rd, wr)
                    if prev is not None and rd >= prev[1] and wr >= prev[2]:
                        dt = (clock - prev[0]) / 1e9
                        self._rate[key] = ((rd - prev[1]) * 1024 / dt, (wr - prev[2]) * 1024 / dt)
                    else:
                        self._rate.pop(key, None)      # first sample or counter reset: no rate yet
                rate = self._rate.get(key)            # same table sample as last scrape: last rate
            if rate is None:
                continue
            if "gpu_xgmi_read_throughput_bytes_per_second" in fams:
                fams["gpu_xgmi_read_throughput_bytes_per_second"].add_metric(ll, rate[0])
            if "gpu_xgmi_write_throughput_bytes_per_second" in fams:
                fams["gpu_xgmi_write_throughput_bytes_per_second"].add_metric(ll, rate[1])


def build_registry(fields: List[str], root: Optional[str] = None, kubernetes: bool = False,
                   pod_socket: str = K.POD_RESOURCES_SOCKET, hostname: str = "") -> CollectorRegistry:
    reg = CollectorRegistry()
    reg.register(GPUCollector(fields, root, hostname=hostname, kubernetes=kubernetes, pod_socket=pod_socket))
    return reg


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-metrics-exporter")
    ap.add_argument("--listen", default=os.environ.get("METRICS_EXPORTER_LISTEN", ":9400"))
    ap.add_argument("--fields", default=os.environ.get("METRICS_EXPORTER_FIELDS"))
    ap.add_argument("--kubernetes", default=os.environ.get("METRICS_EXPORTER_KUBERNETES", "false"))
    a = ap.parse_args(argv)
    from prometheus_client import generate_latest
    from prometheus_client.exposition import CONTENT_TYPE_LATEST

    from ..runtime.manager import _Server
    reg = build_registry(load_fields(a.fields), kubernetes=a.kubernetes == "true",
                         pod_socket=mounts.path(K.POD_RESOURCES_SOCKET), hostname=os.environ.get("NODE_NAME", ""))
    host, _, port = a.listen.rpartition(":")
    srv = _Server((host or "0.0.0.0", int(port)), {"/metrics": lambda: (200, CONTENT_TYPE_LATEST,
                                                                        generate_latest(reg))})
    srv.start()
    log.info("serving GPU metrics on %s", a.listen)
    threading.Event().wait()
    return 0


if __name__ == "__main__":
    sys.exit(main())
