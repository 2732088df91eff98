"""Node status exporter (``amd-validator --component metrics``), reference:
validator/metrics.go:52-320 (same families, ``amd_gpu_operator_`` prefix).

Refresh model: barrier files are watched with inotify (an open/closed barrier is reflected
immediately, not after the reference's 30 s period); the driver check runs every 60 s, the
node-capacity and PCI counts every 30/60 s. New gauges: node time-to-ready (driver ->
validator), per-barrier timestamps, validator GEMM TFLOPS and RCCL all-reduce bus bandwidth
(read from the barrier payloads).
"""

from __future__ import annotations

import logging
import threading
import time
from typing import Any, Dict, Optional

from prometheus_client import CollectorRegistry, Gauge

from .. import devices
from . import components as comp
from . import status as S

log = logging.getLogger("amd-validator.metrics")

STATUS_PERIOD = 30.0
DRIVER_PERIOD = 60.0
PLUGIN_PERIOD = 30.0
PCI_PERIOD = 60.0

BARRIERS = {"driver": (S.DRIVER_READY, S.HOST_DRIVER_READY), "toolkit": (S.TOOLKIT_READY,),
            "hip": (S.HIP_READY,), "plugin": (S.PLUGIN_READY,), "rccl": (S.RCCL_READY,)}


class NodeMetrics:
    def __init__(self, ctx: comp.Context, registry: Optional[CollectorRegistry] = None):
        self.ctx = ctx
        self.registry = registry or CollectorRegistry()
        r, p, node = self.registry, "amd_gpu_operator_", ["node"]
        self.ready_ts = Gauge(p + "node_metrics_ready_ts_seconds", "launch time of the node metrics exporter",
                              node, registry=r)
        self.barrier = {k: Gauge(p + f"node_{k}_ready", f"1 if the {k} barrier of the local node is open", node,
                                 registry=r) for k in BARRIERS}
        self.barrier_ts = Gauge(p + "node_barrier_ts_seconds", "time the barrier was opened", node + ["barrier"],
                                registry=r)
        self.ttr = Gauge(p + "node_time_to_ready_seconds",
                         "driver ready -> last validator barrier (node bring-up critical path)", node, registry=r)
        self.driver_validation = Gauge(p + "node_driver_validation", "1 if the driver check passed", node,
                                       registry=r)
        self.driver_last_success = Gauge(p + "node_driver_validation_last_success_ts_seconds",
                                         "last successful driver check", node, registry=r)
        self.devices_total = Gauge(p + "node_device_plugin_devices_total",
                                   "GPU resources advertised on the node (-1 if unknown)", node, registry=r)
        self.devices_last_success = Gauge(p + "node_device_plugin_validation_last_success_ts_seconds",
                                          "last time GPU resources were found", node, registry=r)
        self.pci_total = Gauge(p + "amd_pci_devices_total", "AMD GPU PCI functions (-1 if unknown)", node,
                               registry=r)
        self.gemm_tflops = Gauge(p + "validator_gemm_tflops",
                                 "validator MFMA GEMM throughput on `gpus` GPUs at once (scope node = aggregate, "
                                 "per_gpu = mean per GPU)", node + ["scope", "dtype", "gpus"], registry=r)
        self.gemm_gpu_tflops = Gauge(p + "validator_gemm_gpu_tflops",
                                     "validator MFMA GEMM throughput of one GPU (its best over the sweep's sets)",
                                     node + ["gpu", "dtype", "m", "n", "k"], registry=r)
        self.dev_unhealthy = Gauge(p + "node_device_unhealthy",
                                   "1 for a device the device plugin withdrew from the kubelet, with its reason "
                                   "(RAS uncorrectable errors, retired HBM pages, agent lost, driver not live)",
                                   node + ["device", "bdf", "reason"], registry=r)
        self.dev_unhealthy_total = Gauge(p + "node_devices_unhealthy", "devices the device plugin reports Unhealthy",
                                         node, registry=r)
        self.gemm_bad_tile = Gauge(p + "validator_gemm_bad_tile",
                                   "1 for each wrong GEMM output tile the last failed HIP validation found, with the "
                                   "GPU, the XCD and the CU that computed it (ABFT check of amd-gemm-validate)",
                                   node + ["gpu", "dtype", "tile", "xcd", "cu"], registry=r)
        self.hip_failure_ts = Gauge(p + "validator_hip_last_failure_ts_seconds",
                                    "time of the last failed HIP validation (0: the last one passed)", node,
                                    registry=r)
        self.gemm_checked = Gauge(p + "validator_gemm_checked_fraction",
                                  "fraction of the validator GEMM's output elements verified (ABFT tile checksums; "
                                  "the least covered GEMM of the last passing run)", node, registry=r)
        self.gemm_abft_ratio = Gauge(p + "validator_gemm_abft_worst_ratio",
                                     "largest |checksum - expected| / tolerance of the last passing run (< 1)",
                                     node, registry=r)
        self.gemm_eff = Gauge(p + "validator_gemm_scaling_efficiency",
                              "aggregate GEMM TFLOP/s on `gpus` GPUs / (gpus x the 1-GPU figure)",
                              node + ["dtype", "gpus"], registry=r)
        self.busbw = Gauge(p + "validator_allreduce_busbw_gbps", "validator RCCL all-reduce peak bus bandwidth",
                           node + ["ranks"], registry=r)
        self.xgmi_link = Gauge(p + "validator_xgmi_link_gbps",
                               "xGMI bandwidth of one ordered GPU pair (src -> dst) from the fabric pod's link matrix; "
                               "mode isolated = that pair alone, concurrent = every pair at once",
                               node + ["src", "dst", "mode"], registry=r)
        self._stop = threading.Event()
        self.ready_ts.labels(ctx.node_name).set(time.time())

    # -- collectors ---------------------------------------------------------------------------
    def refresh_status(self) -> None:
        n = self.ctx.node_name
        sd = self.ctx.status
        for k, files in BARRIERS.items():
            present = [sd.read(f) for f in files]
            present = [d for d in present if d is not None]
            self.barrier[k].labels(n).set(1 if present else 0)
            if present:
                self.barrier_ts.labels(n, k).set(min(d["ts"] for d in present))
        ttr = S.time_to_ready(sd)
        if ttr is not None:
            self.ttr.labels(n).set(ttr)
        hip = sd.read(S.HIP_READY) or {}
        by = hip.get("tflops_by_dtype_gpus") or {}
        if by:                                        # the 1/2/4/8-GPU sweep, per dtype
            for dtype, per in by.items():
                for gpus, v in per.items():
                    self.gemm_tflops.labels(n, "node", dtype, str(gpus)).set(v["total_tflops"])
                    self.gemm_tflops.labels(n, "per_gpu", dtype, str(gpus)).set(v["per_gpu_tflops"])
                    if "efficiency" in v:
                        self.gemm_eff.labels(n, dtype, str(gpus)).set(v["efficiency"])
        elif "gemm_tflops_total" in hip:
            g = str(hip.get("gpus") or "")
            self.gemm_tflops.labels(n, "node", "bf16", g).set(hip["gemm_tflops_total"])
            self.gemm_tflops.labels(n, "per_gpu", "bf16", g).set(hip.get("gemm_tflops_per_gpu", 0))
        if "checked_fraction" in hip:
            self.gemm_checked.labels(n).set(hip["checked_fraction"])
            self.gemm_abft_ratio.labels(n).set(hip.get("abft_worst_ratio", 0.0))
        for line in hip.get("gpu_tflops") or []:      # one series per GPU: a GPU failing the median shows
            for gpu, v in (line.get("tflops") or {}).items():
                self.gemm_gpu_tflops.labels(n, str(gpu), comp._dtype_key(line.get("dtype", "bf16")), str(line.get("m")),
                                            str(line.get("n")), str(line.get("k"))).set(v)
        self.refresh_device_health()
        self.refresh_hip_failure()
        rc = sd.read(S.RCCL_READY) or {}
        if rc.get("peak_busbw_gbps") is not None:
            self.busbw.labels(n, str(rc.get("ranks"))).set(rc["peak_busbw_gbps"])
        links = rc.get("links") or {}
        for mode in ("isolated", "concurrent"):
            for src, row in enumerate(links.get(f"{mode}_gbps") or []):
                for dst, v in enumerate(row):
                    if src != dst:
                        self.xgmi_link.labels(n, str(src), str(dst), mode).set(v)
        for ranks, bw in (rc.get("busbw_by_ranks") or {}).items():     # the 2/4/8-rank sweep
            if bw is not None:
                self.busbw.labels(n, str(ranks)).set(bw)

    def refresh_hip_failure(self) -> None:
        n = self.ctx.node_name
        doc = self.ctx.status.read(S.HIP_LAST_FAILURE)
        self.gemm_bad_tile.clear()
        if not doc:
            self.hip_failure_ts.labels(n).set(0)
            return
        self.hip_failure_ts.labels(n).set(doc.get("ts", 0))
        for f in doc.get("failures") or []:
            w = f.get("where") if isinstance(f, dict) else None
            if not isinstance(w, dict) or "tile" not in w:
                continue
            cu = w.get("cu") or {}
            cu_s = f"se{cu.get('se')}.sh{cu.get('sh')}.cu{cu.get('cu')}" if cu else ""
            xcd = "" if w.get("xcd") is None else str(w.get("xcd"))
            self.gemm_bad_tile.labels(n, str(w.get("device")), comp._dtype_key(str(w.get("dtype", "bf16"))),
                                      ",".join(str(x) for x in w.get("tile") or []), xcd, cu_s).set(1)

    def refresh_device_health(self) -> None:
        """The device plugin's health verdicts (device-health in the status directory)."""
        from ..operands.device_plugin import DEVICE_HEALTH_FILE
        n = self.ctx.node_name
        doc = self.ctx.status.read(DEVICE_HEALTH_FILE) or {}
        devs = doc.get("devices") or {}
        if not isinstance(devs, dict):
            return
        self.dev_unhealthy.clear()
        bad = 0
        for did, d in sorted(devs.items()):
            if isinstance(d, dict) and not d.get("healthy", True):
                bad += 1
                self.dev_unhealthy.labels(n, did, str(d.get("bdf", "")), str(d.get("reason", ""))).set(1)
        self.dev_unhealthy_total.labels(n).set(bad)

    def refresh_driver(self) -> None:
        n = self.ctx.node_name
        try:
            comp.check_driver(self.ctx)
            self.driver_validation.labels(n).set(1)
            self.driver_last_success.labels(n).set(time.time())
        except (comp.ValidationError, OSError, ImportError) as e:
            log.info("driver check failed: %s", e)
            self.driver_validation.labels(n).set(0)

    def refresh_plugin(self) -> None:
        n = self.ctx.node_name
        try:
            node = self.ctx.client.get("v1", "Node", n)
            total = sum(comp.gpu_resources(node, "mixed").values())
            self.devices_total.labels(n).set(total)
            if total:
                self.devices_last_success.labels(n).set(time.time())
        except Exception as e:  # noqa: BLE001
            log.info("node capacity check failed: %s", e)
            self.devices_total.labels(n).set(-1)

    def refresh_pci(self) -> None:
        n = self.ctx.node_name
        try:
            self.pci_total.labels(n).set(len([f for f in devices.scan_pci(self.ctx.sys_root)
                                              if not f["is_virtfn"]]))
        except Exception:  # noqa: BLE001
            self.pci_total.labels(n).set(-1)

    def refresh_all(self) -> None:
        self.refresh_status()
        self.refresh_driver()
        if self.ctx.client is not None:
            self.refresh_plugin()
        self.refresh_pci()

    # -- loops --------------------------------------------------------------------------------
    def _loop(self, period: float, fn) -> None:
        while not self._stop.is_set():
            fn()
            self._stop.wait(period)

    def _watch_barriers(self) -> None:
        names = [f for files in BARRIERS.values() for f in files]
        while not self._stop.is_set():
            missing = [f for f in names if not self.ctx.status.exists(f)]
            # wake on the next barrier creation (inotify); re-check at least every period
            if missing:
                self.ctx.status.wait(missing, any_of=True, timeout=STATUS_PERIOD)
            else:
                self._stop.wait(STATUS_PERIOD)
            self.refresh_status()

    def start(self, port: int) -> int:
        from ..runtime.manager import _Server
        from prometheus_client import generate_latest
        from prometheus_client.exposition import CONTENT_TYPE_LATEST

        self.refresh_all()
        for period, fn in ((DRIVER_PERIOD, self.refresh_driver), (PCI_PERIOD, self.refresh_pci)):
            threading.Thread(target=self._loop, args=(period, fn), daemon=True).start()
        if self.ctx.client is not None:
            threading.Thread(target=self._loop, args=(PLUGIN_PERIOD, self.refresh_plugin), daemon=True).start()
        threading.Thread(target=self._watch_barriers, daemon=True).start()
        srv = _Server(("0.0.0.0", port), {"/metrics": lambda: (200, CONTENT_TYPE_LATEST,
                                                               generate_latest(self.registry))})
        srv.start()
        return srv.port

    def stop(self) -> None:
        self._stop.set()
