"""``amd-validator``: node validator CLI (reference: validator/main.go:207-545).

Component from ``--component`` / ``COMPONENT``: driver, toolkit, hip, plugin, rccl, rdma,
metrics, vfio-pci, mxgpu-manager, mxgpu-devices, sandbox-ready-wait, ready (the validator's
main container). Reference component names cuda / mofed / vgpu-* are accepted too.

Flags / env (reference names kept where they exist): ``--with-wait``/WITH_WAIT,
``--with-workload``/WITH_WORKLOAD, ``--cleanup-all``/CLEANUP_ALL, ``--output-dir``/OUTPUT_DIR,
``--sleep-interval-seconds``/SLEEP_INTERVAL_SECONDS, ``--partition-strategy``/PARTITION_STRATEGY
(MIG_STRATEGY accepted), ``--metrics-port``/METRICS_PORT, ``--node-name``/NODE_NAME,
``--namespace``/OPERATOR_NAMESPACE, ``--default-gpu-workload-config``/DEFAULT_GPU_WORKLOAD_CONFIG,
``--wait-timeout-seconds``/WAIT_TIMEOUT_SECONDS (new: bounds every wait).
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

from . import components as comp
from . import status as S
from ..utils import mounts


def _bool(v: str) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    e = os.environ.get
    ap = argparse.ArgumentParser(prog="amd-validator")
    ap.add_argument("-c", "--component", default=e("COMPONENT", ""))
    ap.add_argument("-w", "--with-wait", default=e("WITH_WAIT", "false"))
    ap.add_argument("-l", "--with-workload", default=e("WITH_WORKLOAD", "true"))
    ap.add_argument("-r", "--cleanup-all", default=e("CLEANUP_ALL", "false"))
    ap.add_argument("-o", "--output-dir", default=e("OUTPUT_DIR", mounts.path(S.DEFAULT_DIR)))
    ap.add_argument("-s", "--sleep-interval-seconds", type=float, default=float(e("SLEEP_INTERVAL_SECONDS", "5")))
    ap.add_argument("--wait-timeout-seconds", type=float, default=float(e("WAIT_TIMEOUT_SECONDS", "3600")))
    ap.add_argument("-m", "--partition-strategy",
                    default=e("PARTITION_STRATEGY", e("MIG_STRATEGY", "single")))
    ap.add_argument("-p", "--metrics-port", type=int, default=int(e("METRICS_PORT", "0")))
    ap.add_argument("-n", "--node-name", default=e("NODE_NAME", ""))
    ap.add_argument("--namespace", default=e("OPERATOR_NAMESPACE", ""))
    ap.add_argument("-g", "--default-gpu-workload-config", default=e("DEFAULT_GPU_WORKLOAD_CONFIG", "vm-passthrough"))
    ap.add_argument("--host-root", default=e("HOST_ROOT", mounts.path("/host")))
    ap.add_argument("--sys-root", default=e("AMD_SYSFS_ROOT", "/"))
    ap.add_argument("--dev-root", default=e("AMD_DEV_ROOT", "/"))
    ap.add_argument("--kubeconfig", default=e("KUBECONFIG", None))
    return ap


def make_context(a, client=None) -> comp.Context:
    return comp.Context(
        status=S.StatusDir(a.output_dir), node_name=a.node_name, namespace=a.namespace, client=client,
        host_root=a.host_root, driver_root=mounts.path("/run/amd/driver"), sys_root=a.sys_root, dev_root=a.dev_root,
        with_wait=_bool(a.with_wait),
        with_workload=_bool(a.with_workload), sleep_interval=a.sleep_interval_seconds,
        wait_timeout=a.wait_timeout_seconds, partition_strategy=a.partition_strategy,
        default_workload=a.default_gpu_workload_config)


NEEDS_CLIENT = {"hip", "cuda", "plugin", "rccl", "metrics", "rdma", "mofed", "vfio-pci", "mxgpu-manager",
                "vgpu-manager", "mxgpu-devices", "vgpu-devices"}


def main(argv=None, client=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    a = build_parser().parse_args(argv)
    if not a.component:
        print("no component given (--component / COMPONENT)", file=sys.stderr)
        return 2
    if a.component not in comp.COMPONENTS and a.component not in ("metrics", "ready"):
        print(f"invalid component specified for validation: {a.component}", file=sys.stderr)
        return 2
    sd = S.StatusDir(a.output_dir)
    if _bool(a.cleanup_all):
        sd.cleanup_all()
    sd.ensure()
    if client is None and a.component in NEEDS_CLIENT and (a.node_name or a.component == "metrics"):
        try:
            from ..k8s.rest import Config, RestClient
            client = RestClient(Config.from_kubeconfig(a.kubeconfig) if a.kubeconfig else Config.auto())
        except Exception as e:  # noqa: BLE001
            if a.component in ("hip", "cuda", "plugin", "rccl") and \
                    os.environ.get("HIP_VALIDATION_MODE", "pod") != "local":
                print(f"cannot reach the Kubernetes API: {e}", file=sys.stderr)
                return 1
            client = None
    ctx = make_context(a, client)

    if a.component == "ready":
        summary = {k: sd.read(f) is not None for k, fs in
                   (("driver", (S.DRIVER_READY, S.HOST_DRIVER_READY)), ("toolkit", (S.TOOLKIT_READY,)),
                    ("hip", (S.HIP_READY,)), ("plugin", (S.PLUGIN_READY,)), ("rccl", (S.RCCL_READY,)))
                   for f in fs}
        ttr = S.time_to_ready(sd)
        print(json.dumps({"event": "all validations are successful", "barriers": summary,
                          "time_to_ready_s": ttr}), flush=True)
        stop = threading.Event()
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        stop.wait()
        return 0
    if a.component == "metrics":
        from .metrics import NodeMetrics
        m = NodeMetrics(ctx)
        port = m.start(a.metrics_port or 8000)
        logging.getLogger("amd-validator").info("node metrics on :%d", port)
        stop = threading.Event()
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        stop.wait()
        m.stop()
        return 0

    t0 = time.monotonic()
    try:
        info = comp.COMPONENTS[a.component](ctx)
    except comp.ValidationError as e:
        print(f"error validating {a.component}: {e}", file=sys.stderr)
        return 1
    print(json.dumps({"component": a.component, "ok": True, "seconds": round(time.monotonic() - t0, 3),
                      "info": info}, default=str), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
