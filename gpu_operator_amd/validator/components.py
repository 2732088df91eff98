"""Validator components: each validates one layer of the node and writes its barrier.

Reference counterparts (validator/main.go): Driver :607-708, Toolkit :775-801, CUDA
:1176-1293 (-> HIP here), Plugin :803-1015, MOFED :847-912 (-> RDMA), VfioPCI :1301-1356,
VGPUManager :1358-1426 (-> MxGPU manager), VGPUDevices :1428-1501 (-> MxGPU devices),
workload-type :405-437. New: RCCL (all-GPU all-reduce over xGMI).

Every wait is event-driven and bounded (the reference's ``--with-wait`` loops forever,
SURVEY.md §7.7 quirk 6; its toolkit validation relies on crash-loop back-off, quirk 6).
"""

from __future__ import annotations

import json
import logging
import os
import shutil
import subprocess
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from .. import devices
from ..k8s import errors
from ..k8s import objects as o
from ..utils import mounts
from . import status as S
from . import workload as W

log = logging.getLogger("amd-validator")

GPU_RESOURCE = "amd.com/gpu"
PARTITION_RESOURCE_PREFIX = "amd.com/partition-"
MELLANOX_LABEL = "feature.node.kubernetes.io/pci-15b3.present"
WORKLOAD_CONFIG_LABEL = "amd.com/gpu.workload.config"


class ValidationError(Exception):
    """A component's check failed. ``failures``: the structured gate failures behind it (GateFailure),
    when the check was a gate."""

    def __init__(self, msg: str, failures: Optional[List["GateFailure"]] = None):
        super().__init__(msg)
        self.failures = list(failures or [])


@dataclass(frozen=True)
class GateFailure:
    """One reason a measurement must not open a barrier. ``kind`` says what failed, so what to do
    about it never depends on the wording of ``text``: ``correctness`` (a wrong result, a failed
    launch, smoke test or probe, a lost worker), ``oom`` (the shape did not fit the free HBM),
    ``floor`` (below the per-GPU TFLOP/s floor), ``relative`` (below the node median), ``efficiency``
    (a scaling step below the gate), ``uniformity`` (the workload's own node-median gate)."""
    kind: str
    text: str
    # where a correctness failure happened, when the workload could say (amd-gemm-validate's ABFT check:
    # device, dtype, tile, workgroup, xcd, cu); not part of the failure's identity
    where: Optional[Dict[str, Any]] = field(default=None, compare=False, hash=False)

    def __str__(self) -> str:
        return self.text


THROUGHPUT_KINDS = frozenset({"floor", "relative", "efficiency", "uniformity"})
# (the fabric gates: "link" -- one xGMI pair below the node median, corrupted or without peer
# access -- and "busbw" -- the all-reduce below its floor)


@dataclass
class Context:
    status: S.StatusDir
    node_name: str = ""
    namespace: str = ""
    client: Any = None
    host_root: str = "/host"         # host filesystem as mounted in the container
    sys_root: str = "/"              # sysfs root (the container's /sys is the host's)
    dev_root: str = "/"
    driver_root: str = "/run/amd/driver"
    with_wait: bool = False
    with_workload: bool = False
    sleep_interval: float = 5.0
    wait_timeout: float = 3600.0     # bound on any --with-wait (the reference waits forever)
    pod_timeout: float = 300.0       # validation pod completion (reference: 60 x 5 s)
    resource_timeout: float = 150.0  # GPU resources in node capacity (reference: 30 x 5 s)
    partition_strategy: str = "single"
    default_workload: str = "vm-passthrough"
    env: Dict[str, str] = field(default_factory=lambda: dict(os.environ))
    run: Callable[..., subprocess.CompletedProcess] = subprocess.run
    clock: Callable[[], float] = time.monotonic
    # VALIDATOR_WAIT_MODE=poll: wait the way the reference validator does -- fixed
    # sleep_interval polls for barriers, node capacity and workload pods
    # (reference validator/main.go:127,556-572,1042-1059,1102-1122). Used by the node bring-up
    # harness (ttr.py) to execute the reference protocol; production waits are event-driven.
    poll_mode: bool = False

    def __post_init__(self):
        if self.env.get("VALIDATOR_WAIT_MODE", "") == "poll":
            self.poll_mode = True


def retry(ctx: Context, what: str, fn: Callable[[], Any]) -> Any:
    """Run ``fn`` once, or until it stops raising (bounded by ctx.wait_timeout) in wait mode."""
    deadline = ctx.clock() + ctx.wait_timeout
    delay = ctx.sleep_interval if ctx.poll_mode else 0.2
    while True:
        try:
            return fn()
        except ValidationError as e:
            if not ctx.with_wait or ctx.clock() >= deadline:
                raise
            log.info("%s not ready (%s); retrying in %.1fs", what, e, delay)
            time.sleep(delay)
            delay = min(ctx.sleep_interval, delay * 2)


def wait_barriers(ctx: Context, names, timeout: Optional[float]) -> bool:
    """Event-driven (inotify) barrier wait; a fixed-period stat loop in poll mode."""
    if not ctx.poll_mode:
        return bool(ctx.status.wait(names, timeout=timeout))
    deadline = None if timeout is None else ctx.clock() + timeout
    while not all(ctx.status.exists(n) for n in names):
        if deadline is not None and ctx.clock() >= deadline:
            return False
        time.sleep(ctx.sleep_interval)
    return True


# ---------------------------------------------------------------------------------------------
# driver
# ---------------------------------------------------------------------------------------------
HOST_DRIVER_MARKERS = ("/usr/bin/amd-smi", "/opt/rocm/bin/amd-smi", "/usr/sbin/amdgpu-install")


def host_driver_installed(ctx: Context) -> bool:
    mode = ctx.env.get("DRIVER_ROOT_MODE", "")
    if mode:
        return mode == "host"
    return any(os.path.exists(ctx.host_root + m) for m in HOST_DRIVER_MARKERS)


def check_driver(ctx: Context) -> Dict[str, Any]:
    st = devices.driver_state(ctx.sys_root, ctx.dev_root)
    if not st["module_loaded"]:
        raise ValidationError("amdgpu module not loaded")
    if not st["live"]:
        raise ValidationError("amdgpu initstate is not live")
    if not st["kfd_present"]:
        raise ValidationError("/dev/kfd missing")
    if st["kfd_gpu_nodes"] == 0:
        raise ValidationError("KFD reports no GPU agents")
    gpus = devices.enumerate_gpus(ctx.sys_root)
    pci = [f for f in devices.scan_pci(ctx.sys_root) if not f["is_virtfn"] and f["driver"] == "amdgpu"]
    bound = {g["pci_bdf"] for g in gpus}
    missing = [f["bdf"] for f in pci if f["bdf"] not in bound]
    # A privileged validator sees every GPU; a device-cgroup-restricted container sees all PCI
    # functions in sysfs but only its own KFD agents (DRIVER_VALIDATION_STRICT=false there).
    if missing and ctx.env.get("DRIVER_VALIDATION_STRICT", "true") == "true":
        raise ValidationError(f"amdgpu-bound GPUs without a KFD agent: {missing}")
    return {"driver_version": st["version"] or "inbox", "gpus": len({g["pci_bdf"] for g in gpus}),
            "kfd_agents": st["kfd_gpu_nodes"], "gfx": sorted({g["gfx_target"] for g in gpus}),
            "hidden_gpus": len(missing),
            "products": sorted({g["product_name"] for g in gpus if g["product_name"]})}


def validate_driver(ctx: Context) -> Dict[str, Any]:
    host = host_driver_installed(ctx)
    if not host:
        # driver container: its startup probe writes .driver-ctr-ready once amdgpu is live
        t = None if not ctx.with_wait else ctx.wait_timeout
        if not ctx.status.exists(S.DRIVER_CTR_READY):
            if not ctx.with_wait:
                raise ValidationError("driver container not ready (.driver-ctr-ready missing)")
            if not wait_barriers(ctx, [S.DRIVER_CTR_READY], t):
                raise ValidationError("timed out waiting for the driver container")
    info = retry(ctx, "driver", lambda: check_driver(ctx))
    info["mode"] = "host" if host else "container"
    name = S.HOST_DRIVER_READY if host else S.DRIVER_READY
    ctx.status.delete(S.DRIVER_READY if host else S.HOST_DRIVER_READY)
    _keep_first_ts(ctx, name, info)
    ctx.status.create(name, info)
    return info


def _keep_first_ts(ctx: Context, name: str, info: Dict[str, Any]) -> None:
    """A re-validated barrier keeps the time the layer was first found ready (the start of node
    time-to-ready) and records the re-check as ``revalidated_ts`` -- as amd-node-validate does."""
    old = ctx.status.read(name)
    if old and isinstance(old.get("ts"), (int, float)):
        info["ts"] = old["ts"]
        info["revalidated_ts"] = time.time()


# ---------------------------------------------------------------------------------------------
# runtime hook (toolkit)
# ---------------------------------------------------------------------------------------------
def check_toolkit(ctx: Context) -> Dict[str, Any]:
    """Inside a container started through the AMD runtime hook with AMD_VISIBLE_DEVICES=all,
    /dev/kfd and the render nodes of every GPU must have been injected."""
    kfd = os.path.join(ctx.dev_root, "dev/kfd")
    if not os.path.exists(kfd):
        raise ValidationError("/dev/kfd not injected into the container")
    dri = os.path.join(ctx.dev_root, "dev/dri")
    render = sorted(x for x in (os.listdir(dri) if os.path.isdir(dri) else []) if x.startswith("renderD"))
    gpus = devices.enumerate_gpus(ctx.sys_root)
    want = {f"renderD{g['drm_render_minor']}" for g in gpus if g["drm_render_minor"] >= 0}
    missing = sorted(want - set(render))
    if missing:
        raise ValidationError(f"render nodes not injected: {missing}")
    return {"render_nodes": len(render), "kfd": True}


def validate_toolkit(ctx: Context) -> Dict[str, Any]:
    info = retry(ctx, "toolkit", lambda: check_toolkit(ctx))
    ctx.status.create(S.TOOLKIT_READY, info)
    return info


# ---------------------------------------------------------------------------------------------
# node shape: GPU model, physical GPUs, GPU pods holding devices
# ---------------------------------------------------------------------------------------------
GEMM_FLOOR_FRACTION = 0.50     # of the model's dense peak: healthy MI355X runs 0.63-0.68 on random data
GEMM_MIN_RELATIVE = 0.85       # of the node median, same dtype and shape: boxes differ ~6 %, GPUs of one box ~2 %
GEMM_MIN_EFFICIENCY = 0.90     # of N x the 1-GPU figure: independent GEMMs on separate GPUs scale at ~1.0
BUSBW_FLOOR_FRACTION = 0.25    # of one xGMI link (model): only when no link matrix was measured
BUSBW_MESH_FRACTION = 0.30     # of the measured mesh bound (smallest per-GPU concurrent link ingress)
LINK_MIN_RELATIVE = 0.80       # of the node median, per link and mode: one degraded xGMI link is named
FABRIC_ANNOTATION = "amd.com/gpu.fabric-validation"   # read for records of older validators only


def _validator_env(ctx: Context) -> Dict[str, str]:
    return {k: v for k, v in ctx.env.items() if k.startswith("VALIDATOR_")}


def _gpus(ctx: Context) -> List[Dict[str, Any]]:
    try:
        return devices.enumerate_gpus(ctx.sys_root)
    except Exception as e:  # noqa: BLE001 - no sysfs access / no native library: callers fall back
        log.info("GPU enumeration failed: %s", e)
        return []


def node_model(ctx: Context, gpus: Optional[List[Dict[str, Any]]] = None):
    """The catalog entry (models/) of this node's GPUs, or None."""
    from .. import models
    for g in (gpus if gpus is not None else _gpus(ctx)):
        hit = models.by_device_id(g.get("device_id", 0))
        if hit:
            return hit[0]
    return None


def physical_gpus(ctx: Context, node: Optional[Dict[str, Any]] = None) -> List[Dict[str, Any]]:
    """One KFD agent per physical GPU (a CPX GPU shows one agent per partition, all on one PCI
    function): the lowest-index agent of each BDF. The HIP device index of that agent is its
    position in KFD order."""
    first: Dict[str, Dict[str, Any]] = {}
    for g in sorted(_gpus(ctx), key=lambda g: g["index"]):
        first.setdefault(g["pci_bdf"], g)
    return list(first.values())


def physical_gpu_count(ctx: Context, node: Optional[Dict[str, Any]] = None) -> int:
    """Physical GPUs of the node: KFD agents grouped by PCI function; without sysfs, the
    labeller's ``amd.com/gpu.count`` label (also physical GPUs); never ``allocatable``, which
    counts time-slicing replicas or partitions."""
    n = len(physical_gpus(ctx, node))
    if n == 0 and node is not None:
        try:
            n = int(o.get_labels(node).get("amd.com/gpu.count", "0") or 0)
        except ValueError:
            n = 0
    return n


def _requests_gpu(pod: Dict[str, Any]) -> bool:
    for c in ((pod.get("spec") or {}).get("containers") or []) + ((pod.get("spec") or {}).get("initContainers") or []):
        res = c.get("resources") or {}
        for k in list((res.get("limits") or {})) + list((res.get("requests") or {})):
            if k == GPU_RESOURCE or k.startswith(PARTITION_RESOURCE_PREFIX):
                return True
    return False


def _pod_start(p: Dict[str, Any]) -> Optional[float]:
    """A pod's ``status.startTime`` (when the kubelet accepted it) as epoch seconds; None if unknown."""
    ts = (p.get("status") or {}).get("startTime")
    if not ts:
        return None
    try:
        import datetime
        return datetime.datetime.fromisoformat(str(ts).replace("Z", "+00:00")).timestamp()
    except ValueError:
        return None


def gpu_pods_on_node(ctx: Context, started_before: Optional[float] = None,
                     later: Optional[List[str]] = None) -> List[str]:
    """Running pods on this node that hold GPU resources (``amd.com/gpu`` or a partition
    resource), excluding the validator's own validation pods. A throughput number taken beside
    them measures the sharing, not the hardware. ``started_before``: only pods whose start time is
    not later than it (unknown start times count: never assume a tenant arrived late); the ones left
    out are appended to ``later``."""
    if ctx.client is None or not ctx.node_name:
        return []
    try:
        pods = ctx.client.list("v1", "Pod", field_selector=f"spec.nodeName={ctx.node_name}")
    except Exception as e:  # noqa: BLE001 - treat as unknown: do not block validation on it
        log.info("listing pods on %s failed: %s", ctx.node_name, e)
        return []
    own = {"amd-hip-validator", "amd-rccl-validator", "amd-device-plugin-validator"}
    out = []
    for p in pods:
        if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
            continue
        if o.get_labels(p).get("app") in own or not _requests_gpu(p):
            continue
        start = _pod_start(p)
        if started_before is not None and start is not None and start > started_before:
            if later is not None:
                later.append(f"{o.namespace(p)}/{o.name(p)}")
            continue
        out.append(f"{o.namespace(p)}/{o.name(p)}")
    return sorted(out)


def _pod_device_ids(ctx: Context) -> Optional[Dict[str, List[str]]]:
    """"namespace/name" -> AMD device ids the kubelet allocated to the pod (pod-resources List, the
    API the metrics exporter attributes GPUs with). None when the socket cannot be queried."""
    from ..operands import kubeletapi as K
    sock = ctx.env.get("POD_RESOURCES_SOCKET") or mounts.path(K.POD_RESOURCES_SOCKET)
    if not os.path.exists(sock):
        return None
    try:
        import grpc
        with grpc.insecure_channel("unix://" + sock) as ch:
            resp = K.pod_resources_stub(ch)(K.PR["ListPodResourcesRequest"](), timeout=5.0)
    except Exception as e:  # noqa: BLE001 - unknown attribution: the caller treats every GPU as held
        log.info("pod-resources query failed: %s", e)
        return None
    out: Dict[str, List[str]] = {}
    for pr in resp.pod_resources:
        ids = [did for c in pr.containers for d in c.devices if d.resource_name.startswith("amd.com/")
               for did in d.device_ids]
        if ids:
            out[f"{pr.namespace}/{pr.name}"] = ids
    return out


def _agent_of(device_id: str, gpus: List[Dict[str, Any]]) -> Optional[Dict[str, Any]]:
    """The KFD agent a device-plugin id names: ``amdgpu-<unique id hex>`` (uuid strategy) or the
    agent index (index strategy); a time-slicing replica ``<id>::<k>`` is its GPU."""
    base = device_id.split("::")[0]
    for g in gpus:
        if (g.get("unique_id") and base == f"amdgpu-{g['unique_id']:016x}") or base == str(g["index"]):
            return g
    return None


def held_gpus(ctx: Context, busy: List[str], gpus: Optional[List[Dict[str, Any]]] = None) -> Dict[str, Any]:
    """Which physical GPUs (PCI functions) the running GPU pods ``busy`` hold. A GPU counts as held
    when any of its agents (CPX partitions share its HBM and power) is allocated to one of them.
    Without a device mapping for every busy pod (no pod-resources socket, an unknown id) every GPU
    is held: the validator never guesses a tenant's GPU is free."""
    gpus = gpus if gpus is not None else _gpus(ctx)
    if not busy:
        return {"held_bdfs": [], "attribution": "none", "by_pod": {}}
    ids = _pod_device_ids(ctx)
    by_pod: Dict[str, List[str]] = {}
    unmapped = []
    for pod in busy:
        agents = [_agent_of(d, gpus) for d in (ids or {}).get(pod, [])]
        if ids is None or not agents or any(a is None for a in agents):
            unmapped.append(pod)
            continue
        by_pod[pod] = sorted({a["pci_bdf"] for a in agents})
    if unmapped:
        return {"held_bdfs": sorted({g["pci_bdf"] for g in gpus}), "attribution": "unattributed",
                "unattributed_pods": unmapped[:16], "by_pod": by_pod}
    return {"held_bdfs": sorted({b for v in by_pod.values() for b in v}), "attribution": "pod-resources",
            "by_pod": by_pod}


def hip_plan(ctx: Context, busy: List[str], gpus: Optional[List[Dict[str, Any]]] = None) -> Dict[str, Any]:
    """The HIP validation plan for this node: the full stabilised GEMM sweep on the GPUs no pod
    holds (``full``: HIP indices, None = every GPU), a correctness-only probe on the held ones
    (``probe``). Reference: the plugin workload asks the scheduler for exactly 1 GPU
    (validator/main.go:978-983) and the CUDA pod runs a microsecond vectorAdd
    (validator/cuda-workload-validation.yaml:20) -- neither touches a GPU someone else was given."""
    gpus = gpus if gpus is not None else _gpus(ctx)
    held = held_gpus(ctx, busy, gpus)
    if not busy:
        return {"full": None, "probe": [], **held}
    hb = set(held["held_bdfs"])
    order = sorted(gpus, key=lambda g: g["index"])
    return {"full": [g["index"] for g in order if g["pci_bdf"] not in hb],
            "probe": [g["index"] for g in order if g["pci_bdf"] in hb], **held}


def _env_float(ctx: Context, key: str) -> Optional[float]:
    v = ctx.env.get(key, "")
    if v == "":
        return None
    try:
        return float(v)
    except ValueError:
        raise ValidationError(f"{key}={v!r} is not a number")


def gemm_floors(ctx: Context, gpus: Optional[List[Dict[str, Any]]] = None) -> Dict[str, float]:
    """Per-GPU TFLOP/s floors of the GEMM probe, by dtype. ``GEMM_MIN_TFLOPS_BF16`` /
    ``GEMM_MIN_TFLOPS_FP8`` (spec.validator.hip.env) win when set (0 = no floor); otherwise
    ``GEMM_FLOOR_FRACTION`` (default GEMM_FLOOR_FRACTION, 0.50) of the node model's dense peak, scaled to the CUs of
    one HIP device (a CPX partition has 1/8 of the GPU). Unknown model: no floor."""
    gpus = gpus if gpus is not None else _gpus(ctx)
    model = node_model(ctx, gpus)
    frac = _env_float(ctx, "GEMM_FLOOR_FRACTION")
    frac = GEMM_FLOOR_FRACTION if frac is None else frac
    share = 1.0
    if model is not None and model.cus and gpus:
        share = min(1.0, min(g["cu_count"] for g in gpus) / model.cus)
    out = {}
    for dtype, key, peak in (("bf16", "GEMM_MIN_TFLOPS_BF16", model.bf16_dense_tflops if model else 0.0),
                             ("fp8", "GEMM_MIN_TFLOPS_FP8", model.fp8_dense_tflops if model else 0.0)):
        v = _env_float(ctx, key)
        out[dtype] = round(v if v is not None else peak * frac * share, 1)
    return out


def busbw_floor(ctx: Context) -> float:
    """The explicit all-reduce bus-bandwidth floor (GB/s): ``RCCL_MIN_BUSBW_GBPS`` when set, else 0 --
    the floor is then mesh-aware (busbw_gate), from the link matrix the same run measures."""
    v = _env_float(ctx, "RCCL_MIN_BUSBW_GBPS")
    return v if v is not None else 0.0


def busbw_gate(ctx: Context, info: Dict[str, Any]) -> Dict[str, Any]:
    """The floor the largest rank count's peak busBW must reach, and its basis (SURVEY §5.8 bounds):
    ``env`` (RCCL_MIN_BUSBW_GBPS), ``measured-mesh`` (RCCL_MIN_BUSBW_MESH_FRACTION, default
    BUSBW_MESH_FRACTION, x the smallest per-GPU ingress with every peer pulling at once -- what a
    collective over this node's links can at best move), or ``model-link`` (BUSBW_FLOOR_FRACTION of
    the model's per-link bandwidth, when no matrix was measured)."""
    explicit = busbw_floor(ctx)
    if explicit:
        return {"min_busbw_gbps": explicit, "basis": "env"}
    mesh = (info.get("links") or {}).get("min_gpu_ingress_gbps")
    if mesh:
        frac = _gate_value(ctx, "RCCL_MIN_BUSBW_MESH_FRACTION", BUSBW_MESH_FRACTION)
        return {"min_busbw_gbps": round(frac * mesh, 1), "basis": "measured-mesh", "measured_mesh_bound_gbps": mesh,
                "fraction": frac}
    model = node_model(ctx)
    return {"min_busbw_gbps": round(model.xgmi_link_gbps * BUSBW_FLOOR_FRACTION, 1) if model else 0.0,
            "basis": "model-link"}


def gate_links(links: Dict[str, Any], min_relative: float) -> List[GateFailure]:
    """The xGMI link matrix's own gate, re-checked here: every ordered GPU pair whose isolated or
    concurrent bandwidth is below ``min_relative`` x the node median of that mode, every pair whose
    copy came back corrupted, every pair without peer access -- each one named ``src->dst``."""
    if not links or links.get("skipped"):
        return []
    bad: List[GateFailure] = []
    for mode in ("isolated", "concurrent"):
        m = links.get(f"{mode}_gbps") or []
        vals = [(s, d, float(v)) for s, row in enumerate(m) for d, v in enumerate(row) if s != d]
        if not vals or not min_relative:
            continue
        med = sorted(v for _, _, v in vals)[len(vals) // 2]
        for s, d, v in vals:
            if med > 0 and v < min_relative * med:
                bad.append(GateFailure("link", f"xGMI link {s}->{d} ({mode}): {v:.1f} GB/s is {v / med:.2f}x the node "
                                               f"median {med:.1f} (floor {min_relative:g}x)"))
    bad += [GateFailure("link", f"xGMI link {x}: copied data corrupted") for x in links.get("corrupt_links") or []]
    bad += [GateFailure("link", f"xGMI link {x}: no peer access") for x in links.get("no_peer_access") or []]
    return bad


# ---------------------------------------------------------------------------------------------
# HIP (matrix-core GEMM + smoke) -- replaces the CUDA vectorAdd validation
# ---------------------------------------------------------------------------------------------
def _dtype_key(name: str) -> str:
    return "fp8" if name.startswith("fp8") else "bf16"


def summarize_gemm(results: List[Dict[str, Any]]) -> Dict[str, Any]:
    agg = [r for r in results if r.get("event") == "aggregate"]
    per = [r for r in results if r.get("event") == "gemm" and not r.get("probe")]
    probe = [r for r in results if r.get("event") == "gemm" and r.get("probe")]
    smoke = [r for r in results if r.get("event") == "hip-smoke"]
    out: Dict[str, Any] = {"gemm": per, "aggregate": agg,
                           "uniformity": [r for r in results if r.get("event") == "uniformity"]}
    plan = next((r for r in results if r.get("event") == "plan"), None)
    if plan is not None:
        out["plan"] = plan
    if probe:
        # tenant-held GPUs: correctness only; a GPU whose HBM the tenant holds is skipped, not failed
        out["probe"] = [{"device": r.get("device"), "ok": bool(r.get("ok")),
                         **({"skipped": "busy: " + str(r.get("error", "out of memory"))} if r.get("oom") else {}),
                         **({"error": r["error"]} if r.get("error") and not r.get("oom") else {})} for r in probe]
    if agg:
        # headline: bf16 before fp8, the largest shape, then the most GPUs
        head = max(agg, key=lambda r: (_dtype_key(r.get("dtype", "bf16")) == "bf16", r["m"] * r["n"] * r["k"],
                                       r.get("gpus", 1)))
        out["gemm_tflops_total"] = head["total_tflops"]
        out["gemm_tflops_per_gpu"] = head["per_gpu_tflops"]
        out["gpus"] = head.get("gpus")
        by: Dict[str, Dict[str, Any]] = {}
        for r in agg:
            big = max(x["m"] * x["n"] * x["k"] for x in agg if x.get("dtype") == r.get("dtype"))
            if r["m"] * r["n"] * r["k"] != big:
                continue
            by.setdefault(_dtype_key(r.get("dtype", "bf16")), {})[str(r.get("gpus", 1))] = {
                "total_tflops": r["total_tflops"], "per_gpu_tflops": r["per_gpu_tflops"],
                **({"efficiency": r["efficiency"]} if "efficiency" in r else {})}
        out["tflops_by_dtype_gpus"] = by
    # every GPU's best TFLOP/s per (dtype, shape): the workload's compact lines, else the per-GPU ones
    lines = [r for r in results if r.get("event") == "gpu_tflops"]
    if not lines and per:
        from .workload_main import gpu_tflops_lines
        lines = gpu_tflops_lines(per)
    if lines:
        out["gpu_tflops"] = [{k: r[k] for k in ("dtype", "m", "n", "k", "tflops")} for r in lines]
    sc = [r for r in results if r.get("event") == "scaling"]
    if sc:
        out["scaling_skipped"] = sorted({r["gpus"] for r in sc if r.get("skipped")})
    if smoke:
        out["smoke_ok"] = all(s.get("ok") for s in smoke)
    # the ABFT coverage of the run: the least covered GEMM and the closest any sum came to its bound
    checked = [r for r in per + probe if "checked_fraction" in r]
    if checked:
        out["checked_fraction"] = min(float(r["checked_fraction"]) for r in checked)
        out["abft_worst_ratio"] = max(float(r.get("abft_worst_ratio", 0.0)) for r in checked)
    out["counters"] = [r for r in results if r.get("event") == "counters"]
    return out


def floor_applies(m: int, n: int, k: int) -> bool:
    """The per-GPU floors are fractions of the dense peak: they apply to shapes that can reach it --
    a full dispatch wave of 256x256 tiles and K >= 4096 (the same rule as amd-gemm-validate)."""
    return (m or 0) * (n or 0) >= 256 * 256 * 256 and (k or 0) >= 4096


def _relative_outliers(per: List[Dict[str, Any]], frac: float, disturbed: frozenset = frozenset()) -> List[str]:
    """GPUs whose best TFLOP/s is below ``frac`` x the node's (upper) median at the same dtype and
    shape: a 40 %-slow GPU passes any absolute floor loose enough for every box, not this. Disturbed
    GPUs (a tenant arrived during the sweep) are neither judged nor part of the median."""
    if not frac:
        return []
    best: Dict[tuple, Dict[Any, float]] = {}
    for r in per:
        if not r.get("ok") or not r.get("tflops") or r.get("device") in disturbed:
            continue
        key = (_dtype_key(r.get("dtype", "bf16")), r.get("m"), r.get("n"), r.get("k"))
        d = best.setdefault(key, {})
        d[r.get("device")] = max(d.get(r.get("device"), 0.0), float(r["tflops"]))
    bad = []
    for (dt, m, n, k), d in sorted(best.items(), key=lambda kv: str(kv[0])):
        if len(d) < 2:
            continue
        med = sorted(d.values())[len(d) // 2]
        for dev, t in sorted(d.items(), key=lambda kv: str(kv[0])):
            if t < frac * med:
                bad.append(f"gemm {dt} {m}x{n}x{k} device {dev}: {t:.1f} TFLOP/s is {t / med:.2f}x the node median "
                           f"{med:.1f} (floor {frac:g}x)")
    return bad


def _line_kind(r: Dict[str, Any]) -> str:
    """The kind of a failing workload line: the workload's own ``kind`` field; a line without one (an
    older workload image) is a correctness failure unless it says out-of-memory structurally."""
    k = r.get("kind")
    if k in THROUGHPUT_KINDS or k in ("correctness", "oom"):
        return k
    return "oom" if r.get("oom") else "correctness"


def _bad_tile(r: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """The location of a wrong GEMM result, from the workload's ABFT fields (amd-gemm-validate names
    the first bad output tile, the workgroup that computed it and -- from the checked dispatch's
    placement record -- its XCD and CU); None for a line without them."""
    if "tile" not in r:
        return None
    return {k: r[k] for k in ("device", "dtype", "tile", "workgroup", "xcd", "cu", "bad_tiles", "variant") if k in r}


def _where_text(w: Dict[str, Any]) -> str:
    cu = w.get("cu") or {}
    on = f"XCD {w['xcd']}" if w.get("xcd") is not None else "several XCDs (split-K pieces)"
    if cu:
        on += f", CU se{cu.get('se')}.sh{cu.get('sh')}.cu{cu.get('cu')}"
    return (f" [bad output tile {w.get('tile')} of {w.get('bad_tiles', 1)}, workgroup {w.get('workgroup')}"
            f" on {on}]")


def _set_devices(info: Dict[str, Any]) -> Dict[tuple, set]:
    """(dtype, m, n, k, gpus) -> the devices whose per-GPU lines belong to that set."""
    out: Dict[tuple, set] = {}
    for r in info["gemm"]:
        out.setdefault((r.get("dtype"), r.get("m"), r.get("n"), r.get("k"), r.get("gpus")), set()).add(r.get("device"))
    return out


def gate_gemm(info: Dict[str, Any], floors: Dict[str, float], busy: List[str] = (),
              min_relative: float = GEMM_MIN_RELATIVE, min_efficiency: float = GEMM_MIN_EFFICIENCY,
              disturbed: frozenset = frozenset()) -> List[GateFailure]:
    """Why a GEMM result must not open hip-ready: failed checks, any GPU of the full run below its
    dtype's floor, below ``min_relative`` x the node median, or a scaling step below
    ``min_efficiency``; on probed (tenant-held) GPUs a failed correctness check -- an allocation
    failure there is a busy skip. Also checked in the pod (--min-tflops, --min-relative,
    --min-efficiency); done here again so an older workload image cannot pass a slow GPU. The full
    run only ever covers GPUs no pod holds (hip_plan), so the floors apply to all of it -- except on
    ``disturbed`` GPUs (a tenant was given them while the sweep ran): their throughput measured the
    sharing, so only their correctness counts, and no set that ran on one is gated on throughput."""
    disturbed = frozenset(disturbed)
    sets = _set_devices(info)

    def touched(r: Dict[str, Any]) -> bool:
        devs = sets.get((r.get("dtype"), r.get("m"), r.get("n"), r.get("k"), r.get("gpus") if r.get("scaling") else None))
        return bool(disturbed) and (devs is None or bool(devs & disturbed))

    bad: List[GateFailure] = []
    for r in info["gemm"]:
        if r.get("ok"):
            continue
        kind = _line_kind(r)
        if kind in THROUGHPUT_KINDS and r.get("device") in disturbed:
            continue
        where = _bad_tile(r) if kind == "correctness" else None
        bad.append(GateFailure(kind, f"gemm {r.get('dtype', 'bf16')} device {r.get('device')}: "
                                     f"{r.get('error', 'check failed')}" + (_where_text(where) if where else ""),
                               where))
    bad += [GateFailure("correctness", f"probe device {p['device']}: {p.get('error', 'check failed')}")
            for p in info.get("probe", []) if not p["ok"] and "skipped" not in p]
    bad += [GateFailure("correctness", f"aggregate {r.get('dtype', 'bf16')} x{r.get('gpus')}: not ok")
            for r in info["aggregate"]
            if r.get("ok") is False and not bad and r.get("efficiency_ok") is not False and not touched(r)]
    if info.get("smoke_ok") is False:
        bad.append(GateFailure("correctness", "hip-smoke failed"))
    for r in info["gemm"]:
        floor = floors.get(_dtype_key(r.get("dtype", "bf16")), 0.0)
        if not floor_applies(r.get("m"), r.get("n"), r.get("k")) or r.get("device") in disturbed:
            continue
        if r.get("ok") and floor and r.get("tflops", 0.0) < floor:
            bad.append(GateFailure("floor", f"gemm {r.get('dtype', 'bf16')} device {r.get('device')}: "
                                            f"{r.get('tflops')} TFLOP/s below the {floor} floor"))
    for r in info["aggregate"]:          # the slowest GPU of each set (per-GPU lines may be cut)
        if touched(r):
            continue
        floor = floors.get(_dtype_key(r.get("dtype", "bf16")), 0.0) if floor_applies(r.get("m"), r.get("n"), r.get("k")) else 0.0
        slow = r.get("min_gpu_tflops", r.get("per_gpu_tflops", 0.0))
        if floor and slow < floor and not bad:
            bad.append(GateFailure("floor", f"aggregate {r.get('dtype', 'bf16')} x{r.get('gpus')}: slowest GPU "
                                            f"{slow} TFLOP/s below the {floor} floor"))
        eff = r.get("efficiency")
        if min_efficiency and eff is not None and (r.get("gpus") or 1) > 1 and eff < min_efficiency and \
                r.get("efficiency_gated", True) is not False:
            bad.append(GateFailure("efficiency", f"aggregate {r.get('dtype', 'bf16')} x{r.get('gpus')}: scaling "
                                                 f"efficiency {eff:.3f} below {min_efficiency:g}"))
    bad += [GateFailure("relative", b) for b in _relative_outliers(info["gemm"], min_relative, disturbed)]
    if not disturbed:         # the workload's median counted the disturbed GPUs: the check above replaces it
        bad += [GateFailure("uniformity", f"uniformity {u.get('dtype')} {u.get('m')}x{u.get('n')}x{u.get('k')}: "
                                          f"slow devices {u.get('slow_devices')} (min ratio {u.get('min_ratio')})")
                for u in info.get("uniformity", []) if u.get("ok") is False]
    return list(dict.fromkeys(bad))


def _hip_env(ctx: Context, floors: Dict[str, float], plan: Dict[str, Any]) -> Dict[str, str]:
    env = _validator_env(ctx)
    for k, v in ctx.env.items():
        if k.startswith(("GEMM_", "HIP_", "HSA_")) and k not in ("HIP_VALIDATION_MODE", "GEMM_VALIDATION_MODE"):
            env[k] = v
    env.setdefault("GEMM_SCALING", "1,2,4,8")
    env["GEMM_MIN_TFLOPS_BF16"] = f"{floors['bf16']:g}"
    env["GEMM_MIN_TFLOPS_FP8"] = f"{floors['fp8']:g}"
    env["GEMM_MIN_RELATIVE"] = f"{_gate_value(ctx, 'GEMM_MIN_RELATIVE', GEMM_MIN_RELATIVE):g}"
    env["GEMM_MIN_EFFICIENCY"] = f"{_gate_value(ctx, 'GEMM_MIN_EFFICIENCY', GEMM_MIN_EFFICIENCY):g}"
    if plan["full"] is not None:
        # tenant GPUs stay out of the full sweep: the free ones, or none at all
        env["GEMM_DEVICES"] = ",".join(map(str, plan["full"])) or "none"
    if plan["probe"]:
        env["GEMM_PROBE_DEVICES"] = ",".join(map(str, plan["probe"]))
    return env


def _gate_value(ctx: Context, key: str, default: float) -> float:
    v = _env_float(ctx, key)
    return default if v is None else v


def _run_local_hip(ctx: Context, floors: Optional[Dict[str, float]] = None,
                   plan: Optional[Dict[str, Any]] = None) -> List[Dict[str, Any]]:
    """The HIP workload in this process's container (HIP_VALIDATION_MODE=local)."""
    from .workload_main import run_hip, stream_run
    floors = floors or {}
    plan = plan or {"full": None, "probe": []}
    t0 = ctx.clock()
    results = run_hip(ctx.env.get("GEMM_SHAPES", "8192").split(","), counters=ctx.env.get("GEMM_COUNTERS") == "1",
                      # the real binaries: return at their last result line, not at their exit
                      run=stream_run if ctx.run is subprocess.run else ctx.run,
                      dtype=ctx.env.get("GEMM_DTYPE", "bf16"), scaling=ctx.env.get("GEMM_SCALING") or None,
                      iters=int(ctx.env.get("GEMM_ITERS", "50")),
                      min_tflops=floors.get("bf16", 0.0), min_tflops_fp8=floors.get("fp8", 0.0),
                      devices=plan["full"], probe_devices=plan["probe"],
                      min_relative=_gate_value(ctx, "GEMM_MIN_RELATIVE", GEMM_MIN_RELATIVE),
                      min_efficiency=_gate_value(ctx, "GEMM_MIN_EFFICIENCY", GEMM_MIN_EFFICIENCY))
    if ctx.poll_mode:
        # the reference spawns the workload pod and polls its phase every sleep_interval, first
        # right after creating it (validator/main.go:1042-1059): it sees the result at the
        # first tick after completion
        ticks = max(1, int(-(-(ctx.clock() - t0) // ctx.sleep_interval)))
        time.sleep(max(0.0, t0 + ticks * ctx.sleep_interval - ctx.clock()))
    return results


def _local_workload(ctx: Context, mode: str) -> Dict[str, Any]:
    if mode == "skip":
        return {"skipped": True}
    info = summarize_gemm(_run_local_hip(ctx))
    if [r for r in info["gemm"] if not r.get("ok")] or info.get("smoke_ok") is False:
        raise ValidationError(f"plugin workload failed: {info}")
    return info


def throughput_only(bad: List[GateFailure]) -> bool:
    """Every gate failure is a throughput gate (floor, node median, scaling efficiency, uniformity);
    none is a wrong result, a failed smoke test, a probe failure or an allocation failure."""
    return bool(bad) and all(b.kind in THROUGHPUT_KINDS for b in bad)


def disturbed_gpus(ctx: Context, plan: Dict[str, Any], gpus: List[Dict[str, Any]],
                   sweep_end: Optional[float] = None) -> Dict[str, Any]:
    """GPUs of the full sweep that a tenant was given while it ran (the HIP pod is privileged and
    requests no GPU resource, so the device plugin kept advertising them): ``devices`` (HIP indices),
    ``pods`` and ``attribution``. A tenant that started after ``sweep_end`` shared nothing with the
    sweep: its GPUs stay gated (``arrived_after``) -- a slow GPU cannot hide behind a pod scheduled
    onto it after the run. Without a device mapping for a running GPU pod every GPU of the sweep
    counts as disturbed (held_gpus never guesses a tenant's GPU is free). Reference: the plugin
    workload asks the scheduler for its GPU (validator/main.go:978-983), so it cannot share one."""
    later: List[str] = []
    now = gpu_pods_on_node(ctx, started_before=None if sweep_end is None else sweep_end + 1.0, later=later)
    if not now:
        return {"devices": [], "pods": [], "attribution": "none", **({"arrived_after": later[:16]} if later else {})}
    held = held_gpus(ctx, now, gpus)
    hb = set(held["held_bdfs"])
    full = None if plan["full"] is None else set(plan["full"])
    devs = sorted(g["index"] for g in gpus if g["pci_bdf"] in hb and (full is None or g["index"] in full))
    if not gpus and held["attribution"] == "unattributed":
        devs = ["all"]
    return {"devices": devs, "pods": now[:16], "attribution": held["attribution"],
            **({"arrived_after": later[:16]} if later else {})}


def validate_hip(ctx: Context) -> Dict[str, Any]:
    """hip-smoke + the MFMA GEMM probe (bf16 and fp8, 1/2/4/8-GPU sweep), gated on correctness, on
    per-GPU throughput floors (models/ defaults, spec.validator.hip.env overrides), on the node
    median and on scaling efficiency. Tenant-safe: GPUs that running pods hold (kubelet
    pod-resources) get a correctness-only probe, never the full sweep (hip_plan); GPUs a tenant was
    given while the sweep ran are re-checked after it and reported ``disturbed``, their throughput
    out of every gate. The pod fails fast: a failing workload ends the pod at once (restartPolicy
    Never, wait_for_pod), its result lines come back with the failure, and the failure is a
    ValidationError naming each gate. A throughput-only failure (every result correct) is measured
    once more, with a fresh plan. The reference gates on vectorAdd's exit code alone
    (validator/main.go:1176-1211)."""
    mode = ctx.env.get("HIP_VALIDATION_MODE", "pod")
    # GEMM_VALIDATION_MODE=dry-run (CPU rehearsals with a kubelet): the pod is planned, scheduled
    # and run, the GEMMs are not; HIP_VALIDATION_MODE=skip without it: nothing is spawned
    dry = ctx.env.get("GEMM_VALIDATION_MODE", "") == "dry-run"
    if mode == "skip" and not dry:      # no GPU work (CPU rehearsals of the node bring-up)
        info = {"skipped": True}
        ctx.status.create(S.HIP_READY, info)
        return info
    gpus = _gpus(ctx)
    floors = gemm_floors(ctx, gpus)
    min_rel = _gate_value(ctx, "GEMM_MIN_RELATIVE", GEMM_MIN_RELATIVE)
    min_eff = _gate_value(ctx, "GEMM_MIN_EFFICIENCY", GEMM_MIN_EFFICIENCY)

    def measure():
        # the plan is taken right before each run: a re-measure never runs on a GPU a tenant now holds
        busy = gpu_pods_on_node(ctx)
        plan = hip_plan(ctx, busy, gpus)
        failed: Optional[W.PodFailed] = None
        if mode == "local":
            results = _run_local_hip(ctx, floors, plan)
        else:
            env = _hip_env(ctx, floors, plan)
            if dry:
                env["GEMM_DRY_RUN"] = "1"
            try:
                results = W.run_workload_pod(ctx.client, "hip-workload-validation.yaml", ctx.namespace, ctx.node_name,
                                             env, timeout=ctx.pod_timeout)["results"]
            except W.PodFailed as e:
                if not e.results:
                    raise ValidationError(f"HIP validation pod failed with no result: {e}"[:1000],
                                          [GateFailure("correctness", str(e)[:400])])
                failed, results = e, e.results
            except TimeoutError as e:
                raise ValidationError(f"HIP validation pod did not finish within {ctx.pod_timeout:.0f}s: {e}",
                                      [GateFailure("correctness", f"timeout after {ctx.pod_timeout:.0f}s")])
            except RuntimeError as e:          # the pod was deleted under the validator
                raise ValidationError(f"HIP validation pod: {e}", [GateFailure("correctness", str(e))])
        sweep_end = time.time()
        info = summarize_gemm(results)
        info["floors_tflops"] = floors
        info["plan"] = {"full": "all" if plan["full"] is None else plan["full"], "probe": plan["probe"],
                        "attribution": plan["attribution"], **({"busy_pods": busy[:16]} if busy else {})}
        if busy:
            info["busy"] = f"{len(busy)} GPU pod(s) on the node hold {len(plan['held_bdfs'])} GPU(s) " \
                           f"({plan['attribution']}): full sweep on {len(plan['full'])} free, probe on {len(plan['probe'])}"
        dist = disturbed_gpus(ctx, plan, gpus, sweep_end) if mode != "local" or ctx.client is not None \
            else {"devices": []}
        # a tenant that held its GPUs before the run is in the plan already (probe only): only the
        # sweep's own GPUs can be disturbed
        devs = frozenset(d for d in dist["devices"] if d != "all")
        if "all" in dist["devices"]:
            devs = frozenset(r.get("device") for r in info["gemm"])
        if devs:
            # recorded in hip-ready: throughput was not gated on these GPUs (correctness was)
            info["disturbed"] = {**dist, "devices": sorted(devs, key=str), "throughput_gated": False}
        bad = gate_gemm(info, floors, busy, min_relative=min_rel, min_efficiency=min_eff, disturbed=devs)
        if failed is not None:
            info["pod_failed"] = {"exit_code": failed.exit_code, "reason": failed.reason}
            if not bad and not devs:
                # the workload failed a gate this validator cannot see in its lines: never pass it
                bad = [GateFailure("correctness", f"workload exited {failed.exit_code} with no failing result line")]
        return info, bad

    info, bad = measure()
    if throughput_only(bad) and ctx.env.get("GEMM_REMEASURE", "1") != "0":
        # a throughput gate alone (every result correct): measure once more -- one more pod in pod
        # mode -- before failing the node, so a transient clock or power event costs one run
        log.warning("HIP validation: %s -- measuring once more", [str(b) for b in bad[:4]])
        first = bad
        info, bad = measure()
        info["remeasured"] = {"first_failure": [str(b) for b in first[:8]],
                              "first_kinds": sorted({b.kind for b in first})}
    if bad:
        _record_hip_failure(ctx, bad)
        raise ValidationError(f"HIP validation failed: {[str(b) for b in bad[:8]]}", bad)
    ctx.status.delete(S.HIP_LAST_FAILURE)
    ctx.status.create(S.HIP_READY, info)
    return info


def _record_hip_failure(ctx: Context, bad: List[GateFailure]) -> None:
    """The node-local record of a failed HIP validation: every gate's kind and text, and where each
    wrong result was computed (GPU, tile, XCD, CU) -- what the node metrics exporter publishes as
    validator_gemm_bad_tile, so a bad CU is visible without reading pod logs. A node-local file: the
    validator needs no write access to Nodes."""
    try:
        ctx.status.create(S.HIP_LAST_FAILURE, {
            "ts": round(time.time(), 3),
            "failures": [{"kind": b.kind, "text": b.text[:300], **({"where": b.where} if b.where else {})}
                         for b in bad[:16]]})
    except OSError as e:
        log.warning("hip-last-failure not written: %s", e)


# ---------------------------------------------------------------------------------------------
# device plugin
# ---------------------------------------------------------------------------------------------
def gpu_resources(node: Dict[str, Any], strategy: str) -> Dict[str, int]:
    cap = ((node.get("status") or {}).get("capacity") or {})
    out = {}
    for k, v in cap.items():
        if k == GPU_RESOURCE or (strategy == "mixed" and k.startswith(PARTITION_RESOURCE_PREFIX)):
            try:
                n = int(v)
            except (TypeError, ValueError):
                continue
            if n > 0:
                out[k] = n
    return out


def wait_gpu_resources(ctx: Context) -> Dict[str, int]:
    """Watch the Node (event-driven) until it advertises GPU resources, bounded."""
    if ctx.poll_mode:
        deadline = ctx.clock() + ctx.resource_timeout
        while True:
            r = gpu_resources(ctx.client.get("v1", "Node", ctx.node_name), ctx.partition_strategy)
            if r:
                return r
            if ctx.clock() >= deadline:
                raise ValidationError(f"no {GPU_RESOURCE} resources on node {ctx.node_name}")
            time.sleep(ctx.sleep_interval)
    done = threading.Event()
    found: Dict[str, int] = {}

    def on_event(ev):
        if o.name(ev.obj) != ctx.node_name:
            return
        r = gpu_resources(ev.obj, ctx.partition_strategy)
        if r:
            found.update(r)
            done.set()
    stop = ctx.client.watch("v1", "Node", on_event, field_selector=f"metadata.name={ctx.node_name}")
    try:
        deadline = ctx.clock() + ctx.resource_timeout
        while not done.is_set():
            r = gpu_resources(ctx.client.get("v1", "Node", ctx.node_name), ctx.partition_strategy)
            if r:
                return r
            remaining = deadline - ctx.clock()
            if remaining <= 0:
                raise ValidationError(f"no {GPU_RESOURCE} resources on node {ctx.node_name} after "
                                      f"{ctx.resource_timeout:.0f}s")
            done.wait(min(remaining, 2.0))
    finally:
        stop()
    return found


def validate_plugin(ctx: Context) -> Dict[str, Any]:
    res = wait_gpu_resources(ctx)
    info: Dict[str, Any] = {"resources": res, "devices": sum(res.values())}
    if ctx.with_workload:
        mode = ctx.env.get("HIP_VALIDATION_MODE", "pod")
        if mode in ("local", "skip"):
            info["workload"] = _local_workload(ctx, mode)
        else:
            # prefer a partition resource (like the reference prefers MIG), else one whole GPU
            name = next((k for k in sorted(res) if k.startswith(PARTITION_RESOURCE_PREFIX)), GPU_RESOURCE)
            try:
                out = W.run_workload_pod(ctx.client, "plugin-workload-validation.yaml", ctx.namespace, ctx.node_name,
                                         _validator_env(ctx), timeout=ctx.pod_timeout, gpu_limit={name: 1})
            except W.PodFailed as e:
                raise ValidationError(f"plugin workload failed on its {name}: {e}"[:1000],
                                      [GateFailure("correctness", f"plugin workload exit {e.exit_code}")])
            except (TimeoutError, RuntimeError) as e:
                raise ValidationError(f"plugin workload pod: {e}", [GateFailure("correctness", str(e))])
            info["workload"] = summarize_gemm(out["results"])
    ctx.status.create(S.PLUGIN_READY, info)
    return info


# ---------------------------------------------------------------------------------------------
# RCCL all-reduce over xGMI (new)
# ---------------------------------------------------------------------------------------------
def summarize_rccl(results: List[Dict[str, Any]]) -> Dict[str, Any]:
    sweep = [r for r in results if r.get("event") == "allreduce"]
    summ = next((r for r in results if r.get("event") == "summary"), {})
    fabric = next((r for r in results if r.get("event") == "fabric"), {})
    per_ranks = {r["ranks"]: r.get("peak_busbw_gbps") for r in results if r.get("event") == "ranks_summary"}
    debug = next((r for r in results if r.get("event") == "rccl-debug"), {})
    summaries = [r for r in results if r.get("event") == "summary"]
    mx = next((r for r in results if r.get("event") == "xgmi_matrix"), None)
    links = None
    if mx is not None:
        links = {k: mx[k] for k in ("gpus", "skipped", "isolated_gbps", "concurrent_gbps", "median_isolated_gbps",
                                    "median_concurrent_gbps", "gpu_ingress_gbps", "min_gpu_ingress_gbps", "min_ratio",
                                    "slow_links", "corrupt_links", "no_peer_access", "ok") if k in mx}
    return {"sweep": sweep, "ranks": summ.get("ranks"), "peak_busbw_gbps": summ.get("peak_busbw_gbps"),
            **({"links": links} if links is not None else {}),
            "link_bound_gbps": summ.get("link_bound_gbps"), "mesh_bound_gbps": summ.get("mesh_bound_gbps"),
            "busbw_by_ranks": per_ranks, "fabric": fabric, "skipped": bool(summ.get("skipped")),
            "algo_proto": debug.get("algo_proto"),
            "ok": bool(summaries) and all(s.get("ok") for s in summaries) and all(r.get("ok") for r in sweep)
            and fabric.get("ok", True) is not False}


def _run_rccl_local(ctx: Context, ngpu: int, floor: float) -> List[Dict[str, Any]]:
    from .workload_main import RCCL_MAX_BYTES, RCCL_STEP_TIMEOUT_S, run_rccl
    ranks = ctx.env.get("RCCL_RANKS") or ",".join(str(n) for n in (2, 4, 8) if n <= ngpu) or str(ngpu)
    # the same sweep (up to 8 GiB), link matrix, gates and hang guard as the fabric pod's
    return run_rccl(int(ctx.env.get("RCCL_MAX_BYTES", RCCL_MAX_BYTES)), ctx.env.get("RCCL_DTYPE", "bf16"), ranks=ranks,
                    min_busbw=floor or None,
                    step_timeout=float(ctx.env.get("RCCL_TIMEOUT_S", RCCL_STEP_TIMEOUT_S)),
                    min_link_relative=_gate_value(ctx, "RCCL_MIN_LINK_RELATIVE", LINK_MIN_RELATIVE),
                    mesh_fraction=None if floor else _gate_value(ctx, "RCCL_MIN_BUSBW_MESH_FRACTION", BUSBW_MESH_FRACTION))


def judge_rccl(ctx: Context, results: List[Dict[str, Any]]) -> tuple:
    """The fabric pod's lines -> (info, failures): the link matrix gate (each bad link named), the
    busBW floor of the largest rank count (busbw_gate), and whatever else the workload failed on (a
    wrong all-reduce result, a timeout) -- the binary gates the same way in the pod; this re-checks
    so an older workload image cannot pass a bad fabric."""
    info = summarize_rccl(results)
    gate = busbw_gate(ctx, info)
    info["min_busbw_gbps"] = gate["min_busbw_gbps"]
    info["busbw_floor"] = gate
    bad = gate_links(info.get("links") or {}, _gate_value(ctx, "RCCL_MIN_LINK_RELATIVE", LINK_MIN_RELATIVE))
    peak, floor = info.get("peak_busbw_gbps"), gate["min_busbw_gbps"]
    if not info["skipped"] and floor and peak is not None and peak < floor:
        bad.append(GateFailure("busbw", f"peak busBW {peak} GB/s below the {floor} GB/s floor ({gate['basis']})"))
    if not info["ok"] and not bad:
        why = next((r.get("reason") or r.get("error") for r in results
                    if r.get("event") in ("summary", "timeout", "async_error") and (r.get("reason") or r.get("error"))),
                   None)
        wrong = [r for r in info["sweep"] if not r.get("ok")]
        if wrong:
            why = f"{len(wrong)} all-reduce size(s) with wrong results, first at {wrong[0].get('bytes')} B on " \
                  f"{wrong[0].get('ranks')} ranks"
        bad.append(GateFailure("correctness", f"RCCL workload failed: {why or 'no passing summary'}"))
    if bad:
        info["ok"] = False
        info["error"] = "; ".join(str(b) for b in bad[:8])
    return info, bad


def run_topology_check(ctx: Context) -> Dict[str, Any]:
    """xGMI topology + hive check with no GPU work (``amd-rccl-validate --topology-only``), in
    this container: KFD io_links from sysfs, every GPU in one hive, 7 links per GPU on a full
    MI355X node."""
    from .workload_main import binary, _json_lines
    try:
        p = ctx.run([binary("amd-rccl-validate"), "--topology-only", "--sys-root", ctx.sys_root],
                    capture_output=True, text=True, timeout=60)
    except (OSError, FileNotFoundError, subprocess.TimeoutExpired) as e:
        raise ValidationError(f"topology check could not run: {e}")
    lines = _json_lines(p.stdout)
    fabric = next((x for x in lines if x.get("event") == "fabric"), None)
    if fabric is None:
        raise ValidationError(f"topology check printed no fabric line (exit {p.returncode})")
    return fabric


def _last_full_fabric(ctx: Context, node: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """The last full collective result: the node-local record, else the Node annotation an older
    validator wrote (read-only: the validator no longer writes Nodes)."""
    rec = ctx.status.read(S.FABRIC_LAST_FULL)
    if rec is not None:
        return rec
    raw = ((node.get("metadata") or {}).get("annotations") or {}).get(FABRIC_ANNOTATION)
    try:
        return json.loads(raw) if raw else None
    except ValueError:
        return None


def _record_full_fabric(ctx: Context, info: Dict[str, Any]) -> None:
    """Keep the last full collective result on the node (survives validator restarts), so a
    topology-only pass on a busy node can report when the fabric was last measured. A node-local
    file, not a Node annotation: the validator DaemonSet needs no write access to Nodes."""
    ctx.status.create(S.FABRIC_LAST_FULL, {
        "ts": round(time.time(), 3), "ranks": info.get("ranks"), "peak_busbw_gbps": info.get("peak_busbw_gbps"),
        "busbw_by_ranks": {str(k): v for k, v in (info.get("busbw_by_ranks") or {}).items()},
        **({"links": {k: (info.get("links") or {}).get(k) for k in ("min_gpu_ingress_gbps", "min_ratio",
                                                                      "median_isolated_gbps", "slow_links")}}
           if info.get("links") else {}),
        "ok": bool(info.get("ok"))})


def plan_rccl_pod(ctx: Context, node: Dict[str, Any], phys: List[Dict[str, Any]]) -> Dict[str, Any]:
    """How the fabric pod gets every physical GPU of the node.

    * whole GPUs advertised one-to-one (no time-slicing, no partitions): request them through
      the scheduler, ``amd.com/gpu: N`` -- the pod cannot start beside a GPU pod;
    * anything else (time-slicing replicas, CPX partitions, the mixed strategy): the advertised
      resource does not map to physical GPUs (8 replicas may all be GPU 0), so the pod requests
      none, runs privileged with every device visible (the hip pod's shape) and pins RCCL to the
      first agent of each physical GPU with HIP_VISIBLE_DEVICES. The caller runs it only when no
      GPU pod holds a device."""
    n = len(phys)
    alloc = ((node.get("status") or {}).get("allocatable") or {})
    try:
        whole = int(alloc.get(GPU_RESOURCE, 0) or 0)
    except (TypeError, ValueError):
        whole = 0
    partitions = any(k.startswith(PARTITION_RESOURCE_PREFIX) for k in alloc)
    agents_per_gpu = 1
    gpus = _gpus(ctx)
    if gpus and n:
        agents_per_gpu = max(1, len(gpus) // n)
    if whole == n and not partitions and agents_per_gpu == 1:
        return {"shape": "scheduled", "gpu_limit": {GPU_RESOURCE: n}, "env": {}, "privileged": False}
    visible = ",".join(str(g["index"]) for g in phys) if phys else ""
    env = {"AMD_VISIBLE_DEVICES": "all"}
    if visible and agents_per_gpu > 1:
        env["HIP_VISIBLE_DEVICES"] = visible
    return {"shape": "privileged-all", "gpu_limit": None, "env": env, "privileged": True,
            "reason": f"allocatable {GPU_RESOURCE}={whole} over {n} physical GPU(s)"
                      + (f", {agents_per_gpu} agents per GPU" if agents_per_gpu > 1 else "")
                      + (", partition resources" if partitions else "")}


def validate_rccl(ctx: Context) -> Dict[str, Any]:
    """The xGMI fabric proof over every PHYSICAL GPU of the node (KFD agents by PCI function;
    allocatable counts replicas or partitions). On a node where GPU pods already hold devices the
    collective cannot run (it would fight them, or never schedule): the topology/hive check runs
    instead and the last full result (Node annotation) is reported with its timestamp."""
    node = ctx.client.get("v1", "Node", ctx.node_name)
    phys = physical_gpus(ctx, node)
    ngpu = len(phys) or physical_gpu_count(ctx, node)
    if ngpu < 2:
        info = {"skipped": f"{ngpu} physical GPU(s): no fabric to validate", "ok": True}
        ctx.status.create(S.RCCL_READY, info)
        return info
    floor = busbw_floor(ctx)
    mode = ctx.env.get("HIP_VALIDATION_MODE", "pod")
    if mode == "local":
        info, bad = judge_rccl(ctx, _run_rccl_local(ctx, ngpu, floor))
        if bad and not info.get("skipped"):
            raise ValidationError(f"RCCL fabric validation failed: {[str(b) for b in bad[:8]]}", bad)
        if not info["skipped"]:
            _record_full_fabric(ctx, info)
        ctx.status.create(S.RCCL_READY, info)
        return info
    busy = gpu_pods_on_node(ctx)
    # RCCL_VALIDATION_MODE=dry-run (CPU rehearsals with a kubelet): the pod is planned, scheduled
    # and run, the collective is not; HIP_VALIDATION_MODE=skip without it: nothing is spawned
    dry = ctx.env.get("RCCL_VALIDATION_MODE", "") == "dry-run"
    if mode == "skip" and not dry:
        info = {"skipped": "HIP_VALIDATION_MODE=skip", "ok": True, "physical_gpus": ngpu,
                "planned": "topology-only" if busy else plan_rccl_pod(ctx, node, phys)["shape"]}
        ctx.status.create(S.RCCL_READY, info)
        return info
    if busy:
        return _topology_only(ctx, node, ngpu, busy,
                              f"{len(busy)} GPU pod(s) hold devices: the collective runs when the node is free")
    plan = plan_rccl_pod(ctx, node, phys)
    env = _validator_env(ctx)
    env.update({k: v for k, v in ctx.env.items() if k.startswith(("RCCL_", "NCCL_"))})
    env.update(plan["env"])
    # the rank sweep stops at the node's physical GPU count; the busBW floor (spec.validator.rccl.env
    # RCCL_MIN_BUSBW_GBPS, else a fraction of the mesh bound the pod's link matrix measures) gates the
    # largest rank count; the link matrix names any pair below RCCL_MIN_LINK_RELATIVE x the median
    env.setdefault("RCCL_RANKS", ",".join(str(n) for n in (2, 4, 8) if n <= ngpu) or str(ngpu))
    if ngpu not in [int(x) for x in env["RCCL_RANKS"].split(",") if x]:
        env["RCCL_RANKS"] += f",{ngpu}"
    if floor:
        env["RCCL_MIN_BUSBW_GBPS"] = f"{floor:g}"
    else:
        env["RCCL_MIN_BUSBW_MESH_FRACTION"] = f"{_gate_value(ctx, 'RCCL_MIN_BUSBW_MESH_FRACTION', BUSBW_MESH_FRACTION):g}"
    env["RCCL_MIN_LINK_RELATIVE"] = f"{_gate_value(ctx, 'RCCL_MIN_LINK_RELATIVE', LINK_MIN_RELATIVE):g}"
    if dry:
        env["RCCL_DRY_RUN"] = "1"

    def tenant_arrived(pod: Dict[str, Any]) -> Optional[str]:
        # the busy check above and the pod's start are not atomic: a tenant scheduled in between
        # leaves a scheduled-shape pod waiting for GPUs it will not get -- give the node back
        started = any(((cs.get("state") or {}).get("running") or (cs.get("state") or {}).get("terminated"))
                      for cs in ((pod.get("status") or {}).get("initContainerStatuses") or []))
        if started:
            return None
        now = gpu_pods_on_node(ctx)
        return f"GPU pod(s) {now[:8]} started before the fabric pod" if now else None
    try:
        out = W.run_workload_pod(ctx.client, "rccl-workload-validation.yaml", ctx.namespace, ctx.node_name,
                                 env, timeout=ctx.pod_timeout, gpu_limit=plan["gpu_limit"],
                                 privileged=plan["privileged"], abort_check=tenant_arrived)
    except W.WorkloadAborted as e:
        return _topology_only(ctx, node, ngpu, gpu_pods_on_node(ctx), f"fabric pod withdrawn: {e}")
    except W.PodFailed as e:
        now = gpu_pods_on_node(ctx)
        if e.admission or now:
            return _topology_only(ctx, node, ngpu, now, f"fabric pod not admitted beside GPU pod(s): {e}"[:400])
        if not e.results:
            raise ValidationError(f"RCCL fabric validation failed: {e}"[:1000], [GateFailure("correctness", str(e)[:400])])
        out = {"results": e.results}                 # the workload's own lines say what failed
    except (RuntimeError, TimeoutError) as e:
        raise ValidationError(f"RCCL fabric validation failed: {e}", [GateFailure("correctness", str(e)[:400])])
    info, bad = judge_rccl(ctx, out["results"])
    info.update(mode="full", physical_gpus=ngpu, pod_shape=plan["shape"])
    if plan.get("reason"):
        info["pod_shape_reason"] = plan["reason"]
    if plan["privileged"]:
        # the privileged-all pod holds no GPU resource: the device plugin kept advertising the GPUs,
        # so a tenant may have started during the collective -- its numbers (and any failure) then
        # measure the sharing, not the fabric
        after = gpu_pods_on_node(ctx)
        if after:
            return _topology_only(ctx, node, ngpu, after, "GPU pod(s) started during the collective: not measured",
                                  disturbed={k: info.get(k) for k in ("ok", "peak_busbw_gbps", "error") if k in info})
    if bad:
        raise ValidationError(f"RCCL fabric validation failed: {[str(b) for b in bad[:8]]}", bad)
    if not info["skipped"]:
        _record_full_fabric(ctx, info)
    ctx.status.create(S.RCCL_READY, info)
    return info


def _topology_only(ctx: Context, node: Dict[str, Any], ngpu: int, busy: List[str], reason: str,
                   **extra) -> Dict[str, Any]:
    """The fabric check without a collective (a node whose GPUs pods hold): topology and hive from
    sysfs, plus the last full result with its timestamp."""
    fabric = run_topology_check(ctx)
    if fabric.get("ok") is False:
        raise ValidationError(f"xGMI topology check failed: {fabric.get('reason', fabric)}")
    info = {"mode": "topology-only", "physical_gpus": ngpu, "fabric": fabric, "ok": True,
            "busy_pods": busy[:16], "last_full": _last_full_fabric(ctx, node), "reason": reason, **extra}
    ctx.status.create(S.RCCL_READY, info)
    return info


# ---------------------------------------------------------------------------------------------
# RDMA (reference: MOFED validation)
# ---------------------------------------------------------------------------------------------
def validate_rdma(ctx: Context) -> Dict[str, Any]:
    if ctx.env.get("RDMA_ENABLED", "false") != "true":
        return {"skipped": "RDMA disabled"}
    if ctx.client is not None and ctx.node_name:
        node = ctx.client.get("v1", "Node", ctx.node_name)
        if o.get_labels(node).get(MELLANOX_LABEL) != "true":
            return {"skipped": "no Mellanox NIC on node"}

    def check():
        if ctx.env.get("USE_HOST_MOFED") == "true":
            if not os.path.isdir(os.path.join(ctx.sys_root, "sys/module/mlx5_core")):
                raise ValidationError("mlx5_core not loaded on host")
        elif not os.path.exists(mounts.path("/run/mellanox/drivers/.driver-ready")):
            raise ValidationError("MOFED driver container not ready")
        return {"rdma": True}
    info = retry(ctx, "rdma", check)
    ctx.status.create(S.RDMA_READY, info)
    return info


# ---------------------------------------------------------------------------------------------
# sandbox components
# ---------------------------------------------------------------------------------------------
def workload_type(ctx: Context) -> str:
    wt = ctx.default_workload
    if ctx.client is not None and ctx.node_name:
        node = ctx.client.get("v1", "Node", ctx.node_name)
        v = o.get_labels(node).get(WORKLOAD_CONFIG_LABEL)
        if v in ("container", "vm-passthrough", "vm-mxgpu"):
            wt = v
    ctx.status.write_raw(S.WORKLOAD_TYPE, wt)
    return wt


def validate_vfio_pci(ctx: Context) -> Dict[str, Any]:
    if workload_type(ctx) != "vm-passthrough":
        return {"skipped": "not a passthrough node"}

    def check():
        fns = [f for f in devices.scan_pci(ctx.sys_root) if not f["is_virtfn"]]
        if not fns:
            raise ValidationError("no AMD GPU PCI functions found")
        bad = [f["bdf"] for f in fns if f["driver"] != "vfio-pci"]
        if bad:
            raise ValidationError(f"not bound to vfio-pci: {bad}")
        return {"devices": len(fns)}
    info = retry(ctx, "vfio-pci", check)
    ctx.status.create(S.VFIO_PCI_READY, info)
    return info


def validate_mxgpu_manager(ctx: Context) -> Dict[str, Any]:
    if workload_type(ctx) != "vm-mxgpu":
        return {"skipped": "not an MxGPU node"}
    host = os.path.isdir(os.path.join(ctx.host_root, "lib/modules")) and \
        ctx.env.get("MXGPU_HOST_DRIVER", "") == "true"

    def check():
        gim = os.path.join(ctx.sys_root, "sys/module/gim")
        if not os.path.isdir(gim):
            raise ValidationError("MxGPU host driver (gim) not loaded")
        return {"gim_version": (open(os.path.join(gim, "version")).read().strip()
                                if os.path.exists(os.path.join(gim, "version")) else "")}
    info = retry(ctx, "mxgpu-manager", check)
    ctx.status.create(S.HOST_MXGPU_MANAGER_READY if host else S.MXGPU_MANAGER_READY, info)
    return info


def validate_mxgpu_devices(ctx: Context) -> Dict[str, Any]:
    if workload_type(ctx) != "vm-mxgpu":
        return {"skipped": "not an MxGPU node"}

    def check():
        vfs = [f for f in devices.scan_pci(ctx.sys_root) if f["is_virtfn"]]
        pfs = [f for f in devices.scan_pci(ctx.sys_root) if not f["is_virtfn"] and f["sriov_numvfs"] > 0]
        if not vfs and not pfs:
            raise ValidationError("no MxGPU virtual functions created")
        return {"virtual_functions": max(len(vfs), sum(f["sriov_numvfs"] for f in pfs))}
    info = retry(ctx, "mxgpu-devices", check)
    ctx.status.create(S.MXGPU_DEVICES_READY, info)
    return info


def sandbox_ready_wait(ctx: Context) -> Dict[str, Any]:
    """Init container of the sandbox device plugin: wait for the workload type, then for the
    barrier its workload needs (reference: assets/state-sandbox-device-plugin/0500_daemonset.yaml:31-50)."""
    if not ctx.status.wait([S.WORKLOAD_TYPE], timeout=ctx.wait_timeout):
        raise ValidationError("workload-type barrier never appeared")
    wt = open(ctx.status.file(S.WORKLOAD_TYPE)).read().strip()
    need = {"vm-passthrough": [S.VFIO_PCI_READY], "vm-mxgpu": [S.MXGPU_DEVICES_READY]}.get(wt, [])
    if need and not ctx.status.wait(need, timeout=ctx.wait_timeout):
        raise ValidationError(f"timed out waiting for {need}")
    return {"workload_type": wt}


COMPONENTS: Dict[str, Callable[[Context], Dict[str, Any]]] = {
    "driver": validate_driver,
    "toolkit": validate_toolkit,
    "hip": validate_hip,
    "cuda": validate_hip,           # reference component name, kept for migration
    "plugin": validate_plugin,
    "rccl": validate_rccl,
    "rdma": validate_rdma,
    "mofed": validate_rdma,         # reference component name
    "vfio-pci": validate_vfio_pci,
    "mxgpu-manager": validate_mxgpu_manager,
    "vgpu-manager": validate_mxgpu_manager,
    "mxgpu-devices": validate_mxgpu_devices,
    "vgpu-devices": validate_mxgpu_devices,
    "sandbox-ready-wait": sandbox_ready_wait,
}
