"""``amd-validator-workload``: what runs inside the spawned validation pods.

    amd-validator-workload hip  [--gemm-shapes 8192,...] [--gemm-dtype bf16|fp8|both] [--counters]
                                [--scaling 1,2,4,8] [--min-tflops X] [--min-tflops-fp8 Y]
                                [--min-relative R] [--min-efficiency E]
                                [--devices I,J,..|none] [--probe-devices K,L,..]
    amd-validator-workload rccl [--ranks 2,4,8] [--processes N] [--max-bytes N] [--dtype float|bf16]
                                [--min-busbw GBPS] [--timeout-s T]

Tenant safety (hip): ``--devices`` are the HIP indices of the GPUs no pod holds -- the full stabilised
sweep runs there only, with HIP_VISIBLE_DEVICES set to them, so the process never opens a context on
a tenant's GPU; ``--probe-devices`` are the held GPUs -- one 1024^3 bf16 GEMM each (no stabilisation,
no sweep, no counters), a correctness probe whose out-of-memory result is reported, not failed.

Runs the native workload binaries (``amd-hip-smoke``, ``amd-gemm-validate``,
``amd-rccl-validate``), optionally collects rocprofv3 counters for one GEMM dispatch
per GEMM dtype (MFMA ops against 2·M·N·K/512, busy cycles, LDS bank conflicts, L2 hit/miss) and
prints JSON result lines. The
same lines go to ``/dev/termination-log`` so the validator reads them back from the pod
status. Exit status is non-zero if any check failed.
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time
from typing import Callable, Dict, List, Optional

BIN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native", "bin")
# One rocprofv3 pass per GEMM dtype (8 SQ + 4 TCC slots per pass on gfx950): the MFMA op counter(s)
# of that dtype, busy cycles, LDS bank conflicts / activity and L2 hits / misses. The f8f6f4
# instruction the fp8 kernel issues is counted under F8 or F6F4 depending on the firmware, so the
# fp8 pass collects both and sums them.
PMC_PASSES = {
    "bf16": {"kernel": "gemm_", "mops": ["SQ_INSTS_VALU_MFMA_MOPS_BF16"]},
    "fp8": {"kernel": "gemm_", "mops": ["SQ_INSTS_VALU_MFMA_MOPS_F8", "SQ_INSTS_VALU_MFMA_MOPS_F6F4"]},
}
PMC_COMMON = ["SQ_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "TCC_HIT_sum", "TCC_MISS_sum"]
PMC_COUNTERS = PMC_PASSES["bf16"]["mops"] + PMC_COMMON      # the bf16 pass (kept for callers)


def rocprofv3_path() -> Optional[str]:
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    return prof if os.path.exists(prof) else None


def binary(name: str) -> str:
    """A workload binary: ``$AMDGO_BIN_DIR`` first (an image that ships them elsewhere; the CPU
    rehearsals' scripted stand-ins), then the in-tree build, then PATH."""
    for d in (os.environ.get("AMDGO_BIN_DIR", ""), BIN_DIR):
        p = os.path.join(d, name) if d else ""
        if p and os.path.exists(p):
            return p
    found = shutil.which(name)
    if found:
        return found
    raise FileNotFoundError(f"{name} not found in {BIN_DIR} or PATH")


def _json_lines(text: str) -> List[Dict]:
    out = []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                out.append(json.loads(line))
            except ValueError:
                pass
    return out


def stream_run(cmd: List[str], capture_output: bool = True, text: bool = True, timeout: Optional[float] = None,
               env: Optional[Dict[str, str]] = None) -> subprocess.CompletedProcess:
    """subprocess.run for a workload binary whose output ends with ``{"event":"done","ok":..}``
    (amd-gemm-validate): returns as soon as that line arrives, with the status it states, and leaves
    the process's exit -- the HIP runtime's and the kernel driver's teardown of its GPU state, about
    0.1 s after the last line on MI355X (tools/hipinit_probe.sh) -- to a reaper thread, so the HIP
    barrier does not wait for it. Without the line (a crash, another binary) it is subprocess.run."""
    import queue
    import threading

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    lines: "queue.Queue[Optional[str]]" = queue.Queue()
    err: List[str] = []

    def pump_out():
        for ln in p.stdout:
            lines.put(ln)
        lines.put(None)

    def pump_err():
        for ln in p.stderr:
            err.append(ln)

    pumps = [threading.Thread(target=f, daemon=True) for f in (pump_out, pump_err)]
    for t in pumps:
        t.start()
    deadline = None if timeout is None else time.monotonic() + timeout
    out: List[str] = []
    while True:
        try:
            ln = lines.get(timeout=None if deadline is None else max(0.0, deadline - time.monotonic()))
        except queue.Empty:
            p.kill()
            p.wait()
            raise subprocess.TimeoutExpired(cmd, timeout, "".join(out), "".join(err))
        if ln is None:
            break
        out.append(ln)
        if '"done"' in ln:
            try:
                d = json.loads(ln)
            except ValueError:
                continue
            if isinstance(d, dict) and d.get("event") == "done":
                threading.Thread(target=p.wait, daemon=True).start()      # reap the exiting child
                return subprocess.CompletedProcess(cmd, 0 if d.get("ok") else 1, "".join(out), "".join(err))
    rc = p.wait(timeout=None if deadline is None else max(1.0, deadline - time.monotonic()))
    pumps[1].join(5.0)                           # the rest of stderr (its pipe closed at exit)
    return subprocess.CompletedProcess(cmd, rc, "".join(out), "".join(err))


def run_json(cmd: List[str], run: Callable = subprocess.run, timeout: float = 600,
             visible: Optional[List[int]] = None) -> (int, List[Dict]):
    """Run a workload binary and parse its JSON lines. ``visible``: HIP_VISIBLE_DEVICES for the
    child; the binary then counts devices from 0 and its ``device`` fields are mapped back to the
    node's HIP indices (``visible_index`` keeps the child's own)."""
    kw = {}
    if visible is not None:
        kw["env"] = dict(os.environ, HIP_VISIBLE_DEVICES=",".join(str(d) for d in visible))
    p = run(cmd, capture_output=True, text=True, timeout=timeout, **kw)
    if p.stderr:
        sys.stderr.write(p.stderr[-4000:])
    lines = [x for x in _json_lines(p.stdout) if x.get("event") != "done"]
    if visible is not None:
        for x in lines:
            if isinstance(x.get("device"), int) and 0 <= x["device"] < len(visible):
                x["visible_index"] = x["device"]
                x["device"] = visible[x["device"]]
            if isinstance(x.get("slow_devices"), list):
                x["slow_devices"] = [visible[d] if isinstance(d, int) and 0 <= d < len(visible) else d
                                     for d in x["slow_devices"]]
    return p.returncode, lines


def _shape_mnk(shape: str):
    parts = [int(x) for x in shape.lower().split("x")]
    return (parts[0],) * 3 if len(parts) == 1 else tuple(parts[:3])


def timed_gemm_kernel(name: str) -> bool:
    """Whether a profiled kernel is the probe's timed GEMM dispatch: any kernel of the GEMM family the
    dispatch picked (256x256 asm pipeline, gemm_mfma_small / _sk, generic) in its timed instantiation --
    not the placement-recording one of the checked dispatch (Rec 1, gemm_tile_common.h), not the ABFT,
    reference or fill kernels. The template argument reads ``3RecE0E`` mangled, ``Rec)0`` demangled."""
    n = name or ""
    return "gemm_" in n and ("3RecE0E" in n or "Rec)0" in n) and "ref_rows" not in n


def _short_kernel(name: str) -> str:
    for fam in ("gemm_mfma_small_sk", "gemm_mfma_small", "gemm_bf16_256x256_w4ap", "gemm_bf16_256x256_w4sp",
                "gemm_bf16_256x256_w4s", "gemm_fp8_256x256_q16ap", "gemm_fp8_256x256_q16p", "gemm_fp8_256x256_q16",
                "gemm_fp8_256x256_w4sp", "gemm_bf16_generic", "gemm_fp8_generic"):
        if fam in name:
            return fam
    return name[:60]


def collect_counters(shape: str, run: Callable = subprocess.run, dtype: str = "bf16",
                     visible: Optional[List[int]] = None) -> List[Dict]:
    """One profiled GEMM dispatch of ``dtype`` under rocprofv3 (counters only: no sys/runtime
    traces, which this pool refuses beside --pmc). Adds the expected MFMA op count
    (2·M·N·K / 512) and whether the measured one matches it."""
    spec = PMC_PASSES[dtype]
    prof = rocprofv3_path()
    if prof is None:
        return [{"event": "counters", "dtype": dtype, "skipped": "rocprofv3 not available"}]
    out = tempfile.mkdtemp(prefix="amdgo-pmc-")
    try:
        cmd = [prof, "--pmc", *spec["mops"], *PMC_COMMON, "--output-format", "csv", "-d", out, "--",
               binary("amd-gemm-validate"), "--shapes", shape, "--iters", "1", "--warmup", "0",
               "--no-stabilise", "--devices", "0", "--check-rows", "1", "--dtype", dtype,
               # the profiler initialises the GPU in the process it starts: no worker processes
               "--launch", "threads"]
        kw = {"env": dict(os.environ, HIP_VISIBLE_DEVICES=",".join(map(str, visible)))} if visible else {}
        p = run(cmd, capture_output=True, text=True, timeout=300, **kw)
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if p.returncode != 0 or not files:
            return [{"event": "counters", "dtype": dtype, "ok": False,
                     "error": f"rocprofv3 exit {p.returncode}: {(p.stderr or '')[-300:]}"}]
        agg: Dict[str, float] = {}
        kernels = set()
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if not timed_gemm_kernel(row.get("Kernel_Name", "")):
                    continue
                kernels.add(_short_kernel(row.get("Kernel_Name", "")))
                agg[row["Counter_Name"]] = agg.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        if not agg:
            return [{"event": "counters", "dtype": dtype, "shape": shape, "ok": False,
                     "error": "no timed GEMM dispatch in the counter records"}]
        m, n, k = _shape_mnk(shape)
        mops = sum(agg.get(c, 0.0) for c in spec["mops"])
        want = 2.0 * m * n * k / 512
        res = {"event": "counters", "dtype": dtype, "kernel": ",".join(sorted(kernels)), "shape": shape, **agg,
               "mfma_mops": mops, "mfma_mops_expected": want, "mfma_mops_match": abs(mops - want) <= 1e-6 * want,
               "lds_conflict_free": agg.get("SQ_LDS_BANK_CONFLICT", 1.0) == 0.0}
        res["ok"] = res["mfma_mops_match"]
        return [res]
    finally:
        shutil.rmtree(out, ignore_errors=True)


PROBE_SHAPE = "1024"      # the correctness probe on GPUs a tenant holds: 6 MiB of operands, ~1 ms


def _parse_devices(spec: Optional[str]) -> Optional[List[int]]:
    """"" / None -> None (every visible GPU); "none" -> [] (no GPU); "0,3" -> [0, 3]."""
    if spec is None or spec.strip() == "":
        return None
    if spec.strip() == "none":
        return []
    return [int(x) for x in spec.split(",") if x.strip()]


def run_hip(shapes: List[str], counters: bool = False, iters: int = 50,
            run: Callable = stream_run, dtype: str = "bf16", scaling: Optional[str] = None,
            min_tflops: float = 0.0, min_tflops_fp8: float = 0.0, devices: Optional[List[int]] = None,
            probe_devices: Optional[List[int]] = None, min_relative: float = 0.0,
            min_efficiency: float = 0.0, dry_run: bool = False) -> List[Dict]:
    """hip-smoke, then the MFMA GEMM probe in ``dtype`` (bf16, fp8 e4m3fn on the double-rate
    16x16x128 matrix-core path, or both) -- clock-stabilised like bench.py, optionally swept over
    ``scaling`` GPU counts ("1,2,4,8") and gated on per-GPU floors, on the node median
    (``min_relative``) and on scaling efficiency -- then optionally one counter-collection pass per
    dtype. ``devices`` (None = all) bounds that full run; ``probe_devices`` get the correctness
    probe only (module docstring)."""
    results: List[Dict] = [{"event": "plan", "devices": "all" if devices is None else devices,
                            "probe_devices": probe_devices or []}]
    if dry_run:
        # GEMM_DRY_RUN=1 (CPU rehearsals of node bring-up): what this pod was given, no GPU work
        results[0].update(skipped="dry-run", hip_visible_devices=os.environ.get("HIP_VISIBLE_DEVICES"),
                          amd_visible_devices=os.environ.get("AMD_VISIBLE_DEVICES"))
        return results
    full = devices is None or len(devices) > 0
    # hip-smoke runs inside the first GEMM process (--smoke: one HIP runtime start, not two)
    if full:
        cmd = [binary("amd-gemm-validate"), "--smoke", "--shapes", ",".join(shapes), "--iters", str(iters)]
        if dtype != "bf16":
            cmd += ["--dtype", dtype]
        if scaling:
            cmd += ["--scaling", scaling]
        if min_tflops:
            cmd += ["--min-tflops", f"{min_tflops:g}"]
        if min_tflops_fp8:
            cmd += ["--min-tflops-fp8", f"{min_tflops_fp8:g}"]
        if min_relative:
            cmd += ["--min-relative", f"{min_relative:g}"]
        if min_efficiency:
            cmd += ["--min-efficiency", f"{min_efficiency:g}"]
        rc, r = run_json(cmd, run, timeout=1200, visible=devices)
        results += r or [{"event": "hip-smoke", "ok": False, "rc": rc}]
        if rc != 0 and not any(x.get("event") == "gemm" for x in r):
            results.append({"event": "gemm", "ok": False, "rc": rc})
    if probe_devices:
        cmd = [binary("amd-gemm-validate"), "--shapes", PROBE_SHAPE, "--dtype", "bf16", "--iters", "3",
               "--warmup", "1", "--no-stabilise", "--check-rows", "16"] + ([] if full else ["--smoke"])
        rc, r = run_json(cmd, run, timeout=120, visible=probe_devices)
        for x in r:
            if x.get("event") != "hip-smoke":
                x["probe"] = True
        results += [x for x in r if x.get("event") in ("gemm", "start", "hip-smoke") or "error" in x]
        if rc != 0 and not any(x.get("event") == "gemm" for x in r):
            results.append({"event": "gemm", "probe": True, "ok": False, "rc": rc})
    results += gpu_tflops_lines(results)
    if counters and full:
        # every shape of the plan, each dtype: the counters follow whichever kernel the dispatch picks
        for d in (["bf16", "fp8"] if dtype == "both" else [dtype]):
            for shape in shapes:
                # the profiler writes its counters from the child's exit path: wait for it (subprocess.run)
                results += collect_counters(shape, subprocess.run if run is stream_run else run, dtype=d,
                                            visible=devices[:1] if devices else None)
    return results


def gpu_tflops_lines(results: List[Dict]) -> List[Dict]:
    """One compact ``gpu_tflops`` line per (dtype, shape): every GPU's best TFLOP/s over the sets it
    ran in (node HIP indices). A summary line: it survives the 4 KiB termination message that the
    per-GPU lines of a 2-dtype x 1/2/4/8 sweep (30 lines) do not, so the validator can export one
    series per GPU (validator_gemm_gpu_tflops)."""
    best: Dict[tuple, Dict[str, float]] = {}
    for r in results:
        if r.get("event") != "gemm" or r.get("probe") or not r.get("ok") or not r.get("tflops"):
            continue
        d = best.setdefault((r.get("dtype", "bf16"), r.get("m"), r.get("n"), r.get("k")), {})
        dev = str(r.get("device"))
        d[dev] = max(d.get(dev, 0.0), float(r["tflops"]))
    return [{"event": "gpu_tflops", "dtype": dt, "m": m, "n": n, "k": k, "tflops": dict(sorted(v.items()))}
            for (dt, m, n, k), v in sorted(best.items(), key=lambda kv: str(kv[0]))]


def hip_ok(results: List[Dict]) -> bool:
    """The pod's exit status: every check, floor, efficiency and uniformity gate of the full run;
    on probed (tenant-held) GPUs only correctness, an out-of-memory result being no failure."""
    for x in results:
        ev = x.get("event")
        if ev == "gemm" and x.get("probe"):
            if not x.get("ok", True) and not x.get("oom"):
                return False
        elif ev in ("gemm", "hip-smoke", "uniformity") and not x.get("ok", True):
            return False
        elif ev == "aggregate" and x.get("ok") is False:
            return False
    return True


# NCCL's numeric algorithm / protocol ids in its TUNING lines (NCCL_ALGO_*, NCCL_PROTO_*)
_ALGOS = {"0": "Tree", "1": "Ring", "2": "CollNetDirect", "3": "CollNetChain", "4": "NVLS", "5": "NVLSTree"}
_PROTOS = {"0": "LL", "1": "LL128", "2": "Simple"}
_RCCL_KEEP = re.compile(r"Algo|algorithm|proto|Channel \d+/\d+|nRanks|Init COMPLETE|Connected all|xGMI|P2P|rings?\b",
                        re.I)


def parse_rccl_debug(text: str, keep: int = 40) -> Dict:
    """Summarise an RCCL ``NCCL_DEBUG=INFO`` log (subsystems INIT,TUNING,GRAPH): the algorithm and
    protocol picked per message size, channel count, transport lines and ranks."""
    algo_proto: Dict[str, int] = {}
    channels = set()
    lines: List[str] = []
    for line in text.splitlines():
        if "NCCL INFO" not in line and "RCCL" not in line:
            continue
        m = re.search(r"Algo\s+(\w+)\s+proto\s+(\w+)", line, re.I) or \
            re.search(r"algorithm\s+(\w+).*?protocol\s+(\w+)", line, re.I)
        if m:
            key = f"{_ALGOS.get(m.group(1), m.group(1))}/{_PROTOS.get(m.group(2), m.group(2))}"
            algo_proto[key] = algo_proto.get(key, 0) + 1
        c = re.search(r"Channel (\d+)/(\d+)", line)
        if c:
            channels.add(int(c.group(2)))
        if _RCCL_KEEP.search(line) and len(lines) < keep:
            lines.append(line.split("NCCL INFO", 1)[-1].strip()[:200])
    return {"event": "rccl-debug", "algo_proto": algo_proto, "channels": max(channels) if channels else None,
            "lines": lines}


def _rccl_env(log_path: str) -> Dict[str, str]:
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,TUNING,GRAPH", NCCL_DEBUG_FILE=log_path)
    return env


RCCL_MAX_BYTES = 8 << 30      # the sweep's largest message (8 B ... 8 GiB), pod and local mode
RCCL_STEP_TIMEOUT_S = 120.0   # the binary's hang guard: bound on one blocking step (init, one size, one check)


def run_rccl(max_bytes: int, dtype: str, run: Callable = subprocess.run, ranks: Optional[str] = None,
             min_busbw: Optional[float] = None, processes: int = 0, min_bytes: int = 1024,
             timeout: float = 1200, step_timeout: float = RCCL_STEP_TIMEOUT_S,
             min_link_relative: Optional[float] = None, mesh_fraction: Optional[float] = None) -> List[Dict]:
    """The xGMI fabric proof: topology + fabric check, then a rank-count sweep in one process
    (``ranks`` "2,4,8") or, with ``processes`` N, one process per GPU joined through
    ncclCommInitRank. RCCL's INFO log is captured and summarised (algorithm/protocol per size).
    ``step_timeout`` is the binary's own watchdog (--timeout-s, a structured timeout line naming the
    phase); ``timeout`` bounds the whole run from here, for a binary that cannot even report."""
    if os.environ.get("RCCL_DRY_RUN") == "1":
        return _rccl_dry_run(ranks)
    base = ["--max-bytes", str(max_bytes), "--dtype", dtype, "--min-bytes", str(min_bytes)]
    if min_busbw:
        base += ["--min-busbw", str(min_busbw)]
    if min_link_relative is not None:
        base += ["--min-link-relative", f"{min_link_relative:g}"]
    if mesh_fraction:
        base += ["--min-busbw-mesh-fraction", f"{mesh_fraction:g}"]
    if step_timeout:
        base += ["--timeout-s", f"{step_timeout:g}"]
    tmp = tempfile.mkdtemp(prefix="amdgo-rccl-")
    try:
        if processes > 0:
            results = _run_rccl_mp(processes, base, tmp, timeout)
        else:
            cmd = [binary("amd-rccl-validate")] + base + (["--ranks", ranks] if ranks else [])
            try:
                p = run(cmd, capture_output=True, text=True, timeout=timeout,
                        env=_rccl_env(os.path.join(tmp, "rccl.%p.log")))
                out, err, rc = p.stdout, p.stderr, p.returncode
            except subprocess.TimeoutExpired as e:       # run() killed it
                out, err, rc = _text(e.stdout), _text(e.stderr), None
            if err:
                sys.stderr.write(err[-4000:])
            results = _json_lines(out)
            if rc is None and not _has_timeout(results):
                results.append(_launcher_timeout(results, timeout, rank=0))
            if rc != 0 and not any(x.get("event") == "summary" for x in results):
                results.append({"event": "summary", "ok": False, "rc": rc,
                                **({"reason": _timeout_reason(results)} if _has_timeout(results) else {})})
        text = ""
        for f in sorted(glob.glob(os.path.join(tmp, "rccl.*.log"))):
            with open(f, errors="replace") as fh:
                text += fh.read()
        results.append(parse_rccl_debug(text))
        return results
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _rccl_dry_run(ranks: Optional[str]) -> List[Dict]:
    """RCCL_DRY_RUN=1 (CPU rehearsals of node bring-up, HIP_VALIDATION_MODE=skip): the pod is
    planned, scheduled and run, the topology/hive check reads the (fake) sysfs, and no collective
    runs. What the pod was given (visible devices, rank list) is reported for the test to check."""
    cmd = [binary("amd-rccl-validate"), "--topology-only", "--sys-root", os.environ.get("AMD_SYSFS_ROOT", "/")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
    results = [x for x in _json_lines(p.stdout) if x.get("event") in ("fabric", "topology")]
    fabric = next((x for x in results if x.get("event") == "fabric"), {"ok": False, "reason": "no fabric line"})
    rl = [int(x) for x in (ranks or "").split(",") if x.strip()]
    results.append({"event": "summary", "ok": bool(fabric.get("ok")), "skipped": "dry-run",
                    "ranks": max(rl) if rl else None, "ranks_planned": rl,
                    "amd_visible_devices": os.environ.get("AMD_VISIBLE_DEVICES"),
                    "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES")})
    return results


def _text(b) -> str:
    return b.decode(errors="replace") if isinstance(b, bytes) else (b or "")


def _has_timeout(lines: List[Dict]) -> bool:
    return any(x.get("event") in ("timeout", "async_error") for x in lines)


def _timeout_reason(lines: List[Dict]) -> str:
    t = next(x for x in lines if x.get("event") in ("timeout", "async_error"))
    what = "timed out" if t["event"] == "timeout" else f"async error {t.get('error', '')}"
    return f"rank {t.get('rank')} of {t.get('ranks')} {what} in {t.get('phase')} ({t.get('bytes', 0)} B)"


def _launcher_timeout(lines: List[Dict], timeout: float, rank: int) -> Dict:
    """A rank the launcher had to kill: the binary's watchdog never reported (stuck in the driver,
    or an older binary). The phase is inferred from its last line."""
    last = next((x for x in reversed(lines) if x.get("event") in ("allreduce", "start")), None)
    phase = "init" if last is None or last.get("event") == "start" else "allreduce"
    return {"event": "timeout", "phase": phase, "rank": rank, "ranks": (last or {}).get("ranks"),
            "bytes": (last or {}).get("bytes", 0), "timeout_s": timeout, "killed_by": "launcher", "ok": False}


def _run_rccl_mp(n: int, base: List[str], tmp: str, timeout: float) -> List[Dict]:
    """Start N ranks of amd-rccl-validate (this process never touches the GPU); rank 0 publishes the
    ncclUniqueId through a file, the others join. Rank 0's lines plus every rank's summary, and a
    structured timeout line for every rank that timed out (its own watchdog's, or the launcher's
    when the rank had to be killed) -- the failure names the collective phase and the ranks."""
    id_file = os.path.join(tmp, "nccl.id")
    procs = []
    for r in range(n):
        cmd = [binary("amd-rccl-validate")] + base + ["--mp-rank", str(r), "--mp-nranks", str(n),
                                                      "--mp-id-file", id_file, "--device", str(r)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      env=_rccl_env(os.path.join(tmp, f"rccl.{r}.log"))))
    outs = []
    deadline = time.monotonic() + timeout
    killed = set()
    for r, p in enumerate(procs):
        try:
            out, err = p.communicate(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            for k, q in enumerate(procs):
                if q.poll() is None:
                    q.kill()
                    killed.add(k)
            out, err = p.communicate()
        if err:
            sys.stderr.write(err[-2000:])
        lines = _json_lines(out)
        if r in killed and not _has_timeout(lines):
            lines.append(dict(_launcher_timeout(lines, timeout, r), ranks=n))
        outs.append((p.returncode, lines))
    results = list(outs[0][1])
    for r, (rc, lines) in enumerate(outs[1:], start=1):
        results += [x for x in lines if x.get("event") in ("summary", "start", "timeout", "async_error") or "error" in x]
    timeouts = [x for _, lines in outs for x in lines if x.get("event") in ("timeout", "async_error")]
    for r, (rc, lines) in enumerate(outs):
        if rc != 0 and not any(x.get("event") == "summary" for x in lines):
            results.append({"event": "summary", "rank": r, "ranks": n, "ok": False, "rc": rc,
                            **({"reason": _timeout_reason(timeouts)} if timeouts else {})})
    return results


TERMINATION_LOG_BYTES = 4000       # kubelet keeps at most 4 KiB of a termination message
_SUMMARY_EVENTS = ("plan", "aggregate", "uniformity", "summary", "timeout", "async_error", "hip-smoke", "counters",
                   "scaling", "fabric", "ranks_summary", "rccl-debug", "gpu_tflops", "xgmi_matrix", "xgmi_link")


def termination_message(results: List[Dict], limit: int = TERMINATION_LOG_BYTES) -> str:
    """The lines the validator reads back from the pod status, whole lines only, most important
    first: summaries (aggregates carry the slowest GPU), then failing per-GPU lines, then passing
    ones -- so a truncated message never hides a failure."""
    def line(r):
        if r.get("event") == "rccl-debug":
            r = {k: v for k, v in r.items() if k != "lines"}
        return json.dumps(r, separators=(",", ":"))
    ordered = [r for r in results if r.get("event") in _SUMMARY_EVENTS]
    ordered += [r for r in results if r.get("event") not in _SUMMARY_EVENTS and r.get("ok") is False]
    ordered += [r for r in results if r.get("event") not in _SUMMARY_EVENTS and r.get("ok") is not False]
    out, size = [], 0
    for r in ordered:
        ln = line(r)
        if size + len(ln) + 1 > limit:
            continue
        out.append(ln)
        size += len(ln) + 1
    return "\n".join(out)


def emit(results: List[Dict], termination_log: Optional[str] = None) -> None:
    if termination_log is None:
        from ..utils import mounts
        termination_log = mounts.path("/dev/termination-log")
    text = "\n".join(json.dumps(r, separators=(",", ":")) for r in results)
    print(text, flush=True)
    if termination_log and os.path.isdir(os.path.dirname(termination_log)):
        try:
            with open(termination_log, "w") as f:
                f.write(termination_message(results))
        except OSError:
            pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="amd-validator-workload")
    sub = ap.add_subparsers(dest="what", required=True)
    h = sub.add_parser("hip")
    h.add_argument("--gemm-shapes", default=os.environ.get("GEMM_SHAPES", "8192"))
    h.add_argument("--iters", type=int, default=int(os.environ.get("GEMM_ITERS", "50")))
    h.add_argument("--counters", action="store_true")
    h.add_argument("--gemm-dtype", choices=["bf16", "fp8", "both"], default=os.environ.get("GEMM_DTYPE", "bf16"))
    h.add_argument("--scaling", default=os.environ.get("GEMM_SCALING", ""),
                   help="GPU counts for the scaling sweep, e.g. 1,2,4,8 (counts above the visible GPUs are skipped)")
    h.add_argument("--min-tflops", type=float, default=float(os.environ.get("GEMM_MIN_TFLOPS_BF16", "0") or 0),
                   help="per-GPU bf16 floor (the validator passes its model default or spec.validator.hip.env)")
    h.add_argument("--min-tflops-fp8", type=float, default=float(os.environ.get("GEMM_MIN_TFLOPS_FP8", "0") or 0))
    h.add_argument("--min-relative", type=float, default=float(os.environ.get("GEMM_MIN_RELATIVE", "0") or 0),
                   help="fail a GPU below this fraction of the node median (same dtype and shape)")
    h.add_argument("--min-efficiency", type=float, default=float(os.environ.get("GEMM_MIN_EFFICIENCY", "0") or 0),
                   help="fail a scaling step N > 1 below this efficiency")
    h.add_argument("--devices", default=os.environ.get("GEMM_DEVICES", ""),
                   help="HIP indices of the GPUs for the full run ('' = all, 'none' = no full run)")
    h.add_argument("--probe-devices", default=os.environ.get("GEMM_PROBE_DEVICES", ""),
                   help="HIP indices of tenant-held GPUs: correctness probe only")
    r = sub.add_parser("rccl")
    r.add_argument("--max-bytes", type=int, default=int(os.environ.get("RCCL_MAX_BYTES", RCCL_MAX_BYTES)))
    r.add_argument("--timeout-s", type=float, default=float(os.environ.get("RCCL_TIMEOUT_S", RCCL_STEP_TIMEOUT_S)),
                   help="the binary's watchdog: bound on one blocking step (0 = none)")
    r.add_argument("--dtype", default=os.environ.get("RCCL_DTYPE", "bf16"),
                   help="all-reduce element type (bf16, the validator's local mode default too)")
    r.add_argument("--ranks", default=os.environ.get("RCCL_RANKS", "2,4,8"))
    r.add_argument("--processes", type=int, default=int(os.environ.get("RCCL_PROCESSES", "0")))
    r.add_argument("--min-busbw", type=float, default=float(os.environ.get("RCCL_MIN_BUSBW_GBPS", "0") or 0))
    r.add_argument("--min-link-relative", type=float,
                   default=float(os.environ.get("RCCL_MIN_LINK_RELATIVE", "0.8") or 0),
                   help="fail an xGMI link (GPU pair) below this fraction of the node median")
    r.add_argument("--min-busbw-mesh-fraction", type=float,
                   default=float(os.environ.get("RCCL_MIN_BUSBW_MESH_FRACTION", "0") or 0),
                   help="without --min-busbw: the busBW floor as a fraction of the measured mesh bound")
    a = ap.parse_args(argv)
    if a.what == "hip":
        results = run_hip(a.gemm_shapes.split(","), counters=a.counters, iters=a.iters, dtype=a.gemm_dtype,
                          scaling=a.scaling or None, min_tflops=a.min_tflops, min_tflops_fp8=a.min_tflops_fp8,
                          devices=_parse_devices(a.devices), probe_devices=_parse_devices(a.probe_devices),
                          min_relative=a.min_relative, min_efficiency=a.min_efficiency,
                          dry_run=os.environ.get("GEMM_DRY_RUN") == "1")
        ok = hip_ok(results)
    else:
        results = run_rccl(a.max_bytes, a.dtype, ranks=a.ranks, min_busbw=a.min_busbw, processes=a.processes,
                           min_link_relative=a.min_link_relative, mesh_fraction=a.min_busbw_mesh_fraction,
                           step_timeout=a.timeout_s)
        ok = all(x.get("ok", False) for x in results if x.get("event") == "summary")
    emit(results)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
