"""``amd-validator-workload``: what runs inside the spawned validation pods.

    amd-validator-workload hip  [--gemm-shapes 8192,...] [--gemm-dtype bf16|fp8|both] [--counters]
                                [--scaling 1,2,4,8] [--min-tflops X] [--min-tflops-fp8 Y]
    amd-validator-workload rccl [--ranks 2,4,8] [--processes N] [--max-bytes N] [--dtype float|bf16]
                                [--min-busbw GBPS]

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
from typing import Callable, Dict, List, Optional

BIN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native", "bin")
# One rocprofv3 pass per GEMM dtype (8 SQ + 4 TCC slots per pass on gfx950): the MFMA op counter(s)
# of that dtype, busy cycles, LDS bank conflicts / activity and L2 hits / misses. The f8f6f4
# instruction the fp8 kernel issues is counted under F8 or F6F4 depending on the firmware, so the
# fp8 pass collects both and sums them.
PMC_PASSES = {
    "bf16": {"kernel": "gemm_bf16_256x256", "mops": ["SQ_INSTS_VALU_MFMA_MOPS_BF16"]},
    "fp8": {"kernel": "gemm_fp8_256x256", "mops": ["SQ_INSTS_VALU_MFMA_MOPS_F8", "SQ_INSTS_VALU_MFMA_MOPS_F6F4"]},
}
PMC_COMMON = ["SQ_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "TCC_HIT_sum", "TCC_MISS_sum"]
PMC_COUNTERS = PMC_PASSES["bf16"]["mops"] + PMC_COMMON      # the bf16 pass (kept for callers)


def rocprofv3_path() -> Optional[str]:
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    return prof if os.path.exists(prof) else None


def binary(name: str) -> str:
    p = os.path.join(BIN_DIR, name)
    if os.path.exists(p):
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


def run_json(cmd: List[str], run: Callable = subprocess.run, timeout: float = 600) -> (int, List[Dict]):
    p = run(cmd, capture_output=True, text=True, timeout=timeout)
    if p.stderr:
        sys.stderr.write(p.stderr[-4000:])
    return p.returncode, _json_lines(p.stdout)


def _shape_mnk(shape: str):
    parts = [int(x) for x in shape.lower().split("x")]
    return (parts[0],) * 3 if len(parts) == 1 else tuple(parts[:3])


def collect_counters(shape: str, run: Callable = subprocess.run, dtype: str = "bf16") -> List[Dict]:
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
               "--no-stabilise", "--devices", "0", "--check-rows", "1", "--dtype", dtype]
        p = run(cmd, capture_output=True, text=True, timeout=300)
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if p.returncode != 0 or not files:
            return [{"event": "counters", "dtype": dtype, "ok": False,
                     "error": f"rocprofv3 exit {p.returncode}: {(p.stderr or '')[-300:]}"}]
        agg: Dict[str, float] = {}
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if spec["kernel"] not in row.get("Kernel_Name", ""):
                    continue
                agg[row["Counter_Name"]] = agg.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        if not agg:
            return [{"event": "counters", "dtype": dtype, "ok": False,
                     "error": f"no {spec['kernel']} dispatch in the counter records"}]
        m, n, k = _shape_mnk(shape)
        mops = sum(agg.get(c, 0.0) for c in spec["mops"])
        want = 2.0 * m * n * k / 512
        res = {"event": "counters", "dtype": dtype, "kernel": spec["kernel"], "shape": shape, **agg,
               "mfma_mops": mops, "mfma_mops_expected": want, "mfma_mops_match": abs(mops - want) <= 1e-6 * want,
               "lds_conflict_free": agg.get("SQ_LDS_BANK_CONFLICT", 1.0) == 0.0}
        res["ok"] = res["mfma_mops_match"]
        return [res]
    finally:
        shutil.rmtree(out, ignore_errors=True)


def run_hip(shapes: List[str], counters: bool = False, iters: int = 50,
            run: Callable = subprocess.run, dtype: str = "bf16", scaling: Optional[str] = None,
            min_tflops: float = 0.0, min_tflops_fp8: float = 0.0) -> List[Dict]:
    """hip-smoke, then the MFMA GEMM probe in ``dtype`` (bf16, fp8 e4m3fn on the double-rate
    16x16x128 matrix-core path, or both) -- clock-stabilised like bench.py, optionally swept over
    ``scaling`` GPU counts ("1,2,4,8") and gated on per-GPU floors -- then optionally one
    counter-collection pass per dtype."""
    results: List[Dict] = []
    rc, r = run_json([binary("amd-hip-smoke")], run)
    results += r or [{"event": "hip-smoke", "ok": False, "rc": rc}]
    cmd = [binary("amd-gemm-validate"), "--shapes", ",".join(shapes), "--iters", str(iters)]
    if dtype != "bf16":
        cmd += ["--dtype", dtype]
    if scaling:
        cmd += ["--scaling", scaling]
    if min_tflops:
        cmd += ["--min-tflops", f"{min_tflops:g}"]
    if min_tflops_fp8:
        cmd += ["--min-tflops-fp8", f"{min_tflops_fp8:g}"]
    rc, r = run_json(cmd, run, timeout=1200)
    results += r
    if rc != 0 and not any(x.get("event") == "gemm" for x in r):
        results.append({"event": "gemm", "ok": False, "rc": rc})
    if counters:
        for d in (["bf16", "fp8"] if dtype == "both" else [dtype]):
            results += collect_counters(shapes[0], run, dtype=d)
    return results


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


def run_rccl(max_bytes: int, dtype: str, run: Callable = subprocess.run, ranks: Optional[str] = None,
             min_busbw: Optional[float] = None, processes: int = 0, min_bytes: int = 1024,
             timeout: float = 1200) -> List[Dict]:
    """The xGMI fabric proof: topology + fabric check, then a rank-count sweep in one process
    (``ranks`` "2,4,8") or, with ``processes`` N, one process per GPU joined through
    ncclCommInitRank. RCCL's INFO log is captured and summarised (algorithm/protocol per size)."""
    if os.environ.get("RCCL_DRY_RUN") == "1":
        return _rccl_dry_run(ranks)
    base = ["--max-bytes", str(max_bytes), "--dtype", dtype, "--min-bytes", str(min_bytes)]
    if min_busbw:
        base += ["--min-busbw", str(min_busbw)]
    tmp = tempfile.mkdtemp(prefix="amdgo-rccl-")
    try:
        if processes > 0:
            results = _run_rccl_mp(processes, base, tmp, timeout)
        else:
            cmd = [binary("amd-rccl-validate")] + base + (["--ranks", ranks] if ranks else [])
            p = run(cmd, capture_output=True, text=True, timeout=timeout, env=_rccl_env(os.path.join(tmp, "rccl.%p.log")))
            if p.stderr:
                sys.stderr.write(p.stderr[-4000:])
            results = _json_lines(p.stdout)
            if p.returncode != 0 and not any(x.get("event") == "summary" for x in results):
                results.append({"event": "summary", "ok": False, "rc": p.returncode})
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


def _run_rccl_mp(n: int, base: List[str], tmp: str, timeout: float) -> List[Dict]:
    """Start N ranks of amd-rccl-validate (this process never touches the GPU); rank 0 publishes the
    ncclUniqueId through a file, the others join. Rank 0's lines plus every rank's summary."""
    id_file = os.path.join(tmp, "nccl.id")
    procs = []
    for r in range(n):
        cmd = [binary("amd-rccl-validate")] + base + ["--mp-rank", str(r), "--mp-nranks", str(n),
                                                      "--mp-id-file", id_file, "--device", str(r)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      env=_rccl_env(os.path.join(tmp, f"rccl.{r}.log"))))
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            out, err = p.communicate()
        if err:
            sys.stderr.write(err[-2000:])
        outs.append((p.returncode, _json_lines(out)))
    results = list(outs[0][1])
    for r, (rc, lines) in enumerate(outs[1:], start=1):
        results += [x for x in lines if x.get("event") in ("summary", "start") or "error" in x]
        if rc != 0 and not any(x.get("event") == "summary" for x in lines):
            results.append({"event": "summary", "rank": r, "ok": False, "rc": rc})
    if outs[0][0] != 0 and not any(x.get("event") == "summary" for x in outs[0][1]):
        results.append({"event": "summary", "rank": 0, "ok": False, "rc": outs[0][0]})
    return results


TERMINATION_LOG_BYTES = 4000       # kubelet keeps at most 4 KiB of a termination message
_SUMMARY_EVENTS = ("aggregate", "summary", "hip-smoke", "counters", "scaling", "fabric", "ranks_summary",
                   "rccl-debug")


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
    r = sub.add_parser("rccl")
    r.add_argument("--max-bytes", type=int, default=int(os.environ.get("RCCL_MAX_BYTES", 1 << 30)))
    r.add_argument("--dtype", default=os.environ.get("RCCL_DTYPE", "float"))
    r.add_argument("--ranks", default=os.environ.get("RCCL_RANKS", "2,4,8"))
    r.add_argument("--processes", type=int, default=int(os.environ.get("RCCL_PROCESSES", "0")))
    r.add_argument("--min-busbw", type=float, default=float(os.environ.get("RCCL_MIN_BUSBW_GBPS", "0") or 0))
    a = ap.parse_args(argv)
    if a.what == "hip":
        results = run_hip(a.gemm_shapes.split(","), counters=a.counters, iters=a.iters, dtype=a.gemm_dtype,
                          scaling=a.scaling or None, min_tflops=a.min_tflops, min_tflops_fp8=a.min_tflops_fp8)
        ok = all(x.get("ok", True) for x in results if x.get("event") in ("gemm", "hip-smoke"))
    else:
        results = run_rccl(a.max_bytes, a.dtype, ranks=a.ranks, min_busbw=a.min_busbw, processes=a.processes)
        ok = all(x.get("ok", False) for x in results if x.get("event") == "summary")
    emit(results)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
