"""In-tree native build for every C++/HIP component of the framework.

Everything is compiled for gfx950 only (``--offload-arch=gfx950``) with ``hipcc``; host-only
C++ (the node agent library and CLIs) is built with ``g++``. Artefacts land in
``gpu_operator_amd/_native/`` so they travel with the repository snapshot to the GPU box
(they are git-ignored, not gpurun-ignored).

Usage::

    python -m gpu_operator_amd._build          # build what is stale
    python -m gpu_operator_amd._build --force  # rebuild everything
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Sequence

REPO = Path(__file__).resolve().parent.parent
NATIVE_SRC = REPO / "native"
OUT = Path(__file__).resolve().parent / "_native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("AMDGO_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    cand = ROCM / "bin" / "hipcc"
    return str(cand) if cand.exists() else "hipcc"


@dataclass
class Target:
    name: str                     # output file name (relative to OUT)
    sources: Sequence[str]        # relative to native/
    kind: str                     # "hip-shared" | "hip-exe" | "cxx-shared" | "cxx-exe" | "pyext"
    flags: List[str] = field(default_factory=list)
    libs: List[str] = field(default_factory=list)
    headers: Sequence[str] = ()   # extra dependency files (relative to native/)

    @property
    def output(self) -> Path:
        return OUT / self.name

    def deps(self) -> List[Path]:
        return [NATIVE_SRC / s for s in list(self.sources) + list(self.headers)]

    def stale(self) -> bool:
        if not self.output.exists():
            return True
        out_m = self.output.stat().st_mtime
        return any(p.stat().st_mtime > out_m for p in self.deps() if p.exists())

    def command(self) -> List[str]:
        srcs = [str(NATIVE_SRC / s) for s in self.sources]
        inc = [f"-I{NATIVE_SRC / 'include'}"]
        if self.kind.startswith("hip"):
            base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wall",
                    "-Wno-unused-function", "-Wno-unused-result"] + inc
            if self.kind == "hip-shared":
                base += ["-fPIC", "-shared"]
            else:
                base += [f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}"]
            return base + self.flags + srcs + ["-o", str(self.output)] + self.libs
        if self.kind == "pyext":
            import pybind11  # noqa: WPS433 (build-time only)
            py_inc = sysconfig.get_paths()["include"]
            suffix_ok = self.name.endswith(sysconfig.get_config_var("EXT_SUFFIX") or ".so")
            assert suffix_ok, self.name
            return (["g++", "-O2", "-std=c++17", "-Wall", "-fPIC", "-shared",
                     f"-I{py_inc}", f"-I{pybind11.get_include()}"] + inc + self.flags + srcs
                    + ["-o", str(self.output)] + self.libs)
        base = ["g++", "-O2", "-std=c++17", "-Wall", "-Wextra"] + inc
        if self.kind == "cxx-shared":
            base += ["-fPIC", "-shared"]
        return base + self.flags + srcs + ["-o", str(self.output)] + self.libs


def _pyext_name(stem: str) -> str:
    return stem + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")


# Production builds read the generated headers with the shipped schedules only; the lab libraries
# read the *_lab.h headers (every schedule), which mask the production ones (tools/gen_*_asm_loop.py).
GEMM_HEADERS = ["include/gemm_tile_common.h", "hip/gemm_bf16_kernels.h", "hip/gemm_bf16_asm_loop.h",
                "hip/gemm_fp8_kernels.h", "hip/gemm_fp8_asm_loop.h", "hip/gemm_w4ap.h", "hip/gemm_small.h",
                "hip/gemm_small_host.h", "hip/gemm_raster_host.h"]
LAB_HEADERS = GEMM_HEADERS + ["hip/gemm_bf16_asm_loop_lab.h", "hip/gemm_fp8_asm_loop_lab.h"]

TARGETS: List[Target] = [
    # GPU compute: validator workloads (GEMM, smoke). Loaded via ctypes by ops/.
    Target("libamdgo_hip.so", ["hip/gemm_bf16.hip", "hip/gemm_fp8.hip", "hip/gemm_abft.hip", "hip/smoke.hip"], "hip-shared",
           headers=GEMM_HEADERS),
    # Node agent library (sysfs/KFD topology, partitions, telemetry, inotify barriers).
    Target(_pyext_name("_amdnode"), ["node/pybind.cpp", "node/amdnode.cpp"], "pyext",
           headers=["include/amdnode.h"]),
    Target("bin/amd-barrier-wait", ["node/barrier_wait.cpp", "node/amdnode.cpp"], "cxx-exe",
           flags=["-static-libstdc++", "-static-libgcc"], headers=["include/amdnode.h"]),
    # Validator workload binaries (run inside the validation pods).
    # (one worker process per GPU: the launcher enumerates the GPUs from KFD sysfs, libamdnode)
    Target("bin/amd-gemm-validate", ["hip/gemm_validate.cpp", "hip/gemm_bf16.hip", "hip/gemm_fp8.hip", "hip/gemm_abft.hip",
                                     "hip/smoke.hip", "node/amdnode.cpp"],
           "hip-exe", flags=["-x", "hip"], headers=GEMM_HEADERS + ["include/amdnode.h"]),
    Target("bin/amd-hip-smoke", ["hip/hip_smoke_main.cpp", "hip/smoke.hip"], "hip-exe", flags=["-x", "hip"]),
    Target("bin/amd-rccl-validate", ["hip/rccl_validate.cpp", "node/amdnode.cpp"], "hip-exe", flags=["-x", "hip"],
           libs=["-lrccl"], headers=["include/amdnode.h"]),
    # OCI runtime shim injecting /dev/kfd + render nodes (legacy) or CDI edits into bundles.
    # Fully static: it runs on the host (via containerd/CRI-O/docker), whatever its glibc.
    Target("bin/amd-container-runtime", ["toolkit/amd_container_runtime.cpp", "node/amdnode.cpp"], "cxx-exe",
           flags=["-static"], headers=["include/amdnode.h", "include/minijson.h"]),
    Target("bin/amd-node-probe", ["node/node_probe.cpp", "node/amdnode.cpp"], "cxx-exe",
           flags=["-static-libstdc++", "-static-libgcc"], headers=["include/amdnode.h"]),
    # driver / toolkit / no-fabric rccl validation without a Python interpreter (validator init containers)
    # (plugin: a TLS GET of its Node -- OpenSSL linked in statically, no runtime dependency on the image's)
    Target("bin/amd-node-validate", ["node/node_validate.cpp", "node/amdnode.cpp"], "cxx-exe",
           flags=["-static-libstdc++", "-static-libgcc", "-s"], headers=["include/amdnode.h", "include/minijson.h"],
           libs=["-Wl,-Bstatic", "-lssl", "-lcrypto", "-Wl,-Bdynamic", "-ldl", "-lpthread"]),
]


# Tools-only: superseded GEMM generations, placement sweeps and knock-out timings for A/B profiling
# (tools/gemm_lab.py). Never loaded by the validator; built on request (`--lab`).
LAB_TARGETS: List[Target] = [
    # one library per dtype: an fp8 schedule edit rebuilds only the fp8 lab
    Target("libamdgo_gemm_lab_bf16.so", ["hip/gemm_bf16_lab.hip"], "hip-shared", headers=LAB_HEADERS),
    Target("libamdgo_gemm_lab_fp8.so", ["hip/gemm_fp8_lab.hip"], "hip-shared", headers=LAB_HEADERS),
    # the hand-scheduled bf16 K pipeline (w4a) next to v44 (tools/asm_lab.py)
    Target("libamdgo_gemm_asmlab.so", ["hip/gemm_bf16_asm_lab.hip"], "hip-shared", headers=LAB_HEADERS),
]


def build(force: bool = False, jobs: int = 4, verbose: bool = False, lab: bool = False) -> List[Path]:
    OUT.mkdir(parents=True, exist_ok=True)
    (OUT / "bin").mkdir(exist_ok=True)
    todo = [t for t in TARGETS + (LAB_TARGETS if lab else []) if force or t.stale()]

    def run(t: Target) -> Path:
        cmd = t.command()
        if verbose:
            print(" ".join(cmd), flush=True)
        t.output.parent.mkdir(parents=True, exist_ok=True)
        proc = subprocess.run(cmd, capture_output=True, text=True)
        if proc.returncode != 0:
            raise RuntimeError(f"build of {t.name} failed:\n{' '.join(cmd)}\n{proc.stderr[-6000:]}")
        return t.output

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        built = list(ex.map(run, todo))
    return built


def main(argv: Sequence[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=4)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--lab", action="store_true", help="also build the tools-only GEMM experiment library")
    a = ap.parse_args(argv)
    if shutil.which(hipcc()) is None and not Path(hipcc()).exists():
        print("hipcc not found", file=sys.stderr)
        return 1
    built = build(force=a.force, jobs=a.jobs, verbose=a.verbose, lab=a.lab)
    for p in built:
        print(f"built {p.relative_to(REPO)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
