"""Run a console script of this package by its installed name, without installing it:

    python -m gpu_operator_amd.cmd.entry amd-validator --component driver

The table is ``[project.scripts]`` of pyproject.toml (a test keeps the two identical). The node
bring-up harness (validator/ttr.py) puts one-line wrappers named after these scripts on PATH, so
the operand entrypoint scripts from the assets run unmodified and exec the same commands a
container image would.
"""

from __future__ import annotations

import importlib
import sys

SCRIPTS = {
    "amd-gpu-operator": "gpu_operator_amd.cmd.operator:main",
    "amd-gpuop-cfg": "gpu_operator_amd.cmd.gpuop_cfg:main",
    "amd-validator": "gpu_operator_amd.validator.main:main",
    "amd-validator-workload": "gpu_operator_amd.validator.workload_main:main",
    "amd-device-plugin": "gpu_operator_amd.operands.device_plugin:main",
    "amd-sandbox-device-plugin": "gpu_operator_amd.operands.sandbox_device_plugin:main",
    "amd-node-labeller": "gpu_operator_amd.operands.node_labeller:main",
    "amd-partition-manager": "gpu_operator_amd.operands.partition_manager:main",
    "amd-metrics-exporter": "gpu_operator_amd.operands.metrics_exporter:main",
    "amd-config-manager": "gpu_operator_amd.operands.config_manager:main",
    "amd-driver-manager": "gpu_operator_amd.operands.driver_manager:main",
    "amdgpu-driver": "gpu_operator_amd.operands.driver_container:main",
    "amd-mxgpu-driver": "gpu_operator_amd.operands.mxgpu_driver:main",
    "amd-mxgpu-device-manager": "gpu_operator_amd.operands.mxgpu_device_manager:main",
    "amd-kata-manager": "gpu_operator_amd.operands.kata_manager:main",
    "amd-ctk": "gpu_operator_amd.toolkit.ctk:main",
}


NATIVE_TOOLS = ("amd-barrier-wait", "amd-hip-smoke", "amd-gemm-validate", "amd-rccl-validate", "amd-node-probe",
                "amd-node-validate", "amd-container-runtime")


def install_wrappers(bin_dir: str) -> str:
    """Put every console script of this package (a one-line ``exec python -m ...entry <name>``
    wrapper) and the native tools on a directory, as a container image's PATH would have them."""
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    native = os.path.join(here, "_native", "bin")
    os.makedirs(bin_dir, exist_ok=True)
    for name in SCRIPTS:
        p = os.path.join(bin_dir, name)
        with open(p, "w") as f:
            f.write(f'#!/bin/sh\nexec "{sys.executable}" -m gpu_operator_amd.cmd.entry {name} "$@"\n')
        os.chmod(p, 0o755)
    for name in NATIVE_TOOLS:
        src, dst = os.path.join(native, name), os.path.join(bin_dir, name)
        if os.path.exists(src) and not os.path.lexists(dst):
            os.symlink(src, dst)
    return bin_dir


def run(name: str, argv=None) -> int:
    target = SCRIPTS.get(name)
    if target is None:
        print(f"unknown console script {name!r}; known: {sorted(SCRIPTS)}", file=sys.stderr)
        return 127
    mod, fn = target.split(":")
    sys.argv[0] = name
    rc = getattr(importlib.import_module(mod), fn)(argv)
    return int(rc or 0)


def main() -> int:
    if len(sys.argv) < 2:
        print("usage: python -m gpu_operator_amd.cmd.entry <console-script> [args...]", file=sys.stderr)
        return 2
    return run(sys.argv[1], sys.argv[2:])


if __name__ == "__main__":
    sys.exit(main())
