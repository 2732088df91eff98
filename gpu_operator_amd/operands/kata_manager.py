"""``amd-kata-manager``: Kata Containers runtime classes for confidential / sandboxed GPU pods.

Counterpart of the reference's external k8s-kata-manager. For
each ``runtimeClasses[]`` entry of the kata config (``spec.kataManager.config``):

1. fetch the guest artifacts (kernel, initrd/rootfs image, ``configuration-<name>.toml``)
   into ``<artifactsDir>/<name>/`` — from an OCI artifact via ``KATA_ARTIFACT_PULL_CMD``
   (default ``oras pull {url} -o {dir}``), or from a local ``file://`` path (air-gapped);
2. when the artifacts carry no Kata configuration, render one: QEMU with VFIO hot-plug on
   PCIe root ports sized for the node's AMD GPUs (MI355X BARs need 64-bit MMIO windows);
3. register containerd handler ``<name>`` (``io.containerd.kata.v2``, ``ConfigPath`` to the
   artifact config, kata pod annotations passed through) and reload containerd.

``--uninstall`` (the preStop hook) removes the handlers; the artifacts stay cached.
"""

from __future__ import annotations

import argparse
import logging
import os
import shlex
import shutil
import subprocess
import sys
import threading
from typing import Callable, Dict, List, Optional

import yaml

from .. import devices
from ..toolkit import runtime_config

log = logging.getLogger("amd-kata-manager")


class KataError(Exception):
    pass


def render_configuration(name: str, adir: str, n_gpus: int) -> str:
    kernel = next((f for f in sorted(os.listdir(adir)) if f.startswith("vmlinu")), "vmlinuz")
    image = next((f for f in sorted(os.listdir(adir)) if f.endswith((".img", ".image"))), "")
    initrd = next((f for f in sorted(os.listdir(adir)) if f.startswith("initrd")), "")
    lines = [f"# rendered by amd-kata-manager for runtime class {name}",
             "[hypervisor.qemu]",
             'path = "/opt/kata/bin/qemu-system-x86_64"',
             f'kernel = "{os.path.join(adir, kernel)}"']
    if image:
        lines.append(f'image = "{os.path.join(adir, image)}"')
    elif initrd:
        lines.append(f'initrd = "{os.path.join(adir, initrd)}"')
    lines += ['machine_type = "q35"',
              "default_memory = 8192",
              f"pcie_root_port = {max(1, n_gpus)}",
              'hot_plug_vfio = "root-port"',
              'cold_plug_vfio = "no-port"',
              "enable_iommu = false",
              'kernel_params = "pci=realloc pci=nocrs"',   # room for the GPUs' 64-bit BARs
              "",
              "[runtime]",
              'internetworking_model = "tcfilter"',
              "sandbox_cgroup_only = true",
              'static_sandbox_resource_mgmt = true', ""]
    return "\n".join(lines)


class KataManager:
    def __init__(self, config: Dict, containerd_config: str, artifacts_dir: Optional[str] = None,
                 pull_cmd: str = "oras pull {url} -o {dir}", run: Callable = subprocess.run,
                 reload: Optional[Callable[[], None]] = None, sys_root: Optional[str] = None):
        self.config = config
        self.artifacts_dir = artifacts_dir or config.get("artifactsDir",
                                                         "/opt/amd-gpu-operator/artifacts/runtimeclasses")
        self.containerd_config = containerd_config
        self.pull_cmd = pull_cmd
        self.run = run
        self.reload = reload
        self.sys_root = sys_root

    def classes(self) -> List[Dict]:
        return list(self.config.get("runtimeClasses") or [])

    def fetch(self, rc: Dict) -> str:
        name = rc["name"]
        dst = os.path.join(self.artifacts_dir, name)
        url = ((rc.get("artifacts") or {}).get("url") or "").strip()
        if not url:
            raise KataError(f"runtime class {name}: no artifacts url")
        os.makedirs(dst, exist_ok=True)
        if url.startswith("file://") or url.startswith("/"):
            src = url[len("file://"):] if url.startswith("file://") else url
            if not os.path.isdir(src):
                raise KataError(f"runtime class {name}: {src} is not a directory")
            for f in os.listdir(src):
                s = os.path.join(src, f)
                if os.path.isfile(s):
                    shutil.copy2(s, os.path.join(dst, f))
        else:
            argv = [a.format(url=url, dir=dst) for a in shlex.split(self.pull_cmd)]
            p = self.run(argv, capture_output=True, text=True, timeout=1800)
            if p.returncode != 0:
                raise KataError(f"runtime class {name}: pulling {url} failed: {(p.stderr or '').strip()[-1000:]}")
        return dst

    def config_path(self, rc: Dict, adir: str) -> str:
        name = rc["name"]
        cand = [f for f in os.listdir(adir) if f.startswith("configuration") and f.endswith(".toml")]
        if cand:
            return os.path.join(adir, sorted(cand)[0])
        n = len({g["bdf"] for g in devices.scan_pci(self.sys_root) if not g["is_virtfn"]}
                ) if self.sys_root is not None else 8
        path = os.path.join(adir, f"configuration-{name}.toml")
        with open(path, "w") as f:
            f.write(render_configuration(name, adir, n))
        return path

    def handlers(self) -> Dict[str, Dict]:
        out = {}
        for rc in self.classes():
            adir = self.fetch(rc)
            out[rc["name"]] = {"runtime_type": "io.containerd.kata.v2",
                               "privileged_without_host_devices": True,
                               "pod_annotations": ["io.katacontainers.*"],
                               "container_annotations": ["io.katacontainers.*"],
                               "options": {"ConfigPath": self.config_path(rc, adir)}}
        return out

    def install(self) -> bool:
        changed = runtime_config.set_containerd_runtimes(self.containerd_config, self.handlers())
        if changed and self.reload:
            self.reload()
        log.info("kata runtime classes %s (%s)", [r["name"] for r in self.classes()],
                 "updated" if changed else "unchanged")
        return changed

    def uninstall(self) -> bool:
        changed = runtime_config.remove_containerd_runtimes(self.containerd_config,
                                                            [r["name"] for r in self.classes()])
        if changed and self.reload:
            self.reload()
        return changed


def main(argv=None, stop: Optional[threading.Event] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-kata-manager")
    ap.add_argument("--config", default="/etc/kata-manager/config.yaml")
    ap.add_argument("--uninstall", action="store_true")
    ap.add_argument("--oneshot", action="store_true")
    a = ap.parse_args(argv)
    with open(a.config) as f:
        cfg = yaml.safe_load(f) or {}
    ctrd = os.environ.get("CONTAINERD_CONFIG", "/etc/containerd/config.toml")

    def reload():
        from ..toolkit.ctk import Installer
        Installer(root="/tmp", runtime="containerd", runtime_config=ctrd,
                  runtime_socket=os.environ.get("CONTAINERD_SOCKET", "/run/containerd/containerd.sock"),
                  restart_mode=os.environ.get("RESTART_MODE", "systemd")).reload_runtime()
    km = KataManager(cfg, ctrd, artifacts_dir=os.environ.get("KATA_ARTIFACTS_DIR"),
                     pull_cmd=os.environ.get("KATA_ARTIFACT_PULL_CMD", "oras pull {url} -o {dir}"),
                     reload=reload, sys_root=os.environ.get("AMD_SYSFS_ROOT", "/"))
    try:
        if a.uninstall:
            km.uninstall()
            return 0
        km.install()
    except KataError as e:
        log.error("%s", e)
        return 1
    if a.oneshot:
        return 0
    (stop or threading.Event()).wait()
    return 0


if __name__ == "__main__":
    sys.exit(main())
