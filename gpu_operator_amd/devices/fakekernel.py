"""A simulated kernel for CPU rehearsals of the containerised-driver path.

The e2e harness (gpu_operator_amd/e2e) runs the driver DaemonSet's containers as processes. On
a CPU-only machine there is no amdgpu to load, so in that mode the harness puts this module on
PATH as ``insmod``, ``rmmod``, ``modprobe``, ``dkms`` and ``chroot``. These act on the fake
sysfs/dev tree of ``AMD_SYSFS_ROOT`` (devices/fakesys.py), the same tree every agent reads:

* loading ``amdgpu`` writes ``sys/module/amdgpu/{initstate=live, version, refcnt=0}`` and
  creates ``dev/kfd``. The KFD topology nodes of the fake GPUs were already laid out by
  ``fakesys.make_node``;
* unloading refuses while ``refcnt`` > 0, as the kernel does, and otherwise removes both;
* ``dkms install`` "builds" (records the version), and ``chroot <root> <cmd...>`` runs ``cmd``.

Never used against a real sysfs: the entry point refuses a root of ``/``.
"""

from __future__ import annotations

import os
import shutil
import sys
from pathlib import Path
from typing import List

COMPANIONS = ("amdkcl", "amdttm", "amddrm_ttm_helper", "amddrm_buddy", "amdxcp")


def _root() -> Path:
    root = os.environ.get("AMD_SYSFS_ROOT", "/")
    if os.path.realpath(root) == "/":
        raise SystemExit("fakekernel: refusing to act on the real / (AMD_SYSFS_ROOT unset or /)")
    return Path(root)


def _mod_name(arg: str) -> str:
    base = os.path.basename(arg)
    for suf in (".ko.xz", ".ko.zst", ".ko"):
        if base.endswith(suf):
            base = base[: -len(suf)]
    return base.replace("-", "_")


def load(name: str) -> int:
    root = _root()
    d = root / "sys/module" / name
    d.mkdir(parents=True, exist_ok=True)
    (d / "refcnt").write_text("0\n")
    if name == "amdgpu":
        built = root / "var/lib/fakekernel/dkms"           # what `dkms install` last built
        ver = os.environ.get("DRIVER_VERSION") or (built.read_text().strip() if built.exists() else "6.12.12")
        (d / "version").write_text(f"{ver}\n")
        (d / "initstate").write_text("live\n")
        (root / "dev").mkdir(parents=True, exist_ok=True)
        (root / "dev/kfd").write_text("")
        for minor in _render_minors(root):             # DRM render nodes of every GPU agent
            (root / "dev/dri").mkdir(parents=True, exist_ok=True)
            (root / "dev/dri" / f"renderD{minor}").write_text("")
    return 0


def _render_minors(root: Path) -> List[int]:
    out = []
    for props in sorted((root / "sys/class/kfd/kfd/topology/nodes").glob("*/properties")):
        for line in props.read_text().splitlines():
            k, _, v = line.partition(" ")
            if k == "drm_render_minor" and int(v or 0) > 0:
                out.append(int(v))
    return out


def unload(name: str) -> int:
    root = _root()
    d = root / "sys/module" / name
    if not d.exists():
        print(f"rmmod: ERROR: Module {name} is not currently loaded", file=sys.stderr)
        return 1
    try:
        users = int((d / "refcnt").read_text().strip() or 0)
    except (OSError, ValueError):
        users = 0
    if users > 0:
        print(f"rmmod: ERROR: Module {name} is in use", file=sys.stderr)
        return 1
    shutil.rmtree(d)
    if name == "amdgpu":
        for p in [root / "dev/kfd"] + list((root / "dev/dri").glob("renderD*")):
            try:
                p.unlink()
            except FileNotFoundError:
                pass
    return 0


def main(argv: List[str]) -> int:
    prog = os.path.basename(argv[0])
    args = argv[1:]
    if prog == "chroot":                   # chroot <newroot> <cmd...>: the command runs "on the host"
        if len(args) < 2:
            return 1
        return main(args[1:])
    if prog == "insmod":
        return load(_mod_name(args[0])) if args else 1
    if prog == "rmmod":
        return max([unload(_mod_name(a)) for a in args if not a.startswith("-")] or [1])
    if prog == "modprobe":
        names = [a for a in args if not a.startswith("-") and "=" not in a]
        if "-r" in args:
            rc = 0
            for n in names:
                rc |= unload(_mod_name(n))
                for c in COMPANIONS:                 # modprobe -r also removes unused dependencies
                    if (_root() / "sys/module" / c).exists():
                        unload(c)
            return rc
        return load(_mod_name(names[0])) if names else 1
    if prog == "dkms":                       # dkms install amdgpu/<version> -k <kernel>
        if len(args) >= 2 and args[0] == "install":
            p = _root() / "var/lib/fakekernel/dkms"
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_text(args[1].split("/", 1)[-1] + "\n")
            return 0
        return 1
    print(f"fakekernel: unknown tool {prog}", file=sys.stderr)
    return 127


def install_tools(bin_dir: str) -> List[str]:
    """Wrappers named after the kernel tools, dispatching to :func:`main`."""
    out = []
    for tool in ("insmod", "rmmod", "modprobe", "dkms", "chroot"):
        p = os.path.join(bin_dir, tool)
        with open(p, "w") as f:
            f.write(f'#!/bin/sh\nexec "{sys.executable}" -c "import sys; from gpu_operator_amd.devices import '
                    f'fakekernel as k; sys.exit(k.main([\'{tool}\'] + sys.argv[1:]))" "$@"\n')
        os.chmod(p, 0o755)
        out.append(p)
    return out


if __name__ == "__main__":
    sys.exit(main(sys.argv))
