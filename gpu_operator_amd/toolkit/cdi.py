"""CDI (Container Device Interface) spec for AMD GPUs: ``amd-ctk cdi generate``.

One device per KFD agent (a whole GPU in SPX, one partition in DPX/QPX/CPX), named by index
and by unique id, plus ``all``. A device's edits are just its DRM render node; the spec-wide
edits add ``/dev/kfd`` (shared by every GPU) — ROCm needs no host libraries injected, unlike
the reference's CUDA driver-library mounts (SURVEY.md §2.3 container-toolkit). Written as JSON
so the native runtime shim (native/toolkit/amd_container_runtime.cpp) parses it directly.
"""

from __future__ import annotations

import json
import os
import stat
from typing import Dict, List, Optional

from .. import devices

CDI_VERSION = "0.6.0"
KIND = "amd.com/gpu"
SPEC_NAME = "amd.com-gpu.json"


def _node(path: str, dev_root: str) -> Dict:
    d: Dict = {"path": path}
    host = os.path.join(dev_root, path.lstrip("/"))
    try:
        st = os.stat(host)
    except OSError:
        return d                        # resolved by the runtime at container creation
    if stat.S_ISCHR(st.st_mode):
        d.update({"type": "c", "major": os.major(st.st_rdev), "minor": os.minor(st.st_rdev)})
    return d


def generate(sys_root: Optional[str] = None, dev_root: str = "/", strategy: str = "index,uuid") -> Dict:
    gpus = devices.enumerate_gpus(sys_root)
    strategies = [s.strip() for s in strategy.split(",") if s.strip()]
    devs: List[Dict] = []
    renders = []
    for g in gpus:
        if g["drm_render_minor"] < 0:
            continue
        node = _node(f"/dev/dri/renderD{g['drm_render_minor']}", dev_root)
        renders.append(node)
        edits = {"deviceNodes": [node],
                 "env": [f"AMD_GPU_UUID_{g['index']}=amdgpu-{g['unique_id']:016x}"]}
        names = []
        if "index" in strategies:
            names.append(str(g["index"]))
        if "uuid" in strategies:
            names.append(f"amdgpu-{g['unique_id']:016x}")
        if "bdf" in strategies and g["compute_partition"] in ("", "SPX"):
            names.append(g["pci_bdf"])
        for n in names:
            devs.append({"name": n, "containerEdits": edits})
    if renders:
        devs.append({"name": "all", "containerEdits": {"deviceNodes": renders}})
    return {"cdiVersion": CDI_VERSION, "kind": KIND,
            "containerEdits": {"deviceNodes": [_node("/dev/kfd", dev_root)]},
            "devices": devs}


def write(spec: Dict, spec_dir: str = "/var/run/cdi") -> str:
    os.makedirs(spec_dir, exist_ok=True)
    path = os.path.join(spec_dir, SPEC_NAME)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(spec, f, indent=2)
    os.chmod(tmp, 0o644)
    os.replace(tmp, path)
    return path


def list_devices(spec_dir: str = "/var/run/cdi") -> List[str]:
    path = os.path.join(spec_dir, SPEC_NAME)
    if not os.path.exists(path):
        return []
    with open(path) as f:
        spec = json.load(f)
    return [f"{spec['kind']}={d['name']}" for d in spec.get("devices", [])]


def create_dev_char_symlinks(dev_root: str = "/", dev_char: str = "/dev/char") -> List[str]:
    """``/dev/char/<major>:<minor>`` links for /dev/kfd and the DRI nodes: systemd's cgroup
    driver resolves device rules through them (reference: createDevCharSymlinks,
    validator/main.go:682-708)."""
    made = []
    os.makedirs(dev_char, exist_ok=True)
    cands = [os.path.join(dev_root, "dev/kfd")]
    dri = os.path.join(dev_root, "dev/dri")
    if os.path.isdir(dri):
        cands += [os.path.join(dri, x) for x in sorted(os.listdir(dri))]
    for p in cands:
        try:
            st = os.stat(p)
        except OSError:
            continue
        if not stat.S_ISCHR(st.st_mode):
            continue
        link = os.path.join(dev_char, f"{os.major(st.st_rdev)}:{os.minor(st.st_rdev)}")
        target = "/" + os.path.relpath(p, dev_root)
        if os.path.islink(link) and os.readlink(link) == target:
            continue
        if os.path.lexists(link):
            os.unlink(link)
        os.symlink(target, link)
        made.append(link)
    return made
