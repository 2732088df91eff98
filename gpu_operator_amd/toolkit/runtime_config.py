"""Register the AMD runtime handlers with containerd / docker / CRI-O (``amd-ctk runtime``).

Reference behaviour: the container-toolkit operand edits the runtime's config so a
RuntimeClass handler named after ``operator.runtimeClass`` runs its runtime wrapper, and
optionally makes it the default. Here the handlers are:

    amd         -> <root>/amd-container-runtime          (mode from amd-container-runtime.conf)
    amd-cdi     -> <root>/amd-container-runtime.cdi      (CDI only; when CDI is enabled)
    amd-legacy  -> <root>/amd-container-runtime.legacy   (KFD topology; when CDI is enabled)

containerd: config v1/v2 (``io.containerd.grpc.v1.cri``) and v3 (containerd 2.x,
``io.containerd.cri.v1.runtime``); the runc handler's options (e.g. ``SystemdCgroup``) are
copied so cgroup handling matches. docker: ``daemon.json`` ``runtimes`` (+ ``features.cdi``).
CRI-O: a drop-in file (``crio.conf.d/99-amd.conf``) owned entirely by us. Every change is
recorded in a state file so ``revert`` restores exactly what was there before.
"""

from __future__ import annotations

import copy
import json
import os
from typing import Any, Dict, List, Optional

import tomli

from . import tomlw

HANDLERS = ("amd", "amd-cdi", "amd-legacy")


def handler_binaries(root: str, name: str, cdi: bool) -> Dict[str, str]:
    base = os.path.join(root, "amd-container-runtime")
    out = {name: base}
    if cdi:
        out[f"{name}-cdi"] = base + ".cdi"
        out[f"{name}-legacy"] = base + ".legacy"
    return out


def _load_state(path: str) -> Dict[str, Any]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _save_state(path: str, st: Dict[str, Any]) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(st, f)


def _write(path: str, text: str) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".amd-tmp"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


# ---------------------------------------------------------------------------------------------
# containerd
# ---------------------------------------------------------------------------------------------
def _cri_path(doc: Dict[str, Any]) -> List[str]:
    ver = int(doc.get("version", 1))
    if ver >= 3:
        return ["plugins", "io.containerd.cri.v1.runtime"]
    if ver == 2:
        return ["plugins", "io.containerd.grpc.v1.cri"]
    return ["plugins", "cri"]


def _dig(d: Dict[str, Any], path: List[str]) -> Dict[str, Any]:
    for p in path:
        d = d.setdefault(p, {})
    return d


def configure_containerd(config: str, binaries: Dict[str, str], default: Optional[str], cdi: bool,
                         cdi_dirs: List[str], state_file: str) -> Dict[str, Any]:
    doc: Dict[str, Any] = {}
    if os.path.exists(config):
        with open(config, "rb") as f:
            doc = tomli.load(f)
    if "version" not in doc:
        doc["version"] = 2
    st = _load_state(state_file)
    cri = _dig(doc, _cri_path(doc))
    ctrd = cri.setdefault("containerd", {})
    runtimes = ctrd.setdefault("runtimes", {})
    base = copy.deepcopy(runtimes.get("runc") or {"runtime_type": "io.containerd.runc.v2"})
    base.setdefault("runtime_type", "io.containerd.runc.v2")
    for name, binary in binaries.items():
        h = copy.deepcopy(base)
        h.setdefault("options", {})["BinaryName"] = binary
        runtimes[name] = h
    if "containerd" not in st:
        st["containerd"] = {"default_runtime_name": ctrd.get("default_runtime_name"),
                            "enable_cdi": cri.get("enable_cdi"), "cdi_spec_dirs": cri.get("cdi_spec_dirs")}
    if default:
        ctrd["default_runtime_name"] = default
    if cdi:
        cri["enable_cdi"] = True
        cri["cdi_spec_dirs"] = cdi_dirs
    st["containerd"]["handlers"] = sorted(binaries)
    _write(config, tomlw.dumps(doc))
    _save_state(state_file, st)
    return doc


def revert_containerd(config: str, state_file: str) -> None:
    if not os.path.exists(config):
        return
    with open(config, "rb") as f:
        doc = tomli.load(f)
    st = _load_state(state_file).get("containerd", {})
    cri = _dig(doc, _cri_path(doc))
    ctrd = cri.setdefault("containerd", {})
    runtimes = ctrd.setdefault("runtimes", {})
    for name in st.get("handlers", HANDLERS):
        runtimes.pop(name, None)
    prev = st.get("default_runtime_name")
    if ctrd.get("default_runtime_name") in (st.get("handlers") or HANDLERS):
        if prev and prev not in (st.get("handlers") or HANDLERS):
            ctrd["default_runtime_name"] = prev
        else:
            ctrd["default_runtime_name"] = "runc"
    for k in ("enable_cdi", "cdi_spec_dirs"):
        if k in st:
            if st[k] is None:
                cri.pop(k, None)
            else:
                cri[k] = st[k]
    _write(config, tomlw.dumps(doc))
    _clear_state(state_file, "containerd")


def _clear_state(state_file: str, key: str) -> None:
    st = _load_state(state_file)
    st.pop(key, None)
    if st:
        _save_state(state_file, st)
    elif os.path.exists(state_file):
        os.unlink(state_file)


# ---------------------------------------------------------------------------------------------
# docker
# ---------------------------------------------------------------------------------------------
def configure_docker(config: str, binaries: Dict[str, str], default: Optional[str], cdi: bool,
                     state_file: str) -> Dict[str, Any]:
    doc: Dict[str, Any] = {}
    if os.path.exists(config) and os.path.getsize(config) > 0:
        with open(config) as f:
            doc = json.load(f)
    st = _load_state(state_file)
    if "docker" not in st:
        st["docker"] = {"default-runtime": doc.get("default-runtime"),
                        "cdi": (doc.get("features") or {}).get("cdi")}
    rts = doc.setdefault("runtimes", {})
    for name, binary in binaries.items():
        rts[name] = {"path": binary, "runtimeArgs": []}
    if default:
        doc["default-runtime"] = default
    if cdi:
        doc.setdefault("features", {})["cdi"] = True
    st["docker"]["handlers"] = sorted(binaries)
    _write(config, json.dumps(doc, indent=4) + "\n")
    _save_state(state_file, st)
    return doc


def revert_docker(config: str, state_file: str) -> None:
    if not os.path.exists(config):
        return
    with open(config) as f:
        doc = json.load(f)
    st = _load_state(state_file).get("docker", {})
    handlers = st.get("handlers") or list(HANDLERS)
    for name in handlers:
        (doc.get("runtimes") or {}).pop(name, None)
    if not doc.get("runtimes"):
        doc.pop("runtimes", None)
    if doc.get("default-runtime") in handlers:
        if st.get("default-runtime") and st["default-runtime"] not in handlers:
            doc["default-runtime"] = st["default-runtime"]
        else:
            doc.pop("default-runtime", None)
    if "cdi" in st and doc.get("features") is not None:
        if st["cdi"] is None:
            doc["features"].pop("cdi", None)
            if not doc["features"]:
                doc.pop("features")
        else:
            doc["features"]["cdi"] = st["cdi"]
    _write(config, json.dumps(doc, indent=4) + "\n")
    _clear_state(state_file, "docker")


# ---------------------------------------------------------------------------------------------
# CRI-O (drop-in owned by us)
# ---------------------------------------------------------------------------------------------
def configure_crio(dropin: str, binaries: Dict[str, str], default: Optional[str]) -> Dict[str, Any]:
    doc: Dict[str, Any] = {"crio": {"runtime": {"runtimes": {}}}}
    rt = doc["crio"]["runtime"]
    if default:
        rt["default_runtime"] = default
    for name, binary in binaries.items():
        rt["runtimes"][name] = {"runtime_path": binary, "runtime_type": "oci",
                                "runtime_root": f"/run/{name}"}
    # put scalars before the runtimes table for a tidy file
    ordered = {"crio": {"runtime": dict(sorted(rt.items(), key=lambda kv: isinstance(kv[1], dict)))}}
    _write(dropin, "# managed by amd-ctk; removed on uninstall\n" + tomlw.dumps(ordered))
    return ordered


def revert_crio(dropin: str) -> None:
    if os.path.exists(dropin):
        os.unlink(dropin)


def configure(runtime: str, config: str, binaries: Dict[str, str], default: Optional[str] = None,
              cdi: bool = False, cdi_dirs: Optional[List[str]] = None, state_file: str = "") -> None:
    state_file = state_file or config + ".amd-state.json"
    if runtime == "containerd":
        configure_containerd(config, binaries, default, cdi, cdi_dirs or ["/etc/cdi", "/var/run/cdi"], state_file)
    elif runtime == "docker":
        configure_docker(config, binaries, default, cdi, state_file)
    elif runtime == "crio":
        configure_crio(config, binaries, default)
    else:
        raise ValueError(f"unsupported runtime {runtime!r}")


def revert(runtime: str, config: str, state_file: str = "") -> None:
    state_file = state_file or config + ".amd-state.json"
    if runtime == "containerd":
        revert_containerd(config, state_file)
    elif runtime == "docker":
        revert_docker(config, state_file)
    elif runtime == "crio":
        revert_crio(config)
    else:
        raise ValueError(f"unsupported runtime {runtime!r}")


def set_containerd_runtimes(config: str, runtimes: Dict[str, Dict[str, Any]]) -> bool:
    """Upsert arbitrary containerd runtime handlers (used by the kata manager). True if changed."""
    doc: Dict[str, Any] = {}
    if os.path.exists(config):
        with open(config, "rb") as f:
            doc = tomli.load(f)
    doc.setdefault("version", 2)
    rts = _dig(doc, _cri_path(doc)).setdefault("containerd", {}).setdefault("runtimes", {})
    changed = False
    for name, h in runtimes.items():
        if rts.get(name) != h:
            rts[name] = h
            changed = True
    if changed:
        _write(config, tomlw.dumps(doc))
    return changed


def remove_containerd_runtimes(config: str, names: List[str]) -> bool:
    if not os.path.exists(config):
        return False
    with open(config, "rb") as f:
        doc = tomli.load(f)
    rts = _dig(doc, _cri_path(doc)).setdefault("containerd", {}).setdefault("runtimes", {})
    gone = [n for n in names if rts.pop(n, None) is not None]
    if gone:
        _write(config, tomlw.dumps(doc))
    return bool(gone)
