"""Asset loader: a state directory of ``NNNN_<kind>.yaml`` manifests -> ordered object list.

Counterpart of the reference's resource manager (reference: controllers/resource_manager.go:
70-187): files are applied in filename order, ``*openshift*`` files only on OpenShift. Unlike
the reference, every object of every kind is kept (the reference holds one slot per kind and
drops the second Role of a state), and a file may hold several
YAML documents.
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional

import yaml

from ..k8s import objects as o

DEFAULT_ASSETS = Path(__file__).resolve().parent.parent / "assets"


@dataclass
class State:
    name: str
    path: str
    objects: List[Dict[str, Any]] = field(default_factory=list)


def assets_dir() -> Path:
    return Path(os.environ.get("AMD_GPU_OPERATOR_ASSETS", str(DEFAULT_ASSETS)))


def load_state(name: str, base: Optional[Path] = None, openshift: bool = False) -> State:
    d = (base or assets_dir()) / name
    if not d.is_dir():
        raise FileNotFoundError(f"state directory {d} missing")
    st = State(name=name, path=str(d))
    for f in sorted(d.iterdir()):
        if f.suffix not in (".yaml", ".yml") or not f.is_file():
            continue
        if "openshift" in f.name and not openshift:
            continue
        with open(f) as fh:
            for doc in yaml.safe_load_all(fh):
                if not doc:
                    continue
                if "kind" not in doc:
                    raise ValueError(f"{f}: manifest without kind")
                doc.setdefault("apiVersion", o.api_version_of(doc["kind"]))
                doc.setdefault("metadata", {})["annotations"] = dict(
                    doc["metadata"].get("annotations") or {})
                doc["metadata"]["annotations"].setdefault("amd.com/asset", f"{name}/{f.name}")
                st.objects.append(doc)
    return st


def load_states(names: List[str], base: Optional[Path] = None, openshift: bool = False) -> List[State]:
    return [load_state(n, base, openshift) for n in names]
