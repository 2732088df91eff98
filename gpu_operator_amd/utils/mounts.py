"""Container mount emulation: where a container path lives on this machine.

In a pod every agent finds its volumes at fixed container paths (``/run/amd/validations``,
``/var/lib/kubelet/device-plugins``, ``/host``, ...). The process-level node harnesses
(``e2e/kubelet.py``, ``validator/ttr.py``) run the same agents as plain processes. Their kubelet
passes a container's volume mounts in ``AMD_MOUNTS``, a JSON list of ``[container_path,
host_path]`` pairs. Every built-in default path an agent opens goes through :func:`path`.
Paths that come from the pod spec (args, env values, ConfigMap scripts) are rewritten by that
kubelet with the same table.

With ``AMD_MOUNTS`` unset (a real container) :func:`path` is the identity.
"""

from __future__ import annotations

import json
import os
from typing import List, Optional, Tuple

_cache: Tuple[Optional[str], List[Tuple[str, str]]] = (None, [])


def table() -> List[Tuple[str, str]]:
    """The mount table of this process, longest container path first."""
    global _cache
    raw = os.environ.get("AMD_MOUNTS")
    if raw == _cache[0]:
        return _cache[1]
    pairs: List[Tuple[str, str]] = []
    if raw:
        for cpath, hpath in json.loads(raw):
            cpath = "/" + str(cpath).strip("/") if str(cpath).strip("/") else "/"
            pairs.append((cpath, str(hpath)))
    pairs.sort(key=lambda p: len(p[0]), reverse=True)
    _cache = (raw, pairs)
    return pairs


def translate(p: str, pairs: Optional[List[Tuple[str, str]]] = None) -> str:
    """Map container path ``p`` through ``pairs`` (longest matching mount wins)."""
    if not p or not p.startswith("/"):
        return p
    for cpath, hpath in (table() if pairs is None else pairs):
        if cpath == "/":
            return os.path.join(hpath, p.lstrip("/")) if p != "/" else hpath
        if p == cpath:
            return hpath
        if p.startswith(cpath + "/"):
            return hpath.rstrip("/") + p[len(cpath):]
    return p


def path(p: str) -> str:
    """The host location of container path ``p`` for this process."""
    return translate(p)


def rewrite_text(text: str, pairs: List[Tuple[str, str]]) -> str:
    """Rewrite every absolute path in a script or argument that starts with a mount's container
    path (the root mount excepted), in one pass so a rewritten path is never rewritten again.
    The match must start a path (no path character before it) and end at a component boundary."""
    import re
    mounts = {c: h.rstrip("/") for c, h in pairs if c != "/"}
    if not mounts:
        return text
    alts = "|".join(re.escape(c) for c in sorted(mounts, key=len, reverse=True))
    rx = re.compile(r"(?<![\w./-])(" + alts + r")(?=$|[/\s\"':;)=])")
    return rx.sub(lambda m: mounts[m.group(1)], text)
