"""Small TOML emitter for container-runtime configs (reading uses ``tomli``).

Covers what containerd / CRI-O configs contain: nested tables, arrays of scalars, arrays of
tables, strings, booleans, integers and floats. Scalars of a table are written before its
sub-tables so the output re-parses to the same document.
"""

from __future__ import annotations

import re
from typing import Any, Dict, List

_BARE = re.compile(r"^[A-Za-z0-9_-]+$")


def _key(k: str) -> str:
    return k if _BARE.match(k) else _str(k)


def _str(s: str) -> str:
    out = s.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n").replace("\t", "\\t")
    return f'"{out}"'


def _scalar(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return repr(v)
    if isinstance(v, str):
        return _str(v)
    if isinstance(v, list):
        return "[" + ", ".join(_scalar(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ", ".join(f"{_key(k)} = {_scalar(x)}" for k, x in v.items()) + "}"
    raise TypeError(f"cannot encode {type(v).__name__} in TOML")


def _is_table_array(v: Any) -> bool:
    return isinstance(v, list) and len(v) > 0 and all(isinstance(x, dict) for x in v)


def dumps(doc: Dict[str, Any]) -> str:
    lines: List[str] = []

    def emit(table: Dict[str, Any], path: List[str]) -> None:
        scalars = [(k, v) for k, v in table.items() if not isinstance(v, dict) and not _is_table_array(v)]
        subs = [(k, v) for k, v in table.items() if isinstance(v, dict)]
        arrays = [(k, v) for k, v in table.items() if _is_table_array(v)]
        if path and (scalars or not subs and not arrays):
            lines.append("")
            lines.append("[" + ".".join(_key(p) for p in path) + "]")
        for k, v in scalars:
            lines.append(f"{_key(k)} = {_scalar(v)}")
        for k, v in subs:
            emit(v, path + [k])
        for k, arr in arrays:
            for item in arr:
                lines.append("")
                lines.append("[[" + ".".join(_key(p) for p in path + [k]) + "]]")
                for ik, iv in item.items():
                    lines.append(f"{_key(ik)} = {_scalar(iv)}")

    emit(doc, [])
    return "\n".join(lines).lstrip("\n") + "\n"
