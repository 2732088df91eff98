"""OpenAPI v3 schema semantics of apiextensions.k8s.io/v1 CustomResourceDefinitions, as the
Kubernetes API server applies them to custom resources -- so the CRD this repo generates is
checked the way a real cluster would check it (round-1 review: "the CRD schema has never been
checked by any API server"):

* :func:`structural_errors` -- the structural-schema rules a v1 CRD must satisfy before the
  API server accepts it (every node typed unless ``x-kubernetes-int-or-string`` or
  ``x-kubernetes-preserve-unknown-fields``; arrays with a single ``items`` schema; no
  ``properties`` next to ``additionalProperties``; ``anyOf`` only in the int-or-string form;
  no ``$ref``/``definitions``/``dependencies``/``patternProperties``/``additionalItems``/
  ``uniqueItems: true``; enums and defaults that validate against their own node);
* :func:`prune` -- unknown fields are dropped unless a node preserves them;
* :func:`apply_defaults` -- ``default`` fills an absent field of a present object;
* :func:`validate` -- type, int-or-string, enum, minimum/maximum, pattern, length, required,
  nullable; messages in the API server's ``<path>: Invalid value: ...`` style.

The order on create/update is the API server's: prune, default, validate.
"""

from __future__ import annotations

import copy
import re
from typing import Any, Dict, List

Schema = Dict[str, Any]

_FORBIDDEN = ("$ref", "definitions", "dependencies", "patternProperties", "additionalItems", "id", "$schema")
_TYPES = {"object", "array", "string", "integer", "number", "boolean"}


def _int_or_string(s: Schema) -> bool:
    return bool(s.get("x-kubernetes-int-or-string"))


def _preserve(s: Schema) -> bool:
    return bool(s.get("x-kubernetes-preserve-unknown-fields"))


# ---------------------------------------------------------------------------------------------
# structural schema
# ---------------------------------------------------------------------------------------------
def structural_errors(s: Schema, path: str = "") -> List[str]:
    errs: List[str] = []
    p = path or "<root>"
    if not isinstance(s, dict):
        return [f"{p}: schema must be an object"]
    for k in _FORBIDDEN:
        if k in s:
            errs.append(f"{p}: {k} is forbidden in a structural schema")
    if s.get("uniqueItems") is True:
        errs.append(f"{p}: uniqueItems cannot be true")
    t = s.get("type")
    if t is not None and t not in _TYPES:
        errs.append(f"{p}.type: unsupported value {t!r}")
    if _int_or_string(s):
        if t is not None:
            errs.append(f"{p}: type must be empty with x-kubernetes-int-or-string")
        any_of = s.get("anyOf")
        if any_of is not None:
            kinds = sorted(x.get("type", "") for x in any_of if isinstance(x, dict))
            if kinds != ["integer", "string"]:
                errs.append(f"{p}.anyOf: with x-kubernetes-int-or-string only integer|string is allowed")
    elif not t and not _preserve(s):
        errs.append(f"{p}.type: Required value: must not be empty for specified fields")
    elif "anyOf" in s or "oneOf" in s or "allOf" in s:
        for key in ("anyOf", "oneOf", "allOf"):
            for i, sub in enumerate(s.get(key) or []):
                if isinstance(sub, dict) and ("type" in sub or "properties" in sub or "items" in sub
                                              or "default" in sub or "description" in sub):
                    errs.append(f"{p}.{key}[{i}]: must only have value validations (no type/properties/"
                                "items/default/description)")
    if "properties" in s and "additionalProperties" in s and s["additionalProperties"] is not False:
        errs.append(f"{p}: additionalProperties and properties are mutually exclusive")
    if t == "array":
        items = s.get("items")
        if not isinstance(items, dict):
            errs.append(f"{p}.items: Required value: must be a single schema for arrays")
        else:
            errs += structural_errors(items, f"{path}.items" if path else "items")
    elif "items" in s:
        errs.append(f"{p}.items: only allowed for type array")
    for name, sub in (s.get("properties") or {}).items():
        errs += structural_errors(sub, f"{path}.properties[{name}]" if path else f"properties[{name}]")
    ap = s.get("additionalProperties")
    if isinstance(ap, dict):
        errs += structural_errors(ap, f"{path}.additionalProperties" if path else "additionalProperties")
    if "enum" in s and not (_preserve(s) and not t):
        for v in s["enum"]:
            e = _check_type(v, s, p)
            if e:
                errs.append(f"{p}.enum: {v!r} {e}")
    if "default" in s:
        errs += [f"{p}.default: {e}" for e in validate(copy.deepcopy(s["default"]), s, "")]
    return errs


# ---------------------------------------------------------------------------------------------
# pruning and defaulting
# ---------------------------------------------------------------------------------------------
def prune(obj: Any, s: Schema) -> Any:
    """Drop fields the schema does not know (in place; returns obj)."""
    if isinstance(obj, dict):
        if _preserve(s) and "properties" not in s and "additionalProperties" not in s:
            return obj
        props = s.get("properties")
        ap = s.get("additionalProperties")
        for k in list(obj):
            if props is not None and k in props:
                prune(obj[k], props[k])
            elif isinstance(ap, dict):
                prune(obj[k], ap)
            elif ap is True or _preserve(s):
                continue
            elif props is not None or ap is False:
                del obj[k]
    elif isinstance(obj, list) and isinstance(s.get("items"), dict):
        for x in obj:
            prune(x, s["items"])
    return obj


def apply_defaults(obj: Any, s: Schema) -> Any:
    """Fill ``default`` into absent fields of present objects (in place; returns obj)."""
    if isinstance(obj, dict):
        for k, sub in (s.get("properties") or {}).items():
            if k not in obj and "default" in sub:
                obj[k] = copy.deepcopy(sub["default"])
            if k in obj and obj[k] is not None:
                apply_defaults(obj[k], sub)
        ap = s.get("additionalProperties")
        if isinstance(ap, dict):
            for k in obj:
                if not (s.get("properties") and k in s["properties"]):
                    apply_defaults(obj[k], ap)
    elif isinstance(obj, list) and isinstance(s.get("items"), dict):
        for x in obj:
            apply_defaults(x, s["items"])
    return obj


# ---------------------------------------------------------------------------------------------
# validation
# ---------------------------------------------------------------------------------------------
def _check_type(v: Any, s: Schema, path: str) -> str:
    if _int_or_string(s):
        return "" if (isinstance(v, (int, str)) and not isinstance(v, bool)) else "must be an integer or a string"
    t = s.get("type")
    if not t:
        return ""
    ok = {"object": isinstance(v, dict), "array": isinstance(v, list), "string": isinstance(v, str),
          "integer": isinstance(v, int) and not isinstance(v, bool),
          "number": isinstance(v, (int, float)) and not isinstance(v, bool),
          "boolean": isinstance(v, bool)}[t]
    return "" if ok else f"must be of type {t}"


def validate(v: Any, s: Schema, path: str = "") -> List[str]:
    p = path or "<root>"
    if v is None:
        return [] if s.get("nullable") else [f"{p}: Invalid value: \"null\": {p} in body must be of type "
                                             f"{s.get('type') or 'any'}"]
    e = _check_type(v, s, p)
    if e:
        return [f"{p}: Invalid value: {v!r}: {p} in body {e}"]
    errs: List[str] = []
    if "enum" in s and v not in s["enum"]:
        errs.append(f"{p}: Unsupported value: {v!r}: supported values: {', '.join(repr(x) for x in s['enum'])}")
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        if "minimum" in s and v < s["minimum"]:
            errs.append(f"{p}: Invalid value: {v}: {p} in body should be greater than or equal to {s['minimum']}")
        if "maximum" in s and v > s["maximum"]:
            errs.append(f"{p}: Invalid value: {v}: {p} in body should be less than or equal to {s['maximum']}")
    if isinstance(v, str):
        if "pattern" in s and not re.search(s["pattern"], v):
            errs.append(f"{p}: Invalid value: {v!r}: {p} in body should match '{s['pattern']}'")
        if "maxLength" in s and len(v) > s["maxLength"]:
            errs.append(f"{p}: Too long: may not be longer than {s['maxLength']}")
        if "minLength" in s and len(v) < s["minLength"]:
            errs.append(f"{p}: Invalid value: {v!r}: {p} in body should be at least {s['minLength']} chars long")
    if isinstance(v, dict):
        props = s.get("properties") or {}
        for r in s.get("required") or []:
            if r not in v:
                errs.append(f"{path + '.' if path else ''}{r}: Required value")
        for k, x in v.items():
            sub = props.get(k)
            if sub is None and isinstance(s.get("additionalProperties"), dict):
                sub = s["additionalProperties"]
            if sub is not None:
                errs += validate(x, sub, f"{path}.{k}" if path else k)
    if isinstance(v, list) and isinstance(s.get("items"), dict):
        for i, x in enumerate(v):
            errs += validate(x, s["items"], f"{p}[{i}]")
        if "maxItems" in s and len(v) > s["maxItems"]:
            errs.append(f"{p}: Too many: {len(v)}: must have at most {s['maxItems']} items")
    return errs


def admit(obj: Dict[str, Any], s: Schema) -> List[str]:
    """What the API server does to a custom resource on create/update: prune, default, validate
    (``metadata``/``apiVersion``/``kind`` are the server's own). Mutates ``obj``; returns errors."""
    body = {k: v for k, v in obj.items() if k not in ("metadata", "apiVersion", "kind")}
    prune(body, s)
    apply_defaults(body, s)
    errs = validate(body, s, "")
    for k in [k for k in obj if k not in ("metadata", "apiVersion", "kind")]:
        del obj[k]
    obj.update(body)
    return errs
