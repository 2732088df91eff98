"""Declarative typed specs for CRDs: one definition drives parsing, defaulting, validation,
serialisation and the OpenAPI v3 schema of the generated CustomResourceDefinition.

This plays the role kubebuilder markers + controller-gen + generated deepcopy play for the
reference (reference: api/v1/clusterpolicy_types.go, api/v1/zz_generated.deepcopy.go,
config/crd/bases/*): a spec class is a dataclass whose fields carry their JSON name,
documentation and validation markers in ``metadata``.

Design rules:
  * every field is optional in Python (``None`` = unset), so "unset" and "false" differ the
    way ``*bool`` does in the reference and defaults live in ``is_enabled()``-style helpers;
  * unknown keys are rejected in strict mode (``from_dict(strict=True)``) and kept in
    ``_extra`` otherwise, so a newer CR round-trips through an older operator;
  * free-form Kubernetes sub-objects (tolerations, resources, relabelings) are typed ``Any``
    and emitted with ``x-kubernetes-preserve-unknown-fields``.
"""

from __future__ import annotations

import copy
import dataclasses
import re
import typing
from typing import Any, Dict, List, Optional, Tuple, Type, TypeVar, get_args, get_origin

T = TypeVar("T", bound="Spec")


class ValidationError(ValueError):
    """A CR field violates its schema (path-qualified message)."""


class IntOrString:
    """Type marker for Kubernetes ``intstr.IntOrString`` / quantity fields: the value is kept as
    given (int or str) and the schema carries ``x-kubernetes-int-or-string``."""


def field(json: Optional[str] = None, *, doc: str = "", enum: Optional[List[Any]] = None,
          pattern: Optional[str] = None, minimum: Optional[int] = None,
          maximum: Optional[int] = None, aliases: Tuple[str, ...] = (),
          required: bool = False, default: Any = None, default_factory: Any = None,
          schema_default: Any = None):
    """Declare a spec field. ``default`` is the *Python* initial value (normally ``None``);
    ``schema_default`` is published in the CRD (applied by the API server)."""
    md = {"json": json, "doc": doc, "enum": enum, "pattern": pattern, "minimum": minimum,
          "maximum": maximum, "aliases": tuple(aliases), "required": required,
          "schema_default": schema_default}
    if default_factory is not None:
        return dataclasses.field(default_factory=default_factory, metadata=md)
    return dataclasses.field(default=default, metadata=md)


def _json_name(f: dataclasses.Field) -> str:
    return f.metadata.get("json") or f.name


def _unwrap_optional(tp):
    if get_origin(tp) is typing.Union:
        args = [a for a in get_args(tp) if a is not type(None)]
        if len(args) == 1:
            return args[0]
    return tp


class Spec:
    """Base class for typed CR sub-objects (subclasses must be ``@dataclass``)."""

    _extra: Dict[str, Any]

    # -- introspection ------------------------------------------------------------------
    @classmethod
    def _fields(cls) -> List[Tuple[dataclasses.Field, Any]]:
        hints = typing.get_type_hints(cls)
        return [(f, _unwrap_optional(hints[f.name])) for f in dataclasses.fields(cls)
                if not f.name.startswith("_")]

    @classmethod
    def _key_map(cls) -> Dict[str, Tuple[dataclasses.Field, Any]]:
        m: Dict[str, Tuple[dataclasses.Field, Any]] = {}
        for f, tp in cls._fields():
            m[_json_name(f)] = (f, tp)
            for a in f.metadata.get("aliases", ()):
                m[a] = (f, tp)
        return m

    # -- parsing --------------------------------------------------------------------------
    @classmethod
    def from_dict(cls: Type[T], data: Optional[Dict[str, Any]], strict: bool = False,
                  path: str = "") -> T:
        data = data or {}
        if not isinstance(data, dict):
            raise ValidationError(f"{path or cls.__name__}: expected object, got {type(data).__name__}")
        kwargs: Dict[str, Any] = {}
        extra: Dict[str, Any] = {}
        keymap = cls._key_map()
        for key, val in data.items():
            if key not in keymap:
                if strict:
                    raise ValidationError(f"{path}.{key}: unknown field" if path else f"{key}: unknown field")
                extra[key] = copy.deepcopy(val)
                continue
            f, tp = keymap[key]
            sub = f"{path}.{key}" if path else key
            if val is None:
                continue
            kwargs[f.name] = _coerce(tp, val, strict, sub)
            _check_markers(f, kwargs[f.name], sub)
        obj = cls(**kwargs)  # type: ignore[call-arg]
        object.__setattr__(obj, "_extra", extra)
        for f, _ in cls._fields():
            if f.metadata.get("required") and getattr(obj, f.name) is None:
                raise ValidationError(f"{path + '.' if path else ''}{_json_name(f)}: required")
        return obj

    # -- serialisation ------------------------------------------------------------------
    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {}
        for f, tp in self._fields():
            v = getattr(self, f.name)
            if v is None:
                continue
            enc = _encode(v)
            if enc == {} and isinstance(v, Spec):
                # keep explicitly-set empty sub-objects only if they carry extra keys
                continue
            out[_json_name(f)] = enc
        out.update(copy.deepcopy(getattr(self, "_extra", {}) or {}))
        return out

    def deepcopy(self: T) -> T:
        return type(self).from_dict(self.to_dict())

    # -- OpenAPI ------------------------------------------------------------------------
    @classmethod
    def openapi(cls) -> Dict[str, Any]:
        props: Dict[str, Any] = {}
        required: List[str] = []
        for f, tp in cls._fields():
            s = _type_schema(tp)
            md = f.metadata
            if md.get("doc"):
                s["description"] = md["doc"]
            if md.get("enum"):
                s["enum"] = list(md["enum"])
            if md.get("pattern"):
                s["pattern"] = md["pattern"]
            if md.get("minimum") is not None:
                s["minimum"] = md["minimum"]
            if md.get("maximum") is not None:
                s["maximum"] = md["maximum"]
            if md.get("schema_default") is not None:
                s["default"] = md["schema_default"]
            props[_json_name(f)] = s
            if md.get("required"):
                required.append(_json_name(f))
        doc = (cls.__doc__ or "").strip().split("\n\n")[0].replace("\n", " ")
        out: Dict[str, Any] = {"type": "object", "properties": props}
        if doc:
            out["description"] = doc
        if required:
            out["required"] = required
        return out


def _check_markers(f: dataclasses.Field, v: Any, path: str) -> None:
    md = f.metadata
    if md.get("enum") and v not in md["enum"]:
        raise ValidationError(f"{path}: {v!r} not in {md['enum']}")
    if md.get("pattern") and isinstance(v, str) and v and not re.fullmatch(md["pattern"], v):
        raise ValidationError(f"{path}: {v!r} does not match {md['pattern']}")
    if md.get("minimum") is not None and isinstance(v, int) and v < md["minimum"]:
        raise ValidationError(f"{path}: {v} < minimum {md['minimum']}")
    if md.get("maximum") is not None and isinstance(v, int) and v > md["maximum"]:
        raise ValidationError(f"{path}: {v} > maximum {md['maximum']}")


def _coerce(tp, val, strict: bool, path: str):
    origin = get_origin(tp)
    if tp is Any:
        return copy.deepcopy(val)
    if tp is IntOrString:
        if isinstance(val, bool) or not isinstance(val, (int, str)):
            raise ValidationError(f"{path}: expected integer or string, got {val!r}")
        return val
    if isinstance(tp, type) and issubclass(tp, Spec):
        return tp.from_dict(val, strict=strict, path=path)
    if origin in (list, List):
        (et,) = get_args(tp) or (Any,)
        if not isinstance(val, list):
            raise ValidationError(f"{path}: expected list")
        return [_coerce(_unwrap_optional(et), x, strict, f"{path}[{i}]") for i, x in enumerate(val)]
    if origin in (dict, Dict):
        kt, vt = get_args(tp) or (str, Any)
        if not isinstance(val, dict):
            raise ValidationError(f"{path}: expected object")
        return {str(k): _coerce(_unwrap_optional(vt), v, strict, f"{path}.{k}") for k, v in val.items()}
    if tp is bool:
        if isinstance(val, bool):
            return val
        if isinstance(val, str) and val.lower() in ("true", "false"):
            return val.lower() == "true"
        raise ValidationError(f"{path}: expected boolean, got {val!r}")
    if tp is int:
        if isinstance(val, bool):
            raise ValidationError(f"{path}: expected integer, got boolean")
        if isinstance(val, int):
            return val
        if isinstance(val, str) and re.fullmatch(r"-?\d+", val):
            return int(val)
        raise ValidationError(f"{path}: expected integer, got {val!r}")
    if tp is str:
        if isinstance(val, (str, int, float)) and not isinstance(val, bool):
            return str(val)
        raise ValidationError(f"{path}: expected string, got {val!r}")
    return val


def _encode(v):
    if isinstance(v, Spec):
        return v.to_dict()
    if isinstance(v, list):
        return [_encode(x) for x in v]
    if isinstance(v, dict):
        return {k: _encode(x) for k, x in v.items()}
    return copy.deepcopy(v)


def _type_schema(tp) -> Dict[str, Any]:
    origin = get_origin(tp)
    if tp is Any:
        return {"x-kubernetes-preserve-unknown-fields": True}
    if tp is IntOrString:
        return {"x-kubernetes-int-or-string": True, "anyOf": [{"type": "integer"}, {"type": "string"}]}
    if isinstance(tp, type) and issubclass(tp, Spec):
        return tp.openapi()
    if origin in (list, List):
        (et,) = get_args(tp) or (Any,)
        return {"type": "array", "items": _type_schema(_unwrap_optional(et))}
    if origin in (dict, Dict):
        _, vt = get_args(tp) or (str, Any)
        return {"type": "object", "additionalProperties": _type_schema(_unwrap_optional(vt))}
    if tp is bool:
        return {"type": "boolean"}
    if tp is int:
        return {"type": "integer", "format": "int32"}
    if tp is str:
        return {"type": "string"}
    return {"x-kubernetes-preserve-unknown-fields": True}
