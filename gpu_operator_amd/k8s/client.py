"""The Kubernetes client interface the operator and node agents are written against.

Two implementations: :class:`gpu_operator_amd.k8s.fake.FakeClient` (in-memory, used by unit
tests, envtest-style multi-node simulations and fault injection) and
:class:`gpu_operator_amd.k8s.rest.RestClient` (the API server over HTTPS).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Protocol

Obj = Dict[str, Any]

ADDED, MODIFIED, DELETED = "ADDED", "MODIFIED", "DELETED"


@dataclass
class WatchEvent:
    type: str            # ADDED | MODIFIED | DELETED
    obj: Obj
    old: Optional[Obj] = None


WatchCallback = Callable[[WatchEvent], None]


class Client(Protocol):
    def get(self, api_version: str, kind: str, name: str, namespace: str = "") -> Obj: ...

    def list(self, api_version: str, kind: str, namespace: str = "",
             label_selector: Any = None, field_selector: Optional[str] = None) -> List[Obj]: ...

    def create(self, obj: Obj) -> Obj: ...

    def update(self, obj: Obj) -> Obj: ...

    def update_status(self, obj: Obj) -> Obj: ...

    def patch(self, api_version: str, kind: str, name: str, patch: Obj, namespace: str = "",
              patch_type: str = "merge") -> Obj: ...

    def delete(self, api_version: str, kind: str, name: str, namespace: str = "",
               propagation: Optional[str] = None, grace_period_seconds: Optional[int] = None) -> None: ...

    def evict(self, name: str, namespace: str, grace_period_seconds: Optional[int] = None) -> None: ...

    def has_kind(self, api_version: str, kind: str) -> bool: ...

    def server_version(self) -> str: ...

    def watch(self, api_version: str, kind: str, callback: WatchCallback,
              namespace: str = "", field_selector: Optional[str] = None) -> Callable[[], None]: ...

    def create_event(self, involved: Obj, reason: str, message: str, type_: str = "Normal") -> None: ...


def merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return patch
    out = dict(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out
