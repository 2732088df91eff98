"""Driver auto-upgrade policy (the role of the reference's vendored k8s-operator-libs
``DriverUpgradePolicySpec``; reference: vendor/github.com/NVIDIA/k8s-operator-libs/api/upgrade/
v1alpha1/upgrade_spec.go:26-110). Same fields and defaults, owned by this project."""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Union

from ..schema import IntOrString, Spec, field


@dataclass
class PodDeletionSpec(Spec):
    """Deletion of pods that use amd.com/gpu resources before the driver restarts."""

    force: Optional[bool] = field("force", schema_default=False)
    timeoutSeconds: Optional[int] = field("timeoutSeconds", minimum=0, schema_default=300)
    deleteEmptyDir: Optional[bool] = field("deleteEmptyDir", schema_default=False)

    def timeout(self) -> int:
        return 300 if self.timeoutSeconds is None else self.timeoutSeconds


@dataclass
class WaitForCompletionSpec(Spec):
    """Wait for selected jobs on the node to finish before the upgrade proceeds."""

    podSelector: Optional[str] = field("podSelector")
    timeoutSeconds: Optional[int] = field("timeoutSeconds", minimum=0, schema_default=0)

    def timeout(self) -> int:
        return self.timeoutSeconds or 0


@dataclass
class DrainSpec(Spec):
    """Node drain during the upgrade."""

    enable: Optional[bool] = field("enable", schema_default=False)
    force: Optional[bool] = field("force", schema_default=False)
    podSelector: Optional[str] = field("podSelector")
    timeoutSeconds: Optional[int] = field("timeoutSeconds", minimum=0, schema_default=300)
    deleteEmptyDir: Optional[bool] = field("deleteEmptyDir", schema_default=False)

    def timeout(self) -> int:
        return 300 if self.timeoutSeconds is None else self.timeoutSeconds


@dataclass
class DriverUpgradePolicySpec(Spec):
    """Rolling, node-by-node amdgpu driver upgrade."""

    autoUpgrade: Optional[bool] = field("autoUpgrade", schema_default=False)
    maxParallelUpgrades: Optional[int] = field("maxParallelUpgrades", minimum=0, schema_default=1)
    maxUnavailable: Optional[IntOrString] = field("maxUnavailable", schema_default="25%",
                                          doc="Absolute number (e.g. 5) or percentage (e.g. 10%).")
    podDeletion: Optional[PodDeletionSpec] = field("podDeletion")
    waitForCompletion: Optional[WaitForCompletionSpec] = field("waitForCompletion")
    drain: Optional[DrainSpec] = field("drain")

    def max_parallel(self) -> int:
        return 1 if self.maxParallelUpgrades is None else self.maxParallelUpgrades

    def max_unavailable_nodes(self, total: int) -> int:
        """Resolve maxUnavailable against ``total`` nodes (percentages round up)."""
        return resolve_int_or_percent(self.maxUnavailable if self.maxUnavailable is not None else "25%",
                                      total)


def resolve_int_or_percent(v: Union[str, int], total: int) -> int:
    s = str(v).strip()
    if s.endswith("%"):
        return int(math.ceil(float(s[:-1]) * total / 100.0))
    return int(s)
