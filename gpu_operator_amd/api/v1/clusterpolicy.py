"""``amd.com/v1`` ClusterPolicy: the single source of truth for every operand on every GPU node.

Same key surface as the reference's ``nvidia.com/v1`` ClusterPolicy
(reference: api/v1/clusterpolicy_types.go:36-84, status :1510-1516), re-targeted at AMD
Instinct operands:

    reference key        -> amd.com/v1 key        (reference key still accepted as alias)
    dcgm                 -> rdc                    RDC daemon (rdcd) instead of DCGM hostengine
    dcgmExporter         -> metricsExporter        amd-smi/RDC Prometheus exporter
    gfd                  -> nodeLabeller           sysfs/KFD node-feature labeller
    mig                  -> partition              compute/memory partition strategy
    migManager           -> partitionManager       SPX/DPX/QPX/CPX x NPS1/NPS4 manager
    vgpuManager          -> mxgpuManager           MxGPU (SR-IOV) host driver
    vgpuDeviceManager    -> mxgpuDeviceManager     MxGPU VF profile manager
    validator.cuda       -> validator.hip          MFMA GEMM probe replaces vectorAdd
    (new)                   validator.rccl         RCCL all-reduce over xGMI

``gds`` has no mature ROCm equivalent: the key is accepted, and enabling it is reported as
unsupported instead of silently ignored.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, ClassVar, Dict, List, Optional

from ..schema import IntOrString, Spec, ValidationError, field
from .upgrade import DriverUpgradePolicySpec

GROUP = "amd.com"
VERSION = "v1"
API_VERSION = f"{GROUP}/{VERSION}"
KIND = "ClusterPolicy"
PLURAL = "clusterpolicies"

# ClusterPolicy status states (reference: api/v1/clusterpolicy_types.go:1496-1507)
STATE_IGNORED = "ignored"
STATE_READY = "ready"
STATE_NOT_READY = "notReady"

IMAGE_PATTERN = r"[a-zA-Z0-9\-]+"
PULL_POLICIES = ["Always", "IfNotPresent", "Never"]
RUNTIMES = ["docker", "crio", "containerd"]
WORKLOADS = ["container", "vm-passthrough", "vm-mxgpu"]
PARTITION_STRATEGIES = ["none", "single", "mixed"]


def _b(v: Optional[bool], default: bool) -> bool:
    return default if v is None else bool(v)


@dataclass
class EnvVar(Spec):
    """An environment variable injected into an operand container."""

    name: Optional[str] = field("name", required=True, doc="Name of the environment variable.")
    value: Optional[str] = field("value", doc="Value of the environment variable.")


@dataclass
class ResourceRequirements(Spec):
    """Compute resources of an operand container."""

    limits: Optional[Dict[str, IntOrString]] = field("limits", doc="Maximum resources allowed.")
    requests: Optional[Dict[str, IntOrString]] = field("requests", doc="Minimum resources required.")


@dataclass
class ImageSpec(Spec):
    """Image coordinates shared by every operand (repository/image:version or @sha256)."""

    IMAGE_ENV: ClassVar[str] = ""

    repository: Optional[str] = field("repository", doc="Image repository.")
    image: Optional[str] = field("image", pattern=IMAGE_PATTERN, doc="Image name.")
    version: Optional[str] = field("version", doc="Image tag or sha256 digest.")
    imagePullPolicy: Optional[str] = field("imagePullPolicy", enum=PULL_POLICIES,
                                           doc="Image pull policy.")
    imagePullSecrets: Optional[List[str]] = field("imagePullSecrets", doc="Image pull secrets.")


@dataclass
class ComponentSpec(ImageSpec):
    """An operand: image + enable switch + container knobs."""

    DEFAULT_ENABLED: ClassVar[bool] = True

    enabled: Optional[bool] = field("enabled", doc="Deploy this operand.")
    resources: Optional[ResourceRequirements] = field("resources", doc="Container resources.")
    args: Optional[List[str]] = field("args", doc="Optional container arguments.")
    env: Optional[List[EnvVar]] = field("env", doc="Optional container environment.")

    def is_enabled(self) -> bool:
        return _b(self.enabled, self.DEFAULT_ENABLED)


# --------------------------------------------------------------------------------------------
# operator / daemonsets / common
# --------------------------------------------------------------------------------------------
@dataclass
class InitContainerSpec(ImageSpec):
    """Base image used by small operator-injected init containers (ROCm base image)."""

    IMAGE_ENV: ClassVar[str] = "ROCM_BASE_IMAGE"


@dataclass
class OperatorSpec(Spec):
    """Operator-wide settings."""

    defaultRuntime: Optional[str] = field("defaultRuntime", enum=RUNTIMES, schema_default="containerd",
                                          doc="Container runtime assumed when a node does not report one.")
    runtimeClass: Optional[str] = field("runtimeClass", schema_default="amd",
                                        doc="RuntimeClass handler configured by the toolkit.")
    initContainer: Optional[InitContainerSpec] = field("initContainer")
    labels: Optional[Dict[str, str]] = field("labels", doc="Labels added to operand pods.")
    annotations: Optional[Dict[str, str]] = field("annotations", doc="Annotations added to operand pods.")
    use_ocp_driver_toolkit: Optional[bool] = field(
        "use_ocp_driver_toolkit", doc="On OpenShift, build amdgpu with the Driver Toolkit image.")

    def default_runtime(self) -> str:
        return self.defaultRuntime or "containerd"

    def runtime_class(self) -> str:
        return self.runtimeClass or "amd"


@dataclass
class RollingUpdateSpec(Spec):
    """Rolling-update knobs of operand DaemonSets."""

    maxUnavailable: Optional[str] = field("maxUnavailable", doc="Absolute number or percentage.")


@dataclass
class DaemonsetsSpec(Spec):
    """Settings applied to every operand DaemonSet."""

    labels: Optional[Dict[str, str]] = field("labels")
    annotations: Optional[Dict[str, str]] = field("annotations")
    tolerations: Optional[List[Any]] = field("tolerations")
    priorityClassName: Optional[str] = field("priorityClassName", schema_default="system-node-critical")
    updateStrategy: Optional[str] = field("updateStrategy", enum=["RollingUpdate", "OnDelete"],
                                          schema_default="RollingUpdate")
    rollingUpdate: Optional[RollingUpdateSpec] = field("rollingUpdate")


@dataclass
class ContainerProbeSpec(Spec):
    """Probe timing of the driver container."""

    initialDelaySeconds: Optional[int] = field("initialDelaySeconds", minimum=0)
    timeoutSeconds: Optional[int] = field("timeoutSeconds", minimum=1)
    periodSeconds: Optional[int] = field("periodSeconds", minimum=1)
    successThreshold: Optional[int] = field("successThreshold", minimum=1)
    failureThreshold: Optional[int] = field("failureThreshold", minimum=1)


@dataclass
class PSPSpec(Spec):
    """PodSecurityPolicy for operands (Kubernetes < 1.25 only)."""

    enabled: Optional[bool] = field("enabled")

    def is_enabled(self) -> bool:
        return _b(self.enabled, False)


@dataclass
class PSASpec(Spec):
    """Pod Security Admission labels on the operator namespace."""

    enabled: Optional[bool] = field("enabled")

    def is_enabled(self) -> bool:
        return _b(self.enabled, False)


@dataclass
class SandboxWorkloadsSpec(Spec):
    """GPU workloads in VMs (KubeVirt/Kata): passthrough or MxGPU virtual functions."""

    enabled: Optional[bool] = field("enabled")
    defaultWorkload: Optional[str] = field("defaultWorkload", enum=WORKLOADS,
                                           aliases=(), schema_default="container")

    def is_enabled(self) -> bool:
        return _b(self.enabled, False)

    def default_workload(self) -> str:
        return self.defaultWorkload or "container"


# --------------------------------------------------------------------------------------------
# driver
# --------------------------------------------------------------------------------------------
@dataclass
class DriverManagerSpec(ImageSpec):
    """amdgpu unload manager init container (evicts GPU pods, optional drain, rmmod)."""

    IMAGE_ENV: ClassVar[str] = "DRIVER_MANAGER_IMAGE"
    env: Optional[List[EnvVar]] = field("env")


@dataclass
class RDMASpec(Spec):
    """Peer-direct RDMA via amdgpu dma-buf (replaces GPUDirect RDMA / nvidia-peermem)."""

    enabled: Optional[bool] = field("enabled")
    useHostMofed: Optional[bool] = field("useHostMofed")

    def is_enabled(self) -> bool:
        return _b(self.enabled, False)


@dataclass
class DriverRepoConfigSpec(Spec):
    configMapName: Optional[str] = field("configMapName", doc="ConfigMap with package repo files.")


@dataclass
class DriverCertConfigSpec(Spec):
    name: Optional[str] = field("name", doc="ConfigMap with custom CA certificates.")


@dataclass
class KernelModuleConfigSpec(Spec):
    name: Optional[str] = field("name", doc="ConfigMap with amdgpu module parameters (amdgpu.conf).")


@dataclass
class DriverSpec(ComponentSpec):
    """amdgpu DKMS driver container."""

    IMAGE_ENV: ClassVar[str] = "DRIVER_IMAGE"

    usePrecompiled: Optional[bool] = field("usePrecompiled",
                                           doc="Use per-kernel precompiled amdgpu images (one DaemonSet per kernel).")
    startupProbe: Optional[ContainerProbeSpec] = field("startupProbe")
    livenessProbe: Optional[ContainerProbeSpec] = field("livenessProbe")
    readinessProbe: Optional[ContainerProbeSpec] = field("readinessProbe")
    rdma: Optional[RDMASpec] = field("rdma")
    upgradePolicy: Optional[DriverUpgradePolicySpec] = field("upgradePolicy")
    manager: Optional[DriverManagerSpec] = field("manager")
    repoConfig: Optional[DriverRepoConfigSpec] = field("repoConfig")
    certConfig: Optional[DriverCertConfigSpec] = field("certConfig")
    kernelModuleConfig: Optional[KernelModuleConfigSpec] = field("kernelModuleConfig")
    blacklistDrivers: Optional[List[str]] = field(
        "blacklistDrivers", doc="Modules to keep unloaded before amdgpu loads (e.g. ast).")

    def use_precompiled(self) -> bool:
        return _b(self.usePrecompiled, False)

    def auto_upgrade(self) -> bool:
        return bool(self.upgradePolicy and self.upgradePolicy.autoUpgrade)


@dataclass
class MxGPUManagerSpec(ComponentSpec):
    """MxGPU (SR-IOV, GIM) host driver for VM workloads."""

    IMAGE_ENV: ClassVar[str] = "MXGPU_MANAGER_IMAGE"
    DEFAULT_ENABLED: ClassVar[bool] = False
    driverManager: Optional[DriverManagerSpec] = field("driverManager")


# --------------------------------------------------------------------------------------------
# runtime hook / device plugin / telemetry / labeller / partitioning
# --------------------------------------------------------------------------------------------
@dataclass
class ToolkitSpec(ComponentSpec):
    """AMD container-runtime hook and CDI spec generator."""

    IMAGE_ENV: ClassVar[str] = "CONTAINER_TOOLKIT_IMAGE"
    installDir: Optional[str] = field("installDir", schema_default="/usr/local/amd",
                                      doc="Host directory the runtime hook is installed to.")

    def install_dir(self) -> str:
        return self.installDir or "/usr/local/amd"


@dataclass
class DevicePluginConfig(Spec):
    name: Optional[str] = field("name", doc="ConfigMap with named device-plugin configs.")
    default: Optional[str] = field("default", doc="Config used when the node has no label.")


@dataclass
class DevicePluginSpec(ComponentSpec):
    """ROCm device plugin advertising amd.com/gpu (and partition resources)."""

    IMAGE_ENV: ClassVar[str] = "DEVICE_PLUGIN_IMAGE"
    config: Optional[DevicePluginConfig] = field("config")


@dataclass
class SandboxDevicePluginSpec(ComponentSpec):
    """KubeVirt device plugin for passthrough PFs and MxGPU VFs."""

    IMAGE_ENV: ClassVar[str] = "SANDBOX_DEVICE_PLUGIN_IMAGE"
    DEFAULT_ENABLED: ClassVar[bool] = False


@dataclass
class MetricsConfig(Spec):
    name: Optional[str] = field("name", doc="ConfigMap with the metrics field list (CSV).")


@dataclass
class ServiceMonitorConfig(Spec):
    enabled: Optional[bool] = field("enabled")
    interval: Optional[str] = field("interval", pattern=r"^(0|(([0-9]+)y)?(([0-9]+)w)?(([0-9]+)d)?"
                                    r"(([0-9]+)h)?(([0-9]+)m)?(([0-9]+)s)?(([0-9]+)ms)?)$")
    honorLabels: Optional[bool] = field("honorLabels")
    additionalLabels: Optional[Dict[str, str]] = field("additionalLabels")
    relabelings: Optional[List[Any]] = field("relabelings")

    def is_enabled(self) -> bool:
        return _b(self.enabled, False)


@dataclass
class MetricsExporterSpec(ComponentSpec):
    """Prometheus exporter of GPU telemetry (power, temperature, utilisation, HBM, xGMI, ECC)."""

    IMAGE_ENV: ClassVar[str] = "METRICS_EXPORTER_IMAGE"
    config: Optional[MetricsConfig] = field("config")
    serviceMonitor: Optional[ServiceMonitorConfig] = field("serviceMonitor")


@dataclass
class RDCSpec(ComponentSpec):
    """Standalone RDC daemon (rdcd) the exporter can attach to."""

    IMAGE_ENV: ClassVar[str] = "RDC_IMAGE"
    hostPort: Optional[int] = field("hostPort", minimum=1, maximum=65535, schema_default=50051)

    def host_port(self) -> int:
        return self.hostPort or 50051


@dataclass
class NodeStatusExporterSpec(ComponentSpec):
    """Node readiness exporter (validator in metrics mode)."""

    IMAGE_ENV: ClassVar[str] = "VALIDATOR_IMAGE"
    DEFAULT_ENABLED: ClassVar[bool] = False


@dataclass
class NodeLabellerSpec(ComponentSpec):
    """Node-feature labeller: product, gfx target, CU count, VRAM, partition modes, xGMI hive."""

    IMAGE_ENV: ClassVar[str] = "NODE_LABELLER_IMAGE"


@dataclass
class PartitionSpec(Spec):
    """How partitioned GPUs are exposed as resources (the role of MIGSpec)."""

    strategy: Optional[str] = field("strategy", enum=PARTITION_STRATEGIES, schema_default="single")

    def get_strategy(self) -> str:
        return self.strategy or "single"


@dataclass
class PartitionConfigSpec(Spec):
    name: Optional[str] = field("name", doc="ConfigMap with named partition layouts.")
    default: Optional[str] = field("default", doc="Layout applied to unlabelled nodes.")


@dataclass
class GPUClientsConfigSpec(Spec):
    name: Optional[str] = field("name", doc="ConfigMap listing host services that hold the GPU.")


@dataclass
class PartitionManagerSpec(ComponentSpec):
    """Compute (SPX/DPX/QPX/CPX) and memory (NPS1/NPS4) partition manager."""

    IMAGE_ENV: ClassVar[str] = "PARTITION_MANAGER_IMAGE"
    config: Optional[PartitionConfigSpec] = field("config")
    gpuClientsConfig: Optional[GPUClientsConfigSpec] = field("gpuClientsConfig")


# --------------------------------------------------------------------------------------------
# validator
# --------------------------------------------------------------------------------------------
@dataclass
class ValidatorComponentSpec(Spec):
    env: Optional[List[EnvVar]] = field("env")


@dataclass
class ValidatorSpec(ComponentSpec):
    """Node validator: driver, runtime hook, HIP GEMM, device plugin and RCCL probes."""

    IMAGE_ENV: ClassVar[str] = "VALIDATOR_IMAGE"
    plugin: Optional[ValidatorComponentSpec] = field("plugin")
    toolkit: Optional[ValidatorComponentSpec] = field("toolkit")
    driver: Optional[ValidatorComponentSpec] = field("driver")
    hip: Optional[ValidatorComponentSpec] = field("hip", aliases=("cuda",))
    rccl: Optional[ValidatorComponentSpec] = field("rccl")
    vfioPCI: Optional[ValidatorComponentSpec] = field("vfioPCI")
    mxgpuManager: Optional[ValidatorComponentSpec] = field("mxgpuManager", aliases=("vgpuManager",))
    mxgpuDevices: Optional[ValidatorComponentSpec] = field("mxgpuDevices", aliases=("vgpuDevices",))

    def component(self, name: str) -> ValidatorComponentSpec:
        v = getattr(self, name, None)
        return v if v is not None else ValidatorComponentSpec()


# --------------------------------------------------------------------------------------------
# sandbox
# --------------------------------------------------------------------------------------------
@dataclass
class VFIOManagerSpec(ComponentSpec):
    """Binds AMD GPUs (vendor 0x1002) to vfio-pci for passthrough."""

    IMAGE_ENV: ClassVar[str] = "VFIO_MANAGER_IMAGE"
    DEFAULT_ENABLED: ClassVar[bool] = False
    driverManager: Optional[DriverManagerSpec] = field("driverManager")


@dataclass
class MxGPUDevicesConfigSpec(Spec):
    name: Optional[str] = field("name", doc="ConfigMap with named VF layouts.")
    default: Optional[str] = field("default", doc="Layout applied to unlabelled nodes.")


@dataclass
class MxGPUDeviceManagerSpec(ComponentSpec):
    """Creates MxGPU virtual functions according to a named layout."""

    IMAGE_ENV: ClassVar[str] = "MXGPU_DEVICE_MANAGER_IMAGE"
    DEFAULT_ENABLED: ClassVar[bool] = False
    config: Optional[MxGPUDevicesConfigSpec] = field("config")


@dataclass
class CDIConfigSpec(Spec):
    """Container Device Interface as the device-injection mechanism."""

    enabled: Optional[bool] = field("enabled")
    default: Optional[bool] = field("default")

    def is_enabled(self) -> bool:
        return _b(self.enabled, False)

    def is_default(self) -> bool:
        return _b(self.default, False)


@dataclass
class KataArtifacts(Spec):
    url: Optional[str] = field("url", required=True)
    pullSecret: Optional[str] = field("pullSecret")


@dataclass
class KataRuntimeClass(Spec):
    name: Optional[str] = field("name", required=True)
    nodeSelector: Optional[Dict[str, str]] = field("nodeSelector")
    artifacts: Optional[KataArtifacts] = field("artifacts", required=True)


@dataclass
class KataConfig(Spec):
    artifactsDir: Optional[str] = field("artifactsDir",
                                        schema_default="/opt/amd-gpu-operator/artifacts/runtimeclasses")
    runtimeClasses: Optional[List[KataRuntimeClass]] = field("runtimeClasses")


@dataclass
class KataManagerSpec(ComponentSpec):
    """Installs Kata guest artifacts and configures containerd runtime handlers."""

    IMAGE_ENV: ClassVar[str] = "KATA_MANAGER_IMAGE"
    DEFAULT_ENABLED: ClassVar[bool] = False
    config: Optional[KataConfig] = field("config")


@dataclass
class GDSSpec(ComponentSpec):
    """GPUDirect Storage: no ROCm equivalent. Accepted for migration, never deployed."""

    IMAGE_ENV: ClassVar[str] = "GDS_IMAGE"
    DEFAULT_ENABLED: ClassVar[bool] = False


# --------------------------------------------------------------------------------------------
# top level
# --------------------------------------------------------------------------------------------
@dataclass
class ClusterPolicySpec(Spec):
    """Desired state of the AMD GPU operator."""

    operator: Optional[OperatorSpec] = field("operator")
    daemonsets: Optional[DaemonsetsSpec] = field("daemonsets")
    driver: Optional[DriverSpec] = field("driver")
    toolkit: Optional[ToolkitSpec] = field("toolkit")
    devicePlugin: Optional[DevicePluginSpec] = field("devicePlugin")
    metricsExporter: Optional[MetricsExporterSpec] = field("metricsExporter", aliases=("dcgmExporter",))
    rdc: Optional[RDCSpec] = field("rdc", aliases=("dcgm",))
    nodeStatusExporter: Optional[NodeStatusExporterSpec] = field("nodeStatusExporter")
    nodeLabeller: Optional[NodeLabellerSpec] = field("nodeLabeller", aliases=("gfd",))
    partition: Optional[PartitionSpec] = field("partition", aliases=("mig",))
    partitionManager: Optional[PartitionManagerSpec] = field("partitionManager", aliases=("migManager",))
    psp: Optional[PSPSpec] = field("psp")
    psa: Optional[PSASpec] = field("psa")
    validator: Optional[ValidatorSpec] = field("validator")
    gds: Optional[GDSSpec] = field("gds")
    sandboxWorkloads: Optional[SandboxWorkloadsSpec] = field("sandboxWorkloads")
    vfioManager: Optional[VFIOManagerSpec] = field("vfioManager")
    sandboxDevicePlugin: Optional[SandboxDevicePluginSpec] = field("sandboxDevicePlugin")
    mxgpuManager: Optional[MxGPUManagerSpec] = field("mxgpuManager", aliases=("vgpuManager",))
    mxgpuDeviceManager: Optional[MxGPUDeviceManagerSpec] = field("mxgpuDeviceManager",
                                                                 aliases=("vgpuDeviceManager",))
    cdi: Optional[CDIConfigSpec] = field("cdi")
    kataManager: Optional[KataManagerSpec] = field("kataManager")

    def __post_init__(self):
        # Materialise every sub-spec so callers never need None checks (the Go structs are
        # value types; only the explicitly nullable ones stay None).
        hints = {f.name: tp for f, tp in self._fields()}
        for name, tp in hints.items():
            if getattr(self, name) is None:
                setattr(self, name, tp())


@dataclass
class Condition(Spec):
    type: Optional[str] = field("type", required=True)
    status: Optional[str] = field("status", enum=["True", "False", "Unknown"], required=True)
    reason: Optional[str] = field("reason")
    message: Optional[str] = field("message")
    lastTransitionTime: Optional[str] = field("lastTransitionTime")


@dataclass
class ClusterPolicyStatus(Spec):
    """Observed state of the operator."""

    state: Optional[str] = field("state", enum=[STATE_IGNORED, STATE_READY, STATE_NOT_READY])
    namespace: Optional[str] = field("namespace")
    notReadyStates: Optional[List[str]] = field("notReadyStates", doc="States not yet ready.")
    conditions: Optional[List[Condition]] = field("conditions")


class ClusterPolicy:
    """Typed view of a ClusterPolicy object (metadata stays a plain dict)."""

    def __init__(self, obj: Dict[str, Any], strict: bool = False):
        if obj.get("apiVersion") not in (None, API_VERSION):
            raise ValidationError(f"apiVersion {obj.get('apiVersion')!r} is not {API_VERSION}")
        self.metadata: Dict[str, Any] = dict(obj.get("metadata") or {})
        self.spec = ClusterPolicySpec.from_dict(obj.get("spec") or {}, strict=strict, path="spec")
        self.status = ClusterPolicyStatus.from_dict(obj.get("status") or {}, path="status")
        validate_spec(self.spec)

    @property
    def name(self) -> str:
        return self.metadata.get("name", "")

    @property
    def uid(self) -> str:
        return self.metadata.get("uid", "")

    def set_status(self, state: str, namespace: str) -> None:
        self.status.state = state
        self.status.namespace = namespace

    def to_dict(self) -> Dict[str, Any]:
        return {"apiVersion": API_VERSION, "kind": KIND, "metadata": dict(self.metadata),
                "spec": self.spec.to_dict(), "status": self.status.to_dict()}


def validate_spec(spec: ClusterPolicySpec) -> None:
    """Cross-field rules the OpenAPI schema cannot express."""
    kc = spec.kataManager.config
    if kc and kc.runtimeClasses:
        names = [rc.name for rc in kc.runtimeClasses]
        if len(set(names)) != len(names):
            raise ValidationError("spec.kataManager.config.runtimeClasses: duplicate names")


# --------------------------------------------------------------------------------------------
# image resolution (reference: api/v1/clusterpolicy_types.go:1552-1640)
# --------------------------------------------------------------------------------------------
def _image_path(repository: str, image: str, version: str, env_name: str) -> str:
    crd_path = ""
    if not repository and not version:
        if image:
            crd_path = image          # already a full reference (e.g. rendered by kbld)
    else:
        sep = "@" if version.startswith("sha256:") else ":"
        crd_path = f"{repository}/{image}{sep}{version}"
    if crd_path:
        return crd_path
    env_val = os.environ.get(env_name, "")
    if env_val:
        return env_val
    raise ValueError(f"empty image path: set it in the ClusterPolicy or via env {env_name}")


def image_path(spec: ImageSpec) -> str:
    """Image for an operand: CR repository/image:version (or @sha256) -> env ``*_IMAGE`` -> error."""
    if not isinstance(spec, ImageSpec) or not type(spec).IMAGE_ENV:
        raise TypeError(f"invalid type to construct image path: {type(spec).__name__}")
    return _image_path(spec.repository or "", spec.image or "", spec.version or "", type(spec).IMAGE_ENV)


def image_pull_policy(policy: Optional[str]) -> str:
    return policy if policy in PULL_POLICIES else "IfNotPresent"
