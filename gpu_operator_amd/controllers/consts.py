"""Label / annotation / name constants of the AMD operator's node and object protocols.

Counterparts of the reference's constants (reference: controllers/state_manager.go:27-101,
controllers/object_controls.go:40-145), re-keyed to ``amd.com/`` and PCI vendor 0x1002.
"""

from __future__ import annotations

from typing import Dict

PREFIX = "amd.com"
PLACEHOLDER = "FILLED_BY_OPERATOR"

# --- node labels written by the operator ----------------------------------------------------
COMMON_GPU_LABEL = f"{PREFIX}/gpu.present"
OPERANDS_LABEL = f"{PREFIX}/gpu.deploy.operands"
PARTITION_MANAGER_DEPLOY_LABEL = f"{PREFIX}/gpu.deploy.partition-manager"
WORKLOAD_CONFIG_LABEL = f"{PREFIX}/gpu.workload.config"
PARTITION_CONFIG_LABEL = f"{PREFIX}/gpu.partition.config"
PARTITION_STATE_LABEL = f"{PREFIX}/gpu.partition.state"
PARTITION_CAPABLE_LABEL = f"{PREFIX}/gpu.partition.capable"
DEVICE_PLUGIN_CONFIG_LABEL = f"{PREFIX}/device-plugin.config"
MXGPU_CONFIG_LABEL = f"{PREFIX}/mxgpu.config"
GPU_PRODUCT_LABEL = f"{PREFIX}/gpu.product"
GPU_FAMILY_LABEL = f"{PREFIX}/gpu.family"
MXGPU_HOST_DRIVER_LABEL = f"{PREFIX}/mxgpu.host-driver-version"
DRIVER_AUTO_UPGRADE_ANNOTATION = f"{PREFIX}/gpu-driver-upgrade-enabled"
PRECOMPILED_LABEL = f"{PREFIX}/precompiled"
LAST_APPLIED_HASH_ANNOTATION = f"{PREFIX}/last-applied-hash"
KATA_RUNTIME_CLASS_LABEL = f"{PREFIX}/kata-runtime-class"
KATA_CONFIG_HASH_ANNOTATION = f"{PREFIX}/kata-manager-config-hash"

WORKLOAD_CONTAINER = "container"
WORKLOAD_VM_PASSTHROUGH = "vm-passthrough"
WORKLOAD_VM_MXGPU = "vm-mxgpu"

# --- NFD labels -----------------------------------------------------------------------------
NFD_PREFIX = "feature.node.kubernetes.io/"
NFD_KERNEL_LABEL = "feature.node.kubernetes.io/kernel-version.full"
NFD_OS_ID_LABEL = "feature.node.kubernetes.io/system-os_release.ID"
NFD_OS_VERSION_LABEL = "feature.node.kubernetes.io/system-os_release.VERSION_ID"
NFD_OSTREE_LABEL = "feature.node.kubernetes.io/system-os_release.OSTREE_VERSION"

# A node has an AMD GPU when NFD reports PCI vendor 0x1002 in one of the GPU classes:
# 0300 (VGA/display), 0380 (display controller: Instinct), 1200 (processing accelerator).
GPU_NODE_LABELS: Dict[str, str] = {
    "feature.node.kubernetes.io/pci-1002.present": "true",
    "feature.node.kubernetes.io/pci-0300_1002.present": "true",
    "feature.node.kubernetes.io/pci-0380_1002.present": "true",
    "feature.node.kubernetes.io/pci-1200_1002.present": "true",
}

# Per workload-config operand deploy labels (reference: state_manager.go:72-95)
GPU_STATE_LABELS: Dict[str, Dict[str, str]] = {
    WORKLOAD_CONTAINER: {
        f"{PREFIX}/gpu.deploy.driver": "true",
        f"{PREFIX}/gpu.deploy.node-labeller": "true",
        f"{PREFIX}/gpu.deploy.container-toolkit": "true",
        f"{PREFIX}/gpu.deploy.device-plugin": "true",
        f"{PREFIX}/gpu.deploy.rdc": "true",
        f"{PREFIX}/gpu.deploy.metrics-exporter": "true",
        f"{PREFIX}/gpu.deploy.node-status-exporter": "true",
        f"{PREFIX}/gpu.deploy.operator-validator": "true",
    },
    WORKLOAD_VM_PASSTHROUGH: {
        f"{PREFIX}/gpu.deploy.sandbox-device-plugin": "true",
        f"{PREFIX}/gpu.deploy.sandbox-validator": "true",
        f"{PREFIX}/gpu.deploy.vfio-manager": "true",
        f"{PREFIX}/gpu.deploy.kata-manager": "true",
    },
    WORKLOAD_VM_MXGPU: {
        f"{PREFIX}/gpu.deploy.sandbox-device-plugin": "true",
        f"{PREFIX}/gpu.deploy.mxgpu-manager": "true",
        f"{PREFIX}/gpu.deploy.mxgpu-device-manager": "true",
        f"{PREFIX}/gpu.deploy.sandbox-validator": "true",
    },
}

# Product families that support compute/memory partitioning (CDNA3/CDNA4 Instinct). The
# labeller publishes amd.com/gpu.partition.capable from sysfs (available_compute_partition);
# the family list is only a fallback for nodes labelled before the labeller ran.
from ..models import PARTITION_CAPABLE_FAMILIES  # noqa: E402  (cdna3, cdna4)
PARTITION_DISABLED_CONFIG = "spx-nps1"

# --- operator namespace handling --------------------------------------------------------------
OCP_SUGGESTED_NAMESPACE = "amd-gpu-operator"
OCP_MONITORING_LABEL = "openshift.io/cluster-monitoring"
# OpenShift cluster proxy with a user CA bundle (reference: object_controls.go:53-60, 931-961):
# the Cluster Network Operator fills a ConfigMap labelled inject-trusted-cabundle, which the
# driver container mounts where RHEL's ca-trust looks for the extracted PEM bundle.
TRUSTED_CA_CONFIGMAP = "amd-gpu-operator-trusted-ca"
TRUSTED_CA_INJECT_LABEL = "config.openshift.io/inject-trusted-cabundle"
TRUSTED_CA_BUNDLE_KEY = "ca-bundle.crt"
TRUSTED_CA_MOUNT_DIR = "/etc/pki/ca-trust/extracted/pem"
TRUSTED_CA_CERT_FILE = "tls-ca-bundle.pem"
POD_SECURITY_PREFIX = "pod-security.kubernetes.io/"
POD_SECURITY_MODES = ("enforce", "audit", "warn")

# --- DaemonSet names ------------------------------------------------------------------------
DS_DRIVER = "amdgpu-driver-daemonset"
DS_TOOLKIT = "amd-container-toolkit-daemonset"
DS_VALIDATOR = "amd-operator-validator"
DS_DEVICE_PLUGIN = "amd-device-plugin-daemonset"
DS_RDC = "amd-rdc"
DS_METRICS_EXPORTER = "amd-metrics-exporter"
DS_NODE_LABELLER = "amd-node-labeller"
DS_PARTITION_MANAGER = "amd-partition-manager"
DS_NODE_STATUS_EXPORTER = "amd-node-status-exporter"
DS_MXGPU_MANAGER = "amd-mxgpu-manager-daemonset"
DS_MXGPU_DEVICE_MANAGER = "amd-mxgpu-device-manager"
DS_SANDBOX_VALIDATOR = "amd-sandbox-validator"
DS_VFIO_MANAGER = "amd-vfio-manager"
DS_SANDBOX_DEVICE_PLUGIN = "amd-sandbox-device-plugin-daemonset"
DS_KATA_MANAGER = "amd-kata-manager"

# --- node-side paths ------------------------------------------------------------------------
VALIDATIONS_DIR = "/run/amd/validations"
DRIVER_ROOT = "/run/amd/driver"

# --- ordered states (reference: state_manager.go:784-801) -----------------------------------
STATES = [
    "pre-requisites",
    "state-operator-metrics",
    "state-driver",
    "state-container-toolkit",
    "state-operator-validation",
    "state-device-plugin",
    "state-rdc",
    "state-metrics-exporter",
    "state-node-labeller",
    "state-partition-manager",
    "state-node-status-exporter",
    # sandbox workload states
    "state-mxgpu-manager",
    "state-mxgpu-device-manager",
    "state-sandbox-validation",
    "state-vfio-manager",
    "state-sandbox-device-plugin",
    "state-kata-manager",
]

# Runtime defaults (reference: object_controls.go:40-145)
RUNTIME_CONFIG = {
    "containerd": ("/etc/containerd/config.toml", "/run/containerd/containerd.sock"),
    "docker": ("/etc/docker/daemon.json", "/var/run/docker.sock"),
    "crio": ("/etc/crio/crio.conf.d/99-amd.conf", "/var/run/crio/crio.sock"),
}
CRIO_HOOKS_DIR = "/run/containers/oci/hooks.d"
