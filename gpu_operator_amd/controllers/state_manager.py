"""ClusterPolicy state manager: per-reconcile cluster discovery, GPU-node labelling and the
ordered walk over the 17 operand states.

Counterpart of the reference's ``ClusterPolicyController`` (reference:
controllers/state_manager.go:134-1004). The reference keeps it in a process-global variable
that the upgrade reconciler reads concurrently (SURVEY.md §5.2 latent race, §7.7 quirk 2).
Here a ``StateManager`` is owned by exactly one reconciler; what other controllers need is
published as an immutable :class:`ClusterSnapshot` through a lock-protected holder.
"""

from __future__ import annotations

import contextlib
import logging
import os
import re
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional, Tuple

from ..api.v1 import clusterpolicy as cp
from ..k8s import errors
from ..k8s import objects as o
from . import consts as C
from . import object_controls as oc
from .resource_manager import State, load_states

log = logging.getLogger("amd-gpu-operator.state")


@dataclass(frozen=True)
class ClusterSnapshot:
    """Read-only facts the ClusterPolicy reconcile derived, shared with other controllers."""

    namespace: str = ""
    openshift: str = ""
    k8s_version: str = ""
    runtime: str = "containerd"
    sandbox_enabled: bool = False
    gpu_nodes: int = 0
    dtk_enabled: bool = False
    driver_app_labels: Tuple[Tuple[str, str], ...] = (("app", C.DS_DRIVER),)


class SnapshotHolder:
    def __init__(self):
        self._lock = threading.Lock()
        self._snap = ClusterSnapshot()

    def set(self, snap: ClusterSnapshot) -> None:
        with self._lock:
            self._snap = snap

    def get(self) -> ClusterSnapshot:
        with self._lock:
            return self._snap


# ---------------------------------------------------------------------------------------------
# node label helpers (reference: state_manager.go:228-414)
# ---------------------------------------------------------------------------------------------
def has_gpu_labels(labels: Dict[str, str]) -> bool:
    return any(labels.get(k) == v for k, v in C.GPU_NODE_LABELS.items())


def has_common_gpu_label(labels: Dict[str, str]) -> bool:
    return labels.get(C.COMMON_GPU_LABEL) == "true"


def has_nfd_labels(labels: Dict[str, str]) -> bool:
    return any(k.startswith(C.NFD_PREFIX) for k in labels)


def has_operands_disabled(labels: Dict[str, str]) -> bool:
    return labels.get(C.OPERANDS_LABEL) == "false"


def is_partition_capable(labels: Dict[str, str]) -> bool:
    """From the labeller's sysfs-derived label; the product family is only a fallback
    (the reference string-matches product names)."""
    v = labels.get(C.PARTITION_CAPABLE_LABEL)
    if v is not None:
        return v == "true"
    return labels.get(C.GPU_FAMILY_LABEL, "").lower() in C.PARTITION_CAPABLE_FAMILIES


def workload_config(labels: Dict[str, str], sandbox_enabled: bool, default: str) -> Tuple[str, Optional[str]]:
    if not sandbox_enabled:
        return C.WORKLOAD_CONTAINER, None
    v = labels.get(C.WORKLOAD_CONFIG_LABEL)
    if v is None:
        return default, "no GPU workload config label"
    if v not in C.GPU_STATE_LABELS:
        return default, f"invalid GPU workload config {v!r}"
    return v, None


def remove_all_gpu_state_labels(labels: Dict[str, str]) -> bool:
    modified = False
    for lm in C.GPU_STATE_LABELS.values():
        for k in lm:
            if k in labels:
                del labels[k]
                modified = True
    if C.PARTITION_MANAGER_DEPLOY_LABEL in labels:
        del labels[C.PARTITION_MANAGER_DEPLOY_LABEL]
        modified = True
    return modified


def update_gpu_state_labels(labels: Dict[str, str], config: str) -> bool:
    """Add the deploy labels of ``config``, drop the ones of other configs; honour
    ``amd.com/gpu.deploy.operands=false`` and user-set values of required labels."""
    if has_operands_disabled(labels):
        return remove_all_gpu_state_labels(labels)
    modified = False
    wanted = C.GPU_STATE_LABELS[config]
    for other, lm in C.GPU_STATE_LABELS.items():
        if other == config:
            continue
        for k in lm:
            if k not in wanted and k in labels:
                del labels[k]
                modified = True
    for k, v in wanted.items():
        if k not in labels:
            labels[k] = v
            modified = True
    if config == C.WORKLOAD_CONTAINER:
        if is_partition_capable(labels) and C.PARTITION_MANAGER_DEPLOY_LABEL not in labels:
            labels[C.PARTITION_MANAGER_DEPLOY_LABEL] = "true"
            modified = True
    elif C.PARTITION_MANAGER_DEPLOY_LABEL in labels:
        del labels[C.PARTITION_MANAGER_DEPLOY_LABEL]
        modified = True
    return modified


def runtime_of(node: Dict[str, Any]) -> Optional[str]:
    rv = ((node.get("status") or {}).get("nodeInfo") or {}).get("containerRuntimeVersion", "")
    if rv.startswith("docker"):
        return "docker"
    if rv.startswith("containerd"):
        return "containerd"
    if rv.startswith("cri-o"):
        return "crio"
    return None


def node_os_tag(labels: Dict[str, str]) -> str:
    osid, ver = labels.get(C.NFD_OS_ID_LABEL), labels.get(C.NFD_OS_VERSION_LABEL)
    return f"{osid}{ver}" if osid and ver else ""


def parse_k8s_minor(version: str) -> int:
    m = re.match(r"v?(\d+)\.(\d+)", version or "")
    return int(m.group(2)) if m else 99


# ---------------------------------------------------------------------------------------------
class StateManager:
    """The ``n`` every control function and transform receives."""

    def __init__(self, client, namespace: Optional[str] = None, metrics=None,
                 assets_base=None, snapshot: Optional[SnapshotHolder] = None):
        self.client = client
        self.namespace = namespace if namespace is not None else os.environ.get("OPERATOR_NAMESPACE", "")
        if not self.namespace:
            raise RuntimeError("OPERATOR_NAMESPACE is not set; the operator cannot proceed")
        self.metrics = metrics
        self.assets_base = assets_base
        self.snapshot = snapshot or SnapshotHolder()
        self.states: List[State] = []
        self.openshift = ""
        self.k8s_version = ""
        # per reconcile
        self.owner: Dict[str, Any] = {}
        self.cp: Optional[cp.ClusterPolicy] = None
        self.spec: cp.ClusterPolicySpec = cp.ClusterPolicySpec()
        self.runtime = "containerd"
        self.sandbox_enabled = False
        self.default_workload = C.WORKLOAD_CONTAINER
        self.has_gpu_nodes = False
        self.has_nfd = False
        self.gpu_node_count = 0
        self.kernel_map: Dict[str, str] = {}
        self.os_tags: List[str] = []
        self.rhcos_versions: Dict[str, bool] = {}
        self.dtk_images: Dict[str, str] = {}
        self.dtk_requested = False
        self._dtk_enabled = False
        self._proxy: Dict[str, str] = {}
        self._proxy_trusted_ca = ""
        # current fan-out variant
        self.current_kernel: Optional[str] = None
        self.current_rhcos: Optional[str] = None
        self.current_os: Optional[str] = None
        self._variant_kind: Optional[str] = None

    # -- discovery ------------------------------------------------------------------------
    def _first_init(self) -> None:
        try:
            cv = self.client.get("config.openshift.io/v1", "ClusterVersion", "version")
            self.openshift = ((cv.get("status") or {}).get("desired") or {}).get("version", "") or "unknown"
        except (errors.NotFound, errors.NoKindMatch):
            self.openshift = ""
        self.k8s_version = self.client.server_version()
        if not re.match(r"v?\d+\.\d+", self.k8s_version or ""):
            raise RuntimeError(f"kubernetes version {self.k8s_version!r} is not a semantic version")
        self.states = load_states(C.STATES, self.assets_base, openshift=bool(self.openshift))
        log.info("kubernetes %s, openshift %s, %d states loaded", self.k8s_version,
                 self.openshift or "no", len(self.states))

    def init(self, owner: Dict[str, Any]) -> None:
        if not self.states:
            self._first_init()
        self.owner = owner
        self.cp = cp.ClusterPolicy(owner)
        self.spec = self.cp.spec
        self.current_kernel = self.current_rhcos = self.current_os = None

        sw = self.spec.sandboxWorkloads
        self.sandbox_enabled = sw.is_enabled()
        dw = sw.default_workload()
        self.default_workload = dw if dw in C.GPU_STATE_LABELS else C.WORKLOAD_CONTAINER

        use_dtk = self.spec.operator.use_ocp_driver_toolkit
        self.dtk_requested = bool(self.openshift) and (use_dtk is None or use_dtk)
        self.rhcos_versions = {}
        self.dtk_images = {}
        self._dtk_enabled = False

        if self.spec.psp.is_enabled() or self.spec.psa.is_enabled():
            self._set_pod_security_labels()

        self.has_nfd, self.gpu_node_count = self.label_gpu_nodes()
        self.has_gpu_nodes = self.gpu_node_count > 0
        self.apply_driver_auto_upgrade_annotation()
        self.runtime = self.detect_runtime()
        self.os_tags = self._gpu_node_os_tags()
        self.kernel_map = {}
        if self.spec.driver.is_enabled() and self.spec.driver.use_precompiled():
            self.kernel_map = self.kernel_versions_map()
        if self.openshift:
            self._init_ocp()
        if self.metrics:
            self.metrics.set_dtk(self.openshift, self.dtk_requested, self._dtk_enabled)
        self.snapshot.set(ClusterSnapshot(
            namespace=self.namespace, openshift=self.openshift, k8s_version=self.k8s_version,
            runtime=self.runtime, sandbox_enabled=self.sandbox_enabled, gpu_nodes=self.gpu_node_count,
            dtk_enabled=self._dtk_enabled,
            driver_app_labels=(("app", C.DS_DRIVER),) if not self._dtk_enabled
            else (("openshift.driver-toolkit", "true"),)))

    def _set_pod_security_labels(self) -> None:
        if self.openshift and self.namespace != C.OCP_SUGGESTED_NAMESPACE:
            log.info("not the suggested namespace on OpenShift; not setting PSA labels")
            return
        ns = self.client.get("v1", "Namespace", self.namespace)
        labels = o.get_labels(ns)
        patch = {k: "privileged" for k in (C.POD_SECURITY_PREFIX + m for m in C.POD_SECURITY_MODES)
                 if labels.get(k) != "privileged"}
        if patch:
            self.client.patch("v1", "Namespace", self.namespace, {"metadata": {"labels": patch}})

    def _init_ocp(self) -> None:
        if self.spec.driver.use_precompiled():
            self._dtk_enabled = False
        elif self.dtk_requested:
            broken = False
            try:
                ist = self.client.get("image.openshift.io/v1", "ImageStream", "driver-toolkit", "openshift")
                for tag in (ist.get("spec") or {}).get("tags") or []:
                    name = tag.get("name") or ""
                    if not name:
                        # a nameless tag: the ImageStream an OpenShift upgrade left broken (RHBZ#2015024;
                        # reference controllers/object_controls.go:3301-3319) -- flagged, never indexed
                        broken = True
                        continue
                    frm = (tag.get("from") or {}).get("name")
                    if name == "latest" or not frm:
                        continue
                    self.dtk_images[name] = frm
                has_is = True
            except (errors.NotFound, errors.NoKindMatch):
                has_is = False
            if broken:
                log.warning("the driver-toolkit ImageStream has a tag without a name (RHBZ#2015024): it is broken")
            self._dtk_enabled = has_is and bool(self.rhcos_versions)
            if self.metrics:
                self.metrics.dtk_imagestream_missing.set(0 if has_is else 1)
                self.metrics.dtk_imagestream_broken.set(1 if broken else 0)
                self.metrics.dtk_nfd_too_old.set(1 if self.has_gpu_nodes and not self.rhcos_versions else 0)
                missing = [v for v in self.rhcos_versions if v not in self.dtk_images]
                self.metrics.dtk_rhcos_tags_missing.set(1 if missing else 0)
        try:
            px = self.client.get("config.openshift.io/v1", "Proxy", "cluster")
            spec = px.get("spec") or {}
            self._proxy = {k: v for k, v in (("HTTP_PROXY", spec.get("httpProxy")),
                                              ("HTTPS_PROXY", spec.get("httpsProxy")),
                                              ("NO_PROXY", spec.get("noProxy"))) if v}
            self._proxy_trusted_ca = ((spec.get("trustedCA") or {}).get("name") or "") if self.openshift else ""
        except (errors.NotFound, errors.NoKindMatch):
            self._proxy = {}
            self._proxy_trusted_ca = ""
        if self._proxy_trusted_ca:
            self.ensure_trusted_ca_configmap()
        if self.namespace == C.OCP_SUGGESTED_NAMESPACE:
            ns = self.client.get("v1", "Namespace", self.namespace)
            if C.OCP_MONITORING_LABEL not in o.get_labels(ns):
                self.client.patch("v1", "Namespace", self.namespace,
                                  {"metadata": {"labels": {C.OCP_MONITORING_LABEL: "true"}}})

    # -- node labelling (reference: labelGPUNodes :473-572) ---------------------------------
    def label_gpu_nodes(self) -> Tuple[bool, int]:
        nodes = self.client.list("v1", "Node")
        cluster_has_nfd = False
        gpu_nodes = 0
        pm = self.spec.partitionManager
        for node in nodes:
            labels = o.get_labels(node)
            before = dict(labels)
            cluster_has_nfd = cluster_has_nfd or has_nfd_labels(labels)
            config, warn = workload_config(labels, self.sandbox_enabled, self.default_workload)
            if warn:
                log.info("node %s: %s; using %s", o.name(node), warn, config)
            if not has_common_gpu_label(labels) and has_gpu_labels(labels):
                labels[C.COMMON_GPU_LABEL] = "true"
            elif has_common_gpu_label(labels) and not has_gpu_labels(labels):
                labels[C.COMMON_GPU_LABEL] = "false"
                remove_all_gpu_state_labels(labels)
            if has_common_gpu_label(labels):
                update_gpu_state_labels(labels, config)
                if pm.is_enabled() and is_partition_capable(labels) and C.PARTITION_CONFIG_LABEL not in labels \
                        and pm.config is not None and pm.config.default:
                    labels[C.PARTITION_CONFIG_LABEL] = pm.config.default
                gpu_nodes += 1
                if self.dtk_requested:
                    rv = labels.get(C.NFD_OSTREE_LABEL)
                    if rv:
                        self.rhcos_versions[rv] = True
            if labels != before:
                patch = {k: v for k, v in labels.items() if before.get(k) != v}
                patch.update({k: None for k in before if k not in labels})
                self.client.patch("v1", "Node", o.name(node), {"metadata": {"labels": patch}})
                log.info("node %s: labels updated %s", o.name(node), sorted(patch))
        if self.metrics:
            self.metrics.gpu_nodes_total.set(gpu_nodes)
        return cluster_has_nfd, gpu_nodes

    def apply_driver_auto_upgrade_annotation(self) -> None:
        want = self.spec.driver.auto_upgrade() and not self.sandbox_enabled
        for node in self.client.list("v1", "Node", label_selector={C.COMMON_GPU_LABEL: "true"}):
            anns = o.get_annotations(node)
            cur = anns.get(C.DRIVER_AUTO_UPGRADE_ANNOTATION)
            if want and cur != "true":
                patch = {C.DRIVER_AUTO_UPGRADE_ANNOTATION: "true"}
            elif not want and cur is not None:
                patch = {C.DRIVER_AUTO_UPGRADE_ANNOTATION: None}
            else:
                continue
            self.client.patch("v1", "Node", o.name(node), {"metadata": {"annotations": patch}})
        if self.metrics:
            self.metrics.driver_auto_upgrade_enabled.set(1 if want else 0)

    def detect_runtime(self) -> str:
        if self.openshift:
            return "crio"
        runtime = None
        for node in self.client.list("v1", "Node", label_selector={C.COMMON_GPU_LABEL: "true"}):
            rt = runtime_of(node)
            if rt is None:
                continue
            runtime = rt
            if rt == "containerd":
                break
        return runtime or self.spec.operator.default_runtime()

    def kernel_versions_map(self) -> Dict[str, str]:
        km: Dict[str, str] = {}
        for node in self.client.list("v1", "Node", label_selector={C.COMMON_GPU_LABEL: "true"}):
            labels = o.get_labels(node)
            kernel = labels.get(C.NFD_KERNEL_LABEL)
            if not kernel:
                raise errors.NotFound(f"node {o.name(node)} has no {C.NFD_KERNEL_LABEL} label; is NFD running?")
            os_tag = node_os_tag(labels)
            if kernel in km and km[kernel] != os_tag:
                raise ValueError(f"kernel {kernel} found on different OS versions ({km[kernel]}, {os_tag})")
            km[kernel] = os_tag
        return km

    def _gpu_node_os_tags(self) -> List[str]:
        tags = set()
        for node in self.client.list("v1", "Node", label_selector={C.COMMON_GPU_LABEL: "true"}):
            t = node_os_tag(o.get_labels(node))
            if t:
                tags.add(t)
        return sorted(tags)

    # -- state predicates ------------------------------------------------------------------
    def is_state_enabled(self, name: str) -> bool:
        s = self.spec
        sb = self.sandbox_enabled
        return {
            "pre-requisites": True,
            "state-operator-metrics": True,
            "state-driver": s.driver.is_enabled(),
            "state-container-toolkit": s.toolkit.is_enabled(),
            "state-operator-validation": True,
            "state-device-plugin": s.devicePlugin.is_enabled(),
            "state-rdc": s.rdc.is_enabled(),
            "state-metrics-exporter": s.metricsExporter.is_enabled(),
            "state-node-labeller": s.nodeLabeller.is_enabled(),
            "state-partition-manager": s.partitionManager.is_enabled(),
            "state-node-status-exporter": s.nodeStatusExporter.is_enabled(),
            "state-mxgpu-manager": sb and s.mxgpuManager.is_enabled(),
            "state-mxgpu-device-manager": sb and s.mxgpuDeviceManager.is_enabled(),
            "state-sandbox-validation": sb,
            "state-vfio-manager": sb and s.vfioManager.is_enabled(),
            "state-sandbox-device-plugin": sb and s.sandboxDevicePlugin.is_enabled(),
            "state-kata-manager": sb and s.kataManager.is_enabled(),
        }.get(name, False)

    # -- helpers used by transforms ----------------------------------------------------------
    def k8s_minor(self) -> int:
        return parse_k8s_minor(self.k8s_version)

    def driver_auto_upgrade(self) -> bool:
        return self.spec.driver.auto_upgrade() and not self.sandbox_enabled

    def dtk_enabled(self) -> bool:
        return self._dtk_enabled

    def cluster_proxy(self) -> Dict[str, str]:
        return dict(self._proxy)

    def trusted_ca_configmap(self) -> str:
        """Name of the CA-bundle ConfigMap the driver container mounts ("" without a proxy CA)."""
        return C.TRUSTED_CA_CONFIGMAP if self._proxy_trusted_ca else ""

    def ensure_trusted_ca_configmap(self) -> None:
        """Get-or-create the ConfigMap the cluster network operator injects the proxy's CA bundle
        into (reference: getOrCreateTrustedCAConfigMap, object_controls.go:971-1010). Never
        updated afterwards: its data belongs to the injector."""
        try:
            self.client.get("v1", "ConfigMap", C.TRUSTED_CA_CONFIGMAP, self.namespace)
            return
        except errors.NotFound:
            pass
        cm = {"apiVersion": "v1", "kind": "ConfigMap",
              "metadata": {"name": C.TRUSTED_CA_CONFIGMAP, "namespace": self.namespace,
                           "labels": {C.TRUSTED_CA_INJECT_LABEL: "true"}},
              "data": {C.TRUSTED_CA_BUNDLE_KEY: ""}}
        o.set_controller_reference(self.owner, cm)
        try:
            self.client.create(cm)
            log.info("created trusted CA bundle ConfigMap %s/%s", self.namespace, C.TRUSTED_CA_CONFIGMAP)
        except errors.AlreadyExists:
            pass

    def node_os_tag(self) -> str:
        if self.current_os:
            return self.current_os
        if self.current_kernel:
            return self.kernel_map.get(self.current_kernel, "")
        return self.os_tags[0] if self.os_tags else ""

    def template_name(self, obj) -> str:
        return o.name(obj)

    # -- DaemonSet fan-out (reference: precompiledDriverDaemonsets :3405-3436, DTK :3442) ------
    def daemonset_variants(self, base: str) -> Optional[List[Dict[str, str]]]:
        if base == C.DS_DRIVER:
            if self.spec.driver.use_precompiled():
                return [{"kind": "precompiled", "kernel": k, "os": v} for k, v in sorted(self.kernel_map.items())]
            if self._dtk_enabled:
                return [{"kind": "dtk", "rhcos": r} for r in sorted(self.rhcos_versions)]
            if len(self.os_tags) > 1:
                return [{"kind": "os", "os": t} for t in self.os_tags]
        if base == C.DS_MXGPU_MANAGER and len(self.os_tags) > 1:
            return [{"kind": "os", "os": t} for t in self.os_tags]
        return None

    def variant_name(self, base: str, v: Dict[str, str]) -> str:
        from .transforms import sanitize_kernel_version
        if v["kind"] == "precompiled":
            return f"{base}-{sanitize_kernel_version(v['kernel'])}-{v['os']}"
        if v["kind"] == "dtk":
            return f"{base}-{v['rhcos'].replace('.', '')}"
        return f"{base}-{v['os']}"

    @contextlib.contextmanager
    def variant(self, v: Dict[str, str]) -> Iterator[None]:
        self.current_kernel = v.get("kernel")
        self.current_rhcos = v.get("rhcos")
        self.current_os = v.get("os")
        self._variant_kind = v["kind"]
        try:
            yield
        finally:
            self.current_kernel = self.current_rhcos = self.current_os = None
            self._variant_kind = None

    @property
    def variant_kind(self) -> Optional[str]:
        return self._variant_kind

    def daemonset_variants_existing(self, base: str) -> List[Dict[str, Any]]:
        return [d for d in self.client.list("apps/v1", "DaemonSet", self.namespace, label_selector={"app": base})
                if o.name(d) != base]

    FANOUT_BASES = (C.DS_DRIVER, C.DS_MXGPU_MANAGER)

    def cleanup_stale_variants(self, base: str, variants: Optional[List[Dict[str, str]]]) -> bool:
        """Delete DaemonSets of other flavours/kernels/OSes; True while their pods remain."""
        want = {base} if variants is None else {self.variant_name(base, v) for v in variants}
        pending = False
        existing = self.client.list("apps/v1", "DaemonSet", self.namespace, label_selector={"app": base})
        for ds in existing:
            if o.name(ds) in want:
                continue
            st = ds.get("status") or {}
            if o.name(ds) != base and st.get("desiredNumberScheduled", 0) > 0 and \
                    self.spec.driver.use_precompiled() and o.get_labels(ds).get(C.PRECOMPILED_LABEL) == "true":
                # a kernel that still has nodes must not lose its driver mid-flight
                kernel = ((ds["spec"]["template"]["spec"].get("nodeSelector") or {}).get(C.NFD_KERNEL_LABEL))
                if kernel in self.kernel_map:
                    continue
            try:
                self.client.delete("apps/v1", "DaemonSet", o.name(ds), self.namespace)
                log.info("deleted stale driver DaemonSet %s", o.name(ds))
            except errors.NotFound:
                pass
        live = {o.name(d) for d in self.client.list("apps/v1", "DaemonSet", self.namespace,
                                                    label_selector={"app": base})}
        for pod in self.client.list("v1", "Pod", self.namespace, label_selector={"app": base}):
            ref = o.controller_of(pod)
            if ref and ref.get("kind") == "DaemonSet" and ref.get("name") not in live:
                pending = True
        return pending

    # -- walk --------------------------------------------------------------------------------
    def step(self, state: State) -> str:
        result = oc.READY
        for obj in state.objects:
            st = oc.apply_object(self, state, obj)
            if st == oc.NOT_READY:
                result = oc.NOT_READY
            elif st == oc.DISABLED and result == oc.READY:
                result = oc.DISABLED
        return result
