"""Per-operand DaemonSet transforms: turn an asset template into the DaemonSet the
ClusterPolicy asks for (image, pull policy/secrets, resources, args, env, runtime wiring and
operand-specific knobs).

One function per operand DaemonSet, dispatched by name, as in the reference
(reference: controllers/object_controls.go:654-698 and the Transform* functions at
:749-2030). Differences by design:

  * errors are never swallowed (the reference's TransformDevicePlugin drops the
    config-manager error, object_controls.go:1234-1237);
  * the driver's repo/cert mounts follow the *GPU node's* OS (from NFD labels), not the
    operator pod's /host-etc/os-release (quirk 7);
  * every transform is a pure function of (template, spec, context) so the golden tests can
    pin its output.
"""

from __future__ import annotations

import json
import re
from typing import Any, Callable, Dict, List, Optional

import yaml

from ..api.v1 import clusterpolicy as cp
from ..k8s import objects as o
from . import consts as C

Obj = Dict[str, Any]


class TransformError(Exception):
    pass


# ---------------------------------------------------------------------------------------------
# shared helpers (reference: object_controls.go:2033-2289, 3041-3080)
# ---------------------------------------------------------------------------------------------
def _container(obj: Obj, name: str, init: bool = False) -> Obj:
    c = o.find_container(obj, name, init=init)
    if c is None:
        kind = "init container" if init else "container"
        raise TransformError(f"{kind} {name!r} missing from DaemonSet {o.name(obj)} manifest")
    return c


def _add_pull_secrets(obj: Obj, secrets: Optional[List[str]]) -> None:
    if not secrets:
        return
    ps = o.pod_spec(obj).setdefault("imagePullSecrets", [])
    have = {s.get("name") for s in ps}
    for s in secrets:
        if s not in have:
            ps.append({"name": s})
            have.add(s)


def apply_component(obj: Obj, container: Obj, spec: cp.ComponentSpec, image: Optional[str] = None) -> None:
    """Image, pull policy/secrets, resources, args and env of a component's main container."""
    container["image"] = image or cp.image_path(spec)
    container["imagePullPolicy"] = cp.image_pull_policy(spec.imagePullPolicy)
    _add_pull_secrets(obj, spec.imagePullSecrets)
    if spec.resources is not None:
        res = {}
        if spec.resources.limits:
            res["limits"] = dict(spec.resources.limits)
        if spec.resources.requests:
            res["requests"] = dict(spec.resources.requests)
        container["resources"] = res
    if spec.args:
        container["args"] = list(spec.args)
    for e in spec.env or []:
        o.set_env(container, e.name, e.value or "")


def set_runtime_class(obj: Obj, runtime: str, runtime_class: str) -> None:
    """RuntimeClass only applies on containerd (CRI-O uses OCI hooks, docker its default
    runtime), as in the reference's setRuntimeClass."""
    if runtime == "containerd":
        o.pod_spec(obj)["runtimeClassName"] = runtime_class


def set_probe(container: Obj, kind: str, probe: Optional[cp.ContainerProbeSpec]) -> None:
    if probe is None:
        return
    p = container.setdefault(kind, {})
    for f in ("initialDelaySeconds", "timeoutSeconds", "periodSeconds", "successThreshold",
              "failureThreshold"):
        v = getattr(probe, f)
        if v is not None:
            p[f] = v


def transform_validation_init_containers(obj: Obj, spec: cp.ClusterPolicySpec) -> None:
    """Point every ``*-validation`` init container at the validator image; drop the RDMA
    validation when RDMA is off (reference: transformValidationInitContainer)."""
    inits = o.containers(obj, init=True)
    kept = []
    for c in inits:
        if "validation" not in c.get("name", ""):
            kept.append(c)
            continue
        if c["name"] == "rdma-validation":
            if not spec.driver.rdma or not spec.driver.rdma.is_enabled():
                continue
            o.set_env(c, "RDMA_ENABLED", "true")
            if spec.driver.rdma.useHostMofed:
                o.set_env(c, "USE_HOST_MOFED", "true")
        c["image"] = cp.image_path(spec.validator)
        if spec.validator.imagePullPolicy:
            c["imagePullPolicy"] = cp.image_pull_policy(spec.validator.imagePullPolicy)
        kept.append(c)
    o.pod_spec(obj)["initContainers"] = kept
    _add_pull_secrets(obj, spec.validator.imagePullSecrets)


def transform_driver_manager(obj: Obj, mgr: Optional[cp.DriverManagerSpec], spec: cp.ClusterPolicySpec,
                             auto_upgrade: bool = False) -> None:
    c = o.find_container(obj, "amd-driver-manager", init=True)
    if c is None:
        return
    mgr = mgr or cp.DriverManagerSpec()
    c["image"] = cp.image_path(mgr)
    c["imagePullPolicy"] = cp.image_pull_policy(mgr.imagePullPolicy)
    _add_pull_secrets(obj, mgr.imagePullSecrets)
    pol = spec.driver.upgradePolicy
    if auto_upgrade and pol is not None:
        # The upgrade controller already evicts/drains: the manager only unloads.
        o.set_env(c, "ENABLE_GPU_POD_EVICTION", "false")
        o.set_env(c, "ENABLE_AUTO_DRAIN", "false")
    elif pol is not None and pol.drain is not None:
        d = pol.drain
        o.set_env(c, "ENABLE_AUTO_DRAIN", "true" if d.enable else "false")
        o.set_env(c, "DRAIN_USE_FORCE", "true" if d.force else "false")
        o.set_env(c, "DRAIN_POD_SELECTOR_LABEL", d.podSelector or "")
        o.set_env(c, "DRAIN_TIMEOUT_SECONDS", f"{d.timeout()}s")
        o.set_env(c, "DRAIN_DELETE_EMPTYDIR_DATA", "true" if d.deleteEmptyDir else "false")
    for e in mgr.env or []:
        o.set_env(c, e.name, e.value or "")


def apply_runtime_mounts(obj: Obj, container: Obj, runtime: str, env_prefix: str = "") -> None:
    """Mount the container runtime's config directory and socket and export their paths."""
    cfg, sock = C.RUNTIME_CONFIG[runtime]
    cfg_dir, cfg_file = cfg.rsplit("/", 1)
    sock_dir, sock_file = sock.rsplit("/", 1)
    o.set_env(container, "RUNTIME", runtime)
    o.set_env(container, f"{env_prefix}RUNTIME_CONFIG", f"/runtime/config-dir/{cfg_file}")
    o.set_env(container, f"{env_prefix}RUNTIME_SOCKET", f"/runtime/sock-dir/{sock_file}")
    o.add_volume(obj, o.host_path_volume("runtime-config", cfg_dir, "DirectoryOrCreate"))
    o.add_volume(obj, o.host_path_volume("runtime-socket", sock_dir))
    o.add_volume_mount(container, {"name": "runtime-config", "mountPath": "/runtime/config-dir/"})
    o.add_volume_mount(container, {"name": "runtime-socket", "mountPath": "/runtime/sock-dir/"})


def sanitize_kernel_version(kernel: str) -> str:
    """DNS-1123-safe kernel string for per-kernel DaemonSet names (reference:
    getSanitizedKernelVersion, object_controls.go:2423-2428)."""
    s = re.sub(r"x86_64|aarch64", "", kernel).replace("_", ".").rstrip(".")
    return s.lower()


# ---------------------------------------------------------------------------------------------
# driver (reference: TransformDriver :837-882, transformDriverContainer :2718-2948)
# ---------------------------------------------------------------------------------------------
OS_REPO_DIRS = {
    "ubuntu": "/etc/apt/sources.list.d", "debian": "/etc/apt/sources.list.d",
    "rhel": "/etc/yum.repos.d", "rocky": "/etc/yum.repos.d", "centos": "/etc/yum.repos.d",
    "almalinux": "/etc/yum.repos.d", "ol": "/etc/yum.repos.d", "rhcos": "/etc/yum.repos.d",
    "fedora": "/etc/yum.repos.d", "sles": "/etc/zypp/repos.d", "sle": "/etc/zypp/repos.d",
    "azurelinux": "/etc/yum.repos.d",
}
OS_CERT_DIRS = {
    "ubuntu": "/usr/local/share/ca-certificates", "debian": "/usr/local/share/ca-certificates",
    "rhel": "/etc/pki/ca-trust/extracted/pem", "rocky": "/etc/pki/ca-trust/extracted/pem",
    "centos": "/etc/pki/ca-trust/extracted/pem", "almalinux": "/etc/pki/ca-trust/extracted/pem",
    "rhcos": "/etc/pki/ca-trust/extracted/pem", "fedora": "/etc/pki/ca-trust/extracted/pem",
    "sles": "/etc/pki/trust/anchors", "sle": "/etc/pki/trust/anchors",
    "azurelinux": "/etc/pki/ca-trust/extracted/pem",
}


def _os_id(os_tag: str) -> str:
    m = re.match(r"([a-z]+)", os_tag or "")
    return m.group(1) if m else ""


def resolve_driver_image(spec: cp.ImageSpec, os_tag: str, precompiled: bool = False,
                         kernel: str = "") -> str:
    """``repo/image:version-<os>`` (+ ``-<kernel>`` before the OS tag for precompiled
    images); a digest is used verbatim (reference: resolveDriverTag :2565-2619)."""
    if precompiled:
        if not spec.repository and not spec.version:
            if not spec.image:
                raise TransformError("precompiled drivers need driver.repository/image/version")
            image = f"{spec.image}-{kernel}"
        else:
            image = f"{spec.repository}/{spec.image}:{spec.version}-{kernel}"
    else:
        image = cp.image_path(spec)
    if "sha256:" not in image:
        if not os_tag:
            raise TransformError("cannot resolve driver image: GPU node OS unknown (NFD labels missing)")
        image = f"{image}-{os_tag}"
    return image


def transform_driver(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    transform_driver_manager(obj, spec.driver.manager, spec, n.driver_auto_upgrade())
    c = _container(obj, "amdgpu-driver-ctr")
    os_tag = n.node_os_tag()
    precompiled = spec.driver.use_precompiled()
    image = resolve_driver_image(spec.driver, os_tag, precompiled, n.current_kernel or "")
    apply_component(obj, c, spec.driver, image=image)
    set_probe(c, "startupProbe", spec.driver.startupProbe)
    set_probe(c, "livenessProbe", spec.driver.livenessProbe)
    set_probe(c, "readinessProbe", spec.driver.readinessProbe)

    if spec.driver.rdma and spec.driver.rdma.is_enabled():
        o.set_env(c, "RDMA_ENABLED", "true")
        if spec.driver.rdma.useHostMofed:
            o.set_env(c, "USE_HOST_MOFED", "true")
            for v in o.pod_spec(obj).get("volumes", []):
                if v["name"] == "run-mellanox-drivers":
                    v["hostPath"]["path"] = "/run/mellanox/drivers"
    if spec.driver.blacklistDrivers:
        o.set_env(c, "BLACKLIST_DRIVERS", ",".join(spec.driver.blacklistDrivers))

    os_id = _os_id(os_tag)
    if spec.driver.repoConfig and spec.driver.repoConfig.configMapName:
        dest = OS_REPO_DIRS.get(os_id)
        if dest is None:
            raise TransformError(f"no package repository directory known for OS {os_id!r}")
        o.add_volume(obj, {"name": "repo-config", "configMap": {"name": spec.driver.repoConfig.configMapName}})
        o.add_volume_mount(c, {"name": "repo-config", "mountPath": dest, "readOnly": True})
    if spec.driver.certConfig and spec.driver.certConfig.name:
        dest = OS_CERT_DIRS.get(os_id)
        if dest is None:
            raise TransformError(f"no certificate directory known for OS {os_id!r}")
        o.add_volume(obj, {"name": "cert-config", "configMap": {"name": spec.driver.certConfig.name}})
        o.add_volume_mount(c, {"name": "cert-config", "mountPath": dest, "readOnly": True})
    if spec.driver.kernelModuleConfig and spec.driver.kernelModuleConfig.name:
        o.add_volume(obj, {"name": "kernel-module-config",
                           "configMap": {"name": spec.driver.kernelModuleConfig.name,
                                         "items": [{"key": "amdgpu.conf", "path": "amdgpu.conf"}]}})
        o.add_volume_mount(c, {"name": "kernel-module-config", "mountPath": "/drivers", "readOnly": True})
        o.set_env(c, "KERNEL_MODULE_PARAMS", "/drivers/amdgpu.conf")

    if n.openshift:
        o.set_env(c, "OPENSHIFT_VERSION", n.openshift)
        if n.variant_kind == "dtk":
            add_driver_toolkit_sidecar(obj, c, n)
        proxy = n.cluster_proxy()
        for k, v in proxy.items():
            o.set_env(c, k, v)
        ca = n.trusted_ca_configmap() if hasattr(n, "trusted_ca_configmap") else ""
        if ca:
            # the proxy's user CA bundle, where the driver container's package manager trusts it
            o.add_volume(obj, {"name": ca, "configMap": {"name": ca, "items": [
                {"key": C.TRUSTED_CA_BUNDLE_KEY, "path": C.TRUSTED_CA_CERT_FILE}]}})
            o.add_volume_mount(c, {"name": ca, "mountPath": C.TRUSTED_CA_MOUNT_DIR, "readOnly": True})
    apply_variant_identity(obj, n)


def split_os_tag(os_tag: str):
    m = re.match(r"^([a-z]+)(.*)$", os_tag or "")
    return (m.group(1), m.group(2)) if m else ("", "")


def apply_variant_identity(obj: Obj, n) -> None:
    """Make a fanned-out DaemonSet variant-specific: name suffix, identity labels and the node
    selector that pins it to its kernel (precompiled; reference:
    transformPrecompiledDriverDaemonset :2430-2442), RHCOS version (DTK) or OS (a cluster
    mixing node OSes gets one driver DaemonSet per OS instead of assuming the first node's,
    SURVEY.md §7.7 quirk 4)."""
    kind = n.variant_kind
    if not kind:
        return
    base = o.name(obj)
    sel = o.pod_spec(obj).setdefault("nodeSelector", {})
    if kind == "precompiled":
        o.labels(obj)[C.PRECOMPILED_LABEL] = "true"
        o.pod_template_meta(obj).setdefault("labels", {})[C.PRECOMPILED_LABEL] = "true"
        sel[C.NFD_KERNEL_LABEL] = n.current_kernel
        v = {"kind": kind, "kernel": n.current_kernel, "os": n.kernel_map.get(n.current_kernel, "")}
    elif kind == "dtk":
        v = {"kind": kind, "rhcos": n.current_rhcos}
    else:
        osid, ver = split_os_tag(n.current_os)
        sel[C.NFD_OS_ID_LABEL] = osid
        sel[C.NFD_OS_VERSION_LABEL] = ver
        v = {"kind": kind, "os": n.current_os}
    o.meta(obj)["name"] = n.variant_name(base, v)


def add_driver_toolkit_sidecar(obj: Obj, driver_ctr: Obj, n) -> None:
    """OpenShift Driver Toolkit: build amdgpu against the RHCOS kernel from the DTK image
    (one DaemonSet per RHCOS version; reference: transformOpenShiftDriverToolkitContainer)."""
    rhcos = n.current_rhcos
    image = n.dtk_images.get(rhcos)
    if not image:
        raise TransformError(f"no driver-toolkit image for RHCOS {rhcos}")
    o.labels(obj)["openshift.driver-toolkit"] = "true"
    o.labels(obj)["openshift.driver-toolkit.rhcos"] = rhcos
    tmeta = o.pod_template_meta(obj).setdefault("labels", {})
    tmeta["openshift.driver-toolkit"] = "true"
    tmeta["openshift.driver-toolkit.rhcos"] = rhcos
    o.pod_spec(obj).setdefault("nodeSelector", {})[C.NFD_OSTREE_LABEL] = rhcos
    o.set_env(driver_ctr, "RHCOS_VERSION", rhcos)
    o.set_env(driver_ctr, "USE_DRIVER_TOOLKIT", "true")
    o.add_volume(obj, {"name": "shared-amd-driver-toolkit", "emptyDir": {}})
    o.add_volume_mount(driver_ctr, {"name": "shared-amd-driver-toolkit", "mountPath": "/mnt/shared-amd-driver-toolkit"})
    sidecar = {"name": "openshift-driver-toolkit-ctr", "image": image,
               "command": ["bash", "-xc"],
               "args": ["until [ -f /mnt/shared-amd-driver-toolkit/dir_prepared ]; do sleep 1; done; "
                        "exec /mnt/shared-amd-driver-toolkit/amdgpu-dtk-build"],
               "securityContext": {"privileged": True, "seLinuxOptions": {"level": "s0"}},
               "env": [{"name": "RHCOS_VERSION", "value": rhcos}],
               "volumeMounts": [{"name": "shared-amd-driver-toolkit",
                                 "mountPath": "/mnt/shared-amd-driver-toolkit"}]}
    o.remove_container(obj, "openshift-driver-toolkit-ctr")
    o.containers(obj).append(sidecar)


def transform_mxgpu_manager(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_driver_manager(obj, spec.mxgpuManager.driverManager, spec)
    c = _container(obj, "amd-mxgpu-manager-ctr")
    image = resolve_driver_image(spec.mxgpuManager, n.node_os_tag())
    apply_component(obj, c, spec.mxgpuManager, image=image)
    apply_variant_identity(obj, n)


# ---------------------------------------------------------------------------------------------
# runtime hook (reference: TransformToolkit :1052-1184)
# ---------------------------------------------------------------------------------------------
def transform_toolkit(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    c = _container(obj, "amd-container-toolkit-ctr")
    apply_component(obj, c, spec.toolkit)
    install_dir = spec.toolkit.install_dir()
    o.set_env(c, "ROOT", install_dir)
    for v in o.pod_spec(obj).get("volumes", []):
        if v["name"] == "toolkit-install-dir":
            v["hostPath"]["path"] = install_dir
    for m in c.get("volumeMounts", []):
        if m["name"] == "toolkit-install-dir":
            m["mountPath"] = install_dir
    o.set_env(c, "RUNTIME_CLASS", spec.operator.runtime_class())
    runtime = n.runtime
    apply_runtime_mounts(obj, c, runtime)
    if runtime == "crio":
        o.set_env(c, "CRIO_HOOKS_DIR", "/usr/share/containers/oci/hooks.d")
    if spec.cdi.is_enabled():
        o.set_env(c, "CDI_ENABLED", "true")
        o.set_env(c, "AMD_RUNTIME_MODE", "cdi" if spec.cdi.is_default() else "auto")
    else:
        o.set_env(c, "AMD_RUNTIME_MODE", "legacy")


# ---------------------------------------------------------------------------------------------
# device plugin (reference: TransformDevicePlugin :1187-1256, handleDevicePluginConfig)
# ---------------------------------------------------------------------------------------------
def _config_manager(obj: Obj, main: Obj, image: str, cm_name: str, default: str, label: str,
                    mount_target: str, config_env: str, process: str) -> None:
    """config-manager init + sidecar: pick the named config from a ConfigMap according to a
    node label, write it to a shared dir and signal the main process on change."""
    common_env = [{"name": "NODE_NAME", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
                  {"name": "NODE_LABEL", "value": label},
                  {"name": "CONFIG_FILE_SRCDIR", "value": "/available-configs"},
                  {"name": "CONFIG_FILE_DST", "value": f"/config/{mount_target}"},
                  {"name": "DEFAULT_CONFIG", "value": default},
                  {"name": "FALLBACK_STRATEGIES", "value": "named,single"},
                  {"name": "SEND_SIGNAL", "value": "true"},
                  {"name": "SIGNAL", "value": "1"},
                  # the program the entrypoint execs: the main container's command is `sh -c`
                  {"name": "PROCESS_TO_SIGNAL", "value": process}]
    mounts = [{"name": "available-configs", "mountPath": "/available-configs"},
              {"name": "config", "mountPath": "/config"}]
    init = {"name": "config-manager-init", "image": image, "command": ["amd-config-manager"],
            "env": common_env + [{"name": "ONESHOT", "value": "true"}], "volumeMounts": mounts}
    side = {"name": "config-manager", "image": image, "command": ["amd-config-manager"],
            "env": common_env + [{"name": "ONESHOT", "value": "false"}], "volumeMounts": mounts,
            "securityContext": {"privileged": True}}
    o.remove_container(obj, "config-manager-init", init=True)
    o.remove_container(obj, "config-manager")
    o.containers(obj, init=True).append(init)
    o.containers(obj).append(side)
    o.pod_spec(obj)["shareProcessNamespace"] = True
    o.add_volume(obj, {"name": "available-configs", "configMap": {"name": cm_name}})
    o.add_volume(obj, {"name": "config", "emptyDir": {}})
    o.add_volume_mount(main, {"name": "config", "mountPath": "/config"})
    o.set_env(main, config_env, f"/config/{mount_target}")


def transform_device_plugin(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    c = _container(obj, "amd-device-plugin")
    apply_component(obj, c, spec.devicePlugin)
    o.set_env(c, "PARTITION_STRATEGY", spec.partition.get_strategy())
    if spec.cdi.is_enabled():
        o.set_env(c, "CDI_ENABLED", "true")
        o.set_env(c, "DEVICE_LIST_STRATEGY", "cdi-annotations" if spec.cdi.is_default() else "device-specs")
        o.set_env(c, "CDI_ANNOTATION_PREFIX", "amd.cdi.k8s.io/")
    if spec.driver.rdma and spec.driver.rdma.is_enabled():
        o.set_env(c, "RDMA_ENABLED", "true")
    cfg = spec.devicePlugin.config
    if cfg is not None and cfg.name:
        _config_manager(obj, c, c["image"], cfg.name, cfg.default or "", C.DEVICE_PLUGIN_CONFIG_LABEL,
                        "config.yaml", "CONFIG_FILE", "amd-device-plugin")
    set_runtime_class(obj, n.runtime, spec.operator.runtime_class())


def transform_sandbox_device_plugin(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    c = _container(obj, "amd-sandbox-device-plugin-ctr")
    apply_component(obj, c, spec.sandboxDevicePlugin)


# ---------------------------------------------------------------------------------------------
# telemetry (reference: TransformDCGM :1441-1494, TransformDCGMExporter :1302-1438)
# ---------------------------------------------------------------------------------------------
def transform_rdc(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    c = _container(obj, "amd-rdc-ctr")
    apply_component(obj, c, spec.rdc)
    port = spec.rdc.host_port()
    for p in c.get("ports", []):
        if p.get("name") == "rdc":
            p["hostPort"] = port
            p["containerPort"] = port
    c["args"] = list(spec.rdc.args) if spec.rdc.args else ["-u", "-p", str(port)]
    set_runtime_class(obj, n.runtime, spec.operator.runtime_class())


def transform_metrics_exporter(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    c = _container(obj, "amd-metrics-exporter")
    apply_component(obj, c, spec.metricsExporter)
    # Unlike dcgm-exporter (reference :1352-1355, which needs the DCGM host engine and so joins
    # the host network when DCGM runs standalone), amd-metrics-exporter reads the kernel and PMFW
    # telemetry (hwmon, gpu_metrics incl. per-link xGMI counters) natively, so it never attaches
    # to rdcd: the RDC state is for RDC's own clients (rdci, job stats) and widens nothing here.
    cfg = spec.metricsExporter.config
    if cfg is not None and cfg.name:
        for v in o.pod_spec(obj).get("volumes", []):
            if v["name"] == "fields":
                v["configMap"] = {"name": cfg.name}
        o.set_env(c, "METRICS_EXPORTER_FIELDS", "/etc/amd-metrics-exporter/fields.csv")
    if n.openshift:
        _add_pod_resources_relabel(obj, spec)
    set_runtime_class(obj, n.runtime, spec.operator.runtime_class())


RELABEL_INIT = "init-pod-resources-relabel"
RELABEL_CONFIGMAP = "amd-metrics-exporter-relabel"


def _add_pod_resources_relabel(obj: Obj, spec: cp.ClusterPolicySpec) -> None:
    """OpenShift: a privileged init container relabels /var/lib/kubelet/pod-resources container_file_t
    (the script of 0850_configmap_openshift.yaml), so the exporter container itself needs no privilege
    to reach the pod-resources socket (reference: object_controls.go:1393-1431, which does the same for
    dcgm-exporter with the operator's init-container image)."""
    ps = o.pod_spec(obj)
    inits = [x for x in ps.get("initContainers", []) if x.get("name") != RELABEL_INIT]
    init_spec = spec.operator.initContainer or cp.InitContainerSpec()
    try:
        image = cp.image_path(init_spec)
    except (ValueError, TypeError):
        image = cp.image_path(spec.validator)      # no ROCm base image configured: the validator image has chcon
    inits.append({"name": RELABEL_INIT, "image": image,
                  "imagePullPolicy": cp.image_pull_policy(init_spec.imagePullPolicy),
                  "command": ["/bin/entrypoint.sh"], "securityContext": {"privileged": True},
                  "volumeMounts": [{"name": "pod-gpu-resources", "mountPath": "/var/lib/kubelet/pod-resources"},
                                   {"name": "relabel-entrypoint", "mountPath": "/bin/entrypoint.sh", "readOnly": True,
                                    "subPath": "entrypoint.sh"}]})
    ps["initContainers"] = inits
    vols = [v for v in ps.get("volumes", []) if v.get("name") != "relabel-entrypoint"]
    vols.append({"name": "relabel-entrypoint", "configMap": {"name": RELABEL_CONFIGMAP, "defaultMode": 0o700}})
    ps["volumes"] = vols


def transform_node_status_exporter(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    c = _container(obj, "amd-node-status-exporter")
    apply_component(obj, c, spec.nodeStatusExporter)


# ---------------------------------------------------------------------------------------------
# labeller / partitioning (reference: TransformGPUDiscoveryPlugin :749-807, TransformMIGManager)
# ---------------------------------------------------------------------------------------------
def transform_node_labeller(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    c = _container(obj, "amd-node-labeller")
    apply_component(obj, c, spec.nodeLabeller)
    o.set_env(c, "PARTITION_STRATEGY", spec.partition.get_strategy())
    set_runtime_class(obj, n.runtime, spec.operator.runtime_class())


def transform_partition_manager(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_validation_init_containers(obj, spec)
    c = _container(obj, "amd-partition-manager")
    pm = spec.partitionManager
    apply_component(obj, c, pm)
    if pm.config is not None and pm.config.name:
        for v in o.pod_spec(obj).get("volumes", []):
            if v["name"] == "partition-config":
                v["configMap"] = {"name": pm.config.name}
    if pm.config is not None and pm.config.default:
        o.set_env(c, "DEFAULT_PARTITION_CONFIG", pm.config.default)
    if pm.gpuClientsConfig is not None and pm.gpuClientsConfig.name:
        for v in o.pod_spec(obj).get("volumes", []):
            if v["name"] == "gpu-clients":
                v["configMap"] = {"name": pm.gpuClientsConfig.name}
    if spec.cdi.is_enabled():
        o.set_env(c, "CDI_ENABLED", "true")
    o.set_env(c, "PARTITION_STRATEGY", spec.partition.get_strategy())
    # An NPS change needs amdgpu reloaded. When the driver container owns the module, only it has
    # the module tree that loaded it (precompiled .ko under /opt/amdgpu or its DKMS build): the
    # partition manager asks it through a request file in the shared /run/amd/driver and waits for
    # its answer (operands/driver_container.py, serve_reloads). With a host driver the agent's
    # default (modprobe via /host) applies. A user-set DRIVER_RELOAD_CMD wins.
    if spec.driver.is_enabled() and not any(e.get("name") == "DRIVER_RELOAD_CMD" for e in c.get("env", [])):
        o.set_env(c, "DRIVER_RELOAD_VIA", "driver-container")


# ---------------------------------------------------------------------------------------------
# validators (reference: TransformValidator :1803-1981, TransformSandboxValidator)
# ---------------------------------------------------------------------------------------------
VALIDATOR_COMPONENTS = {
    "driver-validation": "driver", "toolkit-validation": "toolkit", "hip-validation": "hip",
    "plugin-validation": "plugin", "rccl-validation": "rccl", "vfio-pci-validation": "vfioPCI",
    "mxgpu-manager-validation": "mxgpuManager", "mxgpu-devices-validation": "mxgpuDevices",
}


def _validator_common(obj: Obj, spec: cp.ClusterPolicySpec, n, main_name: str) -> None:
    v = spec.validator
    image = cp.image_path(v)
    main = _container(obj, main_name)
    apply_component(obj, main, v, image=image)
    for c in o.containers(obj, init=True):
        comp = VALIDATOR_COMPONENTS.get(c.get("name", ""))
        c["image"] = image
        c["imagePullPolicy"] = cp.image_pull_policy(v.imagePullPolicy)
        if comp is None:
            continue
        for e in v.component(comp).env or []:
            o.set_env(c, e.name, e.value or "")
        # what the spawned workload pods need to look like the validator itself
        o.set_env(c, "VALIDATOR_IMAGE", image)
        o.set_env(c, "VALIDATOR_IMAGE_PULL_POLICY", cp.image_pull_policy(v.imagePullPolicy))
        if v.imagePullSecrets:
            o.set_env(c, "VALIDATOR_IMAGE_PULL_SECRETS", ",".join(v.imagePullSecrets))
        if n.runtime == "containerd":
            o.set_env(c, "VALIDATOR_RUNTIME_CLASS", spec.operator.runtime_class())


def transform_validator(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    if not spec.devicePlugin.is_enabled():
        # no amd.com/gpu resources will appear: the plugin and RCCL pods could never schedule
        o.remove_container(obj, "plugin-validation", init=True)
        o.remove_container(obj, "rccl-validation", init=True)
    _validator_common(obj, spec, n, "amd-operator-validator")
    pv = o.find_container(obj, "plugin-validation", init=True)
    if pv is not None:
        o.set_env(pv, "PARTITION_STRATEGY", spec.partition.get_strategy())
    set_runtime_class(obj, n.runtime, spec.operator.runtime_class())


def transform_sandbox_validator(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    _validator_common(obj, spec, n, "amd-sandbox-validator")
    for c in o.containers(obj, init=True):
        if o.get_env(c, "DEFAULT_GPU_WORKLOAD_CONFIG") is not None:
            o.set_env(c, "DEFAULT_GPU_WORKLOAD_CONFIG", n.default_workload)


# ---------------------------------------------------------------------------------------------
# sandbox operands
# ---------------------------------------------------------------------------------------------
def transform_vfio_manager(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    transform_driver_manager(obj, spec.vfioManager.driverManager, spec)
    c = _container(obj, "amd-vfio-manager")
    apply_component(obj, c, spec.vfioManager)


def transform_mxgpu_device_manager(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    c = _container(obj, "amd-mxgpu-device-manager")
    apply_component(obj, c, spec.mxgpuDeviceManager)
    for ic in o.containers(obj, init=True):
        ic["image"] = cp.image_path(spec.validator)
    cfg = spec.mxgpuDeviceManager.config
    if cfg is not None and cfg.name:
        for v in o.pod_spec(obj).get("volumes", []):
            if v["name"] == "mxgpu-config":
                v["configMap"] = {"name": cfg.name}
    if cfg is not None and cfg.default:
        o.set_env(c, "DEFAULT_MXGPU_CONFIG", cfg.default)


def kata_config(spec: cp.ClusterPolicySpec) -> Dict[str, Any]:
    cfg = spec.kataManager.config
    d = cfg.to_dict() if cfg is not None else {}
    d.setdefault("artifactsDir", "/opt/amd-gpu-operator/artifacts/runtimeclasses")
    d.setdefault("runtimeClasses", [])
    return d


def transform_kata_manager(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    c = _container(obj, "amd-kata-manager")
    apply_component(obj, c, spec.kataManager)
    cfg = kata_config(spec)
    artifacts = cfg["artifactsDir"]
    o.set_env(c, "KATA_ARTIFACTS_DIR", artifacts)
    for v in o.pod_spec(obj).get("volumes", []):
        if v["name"] == "kata-artifacts":
            v["hostPath"]["path"] = artifacts
    for m in c.get("volumeMounts", []):
        if m["name"] == "kata-artifacts":
            m["mountPath"] = artifacts
    # roll the pods when the config changes (reference: object_controls.go:1666-1677)
    o.pod_template_meta(obj).setdefault("annotations", {})[C.KATA_CONFIG_HASH_ANNOTATION] = \
        o.stable_hash(cfg)
    if n.runtime == "crio":
        o.set_env(c, "RUNTIME", "crio")


# ---------------------------------------------------------------------------------------------
# dispatch + common DaemonSet config (reference: preProcessDaemonSet :654-746)
# ---------------------------------------------------------------------------------------------
TRANSFORMS: Dict[str, Callable[[Obj, cp.ClusterPolicySpec, Any], None]] = {
    C.DS_DRIVER: transform_driver,
    C.DS_MXGPU_MANAGER: transform_mxgpu_manager,
    C.DS_MXGPU_DEVICE_MANAGER: transform_mxgpu_device_manager,
    C.DS_VFIO_MANAGER: transform_vfio_manager,
    C.DS_TOOLKIT: transform_toolkit,
    C.DS_DEVICE_PLUGIN: transform_device_plugin,
    C.DS_SANDBOX_DEVICE_PLUGIN: transform_sandbox_device_plugin,
    C.DS_RDC: transform_rdc,
    C.DS_METRICS_EXPORTER: transform_metrics_exporter,
    C.DS_NODE_STATUS_EXPORTER: transform_node_status_exporter,
    C.DS_NODE_LABELLER: transform_node_labeller,
    C.DS_PARTITION_MANAGER: transform_partition_manager,
    C.DS_VALIDATOR: transform_validator,
    C.DS_SANDBOX_VALIDATOR: transform_sandbox_validator,
    C.DS_KATA_MANAGER: transform_kata_manager,
}


def apply_update_strategy(obj: Obj, spec: cp.ClusterPolicySpec) -> None:
    ds = spec.daemonsets
    if ds.updateStrategy == "OnDelete":
        obj["spec"]["updateStrategy"] = {"type": "OnDelete"}
        return
    if ds.rollingUpdate is None or not ds.rollingUpdate.maxUnavailable:
        return
    if o.name(obj).startswith(C.DS_DRIVER) or o.name(obj).startswith(C.DS_MXGPU_MANAGER):
        return  # a kernel-module DaemonSet is never rolled automatically
    mu = ds.rollingUpdate.maxUnavailable
    if not mu.endswith("%"):
        try:
            mu = int(mu)
        except ValueError as e:
            raise TransformError(f"invalid daemonsets.rollingUpdate.maxUnavailable {mu!r}") from e
    obj["spec"]["updateStrategy"] = {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": mu}}


def apply_common_config(obj: Obj, spec: cp.ClusterPolicySpec) -> None:
    apply_update_strategy(obj, spec)
    ds = spec.daemonsets
    if ds.priorityClassName:
        o.pod_spec(obj)["priorityClassName"] = ds.priorityClassName
    if ds.tolerations:
        o.pod_spec(obj)["tolerations"] = json.loads(json.dumps(ds.tolerations))


def apply_common_metadata(obj: Obj, spec: cp.ClusterPolicySpec) -> None:
    ds = spec.daemonsets
    tm = o.pod_template_meta(obj)
    for k, v in (ds.labels or {}).items():
        if k in ("app", "app.kubernetes.io/part-of"):
            continue   # selectors are immutable
        tm.setdefault("labels", {})[k] = v
    for k, v in (ds.annotations or {}).items():
        tm.setdefault("annotations", {})[k] = v
    for k, v in (spec.operator.labels or {}).items():
        if k not in ("app", "app.kubernetes.io/part-of"):
            tm.setdefault("labels", {}).setdefault(k, v)
    for k, v in (spec.operator.annotations or {}).items():
        tm.setdefault("annotations", {}).setdefault(k, v)


def preprocess_daemonset(obj: Obj, spec: cp.ClusterPolicySpec, n) -> None:
    base = n.template_name(obj)
    t = TRANSFORMS.get(base)
    if t is None:
        return
    apply_common_config(obj, spec)
    t(obj, spec, n)
    apply_common_metadata(obj, spec)


def render_kata_configmap_data(spec: cp.ClusterPolicySpec) -> Dict[str, str]:
    return {"config.yaml": yaml.safe_dump(kata_config(spec), sort_keys=True)}
