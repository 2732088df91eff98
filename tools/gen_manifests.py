#!/usr/bin/env python3
"""Generate the deployable manifests that derive from the code, so they can never drift:

* the ClusterPolicy CRD (OpenAPI v3 schema from ``ClusterPolicySpec``/``ClusterPolicyStatus``)
  -> config/crd/bases/, deployments/amd-gpu-operator/crds/, bundle/manifests/
* the operator's own RBAC (one rule table) -> config/rbac/role.yaml and the Helm chart's
  templates/clusterrole.yaml
* the OLM ClusterServiceVersion (relatedImages + ``*_IMAGE`` env from the chart's values,
  alm-examples from the sample CR) -> bundle/manifests/ and config/manifests/bases/
* the validator's workload-pod ConfigMap (the admin-overridable copy of
  gpu_operator_amd/validator/manifests/*.yaml, the pod templates the validator spawns)
  -> gpu_operator_amd/assets/state-operator-validation/0600_configmap_workloads.yaml

Reference counterpart: controller-gen + operator-sdk.
``python tools/gen_manifests.py`` rewrites them; ``--check`` exits 1 if any is stale (CI).
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path
from typing import Dict, List

import yaml

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from gpu_operator_amd.api.v1 import clusterpolicy as cp  # noqa: E402

VERSION = "v0.1.0"
CHART = ROOT / "deployments" / "amd-gpu-operator"
CRD_NAME = f"{cp.PLURAL}.{cp.GROUP}"
CRD_FILE = f"{cp.GROUP}_{cp.PLURAL}.yaml"


def crd() -> Dict:
    spec_schema = cp.ClusterPolicySpec.openapi()
    status_schema = cp.ClusterPolicyStatus.openapi()
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": CRD_NAME, "annotations": {"amd.com/generated-by": "tools/gen_manifests.py"}},
        "spec": {
            "group": cp.GROUP,
            "names": {"kind": cp.KIND, "listKind": cp.KIND + "List", "plural": cp.PLURAL,
                      "singular": "clusterpolicy", "shortNames": ["cpamd"]},
            "scope": "Cluster",
            "versions": [{
                "name": cp.VERSION, "served": True, "storage": True,
                "subresources": {"status": {}},
                "additionalPrinterColumns": [
                    {"name": "Status", "type": "string", "jsonPath": ".status.state"},
                    {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"}],
                "schema": {"openAPIV3Schema": {
                    "description": "ClusterPolicy: the AMD GPU operator's desired node configuration.",
                    "type": "object",
                    "properties": {
                        "apiVersion": {"type": "string"}, "kind": {"type": "string"},
                        "metadata": {"type": "object"},
                        "spec": spec_schema, "status": status_schema}}},
            }],
        },
    }


def r(groups, resources, verbs):
    return {"apiGroups": groups, "resources": resources, "verbs": verbs}


ALL = ["get", "list", "watch", "create", "update", "patch", "delete"]
RO = ["get", "list", "watch"]

# Everything the controller manager touches (C2/C8/C10; leader election; events).
OPERATOR_RULES: List[Dict] = [
    r(["amd.com"], ["clusterpolicies", "clusterpolicies/finalizers"], ALL),
    r(["amd.com"], ["clusterpolicies/status"], ["get", "update", "patch"]),
    r([""], ["nodes"], ["get", "list", "watch", "update", "patch"]),
    r([""], ["pods"], ["get", "list", "watch", "delete"]),
    r([""], ["pods/eviction"], ["create"]),
    r([""], ["namespaces"], ["get", "list", "watch", "update", "patch"]),
    r([""], ["configmaps", "services", "serviceaccounts", "secrets", "endpoints"], ALL),
    r([""], ["events"], ["create", "patch", "list", "watch"]),
    r(["apps"], ["daemonsets", "deployments", "controllerrevisions"], ALL),
    r(["rbac.authorization.k8s.io"], ["roles", "rolebindings", "clusterroles", "clusterrolebindings"],
      ALL + ["bind", "escalate"]),
    r(["node.k8s.io"], ["runtimeclasses"], ALL),
    r(["policy"], ["podsecuritypolicies"], ALL + ["use"]),
    r(["security.openshift.io"], ["securitycontextconstraints"], ALL + ["use"]),
    r(["monitoring.coreos.com"], ["servicemonitors", "prometheusrules"], ALL),
    r(["coordination.k8s.io"], ["leases"], ALL),
    r(["apiextensions.k8s.io"], ["customresourcedefinitions"], RO),
    r(["config.openshift.io"], ["clusterversions", "proxies"], RO),
    r(["image.openshift.io"], ["imagestreams"], RO),
    r(["nfd.k8s-sigs.io"], ["nodefeaturerules"], ALL),
]


def operator_clusterrole(name: str = "amd-gpu-operator") -> Dict:
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": {"name": name}, "rules": OPERATOR_RULES}


def chart_values() -> Dict:
    with open(CHART / "values.yaml") as f:
        return yaml.safe_load(f)


def image_envs(values: Dict) -> Dict[str, str]:
    """``*_IMAGE`` env of the operator Deployment: the fallback images (reference: CSV env)."""
    out = {}
    for key, env in (("driver", "DRIVER_IMAGE"), ("toolkit", "CONTAINER_TOOLKIT_IMAGE"),
                     ("devicePlugin", "DEVICE_PLUGIN_IMAGE"), ("metricsExporter", "METRICS_EXPORTER_IMAGE"),
                     ("rdc", "RDC_IMAGE"), ("nodeLabeller", "NODE_LABELLER_IMAGE"),
                     ("validator", "VALIDATOR_IMAGE"), ("partitionManager", "PARTITION_MANAGER_IMAGE"),
                     ("vfioManager", "VFIO_MANAGER_IMAGE"), ("mxgpuManager", "MXGPU_MANAGER_IMAGE"),
                     ("mxgpuDeviceManager", "MXGPU_DEVICE_MANAGER_IMAGE"),
                     ("sandboxDevicePlugin", "SANDBOX_DEVICE_PLUGIN_IMAGE"), ("kataManager", "KATA_MANAGER_IMAGE")):
        v = values.get(key) or {}
        if v.get("repository") and v.get("image") and v.get("version"):
            out[env] = f"{v['repository']}/{v['image']}:{v['version']}"
    dm = (values.get("driver") or {}).get("manager") or {}
    if dm.get("image"):
        out["DRIVER_MANAGER_IMAGE"] = f"{dm['repository']}/{dm['image']}:{dm['version']}"
    ic = (values.get("operator") or {}).get("initContainer") or {}
    if ic.get("image"):
        out["ROCM_BASE_IMAGE"] = f"{ic['repository']}/{ic['image']}:{ic['version']}"
    return out


def csv() -> Dict:
    values = chart_values()
    op = values["operator"]
    op_image = f"{op['repository']}/{op['image']}:{op.get('version') or VERSION}"
    envs = image_envs(values)
    with open(ROOT / "config" / "samples" / "amd_v1_clusterpolicy.yaml") as f:
        sample = yaml.safe_load(f)
    sample.pop("status", None)
    related = [{"name": "amd-gpu-operator", "image": op_image}] + [
        {"name": k.lower().replace("_image", "").replace("_", "-"), "image": v} for k, v in sorted(envs.items())]
    deployment = {
        "name": "amd-gpu-operator",
        "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "amd-gpu-operator"}},
                 "template": {"metadata": {"labels": {"app": "amd-gpu-operator"}},
                              "spec": {"serviceAccountName": "amd-gpu-operator",
                                       "priorityClassName": "system-node-critical",
                                       "containers": [{
                                           "name": "amd-gpu-operator", "image": op_image,
                                           "command": ["amd-gpu-operator"],
                                           "args": ["--leader-elect", "--zap-time-encoding=epoch"],
                                           "env": [{"name": "OPERATOR_NAMESPACE", "valueFrom": {
                                               "fieldRef": {"fieldPath": "metadata.namespace"}}}]
                                                  + [{"name": k, "value": v} for k, v in sorted(envs.items())],
                                           "ports": [{"name": "metrics", "containerPort": 8080}],
                                           "livenessProbe": {"httpGet": {"path": "/healthz", "port": 8081},
                                                             "initialDelaySeconds": 15, "periodSeconds": 20},
                                           "readinessProbe": {"httpGet": {"path": "/readyz", "port": 8081},
                                                              "initialDelaySeconds": 5, "periodSeconds": 10}}]}}},
    }
    return {
        "apiVersion": "operators.coreos.com/v1alpha1",
        "kind": "ClusterServiceVersion",
        "metadata": {
            "name": f"amd-gpu-operator.{VERSION}",
            "namespace": "placeholder",
            "annotations": {
                "alm-examples": json.dumps([sample], indent=2),
                "capabilities": "Deep Insights",
                "categories": "AI/Machine Learning, Monitoring",
                "operators.operatorframework.io/builder": "tools/gen_manifests.py",
                "containerImage": op_image,
                "description": "Automates AMD Instinct GPU (MI355X) node provisioning on Kubernetes",
            },
        },
        "spec": {
            "displayName": "AMD GPU Operator",
            "description": "Deploys and validates the amdgpu driver, container runtime hook/CDI, ROCm device "
                           "plugin, node labeller, partition manager, telemetry and the MFMA/RCCL node validator.",
            "version": VERSION.lstrip("v"),
            "maturity": "alpha",
            "minKubeVersion": "1.25.0",
            "keywords": ["amd", "gpu", "rocm", "instinct", "mi355x"],
            "provider": {"name": "AMD GPU operator authors"},
            "links": [{"name": "Source", "url": "https://example.invalid/amd-gpu-operator"}],
            "installModes": [{"type": "OwnNamespace", "supported": True},
                             {"type": "SingleNamespace", "supported": True},
                             {"type": "MultiNamespace", "supported": False},
                             {"type": "AllNamespaces", "supported": False}],
            "relatedImages": related,
            "customresourcedefinitions": {"owned": [{
                "name": CRD_NAME, "kind": cp.KIND, "version": cp.VERSION, "displayName": "ClusterPolicy",
                "description": "Cluster-wide AMD GPU node configuration",
                "statusDescriptors": [{"path": "state", "displayName": "State",
                                       "x-descriptors": ["urn:alm:descriptor:text"]}]}]},
            "install": {"strategy": "deployment", "spec": {
                "clusterPermissions": [{"serviceAccountName": "amd-gpu-operator", "rules": OPERATOR_RULES}],
                "deployments": [deployment]}},
        },
    }


class _NoAliasDumper(yaml.SafeDumper):
    def ignore_aliases(self, data):
        return True


def _yaml(obj) -> str:
    return yaml.dump(obj, Dumper=_NoAliasDumper, sort_keys=False, width=120)


def dump(obj) -> str:
    return "# generated by tools/gen_manifests.py -- do not edit\n" + _yaml(obj)


WORKLOAD_MANIFESTS = ROOT / "gpu_operator_amd" / "validator" / "manifests"


def workloads_configmap() -> str:
    """The validation pod templates, verbatim, as the ConfigMap the validator state deploys."""
    head = ("# generated by tools/gen_manifests.py -- do not edit (source: gpu_operator_amd/validator/manifests/)\n"
            "# Pod templates the validator spawns (mounted at /var/amd/manifests in the validator image\n"
            "# as well; this ConfigMap lets a cluster admin override them without rebuilding the image).\n"
            "apiVersion: v1\nkind: ConfigMap\nmetadata:\n  name: amd-validator-workloads\n"
            "  namespace: FILLED_BY_OPERATOR\n  labels:\n    app: amd-operator-validator\ndata:\n")
    body = ""
    for f in sorted(WORKLOAD_MANIFESTS.glob("*.yaml")):
        body += f"  {f.name}: |-\n" + "".join("    " + ln if ln.strip() else "\n"
                                               for ln in f.read_text().rstrip("\n").splitlines(True)) + "\n"
    return head + body


def outputs() -> Dict[Path, str]:
    c = dump(crd())
    cr = operator_clusterrole()
    chart_cr = ("# generated by tools/gen_manifests.py -- do not edit\n"
                "apiVersion: rbac.authorization.k8s.io/v1\nkind: ClusterRole\nmetadata:\n"
                "  name: {{ include \"amd-gpu-operator.fullname\" . }}\n"
                "  labels:\n    {{- include \"amd-gpu-operator.labels\" . | nindent 4 }}\n"
                + _yaml({"rules": OPERATOR_RULES}))
    s = dump(csv())
    return {
        ROOT / "config" / "crd" / "bases" / CRD_FILE: c,
        CHART / "crds" / CRD_FILE: c,
        ROOT / "bundle" / "manifests" / CRD_FILE: c,
        ROOT / "config" / "rbac" / "role.yaml": dump(cr),
        CHART / "templates" / "clusterrole.yaml": chart_cr,
        ROOT / "bundle" / "manifests" / "amd-gpu-operator.clusterserviceversion.yaml": s,
        ROOT / "config" / "manifests" / "bases" / "amd-gpu-operator.clusterserviceversion.yaml": s,
        ROOT / "gpu_operator_amd" / "assets" / "state-operator-validation" / "0600_configmap_workloads.yaml":
            workloads_configmap(),
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args(argv)
    stale = []
    for path, text in outputs().items():
        cur = path.read_text() if path.exists() else None
        if cur != text:
            stale.append(path)
            if not a.check:
                path.parent.mkdir(parents=True, exist_ok=True)
                path.write_text(text)
    for p in stale:
        print(("stale: " if a.check else "wrote: ") + str(p.relative_to(ROOT)))
    return 1 if (a.check and stale) else 0


if __name__ == "__main__":
    sys.exit(main())
