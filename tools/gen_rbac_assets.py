#!/usr/bin/env python3
"""Emit the per-operand RBAC manifests (ServiceAccount, Role, RoleBinding, ClusterRole,
ClusterRoleBinding, OpenShift SCC) of every state directory under gpu_operator_amd/assets.

Least privilege per operand: each operand's rules are listed here once, in one table, so
reviewing what a node agent may do is a single read. Re-run after editing the table:

    python tools/gen_rbac_assets.py
"""

import os
from pathlib import Path

import yaml

ASSETS = Path(__file__).resolve().parent.parent / "gpu_operator_amd" / "assets"
NS = "FILLED_BY_OPERATOR"

PSP_USE = {"apiGroups": ["policy"], "resources": ["podsecuritypolicies"], "verbs": ["use"],
           "resourceNames": ["amd-gpu-operator-privileged"]}
SCC_USE = {"apiGroups": ["security.openshift.io"], "resources": ["securitycontextconstraints"],
           "verbs": ["use"], "resourceNames": ["privileged"]}


def r(groups, resources, verbs, names=None):
    d = {"apiGroups": groups, "resources": resources, "verbs": verbs}
    if names:
        d["resourceNames"] = names
    return d


NODES_RO = r([""], ["nodes"], ["get", "list", "watch"])
NODES_RW = r([""], ["nodes"], ["get", "list", "watch", "patch", "update"])

# state dir -> (service account, namespaced rules, cluster rules)
OPERANDS = {
    "state-driver": ("amdgpu-driver",
                     [r([""], ["pods", "pods/eviction"], ["get", "list", "watch", "delete", "create"]),
                      r(["apps"], ["daemonsets"], ["get", "list", "watch"]),
                      r([""], ["configmaps"], ["get", "list", "watch"])],
                     [NODES_RW, r([""], ["pods", "pods/eviction"], ["get", "list", "watch", "delete", "create"]),
                      r(["apps"], ["daemonsets", "deployments", "replicasets", "statefulsets"], ["get", "list"])]),
    "state-container-toolkit": ("amd-container-toolkit",
                                [r([""], ["pods"], ["get", "list"])], []),
    "state-operator-validation": ("amd-operator-validator",
                                  [r([""], ["pods"], ["get", "list", "watch", "create", "delete"]),
                                   r(["apps"], ["daemonsets"], ["get", "list"])],
                                  # read-only on nodes: the last full fabric result stays on the node
                                  # (barrier dir file fabric-last-full), no Node writes
                                  [NODES_RO, r([""], ["pods"], ["get", "list"])]),
    "state-device-plugin": ("amd-device-plugin",
                            [r([""], ["configmaps"], ["get", "list", "watch"])],
                            [NODES_RW]),
    "state-rdc": ("amd-rdc", [], []),
    "state-metrics-exporter": ("amd-metrics-exporter",
                               [r([""], ["services", "endpoints", "pods"], ["get", "list", "watch"])],
                               [NODES_RO]),
    "state-node-labeller": ("amd-node-labeller", [r([""], ["configmaps"], ["get", "list", "watch"])],
                            [NODES_RW]),
    "state-partition-manager": ("amd-partition-manager",
                                [r([""], ["configmaps"], ["get", "list", "watch"]),
                                 r([""], ["pods"], ["get", "list", "watch", "delete"]),
                                 r(["apps"], ["daemonsets"], ["get", "list"])],
                                [NODES_RW, r([""], ["pods"], ["get", "list"])]),
    "state-node-status-exporter": ("amd-node-status-exporter",
                                   [r([""], ["pods"], ["get", "list"])], [NODES_RO]),
    "state-mxgpu-manager": ("amd-mxgpu-manager",
                            [r([""], ["pods", "pods/eviction"], ["get", "list", "watch", "delete", "create"]),
                             r(["apps"], ["daemonsets"], ["get", "list"])],
                            [NODES_RW, r([""], ["pods", "pods/eviction"], ["get", "list", "delete", "create"])]),
    "state-mxgpu-device-manager": ("amd-mxgpu-device-manager",
                                   [r([""], ["configmaps"], ["get", "list", "watch"])], [NODES_RW]),
    "state-sandbox-validation": ("amd-sandbox-validator", [r([""], ["pods"], ["get", "list"])],
                                 [NODES_RO]),
    "state-vfio-manager": ("amd-vfio-manager",
                           [r([""], ["pods", "pods/eviction"], ["get", "list", "watch", "delete", "create"]),
                            r(["apps"], ["daemonsets"], ["get", "list"])],
                           [NODES_RW, r([""], ["pods", "pods/eviction"], ["get", "list", "delete", "create"])]),
    "state-sandbox-device-plugin": ("amd-sandbox-device-plugin", [], [NODES_RO]),
    "state-kata-manager": ("amd-kata-manager",
                           [r([""], ["configmaps"], ["get", "list", "watch"])],
                           [NODES_RO, r(["node.k8s.io"], ["runtimeclasses"], ["get", "list"])]),
}


def dump(path: Path, obj) -> None:
    path.write_text(yaml.safe_dump(obj, sort_keys=False))


def main():
    for state, (sa, rules, crules) in OPERANDS.items():
        d = ASSETS / state
        d.mkdir(parents=True, exist_ok=True)
        app = {"app.kubernetes.io/part-of": "amd-gpu-operator"}
        dump(d / "0100_service_account.yaml",
             {"apiVersion": "v1", "kind": "ServiceAccount",
              "metadata": {"name": sa, "namespace": NS, "labels": app}})
        dump(d / "0200_role.yaml",
             {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
              "metadata": {"name": sa, "namespace": NS, "labels": app},
              "rules": [SCC_USE, PSP_USE] + rules})
        dump(d / "0300_rolebinding.yaml",
             {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
              "metadata": {"name": sa, "namespace": NS, "labels": app},
              "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": NS}],
              "roleRef": {"kind": "Role", "name": sa, "apiGroup": "rbac.authorization.k8s.io"}})
        if crules:
            dump(d / "0210_clusterrole.yaml",
                 {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                  "metadata": {"name": sa, "labels": app}, "rules": crules})
            dump(d / "0310_clusterrolebinding.yaml",
                 {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                  "metadata": {"name": sa, "labels": app},
                  "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": NS}],
                  "roleRef": {"kind": "ClusterRole", "name": sa, "apiGroup": "rbac.authorization.k8s.io"}})
        dump(d / "0400_scc_openshift.yaml",
             {"apiVersion": "security.openshift.io/v1", "kind": "SecurityContextConstraints",
              "metadata": {"name": sa, "labels": app},
              "allowHostDirVolumePlugin": True, "allowHostIPC": True, "allowHostNetwork": True,
              "allowHostPID": True, "allowHostPorts": True, "allowPrivilegedContainer": True,
              "allowedCapabilities": ["*"], "readOnlyRootFilesystem": False,
              "runAsUser": {"type": "RunAsAny"}, "seLinuxContext": {"type": "RunAsAny"},
              "fsGroup": {"type": "RunAsAny"}, "supplementalGroups": {"type": "RunAsAny"},
              "users": [f"system:serviceaccount:{NS}:{sa}"], "volumes": ["*"]})
    print(f"wrote RBAC for {len(OPERANDS)} states under {os.path.relpath(ASSETS)}")


if __name__ == "__main__":
    main()
