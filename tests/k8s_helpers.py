"""Shared fixtures for control-plane tests: synthetic AMD GPU nodes and the sample CR."""

import copy
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NS = "amd-gpu-operator"
SAMPLE = os.path.join(ROOT, "config", "samples", "amd_v1_clusterpolicy.yaml")


def sample_cp(**overrides):
    with open(SAMPLE) as f:
        cp = yaml.safe_load(f)
    for path, value in overrides.items():
        cur = cp["spec"]
        keys = path.split(".")
        for k in keys[:-1]:
            cur = cur.setdefault(k, {})
        cur[keys[-1]] = value
    return cp


def gpu_node(name, kernel="6.8.0-45-generic", os_id="ubuntu", os_ver="22.04", runtime="containerd://1.7.13",
             extra_labels=None, gpu=True):
    labels = {"feature.node.kubernetes.io/kernel-version.full": kernel,
              "feature.node.kubernetes.io/system-os_release.ID": os_id,
              "feature.node.kubernetes.io/system-os_release.VERSION_ID": os_ver}
    if gpu:
        labels["feature.node.kubernetes.io/pci-1002.present"] = "true"
    labels.update(extra_labels or {})
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": labels},
            "status": {"nodeInfo": {"containerRuntimeVersion": runtime}}}


def namespace(name=NS):
    return {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name}}


def cluster(nodes=None, cp=None, unserved=("ServiceMonitor", "PrometheusRule")):
    from gpu_operator_amd.k8s.fake import FakeClient

    objs = [namespace()] + list(nodes if nodes is not None else [gpu_node("node-1"), gpu_node("node-2")])
    if cp is not False:
        objs.append(cp or sample_cp())
    return FakeClient(objs, unserved_kinds=set(unserved))


def reconciler(client):
    from gpu_operator_amd.controllers.clusterpolicy_controller import ClusterPolicyReconciler

    os.environ["OPERATOR_NAMESPACE"] = NS
    return ClusterPolicyReconciler(client, namespace=NS)


def run_until_ready(client, rec, sim=None, passes=5, name="cluster-policy"):
    from gpu_operator_amd.k8s.sim import ClusterSim

    sim = sim or ClusterSim(client)
    res = None
    for _ in range(passes):
        res = rec.reconcile(("", name))
        sim.sync()
        st = client.get("amd.com/v1", "ClusterPolicy", name).get("status", {}).get("state")
        if st == "ready":
            return res, st
    return res, client.get("amd.com/v1", "ClusterPolicy", name).get("status", {}).get("state")


def daemonset(client, name):
    return client.get("apps/v1", "DaemonSet", name, NS)


def container(ds, name, init=False):
    key = "initContainers" if init else "containers"
    for c in ds["spec"]["template"]["spec"].get(key) or []:
        if c["name"] == name:
            return c
    return None


def env(c):
    return {e["name"]: e.get("value") for e in c.get("env") or []}


def deepcopy(x):
    return copy.deepcopy(x)
