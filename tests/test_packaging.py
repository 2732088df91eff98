"""Helm chart (rendered by our Go-template engine), generated CRD/RBAC/CSV, kustomize/OLM files,
and the gpuop-cfg configuration validator/migrator."""

import copy
import glob
import json
import os
import subprocess
import sys

import pytest
import yaml

from gpu_operator_amd.api.v1 import clusterpolicy as cp
from gpu_operator_amd.cmd import gpuop_cfg as cfg
from gpu_operator_amd.utils import gotemplate as gt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHART = os.path.join(ROOT, "deployments", "amd-gpu-operator")


# -- template engine --------------------------------------------------------------------------

def _r(src, dot, defines=""):
    t = gt.Template()
    if defines:
        t.add("_h", defines)
    t.add("x", src)
    return t.render("x", dot)


def test_engine_basics():
    dot = {"Values": {"a": {"b": "x", "n": 3, "l": [1, 2], "m": {"k2": "v2", "k1": "v1"}, "e": {}}}}
    assert _r("{{ .Values.a.b }}", dot) == "x"
    assert _r("a  {{- .Values.a.b -}}  b", dot) == "axb"
    assert _r("{{ .Values.a.missing | default \"d\" }}", dot) == "d"
    assert _r("{{ printf \"%s-%d\" .Values.a.b .Values.a.n }}", dot) == "x-3"
    assert _r("{{ range $i, $v := .Values.a.l }}[{{ $i }}:{{ $v }}]{{ end }}", dot) == "[0:1][1:2]"
    assert _r("{{ range $k, $v := .Values.a.m }}{{ $k }}={{ $v }};{{ end }}", dot) == "k1=v1;k2=v2;"
    assert _r("{{ with .Values.a.e }}yes{{ else }}no{{ end }}", dot) == "no"
    assert _r("{{ if and .Values.a.b (not .Values.a.e) }}T{{ else if .Values.a.n }}N{{ else }}F{{ end }}", dot) == "T"
    assert _r("{{ if eq .Values.a.n 4 }}A{{ else if eq .Values.a.n 3 }}B{{ end }}", dot) == "B"
    assert _r("{{- $x := .Values.a.b }}{{ $x | upper | quote }}", dot) == '"X"'
    assert _r("{{ index .Values.a.m \"k1\" }}/{{ (index .Values.a \"m\").k2 }}", dot) == "v1/v2"
    assert _r("{{/* comment */}}ok", dot) == "ok"
    assert _r("{{ toYaml .Values.a.m | nindent 2 }}", dot) == "\n  k1: v1\n  k2: v2"
    assert _r("{{ include \"h\" .Values.a }}", dot, '{{- define "h" -}}<{{ .b }}>{{- end -}}') == "<x>"
    assert _r("{{ \"abcdef\" | trunc 3 }}{{ \"xy-\" | trimSuffix \"-\" }}", dot) == "abcxy"
    assert _r("{{ toYaml (omit .Values.a.m \"k1\") }}", dot) == "k2: v2"
    with pytest.raises(gt.TemplateError):
        _r("{{ nosuchfn 1 }}", dot)
    with pytest.raises(gt.TemplateError):
        _r("{{ if .x }}", dot)


# -- chart ------------------------------------------------------------------------------------

def _objs(values=None):
    return gt.render_objects(CHART, values)


def _by_kind(objs):
    out = {}
    for o in objs:
        out.setdefault(o["kind"], []).append(o)
    return out


def test_chart_default_render():
    k = _by_kind(_objs())
    assert set(k) == {"ServiceAccount", "ClusterRole", "ClusterRoleBinding", "Deployment", "ClusterPolicy", "Job",
                      # the vendored NFD subchart (nfd.enabled=true by default)
                      "Role", "RoleBinding", "ConfigMap", "DaemonSet"}
    assert "SecurityContextConstraints" not in k                    # OpenShift only
    pol = cp.ClusterPolicy(k["ClusterPolicy"][0], strict=True)
    assert pol.spec.driver.is_enabled() and pol.spec.operator.runtimeClass == "amd"
    assert pol.spec.metricsExporter.is_enabled() and not pol.spec.rdc.is_enabled()
    dep = [d for d in k["Deployment"] if d["metadata"]["name"] == "amd-gpu-operator"][0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["DRIVER_IMAGE"] == "registry.example.com/amd/amdgpu-driver:6.12.12"
    assert "OPERATOR_NAMESPACE" in env and "VALIDATOR_IMAGE" in env and "ROCM_BASE_IMAGE" in env
    assert "--leader-elect" in c["args"]
    assert c["readinessProbe"]["httpGet"]["port"] == 8081
    hooks = [j["metadata"]["annotations"]["helm.sh/hook"] for j in k["Job"]]
    assert hooks == ["pre-upgrade"]
    role = [r for r in k["ClusterRole"] if r["metadata"]["name"] == "amd-gpu-operator"][0]
    assert any("clusterpolicies" in r["resources"] for r in role["rules"])


def test_chart_overrides():
    k = _by_kind(_objs({"operator": {"leaderElect": False, "cleanupCRD": True},
                        "nfd": {"nodefeaturerules": True},
                        "devicePlugin": {"config": {"create": True, "default": "ts",
                                                    "data": {"ts": "version: v1\n"}}},
                        "driver": {"usePrecompiled": True}}))
    op = [d for d in k["Deployment"] if d["metadata"]["name"] == "amd-gpu-operator"][0]
    assert "--leader-elect" not in op["spec"]["template"]["spec"]["containers"][0]["args"]
    assert sorted(j["metadata"]["annotations"]["helm.sh/hook"] for j in k["Job"]) == ["pre-delete", "pre-upgrade"]
    assert k["NodeFeatureRule"][0]["spec"]["rules"][0]["labels"]["amd.com/gpu.family.nfd"] == "cdna4"
    cm = [m for m in k["ConfigMap"] if m["metadata"]["name"] == "amd-device-plugin-config"][0]
    assert cm["metadata"]["name"] == "amd-device-plugin-config" and cm["data"]["ts"].startswith("version")
    pol = cp.ClusterPolicy(k["ClusterPolicy"][0], strict=True)
    assert pol.spec.devicePlugin.config.name == "amd-device-plugin-config"
    assert pol.spec.devicePlugin.config.default == "ts"
    assert pol.spec.driver.use_precompiled()


def test_values_sections_are_spec_fields():
    with open(os.path.join(CHART, "values.yaml")) as f:
        values = yaml.safe_load(f)
    spec_keys = {f.metadata.get("json", f.name) for f, _ in cp.ClusterPolicySpec._fields()}
    chart_only = {"platform", "nfd", "node-feature-discovery", "operator"}
    assert set(values) - chart_only <= spec_keys, set(values) - chart_only - spec_keys
    wl = values["node-feature-discovery"]["worker"]["config"]["sources"]["pci"]["deviceClassWhitelist"]
    assert {"0300", "0380", "1200"} <= set(wl)
    with open(os.path.join(CHART, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    assert chart["dependencies"][0]["name"] == "node-feature-discovery"


# -- generated manifests -------------------------------------------------------------------------

def test_generated_manifests_up_to_date():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_manifests.py"), "--check"],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr


def test_crd_schema():
    with open(os.path.join(ROOT, "config", "crd", "bases", "amd.com_clusterpolicies.yaml")) as f:
        crd = yaml.safe_load(f)
    assert crd["spec"]["scope"] == "Cluster" and crd["metadata"]["name"] == "clusterpolicies.amd.com"
    v = crd["spec"]["versions"][0]
    assert v["subresources"] == {"status": {}}
    props = v["schema"]["openAPIV3Schema"]["properties"]["spec"]["properties"]
    for key in ("driver", "toolkit", "devicePlugin", "partitionManager", "kataManager", "cdi", "validator"):
        assert key in props, key
    assert props["rdc"]["properties"]["hostPort"]["maximum"] == 65535
    # chart and bundle carry the same CRD
    for other in (os.path.join(CHART, "crds", "amd.com_clusterpolicies.yaml"),
                  os.path.join(ROOT, "bundle", "manifests", "amd.com_clusterpolicies.yaml")):
        with open(other) as f:
            assert yaml.safe_load(f) == crd


def test_csv_and_kustomize_files_parse():
    with open(os.path.join(ROOT, "bundle", "manifests", "amd-gpu-operator.clusterserviceversion.yaml")) as f:
        csv = yaml.safe_load(f)
    assert cfg.validate_csv(csv)["alm_examples"] == 1
    for p in glob.glob(os.path.join(ROOT, "config", "**", "*.yaml"), recursive=True) + \
            glob.glob(os.path.join(ROOT, "bundle", "**", "*.yaml"), recursive=True):
        with open(p) as f:
            assert list(yaml.safe_load_all(f)), p
    with open(os.path.join(ROOT, "config", "default", "kustomization.yaml")) as f:
        k = yaml.safe_load(f)
    for res in k["resources"]:
        assert os.path.isdir(os.path.join(ROOT, "config", "default", res)), res


# -- gpuop-cfg ---------------------------------------------------------------------------------

def test_validate_clusterpolicy_chart_and_file(tmp_path):
    obj, env = cfg.load_clusterpolicy(None, CHART, None)
    rep = cfg.validate_clusterpolicy(obj, env)
    assert rep["images"]["driver"].endswith("amdgpu-driver:6.12.12")
    assert "rdc" not in rep["images"]                        # disabled operands are not resolved
    # image left empty in the CR and no env fallback -> error
    bad = copy.deepcopy(obj)
    for k in ("repository", "image", "version"):
        bad["spec"]["toolkit"].pop(k)
    with pytest.raises(cfg.ConfigError, match="CONTAINER_TOOLKIT_IMAGE"):
        cfg.validate_clusterpolicy(bad, {})
    assert cfg.validate_clusterpolicy(bad, {"CONTAINER_TOOLKIT_IMAGE": "r/x:1"})["images"]["toolkit"] == "r/x:1"
    # unknown field -> strict parse error
    bad2 = copy.deepcopy(obj)
    bad2["spec"]["driver"]["bogus"] = 1
    with pytest.raises(cfg.ConfigError, match="invalid ClusterPolicy"):
        cfg.validate_clusterpolicy(bad2, env)
    # CLI on a values override file
    vals = tmp_path / "v.yaml"
    vals.write_text("driver:\n  version: '6.14.0'\n")
    assert cfg.main(["validate", "clusterpolicy", "--chart", CHART, "--values", str(vals)]) == 0
    f = tmp_path / "cp.yaml"
    f.write_text(yaml.safe_dump(bad2))
    assert cfg.main(["validate", "clusterpolicy", "--input", str(f)]) == 1


def test_validate_csv_catches_missing_related_image():
    with open(os.path.join(ROOT, "bundle", "manifests", "amd-gpu-operator.clusterserviceversion.yaml")) as f:
        csv = yaml.safe_load(f)
    csv["spec"]["relatedImages"] = [r for r in csv["spec"]["relatedImages"] if "amdgpu-driver" not in r["image"]]
    with pytest.raises(cfg.ConfigError, match="DRIVER_IMAGE"):
        cfg.validate_csv(csv)


def test_convert_nvidia_policy(tmp_path):
    nv = {"apiVersion": "nvidia.com/v1", "kind": "ClusterPolicy", "metadata": {"name": "gpu-cluster-policy"},
          "spec": {"operator": {"defaultRuntime": "containerd", "runtimeClass": "nvidia"},
                   "driver": {"enabled": True, "repository": "nvcr.io/nvidia", "image": "driver",
                              "version": "535", "licensingConfig": {"configMapName": "x"}},
                   "dcgmExporter": {"enabled": True},
                   "gfd": {"enabled": True, "env": [{"name": "GFD_SLEEP_INTERVAL", "value": "60s"}]},
                   "mig": {"strategy": "mixed"},
                   "migManager": {"enabled": True, "config": {"name": "default-mig-parted-config"}},
                   "validator": {"cuda": {"env": [{"name": "WITH_WORKLOAD", "value": "true"}]}},
                   "daemonsets": {"tolerations": [{"key": "nvidia.com/gpu", "operator": "Exists"}]},
                   "gds": {"enabled": True}}}
    out, notes = cfg.convert(nv)
    assert out["apiVersion"] == "amd.com/v1"
    s = out["spec"]
    assert "metricsExporter" in s and "nodeLabeller" in s and s["partition"]["strategy"] == "mixed"
    assert s["daemonsets"]["tolerations"][0]["key"] == "amd.com/gpu"
    assert s["operator"]["runtimeClass"] == "amd"
    assert "repository" not in s["driver"] and "licensingConfig" not in s["driver"]
    assert s["validator"]["hip"]["env"][0]["value"] == "true"
    assert any("GPUDirect Storage" in n for n in notes)
    cp.ClusterPolicy(out)
    f = tmp_path / "nv.yaml"
    f.write_text(yaml.safe_dump(nv))
    assert cfg.main(["convert", "--input", str(f)]) == 0
    with pytest.raises(cfg.ConfigError):
        cfg.convert({"kind": "Pod"})


def test_check_registry_is_offline_safe():
    ok, why = cfg.check_registry("registry.invalid/amd/x:1", timeout=0.5)
    assert not ok and why


# -- self-contained chart: vendored NFD subchart, Chart.lock, OpenShift SCC -----

def test_chart_vendors_nfd_and_installs_offline():
    with open(os.path.join(CHART, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(CHART, "Chart.lock")) as f:
        lock = yaml.safe_load(f)
    dep = chart["dependencies"][0]
    with open(os.path.join(CHART, "charts", dep["name"], "Chart.yaml")) as f:
        sub = yaml.safe_load(f)
    assert sub["name"] == dep["name"] and sub["version"] == dep["version"]          # helm's presence check
    assert dep["repository"].startswith("file://charts/")
    assert lock["dependencies"] == [{k: dep[k] for k in ("name", "version", "repository")}]
    assert lock["digest"] == gt.chart_lock_digest(chart["dependencies"], lock["dependencies"])
    k = _by_kind(gt.render_objects(CHART, include_crds=True))
    conf = [m for m in k["ConfigMap"] if m["metadata"]["name"].endswith("node-feature-discovery-worker-conf")][0]
    worker_conf = yaml.safe_load(conf["data"]["nfd-worker.conf"])
    wl = worker_conf["sources"]["pci"]["deviceClassWhitelist"]
    assert "0380" in wl and "1200" in wl                  # AMD Instinct PF classes (MI300/MI355X)
    ds = k["DaemonSet"][0]["spec"]["template"]["spec"]
    assert any(t.get("key") == "amd.com/gpu" for t in ds["tolerations"])
    crds = {c["metadata"]["name"] for c in k["CustomResourceDefinition"]}
    assert {"nodefeatures.nfd.k8s-sigs.io", "nodefeaturerules.nfd.k8s-sigs.io", "clusterpolicies.amd.com"} <= crds
    off = _by_kind(gt.render_objects(CHART, {"nfd": {"enabled": False}}))
    assert "DaemonSet" not in off and not [d for d in off["Deployment"] if "node-feature" in d["metadata"]["name"]]


def test_chart_lock_digest_matches_helm():
    """The algorithm reproduces a digest Helm itself wrote: the reference's Chart.lock
    (deployments/gpu-operator/Chart.lock:1-6 over Chart.yaml:19-23)."""
    repo = "https://kubernetes-sigs.github.io/node-feature-discovery/charts"
    req = [{"name": "node-feature-discovery", "version": "v0.13.1", "repository": repo, "condition": "nfd.enabled"}]
    locked = [{"name": "node-feature-discovery", "version": "0.13.1", "repository": repo}]
    assert gt.chart_lock_digest(req, locked) == \
        "sha256:8cebf8838e987c231cec03a289deed636e644746464920f799caa35dbcf3bdc6"


def test_operator_scc_renders_only_on_openshift():
    assert "SecurityContextConstraints" not in _by_kind(_objs())
    k = _by_kind(_objs({"platform": {"openshift": True}}))
    scc = k["SecurityContextConstraints"][0]
    assert scc["readOnlyRootFilesystem"] and not scc["allowPrivilegedContainer"] and not scc["allowHostPID"]
    assert scc["users"] == ["system:serviceaccount:amd-gpu-operator:amd-gpu-operator"]


def test_operator_psp_renders_only_below_kubernetes_1_25():
    """The operator pod's restricted PodSecurityPolicy (reference:
    deployments/gpu-operator/templates/podsecuritypolicy.yaml): only with psp.enabled and on a
    cluster older than 1.25, where policy/v1beta1 still exists."""
    on = {"psp": {"enabled": True}}
    k = _by_kind(gt.render_objects(CHART, on, kube="v1.24.3"))
    psp = k["PodSecurityPolicy"][0]
    assert psp["apiVersion"] == "policy/v1beta1" and psp["metadata"]["name"] == "amd-gpu-operator-restricted"
    sp = psp["spec"]
    assert not sp["privileged"] and not sp["hostPID"] and not sp["hostNetwork"] and sp["readOnlyRootFilesystem"]
    assert sp["requiredDropCapabilities"] == ["ALL"] and "hostPath" not in sp["volumes"]
    assert gt.kube_version("v1.24.3+eks")["Minor"] == "24+"
    assert "PodSecurityPolicy" in _by_kind(gt.render_objects(CHART, on, kube="v1.24.3+eks"))   # "24+" minors
    assert "PodSecurityPolicy" not in _by_kind(gt.render_objects(CHART, on, kube="v1.25.0"))
    assert "PodSecurityPolicy" not in _by_kind(gt.render_objects(CHART, on))               # default v1.29
    assert "PodSecurityPolicy" not in _by_kind(gt.render_objects(CHART, {}, kube="v1.24.3"))
