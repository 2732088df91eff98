"""The generated ClusterPolicy CRD checked the way kube-apiserver checks it (k8s/openapi.py):
structural-schema rules, then prune / default / validate of custom resources, over HTTP through
the in-process API server. Parity unpinned against a real kube-apiserver (none here); the
rules implemented are apiextensions.k8s.io/v1's structural-schema and validation semantics."""

import copy
import os

import pytest
import yaml

from gpu_operator_amd.k8s import errors
from gpu_operator_amd.k8s import openapi as OA
from gpu_operator_amd.k8s.apiserver import FakeAPIServer
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.k8s.rest import Config, RestClient
from k8s_helpers import sample_cp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRDS = ["config/crd/bases/amd.com_clusterpolicies.yaml", "deployments/amd-gpu-operator/crds/amd.com_clusterpolicies.yaml",
        "bundle/manifests/amd.com_clusterpolicies.yaml"]


def _crd(path=CRDS[0]):
    with open(os.path.join(ROOT, path)) as f:
        return yaml.safe_load(f)


def _schema():
    return _crd()["spec"]["versions"][0]["schema"]["openAPIV3Schema"]


@pytest.mark.parametrize("path", CRDS)
def test_generated_crds_are_structural(path):
    crd = _crd(path)
    for v in crd["spec"]["versions"]:
        assert OA.structural_errors(v["schema"]["openAPIV3Schema"]) == [], path


def test_structural_rules_catch_bad_schemas():
    bad = {"type": "object", "properties": {
        "a": {"description": "no type"},
        "b": {"type": "array"},
        "c": {"type": "object", "properties": {"x": {"type": "string"}}, "additionalProperties": {"type": "string"}},
        "d": {"type": "string", "enum": ["x", 3]},
        "e": {"type": "integer", "default": "five"},
        "f": {"$ref": "#/definitions/x", "type": "object"},
        "g": {"x-kubernetes-int-or-string": True, "type": "string"},
        "h": {"x-kubernetes-int-or-string": True, "anyOf": [{"type": "integer"}, {"type": "string"}]},
        "i": {"x-kubernetes-preserve-unknown-fields": True},
    }}
    errs = "\n".join(OA.structural_errors(bad))
    for key in ("properties[a].type: Required", "properties[b].items: Required", "mutually exclusive",
                "properties[d].enum: 3", "properties[e].default", "$ref is forbidden",
                "properties[g]: type must be empty"):
        assert key in errs, (key, errs)
    assert "properties[h]" not in errs and "properties[i]" not in errs


def test_prune_default_validate_sample():
    cr = sample_cp()
    cr["spec"]["unknownTopLevel"] = {"x": 1}
    cr["spec"]["driver"]["notAField"] = True
    errs = OA.admit(cr, _schema())
    assert errs == []
    assert "unknownTopLevel" not in cr["spec"] and "notAField" not in cr["spec"]["driver"]
    # free-form sub-objects survive pruning
    cr2 = sample_cp(**{"daemonsets.tolerations": [{"key": "k", "operator": "Exists", "effect": "NoSchedule"}]})
    assert OA.admit(cr2, _schema()) == [] and cr2["spec"]["daemonsets"]["tolerations"][0]["key"] == "k"
    # defaults of present objects are filled in
    assert cr["spec"]["daemonsets"]["updateStrategy"] == "RollingUpdate"
    assert cr["spec"]["driver"]["upgradePolicy"]["maxUnavailable"] == "25%" or \
        "maxUnavailable" in sample_cp()["spec"]["driver"]["upgradePolicy"]


@pytest.mark.parametrize("path,value,needle", [
    ("daemonsets.updateStrategy", "Sometimes", "Unsupported value"),
    ("driver.upgradePolicy.maxParallelUpgrades", -1, "greater than or equal to 0"),
    ("driver.upgradePolicy.maxParallelUpgrades", "two", "must be of type integer"),
    ("driver.enabled", "yes", "must be of type boolean"),
    ("driver.upgradePolicy.maxUnavailable", True, "integer or a string"),
])
def test_invalid_values_rejected(path, value, needle):
    cr = sample_cp(**{path: value})
    errs = OA.admit(cr, _schema())
    assert errs and any(needle in e for e in errs), errs


def test_int_or_string_and_quantities_accept_both():
    for v in (2, "2", "10%"):
        cr = sample_cp(**{"driver.upgradePolicy.maxUnavailable": v})
        assert OA.admit(cr, _schema()) == [], v
    cr = sample_cp(**{"devicePlugin.resources": {"limits": {"cpu": 1, "memory": "200Mi"}, "requests": {"cpu": "500m"}}})
    assert OA.admit(cr, _schema()) == []


@pytest.fixture
def api():
    backing = FakeClient([_crd()])
    srv = FakeAPIServer(backing).start()
    yield RestClient(Config(host=srv.url)), backing
    srv.stop()


def test_api_server_admits_cluster_policy_over_http(api):
    c, backing = api
    cr = sample_cp()
    cr["spec"]["bogus"] = 1
    out = c.create(cr)
    assert "bogus" not in out["spec"] and out["spec"]["daemonsets"]["updateStrategy"] == "RollingUpdate"
    bad = copy.deepcopy(out)
    bad["spec"]["driver"]["upgradePolicy"] = {"maxParallelUpgrades": -3}
    with pytest.raises(errors.Invalid, match="greater than or equal to 0"):
        c.update(bad)
    with pytest.raises(errors.Invalid, match="Unsupported value"):
        c.patch("amd.com/v1", "ClusterPolicy", out["metadata"]["name"], {"spec": {"daemonsets": {"updateStrategy": "x"}}})
    ok = c.patch("amd.com/v1", "ClusterPolicy", out["metadata"]["name"],
                 {"spec": {"driver": {"upgradePolicy": {"maxUnavailable": 1}}}})
    assert ok["spec"]["driver"]["upgradePolicy"]["maxUnavailable"] == 1


def test_api_server_rejects_a_non_structural_crd(api):
    c, _ = api
    crd = _crd()
    crd["metadata"]["name"] = "widgets.example.com"
    crd["spec"]["names"] = {"kind": "Widget", "plural": "widgets", "singular": "widget", "listKind": "WidgetList"}
    crd["spec"]["group"] = "example.com"
    crd["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["spec"] = {"description": "untyped"}
    with pytest.raises(errors.Invalid, match="type: Required value"):
        c.create(crd)
