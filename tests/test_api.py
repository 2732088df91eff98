"""amd.com/v1 ClusterPolicy API: defaults, enable predicates, image resolution, validation."""

import json

import pytest

from gpu_operator_amd.api.schema import ValidationError
from gpu_operator_amd.api.v1 import clusterpolicy as cp
from gpu_operator_amd.api.v1.upgrade import DriverUpgradePolicySpec, resolve_int_or_percent
from k8s_helpers import sample_cp


def spec(d=None, strict=False):
    return cp.ClusterPolicySpec.from_dict(d or {}, strict=strict)


def test_enable_defaults_match_reference_semantics():
    s = spec()
    # on by default (reference: api/v1/clusterpolicy_types.go:1659-1864)
    for comp in (s.driver, s.toolkit, s.devicePlugin, s.metricsExporter, s.nodeLabeller, s.rdc,
                 s.partitionManager):
        assert comp.is_enabled(), type(comp).__name__
    # off by default
    for comp in (s.nodeStatusExporter, s.vfioManager, s.mxgpuManager, s.mxgpuDeviceManager,
                 s.sandboxDevicePlugin, s.kataManager, s.gds):
        assert not comp.is_enabled(), type(comp).__name__
    assert not s.sandboxWorkloads.is_enabled() and not s.psp.is_enabled() and not s.psa.is_enabled()
    assert not s.cdi.is_enabled() and not s.cdi.is_default()
    assert not s.driver.use_precompiled()
    assert s.partition.get_strategy() == "single"
    assert s.operator.runtime_class() == "amd"
    assert s.toolkit.install_dir() == "/usr/local/amd"
    assert s.rdc.host_port() == 50051


def test_explicit_false_differs_from_unset():
    s = spec({"driver": {"enabled": False}, "nodeStatusExporter": {"enabled": True}})
    assert not s.driver.is_enabled()
    assert s.nodeStatusExporter.is_enabled()


def test_reference_keys_are_accepted_as_aliases():
    s = spec({"dcgmExporter": {"enabled": False}, "gfd": {"enabled": False}, "mig": {"strategy": "mixed"},
              "migManager": {"enabled": False}, "dcgm": {"hostPort": 5555},
              "vgpuManager": {"enabled": True}, "vgpuDeviceManager": {"enabled": True},
              "validator": {"cuda": {"env": [{"name": "X", "value": "1"}]}}})
    assert not s.metricsExporter.is_enabled() and not s.nodeLabeller.is_enabled()
    assert s.partition.get_strategy() == "mixed" and not s.partitionManager.is_enabled()
    assert s.rdc.host_port() == 5555
    assert s.mxgpuManager.is_enabled() and s.mxgpuDeviceManager.is_enabled()
    assert s.validator.hip.env[0].name == "X"
    # serialised back under the AMD keys
    out = s.to_dict()
    assert "metricsExporter" in out and "dcgmExporter" not in out
    assert out["validator"]["hip"]["env"] == [{"name": "X", "value": "1"}]


@pytest.mark.parametrize("bad,match", [
    ({"driver": {"imagePullPolicy": "Sometimes"}}, "imagePullPolicy"),
    ({"operator": {"defaultRuntime": "podman"}}, "defaultRuntime"),
    ({"partition": {"strategy": "all"}}, "strategy"),
    ({"driver": {"image": "bad/image"}}, "does not match"),
    ({"rdc": {"hostPort": 0}}, "minimum"),
    ({"driver": {"enabled": "yes"}}, "boolean"),
    ({"driver": {"startupProbe": {"periodSeconds": 0}}}, "minimum"),
    ({"validator": {"plugin": {"env": [{"value": "x"}]}}}, "required"),
    ({"daemonsets": {"updateStrategy": "Recreate"}}, "updateStrategy"),
    ({"metricsExporter": {"serviceMonitor": {"interval": "15 seconds"}}}, "interval"),
])
def test_validation_errors(bad, match):
    with pytest.raises(ValidationError, match=match):
        spec(bad)


def test_strict_mode_rejects_unknown_fields_and_lenient_mode_round_trips_them():
    with pytest.raises(ValidationError, match="unknown"):
        spec({"driver": {"enabledd": True}}, strict=True)
    s = spec({"driver": {"futureKnob": {"a": 1}}})
    assert s.to_dict()["driver"]["futureKnob"] == {"a": 1}


def test_image_path_precedence(monkeypatch):
    d = cp.DriverSpec(repository="r.io/amd", image="amdgpu-driver", version="6.12")
    assert cp.image_path(d) == "r.io/amd/amdgpu-driver:6.12"
    d = cp.DriverSpec(repository="r.io/amd", image="amdgpu-driver", version="sha256:abc")
    assert cp.image_path(d) == "r.io/amd/amdgpu-driver@sha256:abc"
    d = cp.DriverSpec(image="r.io/amd/amdgpu-driver:6.12@sha256:ff")   # kbld-rendered full ref
    assert cp.image_path(d) == "r.io/amd/amdgpu-driver:6.12@sha256:ff"
    monkeypatch.setenv("DRIVER_IMAGE", "env.io/driver:1")
    assert cp.image_path(cp.DriverSpec()) == "env.io/driver:1"
    monkeypatch.delenv("DRIVER_IMAGE")
    with pytest.raises(ValueError, match="DRIVER_IMAGE"):
        cp.image_path(cp.DriverSpec())


def test_every_operand_has_an_image_env_fallback():
    envs = {t.IMAGE_ENV for t in (cp.DriverSpec, cp.ToolkitSpec, cp.DevicePluginSpec, cp.MetricsExporterSpec,
                                  cp.RDCSpec, cp.NodeLabellerSpec, cp.ValidatorSpec, cp.PartitionManagerSpec,
                                  cp.DriverManagerSpec, cp.VFIOManagerSpec, cp.MxGPUManagerSpec,
                                  cp.MxGPUDeviceManagerSpec, cp.SandboxDevicePluginSpec, cp.KataManagerSpec,
                                  cp.InitContainerSpec, cp.NodeStatusExporterSpec)}
    assert "" not in envs and len(envs) == 15   # node-status exporter shares VALIDATOR_IMAGE


def test_pull_policy_defaults():
    assert cp.image_pull_policy(None) == "IfNotPresent"
    assert cp.image_pull_policy("Always") == "Always"


def test_upgrade_policy_defaults_and_max_unavailable():
    p = DriverUpgradePolicySpec.from_dict({"autoUpgrade": True})
    assert p.max_parallel() == 1
    assert p.max_unavailable_nodes(10) == 3            # 25% rounded up
    assert resolve_int_or_percent("10%", 5) == 1
    assert resolve_int_or_percent(4, 100) == 4


def test_sample_cr_parses_strictly_and_round_trips():
    obj = sample_cp()
    p = cp.ClusterPolicy(obj, strict=True)
    again = cp.ClusterPolicy(p.to_dict(), strict=True)
    assert again.spec.to_dict() == p.spec.to_dict()
    assert p.spec.driver.auto_upgrade()
    assert p.spec.kataManager.config.runtimeClasses[0].artifacts.url.startswith("registry.example.com")


def test_duplicate_kata_runtime_classes_rejected():
    obj = sample_cp(**{"kataManager.config.runtimeClasses": [
        {"name": "a", "artifacts": {"url": "x"}}, {"name": "a", "artifacts": {"url": "y"}}]})
    with pytest.raises(ValidationError, match="duplicate"):
        cp.ClusterPolicy(obj)


def test_wrong_api_version_rejected():
    with pytest.raises(ValidationError):
        cp.ClusterPolicy({"apiVersion": "nvidia.com/v1", "kind": "ClusterPolicy", "spec": {}})


def test_openapi_schema_covers_every_spec_key():
    s = cp.ClusterPolicySpec.openapi()
    keys = set(s["properties"])
    for k in ("operator", "daemonsets", "driver", "toolkit", "devicePlugin", "metricsExporter", "rdc",
              "nodeStatusExporter", "nodeLabeller", "partition", "partitionManager", "psp", "psa",
              "validator", "gds", "sandboxWorkloads", "vfioManager", "sandboxDevicePlugin", "mxgpuManager",
              "mxgpuDeviceManager", "cdi", "kataManager"):
        assert k in keys
    drv = s["properties"]["driver"]["properties"]
    assert drv["imagePullPolicy"]["enum"] == ["Always", "IfNotPresent", "Never"]
    assert drv["upgradePolicy"]["properties"]["maxParallelUpgrades"]["minimum"] == 0
    assert s["properties"]["daemonsets"]["properties"]["tolerations"]["items"] == \
        {"x-kubernetes-preserve-unknown-fields": True}
    json.dumps(s)
