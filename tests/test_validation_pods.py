"""The HIP validation pod under real kubelet semantics.

The validator (validate_hip, pod mode) spawns its pod against the process kubelet of the e2e harness
(gpu_operator_amd/e2e/kubelet.py): the pod's init container is the real ``amd-validator-workload hip``
process; only ``amd-gemm-validate`` is the scripted stand-in (gpu_operator_amd/e2e/gemm_standin.py),
which speaks the binary's protocol and gates on the floor the validator passes. Reference
counterpart: validator/main.go:1042-1059 (waitForPod polls the phase only) with the OnFailure pod of
validator/cuda-workload-validation.yaml:13 -- a failing workload there is a 300 s timeout.
"""

import os
import sys
import threading
import time

import pytest

from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.e2e.kubelet import ProcessKubelet
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.validator import components as comp
from gpu_operator_amd.validator import status as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NS = "amd-gpu-operator"
NODE = "n1"
RUNTIME_S = 1.5


@pytest.fixture
def node(tmp_path):
    """A FakeClient cluster with one node, its process kubelet, and the scripted GEMM on its PATH."""
    from gpu_operator_amd.cmd.entry import install_wrappers
    root = str(fakesys.make_node(tmp_path / "root", n_gpus=8))
    standin = tmp_path / "standin"
    standin.mkdir()
    for name, body in (("amd-gemm-validate", f'exec "{sys.executable}" -m gpu_operator_amd.e2e.gemm_standin "$@"\n'),
                       ("rocprofv3", "exit 1\n")):            # no profiler on a CPU node
        p = standin / name
        p.write_text("#!/bin/sh\n" + body)
        p.chmod(0o755)
    wrappers = install_wrappers(str(tmp_path / "bin"))
    state = str(tmp_path / "gemm-runs")
    env = dict(os.environ, PATH=f"{standin}:{wrappers}:{os.environ.get('PATH', '/usr/bin:/bin')}",
               PYTHONPATH=ROOT, AMDGO_BIN_DIR=str(standin), GEMM_STANDIN_STATE=state,
               GEMM_STANDIN_RUNTIME_S=str(RUNTIME_S), AMD_SYSFS_ROOT=root, AMD_DEV_ROOT=root)
    env.pop("KUBECONFIG", None)
    c = FakeClient([{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NS}},
                    {"apiVersion": "v1", "kind": "Node", "metadata": {"name": NODE, "labels": {}},
                     "status": {"capacity": {"amd.com/gpu": "8"}, "allocatable": {"amd.com/gpu": "8"}}}])
    base = f"/tmp/vp-{os.getpid()}-{int(time.time() * 1000) % 100000}"     # unix socket paths: <= 107 chars
    k = ProcessKubelet(c, NODE, base, env, root, root, host_links={}).start()
    yield c, k, root, state
    k.stop()
    k.cleanup()


def _ctx(tmp_path, c, root, script, **env):
    e = {"VALIDATOR_IMAGE": "registry.example.com/amd/amd-gpu-operator-node:v0.1.0", "DRIVER_ROOT_MODE": "host",
         "HIP_VALIDATION_MODE": "pod", **env}
    return comp.Context(status=S.StatusDir(str(tmp_path / "validations")), node_name=NODE, namespace=NS, client=c,
                        host_root=str(tmp_path / "host"), sys_root=root, dev_root=root, env=e, pod_timeout=60)


def _runs(state):
    with open(state) as f:
        return int(f.read())


def _hip_pods(c):
    return [p for p in c.list("v1", "Pod", NS) if o.get_labels(p).get("app") == "amd-hip-validator"]


def _set_script(k, script):
    k.base_env["GEMM_STANDIN_SCRIPT"] = script          # what the kubelet's next pods run with


def test_a_gpu_below_the_floor_fails_the_pod_at_once_and_names_the_device(tmp_path, node):
    """Case (1): the workload fails the floor on GPU 3 -> the init container exits 1, the pod is Failed
    (restartPolicy Never: no crash-loop re-run), and validate_hip raises within the pod's own
    runtime + 5 s with the device and the floor in the error."""
    c, k, root, state = node
    _set_script(k, "slow:3")
    ctx = _ctx(tmp_path, c, root, "slow:3", GEMM_REMEASURE="0")
    t0 = time.monotonic()
    with pytest.raises(comp.ValidationError) as e:
        comp.validate_hip(ctx)
    took = time.monotonic() - t0
    msg = str(e.value)
    assert "device 3" in msg and "floor" in msg and "1258.3" in msg, msg
    assert {f.kind for f in e.value.failures} == {"floor"}
    pods = _hip_pods(c)
    assert len(pods) == 1 and pods[0]["status"]["phase"] == "Failed"
    st = pods[0]["status"]["initContainerStatuses"][0]
    assert st["state"]["terminated"]["exitCode"] == 1 and st["restartCount"] == 0
    assert _runs(state) == 1
    assert took < RUNTIME_S + 5 + 3, took        # + the workload's python start-up on a loaded CPU box
    assert not ctx.status.exists(S.HIP_READY)


def test_a_wrong_tile_fails_at_once_and_names_tile_xcd_and_cu(tmp_path, node):
    """amd-gemm-validate's ABFT check finds a wrong output tile on GPU 3: a correctness failure -- no
    re-measure (a wrong result is not a throughput fluke) -- whose error names the device, the tile,
    the XCD and the CU, with the location structured on the GateFailure."""
    c, k, root, state = node
    _set_script(k, "badtile:3@5.7.2")
    ctx = _ctx(tmp_path, c, root, "badtile:3@5.7.2")
    with pytest.raises(comp.ValidationError) as e:
        comp.validate_hip(ctx)
    msg = str(e.value)
    assert "device 3" in msg and "[5, 7]" in msg and "XCD 2" in msg and "se1.sh0.cu4" in msg, msg
    f = [x for x in e.value.failures if x.kind == "correctness"]
    assert f and f[0].where["tile"] == [5, 7] and f[0].where["xcd"] == 2 and f[0].where["device"] == 3
    assert _runs(state) == 1
    assert not ctx.status.exists(S.HIP_READY)
    # the node-local record and its metric: the bad CU without reading pod logs
    rec = ctx.status.read(S.HIP_LAST_FAILURE)
    assert rec["failures"][0]["where"]["xcd"] == 2
    from prometheus_client import generate_latest
    from gpu_operator_amd.validator.metrics import NodeMetrics
    m = NodeMetrics(ctx)
    m.refresh_status()
    text = generate_latest(m.registry).decode()
    assert ('amd_gpu_operator_validator_gemm_bad_tile{cu="se1.sh0.cu4",dtype="bf16",gpu="3",node="n1",tile="5,7",'
            'xcd="2"} 1.0') in text, [ln for ln in text.splitlines() if "bad_tile" in ln]
    # the next passing validation clears it
    _set_script(k, "fast")
    comp.validate_hip(_ctx(tmp_path, c, root, "fast"))
    assert not ctx.status.exists(S.HIP_LAST_FAILURE)
    m.refresh_status()
    assert "validator_gemm_bad_tile{" not in generate_latest(m.registry).decode()


def test_a_passing_run_records_full_coverage(tmp_path, node):
    c, k, root, state = node
    _set_script(k, "fast")
    ctx = _ctx(tmp_path, c, root, "fast")
    info = comp.validate_hip(ctx)
    assert info["checked_fraction"] == 1.0 and info["abft_worst_ratio"] < 1.0
    assert ctx.status.read(S.HIP_READY)["checked_fraction"] == 1.0


def test_a_slow_first_run_is_measured_once_more_and_passes(tmp_path, node):
    """Case (2): slow on the first run, healthy on the second -> hip-ready after exactly one extra pod."""
    c, k, root, state = node
    _set_script(k, "slow:3;fast")
    ctx = _ctx(tmp_path, c, root, "slow:3;fast")
    info = comp.validate_hip(ctx)
    assert ctx.status.exists(S.HIP_READY) and _runs(state) == 2
    assert info["remeasured"]["first_kinds"] == ["floor"]
    assert any("device 3" in f for f in info["remeasured"]["first_failure"])
    assert info["gemm_tflops_per_gpu"] == 1500.0


def test_a_persistent_throughput_failure_fails_after_one_remeasure(tmp_path, node):
    c, k, root, state = node
    _set_script(k, "slow:5")
    ctx = _ctx(tmp_path, c, root, "slow:5")
    with pytest.raises(comp.ValidationError, match="device 5"):
        comp.validate_hip(ctx)
    assert _runs(state) == 2


def test_a_tenant_scheduled_during_the_sweep_is_disturbed_not_failed(tmp_path, node, monkeypatch):
    """Item 2 / case (iv): a 1-GPU tenant is given GPU 3 while the HIP sweep runs (the HIP pod is
    privileged and requests no GPU, so the device plugin kept advertising it). GPU 3 measures the
    sharing: the post-run re-check marks it disturbed, its throughput is out of the gates, hip-ready
    opens -- no floor failure, no re-measure."""
    c, k, root, state = node
    _set_script(k, "slow:3")
    from gpu_operator_amd import devices as D
    g3 = [g for g in D.enumerate_gpus(root) if g["index"] == 3][0]
    monkeypatch.setattr(comp, "_pod_device_ids",
                        lambda ctx: {"default/train-0": [f"amdgpu-{g3['unique_id']:016x}"]})

    def tenant_arrives():
        for _ in range(400):
            if os.path.exists(state + ".running"):
                break
            time.sleep(0.025)
        c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "train-0", "namespace": "default"},
                  "spec": {"nodeName": NODE,
                           "containers": [{"name": "t", "resources": {"limits": {"amd.com/gpu": "1"}}}]},
                  "status": {"phase": "Running"}})
    th = threading.Thread(target=tenant_arrives)
    k.hold_admission = lambda p: o.name(p) == "train-0"       # the API object is the tenant; no process
    th.start()
    ctx = _ctx(tmp_path, c, root, "slow:3")
    info = comp.validate_hip(ctx)
    th.join()
    assert ctx.status.exists(S.HIP_READY) and _runs(state) == 1
    assert info["disturbed"]["devices"] == [3] and info["disturbed"]["pods"] == ["default/train-0"]
    assert "remeasured" not in info and info.get("pod_failed", {}).get("exit_code") == 1


def test_a_tenant_that_arrives_after_the_sweep_exempts_nothing(tmp_path, node, monkeypatch):
    """the post-run re-check used to exempt every GPU a tenant held at that moment, also one
    scheduled after the sweep ended -- so a genuinely slow GPU could open hip-ready unchecked. A pod whose
    startTime is after the sweep shared nothing with it: GPU 3 stays gated, its slow result fails (after
    the one re-measure a throughput failure gets), and the late tenant is recorded as arrived_after."""
    import datetime
    c, k, root, state = node
    _set_script(k, "slow:3")
    from gpu_operator_amd import devices as D
    g3 = [g for g in D.enumerate_gpus(root) if g["index"] == 3][0]
    monkeypatch.setattr(comp, "_pod_device_ids",
                        lambda ctx: {"default/late-0": [f"amdgpu-{g3['unique_id']:016x}"]})
    late = (datetime.datetime.now(datetime.timezone.utc) + datetime.timedelta(hours=1)).isoformat()

    def tenant_arrives():
        for _ in range(400):
            if os.path.exists(state + ".running"):
                break
            time.sleep(0.025)
        c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "late-0", "namespace": "default"},
                  "spec": {"nodeName": NODE,
                           "containers": [{"name": "t", "resources": {"limits": {"amd.com/gpu": "1"}}}]},
                  "status": {"phase": "Running", "startTime": late}})
    th = threading.Thread(target=tenant_arrives)
    k.hold_admission = lambda p: o.name(p) == "late-0"
    th.start()
    ctx = _ctx(tmp_path, c, root, "slow:3", GEMM_REMEASURE="0")
    with pytest.raises(comp.ValidationError) as e:
        comp.validate_hip(ctx)
    th.join()
    assert "device 3" in str(e.value) and {f.kind for f in e.value.failures} == {"floor"}
    assert not ctx.status.exists(S.HIP_READY)
    # the start-time filter itself
    assert comp.gpu_pods_on_node(ctx) == ["default/late-0"]
    later = []
    assert comp.gpu_pods_on_node(ctx, started_before=time.time(), later=later) == [] and later == ["default/late-0"]
