"""Node validator components against fake sysfs + the fake API server."""

import json
import os
import subprocess
import threading
import time

import pytest

from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.validator import components as comp
from gpu_operator_amd.validator import main as vmain
from gpu_operator_amd.validator import status as S
from gpu_operator_amd.validator.metrics import NodeMetrics

NS = "amd-gpu-operator"


@pytest.fixture
def node_root(tmp_path):
    return str(fakesys.make_node(tmp_path / "root"))


def node_obj(name="n1", gpus=8, labels=None):
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": labels or {}},
            "status": {"capacity": {"amd.com/gpu": str(gpus)}, "allocatable": {"amd.com/gpu": str(gpus)}}}


def ctx_for(tmp_path, root, client=None, **kw):
    env = {"VALIDATOR_IMAGE": "registry.example.com/amd/amd-gpu-operator-node:v0.1.0",
           "DRIVER_ROOT_MODE": kw.pop("driver_mode", "container")}
    env.update(kw.pop("env", {}))
    return comp.Context(status=S.StatusDir(str(tmp_path / "validations")), node_name="n1", namespace=NS,
                        client=client, host_root=str(tmp_path / "host"), sys_root=root, dev_root=root,
                        env=env, **kw)


class FakeKubelet:
    """Completes validation pods with a canned termination message, with kubelet's semantics for
    the pod's restartPolicy: ``exit_code`` 0 -> Succeeded; non-zero -> the init container terminated
    with it and, under ``Never``, the pod Failed -- under ``OnFailure`` the pod stays Pending and the
    container is restarted (restartCount 1, the exit in lastState), as a real kubelet does."""

    def __init__(self, client, messages, exit_code=0):
        self.client, self.messages, self.exit_code = client, messages, exit_code
        self.seen = []
        self.stop = client.watch("v1", "Pod", self.on_event)

    def on_event(self, ev):
        if ev.type != "ADDED":
            return
        pod = ev.obj
        self.seen.append(pod)
        app = o.get_labels(pod).get("app")
        msg = self.messages.get(app, "")
        if isinstance(msg, list):               # one message per pod, the last one repeats
            msg = msg.pop(0) if len(msg) > 1 else msg[0]
        code = self.exit_code.pop(0) if isinstance(self.exit_code, list) and len(self.exit_code) > 1 else \
            (self.exit_code[0] if isinstance(self.exit_code, list) else self.exit_code)

        def finish():
            time.sleep(0.05)
            try:
                p = self.client.get("v1", "Pod", o.name(pod), o.namespace(pod))
            except Exception:  # noqa: BLE001 - the validator withdrew the pod first
                return
            term = {"exitCode": code, "reason": "Completed" if code == 0 else "Error", "message": msg}
            if code == 0:
                p["status"] = {"phase": "Succeeded", "initContainerStatuses": [
                    {"name": "x", "restartCount": 0, "state": {"terminated": term}}]}
            elif (p.get("spec") or {}).get("restartPolicy") == "Never":
                p["status"] = {"phase": "Failed", "initContainerStatuses": [
                    {"name": "x", "restartCount": 0, "state": {"terminated": term}}]}
            else:
                p["status"] = {"phase": "Pending", "initContainerStatuses": [
                    {"name": "x", "restartCount": 1, "state": {"running": {}}, "lastState": {"terminated": term}}]}
            self.client.update_status(p)
        threading.Thread(target=finish).start()


GEMM_MSG = "\n".join(json.dumps(x) for x in [
    {"event": "hip-smoke", "devices": 8, "ok": True},
    {"event": "aggregate", "m": 8192, "n": 8192, "k": 8192, "gpus": 8, "total_tflops": 10900.0,
     "per_gpu_tflops": 1362.5},
    {"event": "gemm", "device": 0, "m": 8192, "n": 8192, "k": 8192, "tflops": 1362.5, "ok": True}])
RCCL_MSG = "\n".join(json.dumps(x) for x in [
    {"event": "allreduce", "ranks": 8, "bytes": 1 << 30, "busbw_gbps": 310.0, "ok": True},
    {"event": "summary", "ranks": 8, "peak_busbw_gbps": 310.0, "ok": True}])


# ---------------------------------------------------------------------------------------------
def test_driver_container_mode_waits_for_driver_ctr_barrier(tmp_path, node_root):
    ctx = ctx_for(tmp_path, node_root, with_wait=True, wait_timeout=5)

    def driver_pod():
        time.sleep(0.2)
        ctx.status.create(S.DRIVER_CTR_READY)
    threading.Thread(target=driver_pod).start()
    info = comp.validate_driver(ctx)
    assert info["mode"] == "container" and info["gpus"] == 8 and info["gfx"] == ["gfx950"]
    assert ctx.status.exists(S.DRIVER_READY) and not ctx.status.exists(S.HOST_DRIVER_READY)
    assert ctx.status.read(S.DRIVER_READY)["products"] == ["AMD Instinct MI355X"]


def test_driver_host_mode(tmp_path, node_root):
    ctx = ctx_for(tmp_path, node_root, driver_mode="host")
    comp.validate_driver(ctx)
    assert ctx.status.exists(S.HOST_DRIVER_READY)


def test_driver_not_live_fails_without_wait(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", live=False))
    ctx = ctx_for(tmp_path, root, driver_mode="host")
    with pytest.raises(comp.ValidationError, match="not loaded|not live"):
        comp.validate_driver(ctx)


def test_driver_wait_is_bounded(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", live=False))
    ctx = ctx_for(tmp_path, root, driver_mode="host", with_wait=True, wait_timeout=0.5, sleep_interval=0.1)
    t0 = time.monotonic()
    with pytest.raises(comp.ValidationError):
        comp.validate_driver(ctx)
    assert time.monotonic() - t0 < 3


def test_toolkit_requires_injected_devices(tmp_path, node_root):
    ctx = ctx_for(tmp_path, node_root)
    assert comp.validate_toolkit(ctx)["render_nodes"] == 8
    os.remove(os.path.join(node_root, "dev/dri/renderD131"))
    with pytest.raises(comp.ValidationError, match="renderD131"):
        comp.check_toolkit(ctx)


def test_hip_spawns_pinned_pod_and_records_results(tmp_path, node_root):
    owner_uid = "cp-uid"
    c = FakeClient([node_obj(), {"apiVersion": "apps/v1", "kind": "DaemonSet",
                                 "metadata": {"name": "amd-operator-validator", "namespace": NS,
                                              "ownerReferences": [{"apiVersion": "amd.com/v1",
                                                                   "kind": "ClusterPolicy", "name": "cp",
                                                                   "uid": owner_uid, "controller": True}]},
                                 "spec": {"template": {"spec": {"tolerations": [{"key": "amd.com/gpu",
                                                                                 "operator": "Exists"}]}}}}])
    k = FakeKubelet(c, {"amd-hip-validator": GEMM_MSG})
    ctx = ctx_for(tmp_path, node_root, client=c, env={"VALIDATOR_RUNTIME_CLASS": "amd"})
    info = comp.validate_hip(ctx)
    pod = k.seen[0]
    assert pod["spec"]["nodeName"] == "n1" and pod["spec"]["runtimeClassName"] == "amd"
    assert pod["metadata"]["ownerReferences"][0]["uid"] == owner_uid
    assert pod["spec"]["tolerations"][0]["key"] == "amd.com/gpu"
    assert all(x["image"].endswith("amd-gpu-operator-node:v0.1.0") for x in pod["spec"]["initContainers"])
    assert info["gemm_tflops_total"] == 10900.0 and info["smoke_ok"]
    assert ctx.status.read(S.HIP_READY)["gemm_tflops_per_gpu"] == 1362.5


def test_hip_failed_pod_fails_validation_fast(tmp_path, node_root):
    """restartPolicy Never: the failing workload fails the pod; the validator returns at once with a
    ValidationError naming the failing check (not a 300 s timeout)."""
    c = FakeClient([node_obj()])
    k = FakeKubelet(c, {"amd-hip-validator": '{"event":"gemm","dtype":"bf16","device":3,"ok":false,'
                                             '"kind":"correctness","error":"check failed: max_rel_err 0.5"}'},
                    exit_code=1)
    ctx = ctx_for(tmp_path, node_root, client=c, pod_timeout=60)
    t0 = time.monotonic()
    with pytest.raises(comp.ValidationError, match="device 3: check failed") as e:
        comp.validate_hip(ctx)
    assert time.monotonic() - t0 < 5 and len(k.seen) == 1          # a correctness failure: no re-measure
    assert [f.kind for f in e.value.failures] == ["correctness"]
    assert k.seen[0]["spec"]["restartPolicy"] == "Never"
    assert not ctx.status.exists(S.HIP_READY)


def test_onfailure_pod_fails_at_the_first_container_exit(tmp_path, node_root, monkeypatch):
    """A pod template with the reference's OnFailure (an admin's ConfigMap override): the kubelet
    restarts the failing init container and the pod never reaches Failed -- wait_for_pod returns at the
    first non-zero exit (lastState), deletes the crash-looping pod, and reports the workload's lines."""
    from gpu_operator_amd.validator import workload as W
    real = W.load_pod_spec

    def onfailure(name):
        t = real(name)
        t["spec"]["restartPolicy"] = "OnFailure"
        return t
    monkeypatch.setattr(W, "load_pod_spec", onfailure)
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-hip-validator": '{"event":"hip-smoke","ok":false,"kind":"correctness"}'}, exit_code=1)
    ctx = ctx_for(tmp_path, node_root, client=c, pod_timeout=60)
    t0 = time.monotonic()
    with pytest.raises(comp.ValidationError, match="hip-smoke failed"):
        comp.validate_hip(ctx)
    assert time.monotonic() - t0 < 5
    assert not [p for p in c.list("v1", "Pod", NS) if o.get_labels(p).get("app") == "amd-hip-validator"]


def test_failed_pod_without_result_lines_names_the_exit(tmp_path, node_root):
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-hip-validator": "Traceback (most recent call last): boom"}, exit_code=2)
    ctx = ctx_for(tmp_path, node_root, client=c, pod_timeout=60)
    with pytest.raises(comp.ValidationError, match="failed with no result.*exited 2"):
        comp.validate_hip(ctx)


def test_hip_pod_timeout_is_a_validation_error(tmp_path, node_root):
    c = FakeClient([node_obj()])                    # no kubelet: the pod never runs
    ctx = ctx_for(tmp_path, node_root, client=c, pod_timeout=0.5)
    with pytest.raises(comp.ValidationError, match="did not finish within 0s|did not finish within 1s"):
        comp.validate_hip(ctx)


def test_plugin_waits_for_capacity_event(tmp_path, node_root):
    n = node_obj(gpus=0)
    n["status"]["capacity"] = {}
    c = FakeClient([n])
    ctx = ctx_for(tmp_path, node_root, client=c, resource_timeout=5)

    def device_plugin_registers():
        time.sleep(0.2)
        cur = c.get("v1", "Node", "n1")
        cur["status"]["capacity"] = {"amd.com/gpu": "8"}
        c.update_status(cur)
    threading.Thread(target=device_plugin_registers).start()
    t0 = time.monotonic()
    info = comp.validate_plugin(ctx)
    assert info["devices"] == 8 and time.monotonic() - t0 < 2
    assert ctx.status.exists(S.PLUGIN_READY)


def test_plugin_times_out(tmp_path, node_root):
    n = node_obj()
    n["status"]["capacity"] = {}
    ctx = ctx_for(tmp_path, node_root, client=FakeClient([n]), resource_timeout=0.3)
    with pytest.raises(comp.ValidationError, match="no amd.com/gpu"):
        comp.validate_plugin(ctx)


def test_plugin_workload_requests_partition_resource_when_mixed(tmp_path, node_root):
    n = node_obj()
    n["status"]["capacity"] = {"amd.com/partition-cpx": "64"}
    c = FakeClient([n])
    k = FakeKubelet(c, {"amd-device-plugin-validator": GEMM_MSG})
    ctx = ctx_for(tmp_path, node_root, client=c, with_workload=True, partition_strategy="mixed")
    comp.validate_plugin(ctx)
    assert k.seen[0]["spec"]["initContainers"][0]["resources"]["limits"] == {"amd.com/partition-cpx": 1}


def test_rccl_requests_all_gpus_and_records_busbw(tmp_path, node_root):
    c = FakeClient([node_obj()])
    k = FakeKubelet(c, {"amd-rccl-validator": RCCL_MSG})
    ctx = ctx_for(tmp_path, node_root, client=c)
    info = comp.validate_rccl(ctx)
    assert k.seen[0]["spec"]["initContainers"][0]["resources"]["limits"] == {"amd.com/gpu": 8}
    assert info["peak_busbw_gbps"] == 310.0 and ctx.status.exists(S.RCCL_READY)


def test_rccl_single_gpu_node_skips(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r1", n_gpus=1))
    ctx = ctx_for(tmp_path, root, client=FakeClient([node_obj(gpus=1)]))
    assert "skipped" in comp.validate_rccl(ctx)


def test_vfio_and_mxgpu_components(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=2, vfio_bound=True))
    c = FakeClient([node_obj(labels={"amd.com/gpu.workload.config": "vm-passthrough"})])
    ctx = ctx_for(tmp_path, root, client=c)
    assert comp.validate_vfio_pci(ctx)["devices"] == 2
    assert open(ctx.status.file(S.WORKLOAD_TYPE)).read() == "vm-passthrough"
    assert comp.sandbox_ready_wait(ctx) == {"workload_type": "vm-passthrough"}
    root2 = str(fakesys.make_node(tmp_path / "r2", n_gpus=2))
    ctx2 = ctx_for(tmp_path, root2, client=c)
    with pytest.raises(comp.ValidationError, match="not bound to vfio-pci"):
        comp.validate_vfio_pci(ctx2)


def test_time_to_ready_and_node_metrics(tmp_path, node_root):
    sd = S.StatusDir(str(tmp_path / "v"))
    t = 1000.0
    sd.create(S.DRIVER_CTR_READY, {"ts": t})
    sd.create(S.DRIVER_READY, {"ts": t + 0.5})
    sd.create(S.TOOLKIT_READY, {"ts": t + 3.0})
    sd.create(S.HIP_READY, {"ts": t + 9.0, "gemm_tflops_total": 10900.0, "gemm_tflops_per_gpu": 1362.5,
                            "gpu_tflops": [{"dtype": "bf16", "m": 8192, "n": 8192, "k": 8192,
                                            "tflops": {str(i): 1650.0 + i for i in range(8)}},
                                           {"dtype": "fp8_e4m3fn", "m": 8192, "n": 8192, "k": 8192,
                                            "tflops": {"0": 3300.0}}],
                            "tflops_by_dtype_gpus": {
                                "bf16": {"1": {"total_tflops": 1400.0, "per_gpu_tflops": 1400.0, "efficiency": 1.0},
                                         "8": {"total_tflops": 10900.0, "per_gpu_tflops": 1362.5,
                                               "efficiency": 0.9732}}}})
    sd.create(S.PLUGIN_READY, {"ts": t + 9.5})
    import json as _json
    sd.write_raw("device-health", _json.dumps({"ts": t, "devices": {
        "amdgpu-a": {"healthy": True, "reason": "", "bdf": "0000:05:00.0"},
        "amdgpu-b": {"healthy": False, "reason": "uncorrectable RAS errors: 1 (umc)", "bdf": "0000:15:00.0"}}}))
    sd.create(S.RCCL_READY, {"ts": t + 14.0, "peak_busbw_gbps": 310.0, "ranks": 8,
                             "busbw_by_ranks": {"2": 141.0, "4": 230.5, "8": 310.0}})
    assert S.time_to_ready(sd) == pytest.approx(14.0)
    ctx = ctx_for(tmp_path, node_root, client=FakeClient([node_obj()]))
    ctx.status = sd
    m = NodeMetrics(ctx)
    m.refresh_all()
    from prometheus_client import generate_latest
    text = generate_latest(m.registry).decode()
    assert 'amd_gpu_operator_node_time_to_ready_seconds{node="n1"} 14.0' in text
    # the device plugin's health verdicts (device-health), one series per withdrawn device with its reason
    assert ('amd_gpu_operator_node_device_unhealthy{bdf="0000:15:00.0",device="amdgpu-b",node="n1",'
            'reason="uncorrectable RAS errors: 1 (umc)"} 1.0') in text
    assert 'amd_gpu_operator_node_devices_unhealthy{node="n1"} 1.0' in text
    assert 'device="amdgpu-a"' not in text
    assert 'amd_gpu_operator_validator_gemm_tflops{dtype="bf16",gpus="8",node="n1",scope="node"} 10900.0' in text
    assert 'amd_gpu_operator_validator_gemm_tflops{dtype="bf16",gpus="1",node="n1",scope="per_gpu"} 1400.0' in text
    assert 'amd_gpu_operator_validator_gemm_scaling_efficiency{dtype="bf16",gpus="8",node="n1"} 0.9732' in text
    assert 'amd_gpu_operator_node_device_plugin_devices_total{node="n1"} 8.0' in text
    assert 'amd_gpu_operator_node_driver_validation{node="n1"} 1.0' in text
    assert 'amd_gpu_operator_amd_pci_devices_total{node="n1"} 8.0' in text
    assert 'amd_gpu_operator_validator_allreduce_busbw_gbps{node="n1",ranks="8"} 310.0' in text
    assert 'amd_gpu_operator_validator_allreduce_busbw_gbps{node="n1",ranks="2"} 141.0' in text
    # one series per GPU (SURVEY §5.5 {gpu,dtype,m,n,k}): a GPU failing the node-median gate is visible
    per_gpu = [ln for ln in text.splitlines() if ln.startswith("amd_gpu_operator_validator_gemm_gpu_tflops{")
               and 'dtype="bf16"' in ln]
    assert len(per_gpu) == 8
    assert ('amd_gpu_operator_validator_gemm_gpu_tflops{dtype="bf16",gpu="3",k="8192",m="8192",n="8192",node="n1"} '
            '1653.0') in text
    assert 'amd_gpu_operator_validator_gemm_gpu_tflops{dtype="fp8",gpu="0",k="8192",m="8192",n="8192",node="n1"} 3300.0' in text


def test_cli_driver_component(tmp_path, node_root, capsys):
    out_dir = str(tmp_path / "vals")
    os.environ["DRIVER_ROOT_MODE"] = "host"
    try:
        rc = vmain.main(["--component", "driver", "--output-dir", out_dir, "--sys-root", node_root,
                         "--dev-root", node_root, "--host-root", str(tmp_path)])
    finally:
        del os.environ["DRIVER_ROOT_MODE"]
    assert rc == 0 and os.path.exists(os.path.join(out_dir, S.HOST_DRIVER_READY))
    assert json.loads(capsys.readouterr().out.strip().splitlines()[-1])["ok"]
    assert vmain.main(["--component", "bogus", "--output-dir", out_dir]) == 2


def test_status_files_atomic_and_cleanup(tmp_path):
    sd = S.StatusDir(str(tmp_path / "v"))
    sd.create(S.DRIVER_READY, {"x": 1})
    sd.create(S.TOOLKIT_READY)
    sd.write_raw(S.WORKLOAD_TYPE, "container")
    assert sd.read(S.DRIVER_READY)["x"] == 1
    sd.cleanup_ready()
    assert not sd.exists(S.DRIVER_READY) and sd.exists(S.WORKLOAD_TYPE)
    sd.cleanup_all()
    assert os.listdir(sd.path) == []


# -- RCCL fabric proof: rank sweep, busBW floor, topology ------------------------------------------
RCCL_SWEEP_MSG = "\n".join(json.dumps(x) for x in [
    {"event": "fabric", "physical_gpus": 8, "single_hive": True, "full_node": True, "min_xgmi_links": 7, "ok": True},
    {"event": "ranks_summary", "ranks": 2, "peak_busbw_gbps": 140.0, "ok": True},
    {"event": "ranks_summary", "ranks": 8, "peak_busbw_gbps": 310.0, "ok": True},
    {"event": "summary", "ranks": 8, "ranks_run": [2, 4, 8], "peak_busbw_gbps": 310.0, "ok": True},
    {"event": "rccl-debug", "algo_proto": {"Ring/Simple": 3}, "channels": 32, "lines": []}])


def _pod_env(pod):
    return {e["name"]: e.get("value") for e in pod["spec"]["initContainers"][0].get("env", [])}


def test_rccl_sweeps_rank_counts_and_passes_the_busbw_floor(tmp_path, node_root):
    c = FakeClient([node_obj()])
    k = FakeKubelet(c, {"amd-rccl-validator": RCCL_SWEEP_MSG})
    ctx = ctx_for(tmp_path, node_root, client=c, env={"RCCL_MIN_BUSBW_GBPS": "250"})
    info = comp.validate_rccl(ctx)
    env = _pod_env(k.seen[0])
    assert env["RCCL_RANKS"] == "2,4,8" and env["RCCL_MIN_BUSBW_GBPS"] == "250"
    assert "amd.com/gpu: 8" not in open(os.path.join(os.path.dirname(comp.__file__), "manifests",
                                                     "rccl-workload-validation.yaml")).read()
    assert info["busbw_by_ranks"] == {2: 140.0, 8: 310.0} and info["algo_proto"] == {"Ring/Simple": 3}
    assert info["fabric"]["full_node"] and info["ok"]


def test_rccl_fails_validation_on_a_split_hive(tmp_path, node_root):
    msg = "\n".join(json.dumps(x) for x in [
        {"event": "fabric", "physical_gpus": 8, "single_hive": False, "ok": False, "reason": "GPUs span 2 xGMI hives"},
        {"event": "summary", "ok": False, "reason": "fabric check failed"}])
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-rccl-validator": msg}, exit_code=1)
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(Exception):
        comp.validate_rccl(ctx)
    assert not ctx.status.exists(S.RCCL_READY)


def test_rccl_ranks_follow_the_node_gpu_count(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r4", n_gpus=4))
    c = FakeClient([node_obj(gpus=4)])
    k = FakeKubelet(c, {"amd-rccl-validator": RCCL_SWEEP_MSG})
    comp.validate_rccl(ctx_for(tmp_path, root, client=c))
    assert _pod_env(k.seen[0])["RCCL_RANKS"] == "2,4"
    assert k.seen[0]["spec"]["initContainers"][0]["resources"]["limits"] == {"amd.com/gpu": 4}


RCCL_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu_operator_amd", "_native",
                        "bin", "amd-rccl-validate")


def _topology(root):
    p = subprocess.run([RCCL_BIN, "--topology-only", "--sys-root", str(root)], capture_output=True, text=True,
                       timeout=30)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, {x["event"]: x for x in lines}


@pytest.mark.skipif(not os.path.exists(RCCL_BIN), reason="amd-rccl-validate not built")
def test_rccl_topology_full_mesh_hive_ok(tmp_path):
    rc, ev = _topology(fakesys.make_node(tmp_path, n_gpus=8))
    assert rc == 0 and ev["fabric"]["ok"] and ev["fabric"]["full_node"] and ev["fabric"]["min_xgmi_links"] == 7
    assert len(ev["topology"]["gpus"]) == 8 and all(len(g["xgmi_peers"]) == 7 for g in ev["topology"]["gpus"])


@pytest.mark.skipif(not os.path.exists(RCCL_BIN), reason="amd-rccl-validate not built")
def test_rccl_topology_split_hive_fails(tmp_path):
    from pathlib import Path
    root = fakesys.make_node(tmp_path, n_gpus=8)
    topo = Path(root) / "sys/class/kfd/kfd/topology/nodes"
    for n in (5, 6, 7, 8):                     # half the GPUs report another hive
        props = topo / str(n) / "properties"
        props.write_text(props.read_text().replace(f"hive_id {0x5A5A_0001}", "hive_id 12345"))
        (Path(root) / "sys/bus/pci/devices").joinpath(f"0000:{0x05 + 0x10 * (n - 1):02x}:00.0",
                                                      "xgmi_hive_info/xgmi_hive_id").write_text("12345\n")
    rc, ev = _topology(root)
    assert rc == 1 and not ev["fabric"]["ok"] and "2 xGMI hives" in ev["fabric"]["reason"]


@pytest.mark.skipif(not os.path.exists(RCCL_BIN), reason="amd-rccl-validate not built")
def test_rccl_topology_missing_link_fails(tmp_path):
    import shutil
    from pathlib import Path
    root = fakesys.make_node(tmp_path, n_gpus=8)
    shutil.rmtree(Path(root) / "sys/class/kfd/kfd/topology/nodes/3/io_links/4")
    rc, ev = _topology(root)
    assert rc == 1 and "6 xGMI links" in ev["fabric"]["reason"]


@pytest.mark.skipif(not os.path.exists(RCCL_BIN), reason="amd-rccl-validate not built")
def test_rccl_topology_single_gpu_is_fine(tmp_path):
    rc, ev = _topology(fakesys.make_node(tmp_path, n_gpus=1))
    assert rc == 0 and ev["fabric"]["ok"] and not ev["fabric"]["full_node"]


def test_rccl_debug_log_summary():
    from gpu_operator_amd.validator.workload_main import parse_rccl_debug
    log = "\n".join([
        "host:1:1 [0] NCCL INFO Channel 00/16 :    0   1   2   3   4   5   6   7",
        "host:1:1 [0] NCCL INFO Channel 15/16 :    0   1   2   3   4   5   6   7",
        "host:1:1 [0] NCCL INFO comm 0x1 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0",
        "host:1:1 [0] NCCL INFO AllReduce: 1048576 Bytes -> Algo 1 proto 2 time 21.5",
        "host:1:1 [0] NCCL INFO AllReduce: 1024 Bytes -> Algo 0 proto 0 time 9.1",
        "host:1:1 [0] NCCL INFO AllReduce: 2048 Bytes -> Algo 0 proto 0 time 9.4",
        "unrelated"])
    d = parse_rccl_debug(log)
    assert d["algo_proto"] == {"Ring/Simple": 1, "Tree/LL": 2} and d["channels"] == 16
    assert any("nRanks 8" in x for x in d["lines"])


def test_rccl_workload_cli_reads_env(monkeypatch):
    from gpu_operator_amd.validator import workload_main as WM
    seen = {}

    def fake(max_bytes, dtype, ranks=None, min_busbw=None, processes=0, **kw):
        seen.update(max_bytes=max_bytes, dtype=dtype, ranks=ranks, min_busbw=min_busbw, processes=processes)
        return [{"event": "summary", "ok": True}]
    monkeypatch.setattr(WM, "run_rccl", fake)
    monkeypatch.setattr(WM, "emit", lambda r: None)
    monkeypatch.setenv("RCCL_MIN_BUSBW_GBPS", "123.5")
    monkeypatch.setenv("RCCL_RANKS", "2,8")
    assert WM.main(["rccl"]) == 0
    # bf16 in the pod, as in local mode
    assert seen == {"max_bytes": 8 << 30, "dtype": "bf16", "ranks": "2,8", "min_busbw": 123.5, "processes": 0}


# -- throughput floors, node shapes, busy nodes ------------------------------
def _gemm_msg(per_gpu, dtype="bf16", gpus=8):
    return "\n".join(json.dumps(x) for x in [
        {"event": "hip-smoke", "devices": gpus, "ok": True},
        {"event": "aggregate", "dtype": dtype, "m": 8192, "n": 8192, "k": 8192, "gpus": gpus,
         "total_tflops": per_gpu * gpus, "per_gpu_tflops": per_gpu, "min_gpu_tflops": per_gpu, "ok": True},
        {"event": "gemm", "dtype": dtype, "device": 0, "m": 8192, "n": 8192, "k": 8192, "tflops": per_gpu,
         "ok": True}])


def test_gemm_floors_come_from_the_model_and_env(tmp_path, node_root):
    f = comp.gemm_floors(ctx_for(tmp_path, node_root))
    assert f == {"bf16": round(2516.6 * 0.50, 1), "fp8": round(5033.2 * 0.50, 1)}   # MI355X dense peaks
    f = comp.gemm_floors(ctx_for(tmp_path, node_root, env={"GEMM_MIN_TFLOPS_BF16": "1200",
                                                           "GEMM_MIN_TFLOPS_FP8": "0"}))
    assert f == {"bf16": 1200.0, "fp8": 0.0}
    cpx = str(fakesys.make_node(tmp_path / "cpx", compute="CPX"))       # a partition has 1/8 of the CUs
    assert comp.gemm_floors(ctx_for(tmp_path, cpx))["bf16"] == round(2516.6 * 0.50 / 8, 1)
    with pytest.raises(comp.ValidationError, match="not a number"):
        comp.gemm_floors(ctx_for(tmp_path, node_root, env={"GEMM_MIN_TFLOPS_BF16": "fast"}))
    # the busBW floor: explicit env, else mesh-aware from the measured link matrix, else the model's link
    ctx = ctx_for(tmp_path, node_root)
    assert comp.busbw_floor(ctx) == 0.0
    assert comp.busbw_gate(ctx, {}) == {"min_busbw_gbps": round(153.6 * 0.25, 1), "basis": "model-link"}
    g = comp.busbw_gate(ctx, {"links": {"min_gpu_ingress_gbps": 700.0}})
    assert g["basis"] == "measured-mesh" and g["min_busbw_gbps"] == 210.0
    assert comp.busbw_gate(ctx_for(tmp_path, node_root, env={"RCCL_MIN_BUSBW_GBPS": "99"}), {})["basis"] == "env"


def test_hip_below_floor_opens_no_barrier(tmp_path, node_root):
    c = FakeClient([node_obj()])
    k = FakeKubelet(c, {"amd-hip-validator": _gemm_msg(600.0)})          # a GPU at ~1/4 of its rate
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(comp.ValidationError, match="below the 1258.3 floor"):
        comp.validate_hip(ctx)
    assert not ctx.status.exists(S.HIP_READY)
    env = _pod_env(k.seen[0])
    assert env["GEMM_MIN_TFLOPS_BF16"] == "1258.3" and env["GEMM_SCALING"] == "1,2,4,8"
    assert env["GEMM_MIN_RELATIVE"] == "0.85" and env["GEMM_MIN_EFFICIENCY"] == "0.9"
    assert "GEMM_DEVICES" not in env and "GEMM_PROBE_DEVICES" not in env       # an idle node: every GPU


def test_hip_throughput_failure_is_measured_once_more(tmp_path, node_root):
    """A throughput gate alone (every result correct) re-measures once before failing the node: a
    transient costs one more run, not a crash-loop back-off. A persistent one still fails."""
    c = FakeClient([node_obj()])
    k = FakeKubelet(c, {"amd-hip-validator": [_gemm_msg(600.0), _gemm_msg(1500.0)]})
    ctx = ctx_for(tmp_path, node_root, client=c)
    info = comp.validate_hip(ctx)
    assert ctx.status.exists(S.HIP_READY) and len(k.seen) == 2
    assert "below the 1258.3 floor" in info["remeasured"]["first_failure"][0]
    # a wrong result is never re-measured
    bad = _gemm_msg(1500.0).replace('"tflops": 1500.0, "ok": true', '"tflops": 1500.0, "ok": false')
    c2 = FakeClient([node_obj()])
    k2 = FakeKubelet(c2, {"amd-hip-validator": bad})
    with pytest.raises(comp.ValidationError, match="check failed"):
        comp.validate_hip(ctx_for(tmp_path / "b", node_root, client=c2))
    assert len(k2.seen) == 1
    # the decision reads each failure's kind, never its wording
    G = comp.GateFailure
    assert comp.throughput_only([G("floor", "anything"), G("efficiency", "x"), G("relative", "y")])
    assert not comp.throughput_only([G("correctness", "below floor: 1 < 2 TFLOP/s"), G("floor", "z")])
    assert not comp.throughput_only([G("oom", "out of memory")]) and not comp.throughput_only([])


def test_hip_records_the_scaling_sweep(tmp_path, node_root):
    msg = "\n".join(json.dumps(x) for x in [
        {"event": "hip-smoke", "devices": 8, "ok": True},
        {"event": "aggregate", "dtype": "bf16", "m": 8192, "n": 8192, "k": 8192, "gpus": 1, "total_tflops": 1550.0,
         "per_gpu_tflops": 1550.0, "min_gpu_tflops": 1550.0, "efficiency": 1.0, "ok": True},
        {"event": "aggregate", "dtype": "bf16", "m": 8192, "n": 8192, "k": 8192, "gpus": 8, "total_tflops": 12168.0,
         "per_gpu_tflops": 1521.0, "min_gpu_tflops": 1510.0, "efficiency": 0.9813, "ok": True},
        {"event": "aggregate", "dtype": "fp8_e4m3fn", "m": 8192, "n": 8192, "k": 8192, "gpus": 1,
         "total_tflops": 3100.0, "per_gpu_tflops": 3100.0, "min_gpu_tflops": 3100.0, "efficiency": 1.0, "ok": True}])
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-hip-validator": msg})
    info = comp.validate_hip(ctx_for(tmp_path, node_root, client=c))
    assert info["gemm_tflops_total"] == 12168.0 and info["gpus"] == 8
    assert info["tflops_by_dtype_gpus"]["bf16"]["8"]["efficiency"] == 0.9813
    assert info["tflops_by_dtype_gpus"]["fp8"]["1"]["per_gpu_tflops"] == 3100.0


def test_rccl_below_floor_opens_no_barrier(tmp_path, node_root):
    msg = "\n".join(json.dumps(x) for x in [
        {"event": "fabric", "physical_gpus": 8, "single_hive": True, "ok": True},
        {"event": "summary", "ranks": 8, "peak_busbw_gbps": 1.0, "ok": True}])   # a pod without the floor
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-rccl-validator": msg})
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(comp.ValidationError, match="below the 38.4 GB/s floor"):
        comp.validate_rccl(ctx)
    assert not ctx.status.exists(S.RCCL_READY)


def test_rccl_full_run_keeps_the_result_on_the_node_without_writing_the_node(tmp_path, node_root):
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-rccl-validator": RCCL_SWEEP_MSG})
    ctx = ctx_for(tmp_path, node_root, client=c)
    comp.validate_rccl(ctx)
    rec = ctx.status.read(S.FABRIC_LAST_FULL)
    assert rec["ok"] and rec["peak_busbw_gbps"] == 310.0 and rec["busbw_by_ranks"]["8"] == 310.0
    assert not (c.get("v1", "Node", "n1")["metadata"].get("annotations") or {})   # no Node write
    ctx.status.cleanup_ready()                      # a validator restart's preStop keeps the record
    assert ctx.status.read(S.FABRIC_LAST_FULL)["peak_busbw_gbps"] == 310.0
    role = open(os.path.join(os.path.dirname(comp.__file__), "..", "assets", "state-operator-validation",
                             "0210_clusterrole.yaml")).read()
    assert "patch" not in role and "update" not in role


def test_rccl_time_slicing_node_asks_for_the_physical_gpus(tmp_path, node_root):
    c = FakeClient([node_obj(gpus=80)])                                 # 8 GPUs x 10 time-slicing replicas
    k = FakeKubelet(c, {"amd-rccl-validator": RCCL_SWEEP_MSG})
    info = comp.validate_rccl(ctx_for(tmp_path, node_root, client=c))
    c0 = k.seen[0]["spec"]["initContainers"][0]
    assert "limits" not in (c0.get("resources") or {}) and c0["securityContext"]["privileged"]
    assert _pod_env(k.seen[0])["AMD_VISIBLE_DEVICES"] == "all" and _pod_env(k.seen[0])["RCCL_RANKS"] == "2,4,8"
    assert info["pod_shape"] == "privileged-all" and info["physical_gpus"] == 8


def test_rccl_cpx_node_pins_one_agent_per_physical_gpu(tmp_path):
    root = str(fakesys.make_node(tmp_path / "cpx", compute="CPX"))
    n = node_obj(gpus=64)
    c = FakeClient([n])
    k = FakeKubelet(c, {"amd-rccl-validator": RCCL_SWEEP_MSG})
    info = comp.validate_rccl(ctx_for(tmp_path, root, client=c))
    env = _pod_env(k.seen[0])
    assert env["RCCL_RANKS"] == "2,4,8" and len(env["HIP_VISIBLE_DEVICES"].split(",")) == 8
    assert env["HIP_VISIBLE_DEVICES"].split(",")[:2] == ["0", "8"]       # first partition of GPU 0, GPU 1
    assert info["physical_gpus"] == 8


def test_busy_node_runs_topology_only_and_keeps_the_last_full_result(tmp_path, node_root):
    n = node_obj()
    n["metadata"]["annotations"] = {comp.FABRIC_ANNOTATION: json.dumps({"ts": 1.0, "peak_busbw_gbps": 305.0,
                                                                         "ok": True})}
    job = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "train-0", "namespace": "default"},
           "spec": {"nodeName": "n1", "containers": [{"name": "t", "resources": {"limits": {"amd.com/gpu": "8"}}}]},
           "status": {"phase": "Running"}}
    c = FakeClient([n, job])
    k = FakeKubelet(c, {"amd-rccl-validator": RCCL_SWEEP_MSG, "amd-hip-validator": _gemm_msg(700.0)})
    ctx = ctx_for(tmp_path, node_root, client=c)
    info = comp.validate_rccl(ctx)
    assert info["mode"] == "topology-only" and info["busy_pods"] == ["default/train-0"]
    assert info["fabric"]["ok"] and info["last_full"]["peak_busbw_gbps"] == 305.0
    assert not [p for p in k.seen if o.get_labels(p).get("app") == "amd-rccl-validator"]   # no collective pod
    assert ctx.status.exists(S.RCCL_READY)
    # every GPU is held (no pod-resources socket: unattributed): no full sweep, a correctness probe on
    # each, and an out-of-memory probe is a busy skip, not a failure
    k.messages["amd-hip-validator"] = _probe_msg(range(8), oom={3})
    hip = comp.validate_hip(ctx)
    env = _pod_env(k.seen[-1])
    assert env["GEMM_DEVICES"] == "none" and env["GEMM_PROBE_DEVICES"] == "0,1,2,3,4,5,6,7"
    assert hip["plan"]["attribution"] == "unattributed" and hip["plan"]["full"] == []
    assert [p["device"] for p in hip["probe"] if "skipped" in p] == [3]
    assert ctx.status.exists(S.HIP_READY)


def _probe_msg(devices, oom=(), bad=()):
    lines = [{"event": "plan", "devices": [], "probe_devices": list(devices)},
             {"event": "hip-smoke", "devices": 1, "ok": True}]
    for d in devices:
        r = {"event": "gemm", "probe": True, "dtype": "bf16", "device": d, "m": 1024, "n": 1024, "k": 1024,
             "tflops": 100.0, "ok": d not in oom and d not in bad}
        if d in oom:
            r.update(oom=True, tflops=0.0, error="out of memory: the shape needs 0.01 GiB, 0.00 GiB of 288 GiB free")
        if d in bad:
            r.update(error="max_rel_err 0.5")
        lines.append(r)
    return "\n".join(json.dumps(x) for x in lines)


def _tenant(name="train-0", gpus=2):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"nodeName": "n1", "containers": [{"name": "t", "resources": {"limits": {"amd.com/gpu": str(gpus)}}}]},
            "status": {"phase": "Running"}}


def test_hip_plan_sweeps_only_the_gpus_no_pod_holds(tmp_path, node_root, monkeypatch):
    """A tenant holds 2 GPUs (pod-resources: device ids of agents 2 and 5): the full sweep runs on
    the 6 free GPUs (GEMM_DEVICES), the 2 held ones get the correctness probe."""
    monkeypatch.setattr(comp, "_pod_device_ids", lambda ctx: {
        "default/train-0": ["amdgpu-1000000000000020", "amdgpu-1000000000000050"],
        "amd-gpu-operator/amd-hip-validator-n1": ["amdgpu-1000000000000000"]})
    c = FakeClient([node_obj(), _tenant()])
    msg = "\n".join(json.dumps(x) for x in [
        {"event": "hip-smoke", "ok": True},
        *[{"event": "gemm", "dtype": "bf16", "device": d, "m": 8192, "n": 8192, "k": 8192, "tflops": 1600.0 + d,
           "ok": True} for d in (0, 1, 3, 4, 6, 7)],
        {"event": "aggregate", "dtype": "bf16", "m": 8192, "n": 8192, "k": 8192, "gpus": 6, "total_tflops": 9621.0,
         "per_gpu_tflops": 1603.5, "min_gpu_tflops": 1600.0, "efficiency": 0.99, "ok": True}]) + "\n" + \
        "\n".join(_probe_msg([2, 5]).splitlines()[2:])
    k = FakeKubelet(c, {"amd-hip-validator": msg})
    ctx = ctx_for(tmp_path, node_root, client=c)
    info = comp.validate_hip(ctx)
    env = _pod_env(next(p for p in k.seen if o.get_labels(p).get("app") == "amd-hip-validator"))
    assert env["GEMM_DEVICES"] == "0,1,3,4,6,7" and env["GEMM_PROBE_DEVICES"] == "2,5"
    assert env["GEMM_MIN_TFLOPS_BF16"] == "1258.3"              # free GPUs keep their floor
    assert info["plan"] == {"full": [0, 1, 3, 4, 6, 7], "probe": [2, 5], "attribution": "pod-resources",
                            "busy_pods": ["default/train-0"]}
    assert ctx.status.exists(S.HIP_READY)


def test_hip_plan_holds_every_partition_of_a_held_gpu(tmp_path, monkeypatch):
    root = str(fakesys.make_node(tmp_path / "cpx", compute="CPX"))
    monkeypatch.setattr(comp, "_pod_device_ids", lambda ctx: {"default/train-0": ["amdgpu-1000000000000013"]})
    ctx = ctx_for(tmp_path, root, client=FakeClient([node_obj(gpus=64), _tenant(gpus=1)]))
    plan = comp.hip_plan(ctx, ["default/train-0"])
    assert plan["probe"] == list(range(8, 16)) and len(plan["full"]) == 56    # GPU 1's 8 partitions


def test_hip_probe_failure_that_is_not_oom_fails_the_node(tmp_path, node_root):
    c = FakeClient([node_obj(), _tenant(gpus=8)])
    k = FakeKubelet(c, {"amd-hip-validator": _probe_msg(range(8), bad={6})})
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(comp.ValidationError, match="probe device 6: max_rel_err"):
        comp.validate_hip(ctx)
    assert not ctx.status.exists(S.HIP_READY)


def test_hip_gpu_below_the_node_median_opens_no_barrier(tmp_path, node_root):
    """Every GPU above the absolute floor, one at 0.8x its 7 siblings: a sick GPU, no hip-ready."""
    per = [{"event": "gemm", "dtype": "bf16", "device": d, "m": 8192, "n": 8192, "k": 8192,
            "tflops": 1300.0 if d == 5 else 1625.0, "ok": True} for d in range(8)]
    msg = "\n".join(json.dumps(x) for x in [{"event": "hip-smoke", "ok": True}, *per])
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-hip-validator": msg})
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(comp.ValidationError, match=r"device 5: 1300.0 TFLOP/s is 0.80x the node median 1625.0"):
        comp.validate_hip(ctx)
    assert not ctx.status.exists(S.HIP_READY)
    # the same spread within 0.85 passes; GEMM_MIN_RELATIVE=0 turns the gate off
    assert not comp._relative_outliers([dict(r, tflops=1400.0) if r["device"] == 5 else r for r in per], 0.85)
    assert not comp._relative_outliers(per, 0.0)


def test_hip_low_scaling_efficiency_opens_no_barrier(tmp_path, node_root):
    msg = "\n".join(json.dumps(x) for x in [
        {"event": "hip-smoke", "ok": True},
        {"event": "aggregate", "dtype": "bf16", "m": 8192, "n": 8192, "k": 8192, "gpus": 1, "total_tflops": 1600.0,
         "per_gpu_tflops": 1600.0, "min_gpu_tflops": 1600.0, "efficiency": 1.0, "ok": True},
        {"event": "aggregate", "dtype": "bf16", "m": 8192, "n": 8192, "k": 8192, "gpus": 8, "total_tflops": 10240.0,
         "per_gpu_tflops": 1280.0, "min_gpu_tflops": 1270.0, "efficiency": 0.8, "ok": True}])
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-hip-validator": msg})
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(comp.ValidationError, match="x8: scaling efficiency 0.800 below 0.9"):
        comp.validate_hip(ctx)
    assert not ctx.status.exists(S.HIP_READY)


def test_rccl_tenant_between_the_busy_check_and_the_fabric_pod_falls_back(tmp_path, node_root):
    """The kubelet rejects the nodeName-bound fabric pod at admission (a tenant took GPUs after the
    busy check): topology-only in seconds, not a failure after the 300 s pod timeout."""
    c = FakeClient([node_obj()])
    k = FakeKubelet(c, {"amd-rccl-validator": ""}, exit_code=1)
    orig = k.on_event

    def admit(ev):                        # the tenant lands as the fabric pod is created
        if ev.type == "ADDED" and o.get_labels(ev.obj).get("app") == "amd-rccl-validator":
            c.create(_tenant(gpus=2))
        orig(ev)
    k.on_event = admit
    c.watch("v1", "Pod", admit)
    ctx = ctx_for(tmp_path, node_root, client=c)
    t = time.monotonic()
    info = comp.validate_rccl(ctx)
    assert time.monotonic() - t < 30
    assert info["mode"] == "topology-only" and info["busy_pods"] == ["default/train-0"]
    # whichever the validator sees first: the admission rejection, or the tenant before the pod started
    assert info["reason"].startswith(("fabric pod not admitted", "fabric pod withdrawn")), info["reason"]
    assert ctx.status.exists(S.RCCL_READY)


def test_termination_message_keeps_summaries_and_failures_first():
    from gpu_operator_amd.validator.workload_main import termination_message
    res = [{"event": "gemm", "device": i, "tflops": 1500.0, "pad": "x" * 200, "ok": True} for i in range(30)]
    res += [{"event": "gemm", "device": 99, "tflops": 10.0, "ok": False},
            {"event": "aggregate", "gpus": 8, "total_tflops": 1.0, "ok": False},
            {"event": "rccl-debug", "algo_proto": {}, "lines": ["y" * 300] * 40}]
    msg = termination_message(res)
    lines = [json.loads(x) for x in msg.splitlines()]
    assert len(msg) <= 4000 and lines[0]["event"] == "aggregate" and "lines" not in lines[1]
    assert lines[2]["device"] == 99 and len(lines) < 33


def test_local_mode_rccl_sweep_matches_the_pod(tmp_path, node_root, monkeypatch):
    """local mode sweeps to 8 GiB with the binary's hang guard, like the pod."""
    from gpu_operator_amd.validator import workload_main as WM
    seen = {}

    def fake(max_bytes, dtype, **kw):
        seen.update(max_bytes=max_bytes, **kw)
        return [{"event": "summary", "ranks": 8, "peak_busbw_gbps": 300.0, "ok": True}]
    monkeypatch.setattr(WM, "run_rccl", fake)
    c = FakeClient([node_obj()])
    ctx = ctx_for(tmp_path, node_root, client=c, env={"HIP_VALIDATION_MODE": "local"})
    comp.validate_rccl(ctx)
    assert seen["max_bytes"] == 8 << 30 and seen["step_timeout"] == 120.0 and seen["ranks"] == "2,4,8"


# -- the xGMI link matrix ----------------------------------------------------------
def _matrix_msg(slow=None, n=8, base=100.0, slow_gbps=55.0, busbw=320.0):
    iso = [[0.0 if s == d else base for d in range(n)] for s in range(n)]
    conc = [[0.0 if s == d else base * 0.9 for d in range(n)] for s in range(n)]
    if slow:
        s, d = slow
        iso[s][d] = slow_gbps
        conc[s][d] = slow_gbps * 0.9
    ingress = [sum(conc[s][d] for s in range(n)) for d in range(n)]
    return "\n".join(json.dumps(x) for x in [
        {"event": "xgmi_matrix", "gpus": n, "isolated_gbps": iso, "concurrent_gbps": conc,
         "median_isolated_gbps": base, "gpu_ingress_gbps": ingress, "min_gpu_ingress_gbps": min(ingress),
         "slow_links": [f"{slow[0]}->{slow[1]}"] if slow else [], "corrupt_links": [], "no_peer_access": [],
         "ok": not slow},
        {"event": "ranks_summary", "ranks": 8, "peak_busbw_gbps": busbw, "ok": True},
        {"event": "summary", "ranks": 8, "ranks_run": [2, 4, 8], "peak_busbw_gbps": busbw, "ok": not slow}])


def test_one_slow_xgmi_link_is_named_and_opens_no_barrier(tmp_path, node_root):
    """A rank output whose link matrix has one slow pair (3 -> 5 at 0.55x the median): no rccl-ready,
    the pair in the error -- an 8-rank all-reduce at a healthy busBW would have hidden it."""
    c = FakeClient([node_obj()])
    k = FakeKubelet(c, {"amd-rccl-validator": _matrix_msg(slow=(3, 5))}, exit_code=1)
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(comp.ValidationError, match=r"3->5") as e:
        comp.validate_rccl(ctx)
    assert {f.kind for f in e.value.failures} == {"link"}
    assert not ctx.status.exists(S.RCCL_READY)
    env = _pod_env(k.seen[0])
    assert env["RCCL_MIN_LINK_RELATIVE"] == "0.8" and env["RCCL_MIN_BUSBW_MESH_FRACTION"] == "0.3"
    assert "RCCL_MIN_BUSBW_GBPS" not in env


def test_healthy_matrix_sets_the_mesh_aware_busbw_floor_and_exports_links(tmp_path, node_root):
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-rccl-validator": _matrix_msg()})
    ctx = ctx_for(tmp_path, node_root, client=c)
    info = comp.validate_rccl(ctx)
    # 7 peers x 90 GB/s concurrent ingress = 630 GB/s measured mesh bound; the floor is 0.3 of it
    assert info["busbw_floor"]["basis"] == "measured-mesh" and info["min_busbw_gbps"] == 189.0
    assert info["links"]["min_gpu_ingress_gbps"] == 630.0 and ctx.status.exists(S.RCCL_READY)
    m = NodeMetrics(ctx)
    m.refresh_status()
    from prometheus_client import generate_latest
    text = generate_latest(m.registry).decode()
    assert 'amd_gpu_operator_validator_xgmi_link_gbps{dst="5",mode="isolated",node="n1",src="3"} 100.0' in text
    assert len([x for x in text.splitlines() if x.startswith("amd_gpu_operator_validator_xgmi_link_gbps{")]) == 2 * 56
    # the same matrix with an all-reduce below 0.3 of the mesh bound: a busBW failure, named as such
    c2 = FakeClient([node_obj()])
    FakeKubelet(c2, {"amd-rccl-validator": _matrix_msg(busbw=150.0)})
    with pytest.raises(comp.ValidationError, match="busBW 150.0 GB/s below the 189.0 GB/s floor .measured-mesh"):
        comp.validate_rccl(ctx_for(tmp_path / "b", node_root, client=c2))


def test_link_gate_names_corrupt_and_unreachable_pairs():
    links = {"isolated_gbps": [[0, 10], [10, 0]], "concurrent_gbps": [[0, 9], [9, 0]],
             "corrupt_links": ["0->1"], "no_peer_access": ["1->0"]}
    got = [str(f) for f in comp.gate_links(links, 0.8)]
    assert got == ["xGMI link 0->1: copied data corrupted", "xGMI link 1->0: no peer access"]
    assert comp.gate_links({"skipped": "1 GPU visible", "ok": True}, 0.8) == []


def test_node_status_alerts_reference_metrics_the_exporter_serves(tmp_path, node_root):
    """Every metric an alert of the node-status PrometheusRule queries is one the node metrics exporter
    registers: a renamed gauge cannot leave an alert that never fires."""
    import re
    import yaml
    rule = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "gpu_operator_amd/assets/state-node-status-exporter/0800_prometheus_rule.yaml")))
    exprs = [r["expr"] for g in rule["spec"]["groups"] for r in g["rules"]]
    used = {m for e in exprs for m in re.findall(r"amd_gpu_operator_\w+", e)}
    ctx = ctx_for(tmp_path, node_root, client=FakeClient([node_obj()]))
    m = NodeMetrics(ctx)
    served = set(m.registry._names_to_collectors)
    assert used and used <= served, sorted(used - served)
    assert {"amd_gpu_operator_validator_gemm_bad_tile", "amd_gpu_operator_node_device_unhealthy"} <= used
