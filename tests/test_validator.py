"""Node validator components against fake sysfs + the fake API server."""

import json
import os
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
    """Completes validation pods with a canned termination message."""

    def __init__(self, client, messages, phase="Succeeded"):
        self.client, self.messages, self.phase = client, messages, phase
        self.seen = []
        self.stop = client.watch("v1", "Pod", self.on_event)

    def on_event(self, ev):
        if ev.type != "ADDED":
            return
        pod = ev.obj
        self.seen.append(pod)
        app = o.get_labels(pod).get("app")
        msg = self.messages.get(app, "")

        def finish():
            time.sleep(0.05)
            p = self.client.get("v1", "Pod", o.name(pod), o.namespace(pod))
            p["status"] = {"phase": self.phase, "initContainerStatuses": [
                {"name": "x", "state": {"terminated": {"exitCode": 0, "message": msg}}}]}
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


def test_hip_failed_pod_fails_validation(tmp_path, node_root):
    c = FakeClient([node_obj()])
    FakeKubelet(c, {"amd-hip-validator": '{"event":"gemm","ok":false}'}, phase="Failed")
    ctx = ctx_for(tmp_path, node_root, client=c)
    with pytest.raises(RuntimeError, match="failed"):
        comp.validate_hip(ctx)
    assert not ctx.status.exists(S.HIP_READY)


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


def test_rccl_single_gpu_node_skips(tmp_path, node_root):
    ctx = ctx_for(tmp_path, node_root, client=FakeClient([node_obj(gpus=1)]))
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
    sd.create(S.HIP_READY, {"ts": t + 9.0, "gemm_tflops_total": 10900.0, "gemm_tflops_per_gpu": 1362.5})
    sd.create(S.PLUGIN_READY, {"ts": t + 9.5})
    sd.create(S.RCCL_READY, {"ts": t + 14.0, "peak_busbw_gbps": 310.0, "ranks": 8})
    assert S.time_to_ready(sd) == pytest.approx(14.0)
    ctx = ctx_for(tmp_path, node_root, client=FakeClient([node_obj()]))
    ctx.status = sd
    m = NodeMetrics(ctx)
    m.refresh_all()
    from prometheus_client import generate_latest
    text = generate_latest(m.registry).decode()
    assert 'amd_gpu_operator_node_time_to_ready_seconds{node="n1"} 14.0' in text
    assert 'amd_gpu_operator_validator_gemm_tflops{node="n1",scope="node"} 10900.0' in text
    assert 'amd_gpu_operator_node_device_plugin_devices_total{node="n1"} 8.0' in text
    assert 'amd_gpu_operator_node_driver_validation{node="n1"} 1.0' in text
    assert 'amd_gpu_operator_amd_pci_devices_total{node="n1"} 8.0' in text
    assert 'amd_gpu_operator_validator_allreduce_busbw_gbps{node="n1",ranks="8"} 310.0' in text


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


def test_time_to_ready_chain_on_fake_node(tmp_path):
    """The node bring-up harness wires the real agents through barriers + fake kubelet."""
    from gpu_operator_amd.devices import fakesys
    from gpu_operator_amd.validator import ttr
    root = str(fakesys.make_node(tmp_path / "node", n_gpus=2))
    r = ttr.run_chain(workdir=str(tmp_path / "wd"), sys_root=root, dev_root=root, hip_mode="skip", timeout=30)
    assert r["errors"] == [] and r["time_to_ready_s"] is not None
    assert r["capacity"] == {"amd.com/gpu": "2"}
    order = list(r["marks_s"])
    assert order.index("driver") < order.index("toolkit_install") < order.index("device_plugin_start") \
        < order.index("plugin_validation") < order.index("ready")
    model = ttr.reference_model(r["steps_s"])
    # the reference's constants alone put it >= 2 poll periods behind
    assert model["time_to_ready_s"] > r["time_to_ready_s"] + 10


def test_time_to_ready_aborts_fast_on_driver_failure(tmp_path):
    import os
    import time
    from gpu_operator_amd.validator import ttr
    empty = tmp_path / "nodriver"
    os.makedirs(empty)
    t0 = time.monotonic()
    r = ttr.run_chain(workdir=str(tmp_path / "wd"), sys_root=str(empty), dev_root=str(empty), hip_mode="skip",
                      timeout=1.0)
    assert r["time_to_ready_s"] is None and r["errors"]
    assert time.monotonic() - t0 < 15


def test_reference_model_constants():
    from gpu_operator_amd.validator import ttr
    m = ttr.reference_model({"driver": 0.5, "toolkit_install": 0.5, "toolkit_validation": 0.1, "hip": 2.0,
                             "device_plugin_start": 0.2})
    # toolkit ready at 6 s; the first validation attempt (0.6 s) fails -> 10 s back-off
    assert m["toolkit_crashloops"] == 1 and m["toolkit_ready_s"] == 6.0
    assert m["time_to_ready_s"] >= 15.0
