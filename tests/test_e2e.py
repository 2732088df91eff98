"""The reference's end-to-end flow (tests/scripts/end-to-end.sh + checks.sh) executed on real
processes: in-process HTTP API server with this repo's CRDs, the operator as its own process,
the DaemonSet controller, and a kubelet that runs every pod on the node as OS processes
(gpu_operator_amd/e2e). CPU rehearsal: fake sysfs with 8 GPUs, no GPU work
(HIP_VALIDATION_MODE=skip); the MI355X run is tests/test_e2e_gpu.py.

Steps (reference script -> here): install-operator.sh, verify-operator.sh (check_pod_ready for
every operand), verify-operand-restarts.sh (check_no_restarts), install-workload.sh +
verify-workload.sh (a pod with an amd.com/gpu limit, allocated through the device plugin's
gRPC Allocate), update-clusterpolicy.sh (env and image version reach the DaemonSet and the
restarted pod), checks.sh test_restart_operator (recovery within 100 s, no operand churn),
disable-operands.sh / verify-disable-operands.sh, enable-operands.sh, uninstall-operator.sh.
"""

import os

import pytest

from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.e2e.harness import E2E
from gpu_operator_amd.utils import mounts

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BARRIER = os.path.join(ROOT, "gpu_operator_amd", "_native", "bin", "amd-barrier-wait")


@pytest.mark.skipif(not os.path.exists(BARRIER), reason="native binaries not built")
def test_reference_end_to_end_flow_on_real_processes(tmp_path):
    node = str(fakesys.make_node(tmp_path / "root", n_gpus=8))
    r = E2E(sys_root=node, dev_root=node, hip_mode="skip", timeout=90).run()
    assert r["ok"], r
    names = [s["name"] for s in r["steps"]]
    assert names == ["install-operator", "verify-operator", "verify-operand-restarts", "install+verify-workload",
                     "exporter-attribution", "update-clusterpolicy", "time-slicing", "restart-operator", "disable-operands", "enable-operands", "uninstall",
                     "install-operator[sandbox]", "verify-operator[sandbox]", "install+verify-workload[sandbox]",
                     "uninstall[sandbox]"]
    assert set(r["operands_ready"]) >= {"amd-container-toolkit-daemonset", "amd-device-plugin-daemonset",
                                        "amd-node-labeller", "amd-metrics-exporter", "amd-operator-validator"}
    st = {s["name"]: s for s in r["steps"]}
    v = st["verify-operator"]["detail"]
    assert {"host-driver-ready", "toolkit-ready", "hip-ready", "plugin-ready"} <= set(v["validations"])
    assert v["amd.com/gpu"] == "8"                   # device plugin -> kubelet ListAndWatch -> Node
    assert st["install+verify-workload"]["detail"]["phase"] == "Succeeded"
    assert "allocated:" in st["install+verify-workload"]["detail"]["log_tail"]
    ex = st["exporter-attribution"]["detail"]
    assert ex["series"] > 0 and ex["attributed_metrics"], ex
    ts = st["time-slicing"]["detail"]
    assert ts["advertised"] == 80 and ts["labels"]["amd.com/gpu.replicas"] == "10"
    assert ts["labels"]["amd.com/gpu.product"].endswith("-SHARED")
    assert r["operator_restart_recovery_s"] < 100
    assert st["disable-operands"]["detail"]["terminated_processes"] >= 6
    m = r["marks_s"]
    # the node-side order the operator's states and the barriers impose
    assert m["clusterpolicy:created"] <= m["amd-container-toolkit-daemonset-e2e-node:sandbox"] \
        < m["amd-operator-validator-e2e-node:sandbox"]
    assert r["time_to_ready_s"] < 30


def test_mount_table_rewrites_container_paths_once():
    pairs = sorted([("/run/amd", "/n/run/amd"), ("/run/amd/validations", "/v"), ("/host", "/h"),
                    ("/bin/entrypoint.sh", "/cm/entrypoint.sh")], key=lambda p: len(p[0]), reverse=True)
    assert mounts.translate("/run/amd/validations/x", pairs) == "/v/x"
    assert mounts.translate("/run/amd/driver", pairs) == "/n/run/amd/driver"
    assert mounts.translate("/run/amdx", pairs) == "/run/amdx"
    text = 'cd /run/amd/validations && exec /bin/entrypoint.sh --root=/host $ROOT/run/amd "/run/amd"'
    assert mounts.rewrite_text(text, pairs) == \
        'cd /v && exec /cm/entrypoint.sh --root=/h $ROOT/run/amd "/n/run/amd"'


@pytest.mark.skipif(not os.path.exists(BARRIER), reason="native binaries not built")
def test_three_node_cluster_on_real_processes():
    """One operator, three nodes (a process kubelet each, fake sysfs with 8 GPUs each): every
    operand DaemonSet fans out to all nodes, one GPU pod per node lands on its node, and
    deploy.operands=false on one node leaves the other nodes' operand pods untouched."""
    from gpu_operator_amd.e2e.harness import MultiNodeE2E
    r = MultiNodeE2E(nodes=3, gpus=8, timeout=90).run()
    assert r["ok"], r
    assert all(v == 3 for v in r["operands_ready"].values()), r["operands_ready"]
    st = {s["name"]: s for s in r["steps"]}
    assert sorted(st["workload-per-node"]["detail"].values()) == ["e2e-node-0", "e2e-node-1", "e2e-node-2"]
    d = st["disable-one-node"]["detail"]
    assert d["node"] == "e2e-node-0" and d["untouched"] == ["e2e-node-1", "e2e-node-2"]


@pytest.mark.skipif(not os.path.exists(BARRIER), reason="native binaries not built")
def test_driver_container_install_and_auto_upgrade_on_real_processes(tmp_path):
    """driver.enabled=true on a node without amdgpu (fake sysfs, the simulated kernel of
    devices/fakekernel.py on PATH): the driver DaemonSet's driver-manager and driver container
    install amdgpu, its startup probe releases the validator (container-driver mode), and a
    driver.version bump runs the upgrade controller's whole state machine -- the Job-managed GPU
    pod is evicted and gone before the driver pod restarts, the new container unloads and loads
    the new version, the node is uncordoned."""
    node = str(fakesys.make_node(tmp_path / "root", n_gpus=8, live=False, kfd=False))
    r = E2E(sys_root=node, dev_root=node, hip_mode="skip", timeout=90, driver="container").run()
    assert r["ok"], r
    st = {s["name"]: s for s in r["steps"]}
    assert "amdgpu-driver-daemonset" in r["operands_ready"]
    assert st["verify-operator"]["detail"]["driver-ready"]["mode"] == "container"
    up = st["driver-upgrade"]["detail"]
    assert (up["from"], up["to"]) == ("6.12.12", "6.12.13")
    assert up["states"][-7:] == ["cordon-required", "wait-for-jobs-required", "pod-deletion-required",
                                 "pod-restart-required", "validation-required", "uncordon-required", "upgrade-done"]


@pytest.mark.skipif(not os.path.exists(BARRIER), reason="native binaries not built")
def test_fabric_validation_on_time_slicing_and_busy_nodes(tmp_path):
    """Whole GPUs: the fabric pod asks for the 8 physical GPUs. Time-slicing x10 (allocatable 80):
    no replica request, every GPU visible, ranks 2,4,8. A GPU pod running during a validator
    restart: topology-only, validator Ready, no collective pod."""
    node = str(fakesys.make_node(tmp_path / "root", n_gpus=8))
    r = E2E(sys_root=node, dev_root=node, hip_mode="skip", timeout=90).run_fabric_shapes()
    assert r["ok"], r
    inst = r["install"]
    assert inst["rccl_pod"]["limits"] == {"amd.com/gpu": 8} and inst["rccl-ready"]["pod_shape"] == "scheduled"
    assert inst["rccl-ready"]["physical_gpus"] == 8 and inst["rccl-ready"]["fabric"]["ok"]
    ts = r["time-slicing"]
    assert ts["allocatable"] == 80
    assert ts["rccl-ready"]["pod_shape"] == "privileged-all" and ts["rccl-ready"]["physical_gpus"] == 8
    assert ts["rccl_pod"]["limits"] is None and ts["rccl_pod"]["privileged"]
    assert ts["rccl_pod"]["env"]["RCCL_RANKS"] == "2,4,8" and ts["rccl_pod"]["env"]["AMD_VISIBLE_DEVICES"] == "all"
    busy = r["busy"]["rccl-ready"]
    assert busy["mode"] == "topology-only" and busy["busy_pods"] == ["default/gpu-busy"] and busy["fabric"]["ok"]


@pytest.mark.skipif(not os.path.exists(BARRIER), reason="native binaries not built")
def test_fabric_validation_on_a_cpx_node(tmp_path):
    """CPX: 64 KFD agents, allocatable amd.com/gpu=64; the fabric pod pins one agent per physical
    GPU (HIP_VISIBLE_DEVICES, 8 entries) and plans ranks 2,4,8."""
    node = str(fakesys.make_node(tmp_path / "root", n_gpus=8, compute="CPX"))
    e = E2E(sys_root=node, dev_root=node, hip_mode="skip", timeout=90)
    e.setup()
    # the node's layout is CPX on purpose: the partition manager keeps it (no re-partition to SPX)
    e.backing.patch("v1", "Node", e.node, {"metadata": {"labels": {"amd.com/gpu.partition.config": "cpx-nps1"}}})
    try:
        e.step("install-operator", e.install_operator)
        v = e.step("verify-operator", lambda: e.verify_operator("install"))
        shape = e._rccl_pod_shape()
    finally:
        e.teardown()
    assert v["amd.com/gpu"] == "64"
    rr = v["rccl-ready"]
    assert rr["physical_gpus"] == 8 and rr["pod_shape"] == "privileged-all"
    vis = shape["env"]["HIP_VISIBLE_DEVICES"].split(",")
    assert len(vis) == 8 and vis[:2] == ["0", "8"] and shape["env"]["RCCL_RANKS"] == "2,4,8"


@pytest.mark.skipif(not os.path.exists(BARRIER), reason="native binaries not built")
def test_validator_beside_tenants_on_real_processes(tmp_path):
    """VERDICT r3 item 1 on real processes (8 fake GPUs, GEMM and collective dry-run): (i) a tenant
    holds 2 GPUs -- the HIP pod's full sweep lists the 6 free ones (from the kubelet's pod-resources),
    the held 2 get the probe; (ii) tenants hold all 8 -- only the probe; (iii) a tenant lands between
    the fabric busy check and the fabric pod -- topology-only within seconds; (iv) a tenant given a GPU
    during the HIP sweep -- that GPU disturbed, no floor failure. Ready in each."""
    node = str(fakesys.make_node(tmp_path / "root", n_gpus=8))
    r = E2E(sys_root=node, dev_root=node, hip_mode="skip", timeout=90).run_tenant_cases()
    assert r["ok"], r
    assert r["idle"]["hip-ready"]["plan"]["full"] == "all" and r["idle"]["rccl-ready"]["mode"] == "full"
    two = r["two-held"]
    full = two["hip_pod_env"]["GEMM_DEVICES"].split(",")
    probe = two["hip_pod_env"]["GEMM_PROBE_DEVICES"].split(",")
    assert len(full) == 6 and len(probe) == 2 and not set(full) & set(probe)
    assert two["hip-ready"]["plan"]["attribution"] == "pod-resources"
    assert two["rccl-ready"]["mode"] == "topology-only"
    held = r["all-held"]
    assert held["hip_pod_env"]["GEMM_DEVICES"] == "none"
    assert held["hip_pod_env"]["GEMM_PROBE_DEVICES"] == "0,1,2,3,4,5,6,7"
    race = r["race"]
    assert race["tenant_started_after_busy_check"] and race["rccl-ready"]["mode"] == "topology-only"
    assert race["rccl-ready"]["busy_pods"] == ["default/tenant-race"] and race["ready_s"] < 30
    # (iv) a tenant given a GPU while the HIP sweep runs (real HIP pod, scripted GEMM): that GPU is
    # disturbed, its slow number out of the gates -- hip-ready, no floor failure, no re-measure
    sweep = r["during-sweep"]
    hip = sweep["hip-ready"]
    assert len(sweep["tenant_gpus"]) == 1 and hip["disturbed"]["devices"] == sweep["tenant_gpus"]
    assert hip["disturbed"]["pods"] == ["default/tenant-sweep"] and hip["disturbed"]["attribution"] == "pod-resources"
    assert "remeasured" not in hip and hip["pod_failed"]["exit_code"] == 1
