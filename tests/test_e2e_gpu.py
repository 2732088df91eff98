"""The reference's end-to-end flow on an MI355X box (tests/test_e2e.py is the CPU rehearsal):
the operator process reconciles a ClusterPolicy on the in-process API server; the node's pods
run as processes against the real GPU. The validator's HIP check runs in pod mode (it creates
the HIP workload pod, which the kubelet runs: the MFMA GEMM probe on the GPU), and the test
workload pod runs ``amd-hip-smoke`` on an ``amd.com/gpu`` the device plugin allocated.
"""

import os

import pytest

from gpu_operator_amd.e2e.harness import E2E

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
def test_reference_end_to_end_flow_on_mi355x():
    r = E2E(sys_root="/", dev_root="/", hip_mode="pod", timeout=150).run()
    assert r["ok"], {k: v for k, v in r.items() if k != "marks_s"}
    st = {s["name"]: s for s in r["steps"]}
    v = st["verify-operator"]["detail"]
    assert int(v["amd.com/gpu"]) >= 1
    assert v["gpu_labels"].get("amd.com/gpu.gfx") == "gfx950" or \
        any(x.endswith("gfx950") for x in v["gpu_labels"].values()), v["gpu_labels"]
    hip = v["hip-ready"]
    # the validator's HIP workload pod ran the MFMA GEMM on this GPU and passed its fp32 check
    assert hip["gemm"] and all(g.get("ok") for g in hip["gemm"]), hip
    assert hip["gemm_tflops_per_gpu"] > 500, hip
    w = st["install+verify-workload"]["detail"]
    assert w["phase"] == "Succeeded", w
    assert r["operator_restart_recovery_s"] < 100
