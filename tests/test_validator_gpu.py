"""The validator's native workload binaries on a real MI355X."""

import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu_operator_amd", "_native", "bin")


def run(*args, timeout=600):
    p = subprocess.run([os.path.join(BIN, args[0]), *args[1:]], capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def test_hip_smoke_binary():
    rc, lines, err = run("amd-hip-smoke")
    assert rc == 0, err
    assert lines[-1]["ok"] and lines[-1]["devices"] >= 1


def test_gemm_validate_binary_checks_and_reports_tflops():
    rc, lines, err = run("amd-gemm-validate", "--shapes", "4096,8192", "--iters", "10")
    assert rc == 0, err
    start = lines[0]
    assert start["gcn_arch"].startswith("gfx950") and start["cus"] == 256
    gemms = [x for x in lines if x["event"] == "gemm"]
    assert gemms and all(g["ok"] for g in gemms)
    agg = [x for x in lines if x["event"] == "aggregate" and x["m"] == 8192][0]
    assert agg["per_gpu_tflops"] > 900           # MI355X bf16 dense, random operands


def test_gemm_validate_binary_fp8_and_both():
    rc, lines, err = run("amd-gemm-validate", "--shapes", "8192", "--dtype", "both", "--iters", "10")
    assert rc == 0, err
    gemms = [x for x in lines if x["event"] == "gemm"]
    assert {g["dtype"] for g in gemms} == {"bf16", "fp8_e4m3fn"} and all(g["ok"] for g in gemms)
    agg = {x["dtype"]: x["per_gpu_tflops"] for x in lines if x["event"] == "aggregate"}
    assert agg["fp8_e4m3fn"] > 1.5 * agg["bf16"]   # the f8f6f4 MFMAs run at 2x the bf16 rate
    rc, lines, err = run("amd-gemm-validate", "--dtype", "fp4")
    assert rc == 2 and "unknown --dtype" in lines[0]["error"]


def test_rccl_validate_binary():
    rc, lines, err = run("amd-rccl-validate", "--max-bytes", str(1 << 26), "--iters", "5", "--warmup", "2")
    assert rc == 0, err
    ev = {x.get("event"): x for x in lines}
    assert ev["fabric"]["ok"] and ev["fabric"]["single_hive"]
    assert ev["topology"]["gpus"][0]["xgmi_links"] == 7          # a GPU of the box's 8-GPU hive
    summ = lines[-1]
    assert summ["event"] == "summary" and summ["ok"]
    assert all(x["ok"] for x in lines if x.get("event") == "allreduce")


def test_rccl_rank_sweep_on_one_gpu_is_a_clean_skip():
    rc, lines, err = run("amd-rccl-validate", "--ranks", "2,4,8", "--max-bytes", str(1 << 20), "--iters", "2")
    assert rc == 0, err
    skipped = [x["ranks"] for x in lines if x.get("event") == "skipped"]
    assert skipped == [2, 4, 8]
    assert lines[-1]["event"] == "summary" and lines[-1]["ok"] and lines[-1]["skipped"]


def test_rccl_multi_process_mode_and_debug_capture():
    from gpu_operator_amd.validator.workload_main import run_rccl
    res = run_rccl(1 << 22, "bf16", processes=1, min_bytes=1 << 20, timeout=300)
    summ = [x for x in res if x.get("event") == "summary"]
    assert summ and all(x["ok"] for x in summ), res
    start = [x for x in res if x.get("event") == "start"][0]
    assert start["mode"] == "multi-process" and start["ranks"] == 1
    assert all(x["ok"] for x in res if x.get("event") == "allreduce")
    dbg = [x for x in res if x.get("event") == "rccl-debug"][0]
    assert isinstance(dbg["algo_proto"], dict) and dbg["lines"]          # RCCL's INFO log was captured


def test_node_probe_on_real_hardware():
    rc, lines, err = run("amd-node-probe")
    assert rc == 0, err
    j = lines[0]
    assert j["driver"]["live"] and j["driver"]["kfd"]
    assert any(g["gfx"] == "gfx950" for g in j["gpus"])


def test_validator_workload_hip_with_counters(tmp_path):
    from gpu_operator_amd.validator import workload_main as W
    results = W.run_hip(["4096"], counters=True, iters=5)
    assert any(r.get("event") == "gemm" and r["ok"] for r in results)
    ctr = [r for r in results if r.get("event") == "counters"]
    assert ctr
    if "skipped" not in ctr[0]:
        assert ctr[0]["SQ_INSTS_VALU_MFMA_MOPS_BF16"] > 0


def test_validator_hip_component_local_mode(tmp_path):
    from gpu_operator_amd.validator import components as comp
    from gpu_operator_amd.validator import status as S
    ctx = comp.Context(status=S.StatusDir(str(tmp_path / "v")), env={"HIP_VALIDATION_MODE": "local",
                                                                      "GEMM_SHAPES": "4096"})
    info = comp.validate_hip(ctx)
    assert info["gemm_tflops_per_gpu"] > 500 and ctx.status.exists(S.HIP_READY)


def test_node_time_to_ready_both_protocols_on_the_gpu():
    """Real processes, real GPU validation: our chain must reach Ready and beat the reference's
    protocol constants executed in the same harness."""
    from gpu_operator_amd.validator import ttr
    r = ttr.run_both(hip_mode="local", gemm_shapes="4096", timeout=120)
    ours, ref = r["ours"], r["reference"]
    assert ours["errors"] == [] and ref["errors"] == [], (ours["errors"], ref["errors"])
    assert ours["gemm_tflops_per_gpu"] and ours["gemm_tflops_per_gpu"] > 300
    assert r["agent_chain_time_to_ready_s"] < r["reference_protocol_time_to_ready_s"]
    assert ours["marks_s"]["kubelet:capacity:amd.com/gpu=1"] < ours["barriers_s"]["plugin-ready"]
