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
    # clock stabilisation ran before the timed dispatches (>= 50 dispatches, or the time cap)
    assert all(g["stabilise_dispatches"] >= 50 for g in gemms)
    agg = [x for x in lines if x["event"] == "aggregate" and x["m"] == 8192][0]
    assert agg["per_gpu_tflops"] > 1200           # MI355X bf16, random operands, steady clock
    assert lines[-1] == {"event": "done", "ok": True}     # where the validator stops reading


def test_gemm_validate_scaling_sweep_on_one_gpu():
    """--scaling 1,2,4,8 on a 1-GPU box: gpus=1 measured (efficiency 1), 2/4/8 clean skips, exit 0."""
    rc, lines, err = run("amd-gemm-validate", "--shapes", "8192", "--iters", "20", "--scaling", "1,2,4,8")
    assert rc == 0, err
    aggs = [x for x in lines if x["event"] == "aggregate"]
    assert [a["gpus"] for a in aggs] == [1] and aggs[0]["efficiency"] == 1.0 and aggs[0]["ok"]
    skipped = [x["gpus"] for x in lines if x["event"] == "scaling" and x.get("skipped")]
    assert skipped == [2, 4, 8]


def test_gemm_validate_gates_on_the_floor():
    rc, lines, err = run("amd-gemm-validate", "--shapes", "4096", "--iters", "5", "--min-tflops", "1000000")
    assert rc == 1
    g = [x for x in lines if x["event"] == "gemm"][0]
    assert not g["ok"] and "below floor" in g["error"]


def test_pod_path_tflops_match_the_bench_protocol():
    """The validator pod's number (amd-gemm-validate, what feeds validator_gemm_tflops and the
    floors) is within 3 % of bench.py's protocol on the same box, for bf16 and fp8."""
    import sys
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from gpu_operator_amd.ops import gemm as G
    args = bench.parse_args(["--steps", "50", "--warmup", "5", "--stabilise-max-s", "6"])
    dev = torch.device("cuda", 0)
    ctx = bench.Ctx(args, torch, None, dev, 0, 0, 1, False, False)
    m = n = k = 8192
    a = G.fill_uniform_(torch.empty((m, k), dtype=torch.bfloat16, device=dev), 1000)
    bt = G.fill_uniform_(torch.empty((n, k), dtype=torch.bfloat16, device=dev), 2000)
    c = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    bf16 = G.tflops(m, n, k, ctx.timed(lambda: G.gemm_bf16(a, bt, c), 50, 5)["elapsed_s"] / 50)
    f8 = torch.float8_e4m3fn
    a8 = G.fill_uniform_fp8_(torch.empty((m, k), dtype=f8, device=dev), 3000)
    b8 = G.fill_uniform_fp8_(torch.empty((n, k), dtype=f8, device=dev), 4000)
    fp8 = G.tflops(m, n, k, ctx.timed(lambda: G.gemm_fp8(a8, b8, c), 50, 5)["elapsed_s"] / 50)
    del a, bt, c, a8, b8
    torch.cuda.synchronize()
    rc, lines, err = run("amd-gemm-validate", "--shapes", "8192", "--dtype", "both", "--iters", "50")
    assert rc == 0, err
    pod = {x["dtype"]: x["per_gpu_tflops"] for x in lines if x["event"] == "aggregate"}
    print(f"bench protocol bf16 {bf16:.1f} fp8 {fp8:.1f}; pod path {pod}")
    assert pod["bf16"] >= 0.97 * bf16, (pod, bf16)
    assert pod["fp8_e4m3fn"] >= 0.97 * fp8, (pod, fp8)


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


def test_counters_follow_the_dispatched_kernel_for_every_shape_and_dtype():
    """GEMM_SHAPES=1024,8192 with --counters -> an ok counters line per shape and
    dtype, MFMA ops matching 2MNK/512 -- 1024^3 runs gemm_mfma_small (v60), 8192^3 the asm pipeline --
    and only the timed dispatch is counted (the checked dispatch's recording kernel is not)."""
    from gpu_operator_amd.validator import workload_main as W
    if W.rocprofv3_path() is None:
        pytest.skip("rocprofv3 not installed")
    results = W.run_hip(["1024", "8192"], counters=True, iters=5, dtype="both")
    ctr = {(r["dtype"], r["shape"]): r for r in results if r.get("event") == "counters"}
    assert set(ctr) == {(d, s) for d in ("bf16", "fp8") for s in ("1024", "8192")}, list(ctr)
    for key, c in ctr.items():
        print(key, c.get("kernel"), c.get("mfma_mops"), c.get("mfma_mops_expected"))
        assert c["ok"] and c["mfma_mops_match"], (key, c)
    assert "gemm_mfma_small" in ctr[("bf16", "1024")]["kernel"] and "gemm_mfma_small" in ctr[("fp8", "1024")]["kernel"]
    assert ctr[("bf16", "8192")]["kernel"] == "gemm_bf16_256x256_w4ap"


def test_validator_workload_hip_with_counters(tmp_path):
    """Counters for both kernels when the pod runs --gemm-dtype both; rocprofv3 ships in this image,
    so a skipped or failed collection fails the test (it cannot pass vacuously)."""
    from gpu_operator_amd.validator import workload_main as W
    results = W.run_hip(["4096"], counters=True, iters=5, dtype="both")
    assert any(r.get("event") == "gemm" and r["ok"] for r in results)
    ctr = {r["dtype"]: r for r in results if r.get("event") == "counters"}
    assert set(ctr) == {"bf16", "fp8"}, ctr
    if W.rocprofv3_path() is None:
        pytest.skip("rocprofv3 not installed")
    for dtype, c in ctr.items():
        assert "skipped" not in c and "error" not in c, c
        assert c["mfma_mops_expected"] == 2 * 4096 ** 3 / 512
        assert c["mfma_mops_match"], (dtype, c)              # MOPS = 2·M·N·K / 512
        assert c["SQ_LDS_BANK_CONFLICT"] == 0, (dtype, c)


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


def test_gemm_validate_reports_out_of_memory_structurally():
    """393216^3: A alone is 309 GB, more than the 288 GB of HBM. The probe checks free HBM before
    allocating and reports a structured out-of-memory line (no kernel launched), exit 1."""
    rc, lines, err = run("amd-gemm-validate", "--shapes", "393216", "--iters", "1", "--warmup", "0", "--no-stabilise",
                         timeout=120)
    assert rc == 1, err
    g = [x for x in lines if x.get("event") == "gemm"][0]
    assert g["oom"] and not g["ok"] and g["error"].startswith("out of memory")
    assert g["need_bytes"] > g["free_bytes"] > 0 and g["need_bytes"] >= 2 * 393216 ** 2 * 2


def test_busy_gpu_oom_probe_is_a_skip_in_validate_hip(tmp_path, monkeypatch):
    """validate_hip, local mode, the box's GPU held by a tenant pod (pod-resources mapping faked):
    the GPU gets only the probe; its allocation failure (shape forced past HBM) is a busy skip and
    hip-ready opens."""
    from gpu_operator_amd import devices as D
    from gpu_operator_amd.k8s.fake import FakeClient
    from gpu_operator_amd.validator import components as comp
    from gpu_operator_amd.validator import status as S
    from gpu_operator_amd.validator import workload_main as WM
    g0 = sorted(D.enumerate_gpus("/"), key=lambda g: g["index"])[0]
    tenant = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "train-0", "namespace": "default"},
              "spec": {"nodeName": "n1", "containers": [{"name": "t", "resources": {"limits": {"amd.com/gpu": "1"}}}]},
              "status": {"phase": "Running"}}
    did = f"amdgpu-{g0['unique_id']:016x}"
    monkeypatch.setattr(comp, "_pod_device_ids", lambda ctx: {"default/train-0": [did]})
    monkeypatch.setattr(WM, "PROBE_SHAPE", "393216")
    ctx = comp.Context(status=S.StatusDir(str(tmp_path / "v")), node_name="n1", client=FakeClient([tenant]),
                       env={"HIP_VALIDATION_MODE": "local", "GEMM_SHAPES": "4096"})
    info = comp.validate_hip(ctx)
    assert info["plan"]["probe"] == [g0["index"]] and g0["index"] not in info["plan"]["full"]
    probe = [p for p in info["probe"] if p["device"] == g0["index"]][0]
    assert probe["skipped"].startswith("busy: out of memory") and ctx.status.exists(S.HIP_READY)


def test_rccl_watchdog_reports_a_missing_peer(tmp_path):
    """Rank 0 of a 2-rank multi-process run whose peer never starts: ncclCommInitRank blocks in the
    bootstrap; the watchdog prints a structured init timeout, aborts and exits 124."""
    rc, lines, err = run("amd-rccl-validate", "--mp-rank", "0", "--mp-nranks", "2", "--mp-id-file",
                         str(tmp_path / "id"), "--device", "0", "--timeout-s", "5", timeout=90)
    assert rc == 124, (rc, lines, err[-2000:])
    t = [x for x in lines if x.get("event") == "timeout"][0]
    assert t["phase"] == "init" and t["ranks"] == 2 and t["rank"] == 0 and t["timeout_s"] == 5.0


def test_gemm_validate_runs_hip_smoke_in_process():
    rc, lines, err = run("amd-gemm-validate", "--smoke", "--shapes", "4096", "--iters", "5", "--no-stabilise")
    assert rc == 0, err
    sm = [x for x in lines if x.get("event") == "hip-smoke"]
    assert len(sm) == 1 and sm[0]["ok"] and sm[0]["devices"] >= 1 and sm[0]["elements"] == 50000


def _tflops(*extra):
    rc, lines, err = run("amd-gemm-validate", "--shapes", "8192", "--iters", "50", *extra)
    assert rc == 0, err
    g = [x for x in lines if x["event"] == "gemm"][0]
    return g, lines


def test_idle_before_the_timed_loop_does_not_droop_the_number():
    """A GPU that waits at the rendezvous (here: 200 ms of host idle injected after it) re-ramps before
    the timed loop, and the window is >= 100 ms: the reported TF/s stays within 2 % of the run
    without the idle."""
    base, lines = _tflops()
    idle, _ = _tflops("--pre-timed-idle-ms", "200")
    print(f"no idle {base['tflops']} TF/s, 200 ms idle {idle['tflops']} TF/s; ramp {idle['ramp_dispatches']}, "
          f"iters {idle['iters']}")
    assert base["iters"] * base["ms"] >= 99.0
    # a 1-GPU set waits for nobody at its rendezvous: no re-ramp; the injected idle gets one
    assert base["ramp_dispatches"] == 0 and idle["ramp_dispatches"] >= 10
    assert abs(idle["tflops"] - base["tflops"]) <= 0.02 * base["tflops"], (base, idle)


def test_bench_reramps_after_the_barrier():
    """bench.py's timed region after a 200 ms idle at the pre-timing barrier: within 2 % of the run
    without it (the re-ramp runs between the barrier and the timed loop)."""
    import sys
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from gpu_operator_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    m = 8192
    a = G.fill_uniform_(torch.empty((m, m), dtype=torch.bfloat16, device=dev), 1000)
    bt = G.fill_uniform_(torch.empty((m, m), dtype=torch.bfloat16, device=dev), 2000)
    c = torch.empty((m, m), dtype=torch.bfloat16, device=dev)
    out = {}
    for idle in (0.0, 200.0):
        args = bench.parse_args(["--steps", "20", "--warmup", "5", "--pre-timed-idle-ms", str(idle)])
        ctx = bench.Ctx(args, torch, None, dev, 0, 0, 1, False, False)
        res = ctx.timed(lambda: G.gemm_bf16(a, bt, c), 20, 5)
        out[idle] = G.tflops(m, m, m, res["elapsed_s"] / 20)
        assert res["ramp_dispatches"] >= 10
    print(f"bench 20 steps: no idle {out[0.0]:.1f}, 200 ms idle {out[200.0]:.1f} TF/s")
    assert abs(out[200.0] - out[0.0]) <= 0.02 * out[0.0], out


def test_gemm_validate_runs_one_worker_process_per_gpu():
    """The default launch: a launcher that never opens the GPU and one worker per GPU meeting at a
    pipe rendezvous. Two workers on the box's one GPU (--devices 0,0) exercise the rendezvous; their
    2-GPU set shares a physical GPU, so it is measured and marked, not gated on efficiency."""
    rc, lines, err = run("amd-gemm-validate", "--shapes", "2048", "--iters", "5", "--devices", "0,0",
                         "--scaling", "1,2", "--min-efficiency", "0.9", "--smoke")
    assert rc == 0, (lines, err)
    start = lines[0]
    assert start["launch"] == "processes" and start["devices"] == 2 and start["gcn_arch"].startswith("gfx950")
    assert [x for x in lines if x["event"] == "hip-smoke"][0] == {"event": "hip-smoke", "devices": 2,
                                                                  "elements": 50000, "ok": True}
    aggs = {a["gpus"]: a for a in lines if a["event"] == "aggregate"}
    assert aggs[1]["ok"] and aggs[2]["ok"] and aggs[2]["shared_gpu"] and aggs[2]["efficiency_gated"] is False
    gemms = [x for x in lines if x["event"] == "gemm" and x.get("gpus") == 2]
    assert len(gemms) == 2 and all(g["ok"] for g in gemms)
    assert lines[-1] == {"event": "done", "ok": True}
    rc, lines, err = run("amd-gemm-validate", "--shapes", "2048", "--iters", "5", "--launch", "threads")
    assert rc == 0 and lines[0]["launch"] == "threads", err


def test_xgmi_link_matrix_on_one_gpu_is_a_clean_skip_and_its_kernels_run():
    """The link matrix needs 2+ GPUs: on the 1-GPU box it is a clean skip. --link-self-test runs the
    peer-read copy, the pattern check and the matrix line on GPU 0 -> GPU 0 (its HBM), so the kernels
    the 8-GPU node uses are exercised here."""
    rc, lines, err = run("amd-rccl-validate", "--links-only", timeout=120)
    assert rc == 0, err
    mx = [x for x in lines if x.get("event") == "xgmi_matrix"][0]
    assert mx["skipped"] and mx["ok"] and lines[-1]["event"] == "summary" and lines[-1]["skipped"]
    rc, lines, err = run("amd-rccl-validate", "--links-only", "--link-self-test", "--link-bytes", str(256 << 20),
                         timeout=120)
    assert rc == 0, (lines, err)
    mx = [x for x in lines if x.get("event") == "xgmi_matrix"][0]
    print(f"GPU0 -> GPU0 copy: isolated {mx['isolated_gbps']} GB/s, concurrent {mx['concurrent_gbps']} GB/s")
    assert mx["self_test"] and mx["ok"] and mx["corrupt_links"] == [] and mx["gpus"] == 1
    assert mx["isolated_gbps"][0][0] > 1000          # an HBM3E copy kernel: TB/s, not PCIe


def test_link_matrix_names_the_throttled_virtual_peer_only():
    """VERDICT r5 item 2 on one GPU: 7 source buffers on GPU 0 pulled by ONE kernel (the concurrent
    phase's shape: one kernel, one stream per destination), source 3 given an eighth of the blocks.
    The throttled peer, and only it, is named; the unthrottled concurrent rates agree within 10 %."""
    rc, lines, err = run("amd-rccl-validate", "--links-only", "--virtual-peers", "7", "--link-bytes", str(128 << 20),
                         timeout=180)
    assert rc == 0, (lines, err)
    mx = [x for x in lines if x.get("event") == "xgmi_matrix"][0]
    conc = [row[0] for row in mx["concurrent_gbps"]]
    print(f"7 virtual peers, concurrent GB/s per source: {conc}; isolated: {[r[0] for r in mx['isolated_gbps']]}")
    assert mx["ok"] and mx["slow_links"] == [] and mx["streams_per_device"] == 1
    assert max(conc) / min(conc) < 1.10, conc
    rc, lines, err = run("amd-rccl-validate", "--links-only", "--virtual-peers", "7", "--throttle-peer", "3",
                         "--link-bytes", str(128 << 20), timeout=180)
    assert rc == 1, (lines, err)
    mx = [x for x in lines if x.get("event") == "xgmi_matrix"][0]
    conc = [row[0] for row in mx["concurrent_gbps"]]
    print(f"throttled v3: concurrent GB/s per source: {conc}")
    assert mx["slow_links"] == ["v3->0"] and mx["kind"] == "link", mx
    others = [c for i, c in enumerate(conc) if i != 3]
    assert max(others) / min(others) < 1.10, others
    assert [x["src"] for x in lines if x.get("event") == "xgmi_link"] == ["v3"]
