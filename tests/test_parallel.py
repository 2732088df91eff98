"""Multi-process paths on CPU (gloo): the all-reduce probe and bench.py's distributed plumbing."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpu_operator_amd.parallel.allreduce import bus_factor, measure_allreduce
    res = []
    for nbytes in (4, 4096, 1 << 20):
        for dtype in (torch.float32, torch.bfloat16):
            r = measure_allreduce(nbytes, dtype=dtype, iters=3, warmup=1)
            res.append((nbytes, str(dtype), r.ok, r.ranks, r.algbw_gbps, r.busbw_gbps))
    out.put((rank, res, bus_factor(world)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_allreduce_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, res, bf in got:
        assert bf == pytest.approx(2 * (world - 1) / world)
        for nbytes, dtype, ok, ranks, algbw, busbw in res:
            assert ok and ranks == world, (rank, nbytes, dtype)
            assert busbw == pytest.approx(algbw * bf)


def test_bench_cpu_rehearsal_two_ranks():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--device", "cpu", "--shape", "64x64x128"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                                   # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["value"] == pytest.approx(d["per_gpu_tflops"] * 2, rel=1e-3, abs=0.02) and d["value"] > 0
    assert d["allreduce_ok"] and d["device"] == "cpu-rehearsal"
    assert d["config"]["parallelism"].startswith("dp2")
    # each rank's own loop next to the MAX-over-ranks headline: a slow rank is visible
    assert 0 < d["per_rank_tflops_min"] <= d["per_rank_tflops_max"] and d["slowest_rank"] in (0, 1)
    assert d["per_rank_tflops_min"] >= d["per_gpu_tflops"] * 0.999


def test_bench_self_launches_n_ranks_without_torchrun():
    """`bench.py --gpus 4` with no WORLD_SIZE must run 4 ranks itself (never a silent 1-rank run)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "2", "--warmup", "1",
           "--device", "cpu", "--shape", "64x64x128"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                                   # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 4 and d["config"]["parallelism"].startswith("dp4")
    assert "allreduce_busbw_gbps" in d and d["allreduce_ok"]
    assert d["metric"].startswith("validator HIP GEMM TFLOPS (bf16 64x64x128")


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--device", "cpu", "--shape", "64x64x64"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert p.returncode == 3 and "WORLD_SIZE" in p.stderr


def test_bench_refuses_more_gpus_than_visible():
    # This container has no GPU: an 8-GPU request must fail loudly instead of running on fewer.
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert p.returncode == 3 and "visible" in p.stderr


def test_bench_time_to_ready_fields_separate_measured_from_modelled(monkeypatch):
    """The bench line carries the time-to-ready split: the harness's simulated waits on the
    validator's path (modelled) and the rest (measured), for both protocols."""
    sys.path.insert(0, ROOT)
    import bench
    from gpu_operator_amd.validator import ttr
    run = {"protocol": "ours", "time_to_ready_s": 1.5, "time_to_ready_modelled_s": 0.9,
           "time_to_ready_measured_s": 0.6, "barriers_s": {}, "errors": []}
    ref = dict(run, protocol="reference", time_to_ready_s=16.5, time_to_ready_modelled_s=0.95,
               time_to_ready_measured_s=15.55)
    monkeypatch.setattr(ttr, "run_both", lambda **kw: {
        "agent_chain_time_to_ready_s": 1.5, "reference_protocol_time_to_ready_s": 16.5, "ours": run,
        "reference": ref, "agent_chain_time_to_ready_measured_s": 0.6, "agent_chain_time_to_ready_modelled_s": 0.9,
        "reference_protocol_time_to_ready_measured_s": 15.55, "reference_protocol_time_to_ready_modelled_s": 0.95})
    out = bench._time_to_ready_extra()
    assert out["time_to_ready_measured_s"] == 0.6 and out["time_to_ready_modelled_s"] == 0.9
    assert out["reference_protocol_time_to_ready_measured_s"] == 15.55
    assert out["reference_protocol_time_to_ready_modelled_s"] == 0.95


def test_bench_launcher_counts_gpus_from_sysfs_without_the_runtime(tmp_path, monkeypatch):
    """The N-rank launcher never initialises the GPU: it counts KFD agents (narrowed by the
    visibility variables); torch only when sysfs has no KFD topology."""
    sys.path.insert(0, ROOT)
    import bench
    from gpu_operator_amd import devices as D
    monkeypatch.setattr(D, "enumerate_gpus", lambda root="/": [{"index": i} for i in range(8)])
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    assert bench._visible_gpus() == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3,5")
    assert bench._visible_gpus() == 3
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: (_ for _ in ()).throw(AssertionError("runtime touched")))
    assert bench._visible_gpus() == 3
