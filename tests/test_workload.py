"""The validation pods' workload driver (validator/workload_main.py) against fake binaries: the
tenant-safe HIP plan (full sweep on free GPUs with HIP_VISIBLE_DEVICES, a correctness probe on held
ones) and the RCCL hang guards (the launcher's structured timeout for a rank that never reports)."""

import json
import os
import stat
import subprocess
import sys
import time

import pytest

from gpu_operator_amd.validator import workload_main as WM


class FakeRun:
    """subprocess.run stand-in: records (cmd, HIP_VISIBLE_DEVICES) and answers per binary."""

    def __init__(self, answers):
        self.answers, self.calls = answers, []

    def __call__(self, cmd, capture_output=True, text=True, timeout=None, env=None):
        vis = (env or {}).get("HIP_VISIBLE_DEVICES")
        self.calls.append((os.path.basename(cmd[0]), cmd[1:], vis))
        out = self.answers[os.path.basename(cmd[0])](cmd, vis)
        return subprocess.CompletedProcess(cmd, 0 if all(x.get("ok", True) for x in out) else 1,
                                           "\n".join(json.dumps(x) for x in out), "")


def _gemm_lines(cmd, vis):
    n = len(vis.split(",")) if vis else 8
    shape = int(cmd[cmd.index("--shapes") + 1])
    out = [{"event": "hip-smoke", "devices": n, "ok": True}] if "--smoke" in cmd else []
    for d in range(n):
        r = {"event": "gemm", "dtype": "bf16", "device": d, "m": shape, "n": shape, "k": shape, "tflops": 1600.0,
             "ok": True}
        if shape == 1024 and d == 1:          # the second held GPU: its tenant took the HBM
            r.update(ok=False, oom=True, tflops=0.0, error="out of memory: the shape needs 0.01 GiB")
        out.append(r)
    if shape != 1024:
        out.append({"event": "uniformity", "dtype": "bf16", "m": shape, "n": shape, "k": shape, "gpus": n,
                    "slow_devices": [0], "ok": True})
    return out


@pytest.fixture
def fake_bins(monkeypatch):
    monkeypatch.setattr(WM, "binary", lambda name: "/fake/" + name)
    return FakeRun({"amd-hip-smoke": lambda cmd, vis: [{"event": "hip-smoke", "ok": True}],
                    "amd-gemm-validate": _gemm_lines})


def test_full_sweep_on_free_gpus_probe_on_held_ones(fake_bins):
    res = WM.run_hip(["8192"], run=fake_bins, devices=[0, 1, 3, 4, 6, 7], probe_devices=[2, 5],
                     scaling="1,2,4,8", min_relative=0.85, min_efficiency=0.9)
    calls = {(c[0], c[2]): c[1] for c in fake_bins.calls}
    full = calls[("amd-gemm-validate", "0,1,3,4,6,7")]
    assert full[full.index("--min-relative") + 1] == "0.85" and full[full.index("--min-efficiency") + 1] == "0.9"
    probe = calls[("amd-gemm-validate", "2,5")]
    assert probe[probe.index("--shapes") + 1] == "1024" and "--no-stabilise" in probe and "--scaling" not in probe
    assert "--smoke" in full and "--smoke" not in probe          # hip-smoke inside the full run's process
    assert [c[0] for c in fake_bins.calls] == ["amd-gemm-validate", "amd-gemm-validate"]
    assert [r for r in res if r.get("event") == "hip-smoke"][0]["ok"]
    full_devs = sorted(r["device"] for r in res if r.get("event") == "gemm" and not r.get("probe"))
    assert full_devs == [0, 1, 3, 4, 6, 7]                      # mapped back from the child's 0..5
    assert next(r for r in res if r.get("event") == "uniformity")["slow_devices"] == [0]
    probed = {r["device"]: r for r in res if r.get("probe")}
    assert sorted(probed) == [2, 5] and probed[5]["oom"] and probed[5]["visible_index"] == 1
    assert WM.hip_ok(res)                                        # an OOM on a held GPU is no failure
    res.append({"event": "gemm", "probe": True, "device": 2, "ok": False, "error": "max_rel_err 0.3"})
    assert not WM.hip_ok(res)


def test_every_gpu_held_runs_the_probe_only(fake_bins):
    res = WM.run_hip(["8192"], run=fake_bins, devices=[], probe_devices=[0, 1], counters=True)
    assert [c[0] for c in fake_bins.calls] == ["amd-gemm-validate"]   # no counters, no full run
    assert "--smoke" in fake_bins.calls[0][1] and fake_bins.calls[0][2] == "0,1"
    assert all(r.get("probe") for r in res if r.get("event") == "gemm")
    assert WM.hip_ok(res) and res[0] == {"event": "plan", "devices": [], "probe_devices": [0, 1]}


def test_cli_reads_the_plan_from_env(monkeypatch):
    seen = {}
    monkeypatch.setattr(WM, "run_hip", lambda shapes, **kw: seen.update(kw) or [{"event": "hip-smoke", "ok": True}])
    monkeypatch.setattr(WM, "emit", lambda r: None)
    monkeypatch.setenv("GEMM_DEVICES", "none")
    monkeypatch.setenv("GEMM_PROBE_DEVICES", "0,3")
    monkeypatch.setenv("GEMM_MIN_RELATIVE", "0.85")
    assert WM.main(["hip"]) == 0
    assert seen["devices"] == [] and seen["probe_devices"] == [0, 3] and seen["min_relative"] == 0.85


HANG = """#!/usr/bin/env python3
import sys, time
args = sys.argv[1:]
rank = int(args[args.index("--mp-rank") + 1]) if "--mp-rank" in args else 0
print('{"event":"start","mode":"multi-process","ranks":2,"rank":%d}' % rank, flush=True)
if rank == 1:
    time.sleep(600)              # a faulted peer: never reports, never exits
print('{"event":"allreduce","ranks":2,"rank":0,"bytes":1024,"busbw_gbps":1.0,"ok":true}', flush=True)
time.sleep(600)                  # rank 0 then blocks in the collective with it
"""


def test_multi_process_launcher_reports_a_hung_rank(tmp_path, monkeypatch):
    fake = tmp_path / "amd-rccl-validate"
    fake.write_text(HANG)
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setattr(WM, "binary", lambda name: str(fake))
    t = time.monotonic()
    res = WM.run_rccl(1 << 20, "float", processes=2, timeout=3, step_timeout=1)
    assert time.monotonic() - t < 20
    touts = [r for r in res if r.get("event") == "timeout"]
    assert {r["rank"] for r in touts} == {0, 1} and all(r["killed_by"] == "launcher" for r in touts)
    by = {r["rank"]: r for r in touts}
    assert by[1]["phase"] == "init" and by[0]["phase"] == "allreduce" and by[0]["bytes"] == 1024
    assert by[0]["ranks"] == 2
    summ = [r for r in res if r.get("event") == "summary"]
    assert summ and not any(s["ok"] for s in summ) and "timed out in" in summ[0]["reason"]
    msg = WM.termination_message(res)
    assert '"event":"timeout"' in msg                             # it reaches the validator


def test_single_process_binary_timeout_is_structured(tmp_path, monkeypatch):
    fake = tmp_path / "amd-rccl-validate"
    fake.write_text(HANG.replace("rank == 1", "True"))
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setattr(WM, "binary", lambda name: str(fake))
    res = WM.run_rccl(1 << 20, "float", ranks="2", timeout=2)
    t = next(r for r in res if r.get("event") == "timeout")
    assert t["phase"] == "init" and t["killed_by"] == "launcher"
    assert next(r for r in res if r.get("event") == "summary")["ok"] is False


def test_rccl_binary_passes_its_watchdog_deadline(monkeypatch):
    seen = []

    def run(cmd, **kw):
        seen.append(cmd)
        return subprocess.CompletedProcess(cmd, 0, '{"event":"summary","ok":true}', "")
    monkeypatch.setattr(WM, "binary", lambda name: "/fake/" + name)
    WM.run_rccl(8 << 30, "bf16", run=run, ranks="2,4,8")
    cmd = seen[0]
    assert cmd[cmd.index("--timeout-s") + 1] == "120" and cmd[cmd.index("--max-bytes") + 1] == str(8 << 30)


def _script(tmp_path, name, body):
    p = tmp_path / name
    p.write_text("#!/bin/sh\n" + body)
    p.chmod(p.stat().st_mode | stat.S_IEXEC)
    return str(p)


def test_stream_run_returns_at_the_done_line(tmp_path):
    """amd-gemm-validate's last line is {"event":"done"}: the HIP step returns there and does not wait
    for the process's exit (its GPU teardown), which a reaper thread collects later."""
    fake = _script(tmp_path, "gemm", 'echo \'{"event":"gemm","ok":true}\'\necho \'{"event":"done","ok":true}\'\n'
                                     'sleep 3\n')
    t = time.monotonic()
    rc, lines = WM.run_json([fake], WM.stream_run, timeout=30)
    assert time.monotonic() - t < 2.0
    assert rc == 0 and lines == [{"event": "gemm", "ok": True}]          # the done line is consumed
    bad = _script(tmp_path, "bad", 'echo \'{"event":"gemm","ok":false}\'\necho \'{"event":"done","ok":false}\'\n')
    assert WM.run_json([bad], WM.stream_run, timeout=30)[0] == 1


def test_stream_run_without_done_line_waits_and_times_out(tmp_path):
    crash = _script(tmp_path, "crash", 'echo \'{"event":"gemm","ok":true}\'\necho boom >&2\nexit 7\n')
    p = WM.stream_run([crash], timeout=30)
    assert p.returncode == 7 and "boom" in p.stderr
    hang = _script(tmp_path, "hang", 'echo \'{"event":"start"}\'\nsleep 30\n')
    t = time.monotonic()
    with pytest.raises(subprocess.TimeoutExpired):
        WM.stream_run([hang], timeout=1.0)
    assert time.monotonic() - t < 5.0


def test_counter_filter_takes_the_timed_gemm_only():
    """The counter pass keeps the timed GEMM dispatch of any family and drops the checked dispatch's
    placement-recording instantiation and the ABFT / reference / fill kernels."""
    f = WM.timed_gemm_kernel
    assert f("_ZN12_GLOBAL__N_122gemm_bf16_256x256_w4apILi19ELb1ELb0ELi8ELi0ELNS_3RecE0EEEvPKDF16bS3_PDF16biii")
    assert not f("_ZN12_GLOBAL__N_122gemm_bf16_256x256_w4apILi19ELb1ELb0ELi8ELi0ELNS_3RecE1EEEvPKDF16bS3_PDF16biii")
    assert f("void (anonymous namespace)::gemm_mfma_small<false, 128, ((anonymous namespace)::Rec)0>(void const*)")
    assert f("void (anonymous namespace)::gemm_fp8_256x256_q16ap<2, true, true, 17, 2, ((anonymous namespace)::Rec)0>()")
    assert not f("void (anonymous namespace)::gemm_fp8_256x256_q16ap<2, true, true, 17, 2, ((anonymous namespace)::Rec)1>()")
    for other in ("(anonymous namespace)::abft_compare(float const*)", "void (anonymous namespace)::abft_expect<unsigned char>()",
                  "(anonymous namespace)::fill_uniform_bf16(bool _Accum*, unsigned int)"):
        assert not f(other)
    assert WM._short_kernel("void (anonymous namespace)::gemm_mfma_small_sk<true, 128, ((anonymous namespace)::Rec)0>") \
        == "gemm_mfma_small_sk"
