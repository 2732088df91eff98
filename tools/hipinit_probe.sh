#!/bin/bash
# HIP start-up / teardown cost on the GPU box (the validator's HIP step): library load and runtime init
# through ctypes, then amd-gemm-validate's wall time to its last result line and to process exit,
# with and without --fast-exit. Output: gpurun_out/r4_hipinit/probe.txt
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r4_hipinit; mkdir -p $O
python3 - > $O/probe.txt 2>&1 <<'PY'
import os, subprocess, time
B = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpu_operator_amd/_native/bin")
code = ("import ctypes,time; t=time.perf_counter(); h=ctypes.CDLL('libamdhip64.so'); t1=time.perf_counter(); "
        "n=ctypes.c_int(); h.hipGetDeviceCount(ctypes.byref(n)); t2=time.perf_counter(); "
        "print('dlopen %.3f init %.3f' % (t1-t, t2-t1))")
for _ in range(2):
    print("ctypes", subprocess.run(["python3", "-c", code], capture_output=True, text=True).stdout.strip())

def run(argv):
    t0 = time.perf_counter()
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, text=True)
    last = t0
    for _ in p.stdout:
        last = time.perf_counter()
    p.wait()
    return round(last - t0, 3), round(time.perf_counter() - t0, 3), p.returncode

base = [os.path.join(B, "amd-gemm-validate"), "--smoke", "--shapes", "8192", "--dtype", "bf16"]
for i in range(3):
    for extra in ([], ["--fast-exit"]):
        print("gemm-validate", " ".join(extra) or "(normal exit)", "last-line / exit / rc:", run(base + extra))
PY
