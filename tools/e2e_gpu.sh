# The reference end-to-end flow on the MI355X box (gpu_operator_amd/e2e), logs of a failed run
# copied under gpurun_out/e2e. Run: gpurun -- bash tools/e2e_gpu.sh
mkdir -p gpurun_out/e2e
timeout -k 10 500 python3 -u -m gpu_operator_amd.e2e --hip-mode pod --timeout 120 --keep > gpurun_out/e2e/e2e.json 2> gpurun_out/e2e/e2e.err
rc=$?
echo e2e_rc=$rc
python3 - <<'PY'
import json, shutil, glob, os
r = json.load(open("gpurun_out/e2e/e2e.json"))
print({k: v for k, v in r.items() if k not in ("steps", "marks_s")})
for s in r.get("steps", []):
    print(s["name"], s["ok"], s["seconds"], s.get("error", ""))
d = r.get("logs_dir")
if d and os.path.isdir(d):
    for f in glob.glob(d + "/operator.*.log"):
        shutil.copy(f, "gpurun_out/e2e/")
    for p in glob.glob(d + "/pods/*/logs"):
        shutil.copytree(p, "gpurun_out/e2e/pods/" + os.path.basename(os.path.dirname(p)), dirs_exist_ok=True)
PY
