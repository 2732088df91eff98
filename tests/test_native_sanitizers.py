"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5.2:
the reference has no race/sanitizer tier; its Go equivalent would be `go test -race`).

libamdnode (sysfs/KFD parsing), the barrier waiter and the OCI runtime shim (JSON parser, bundle
rewrite) are rebuilt with -fsanitize=address,undefined and driven over fake sysfs trees, partition
re-enumeration, malformed inputs and bundles; any sanitizer report fails the test."""

import json
import os
import shutil
import subprocess
import threading

import pytest

from gpu_operator_amd.devices import fakesys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "native")
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


@pytest.fixture(scope="module")
def bins(tmp_path_factory):
    out = tmp_path_factory.mktemp("asan")
    targets = {
        "probe": ["node/node_probe.cpp", "node/amdnode.cpp"],
        "wait": ["node/barrier_wait.cpp", "node/amdnode.cpp"],
        "shim": ["toolkit/amd_container_runtime.cpp", "node/amdnode.cpp"],
    }
    paths = {}
    procs = {}
    for name, srcs in targets.items():
        exe = str(out / name)
        cmd = ["g++", "-std=c++17", f"-I{NATIVE}/include"] + SAN + [os.path.join(NATIVE, s) for s in srcs] + ["-o", exe]
        procs[name] = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        paths[name] = exe
    for name, p in procs.items():
        _, err = p.communicate(timeout=300)
        assert p.returncode == 0, err[-3000:]
    return paths


def _run(cmd, **kw):
    p = subprocess.run(cmd, capture_output=True, text=True, env=kw.pop("env", ENV), timeout=60, **kw)
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    return p


@pytest.mark.parametrize("compute,memory", [("SPX", "NPS1"), ("CPX", "NPS2"), ("QPX", "NPS1")])
def test_node_probe_clean(bins, tmp_path, compute, memory):
    root = fakesys.make_node(tmp_path / "n", compute=compute, memory=memory, sriov_totalvfs=4)
    fakesys.create_vfs(root, "0000:05:00.0", 2, driver="vfio-pci")
    p = _run([bins["probe"], "--root", str(root)])
    assert p.returncode == 0
    doc = json.loads(p.stdout)
    assert len(doc["gpus"]) == 8 * {"SPX": 1, "QPX": 4, "CPX": 8}[compute]


def test_node_probe_malformed_tree(bins, tmp_path):
    root = fakesys.make_node(tmp_path / "n", n_gpus=2)
    props = root / "sys/class/kfd/kfd/topology/nodes/1/properties"
    props.write_text("simd_count\nlocation_id not-a-number\n" + "x" * 5000 + "\n\n  \n")
    (root / "sys/bus/pci/devices/0000:05:00.0/current_compute_partition").write_text("")
    (root / "sys/bus/pci/devices/0000:15:00.0/hwmon/hwmon3/power1_average").write_text("garbage")
    p = _run([bins["probe"], "--root", str(root)])
    assert p.returncode == 0
    empty = tmp_path / "empty"
    empty.mkdir()
    assert _run([bins["probe"], "--root", str(empty)]).returncode == 0


def test_barrier_wait_clean(bins, tmp_path):
    d = tmp_path / "v"
    d.mkdir()
    threading.Timer(0.3, lambda: (d / "toolkit-ready").write_text("{}")).start()
    assert _run([bins["wait"], "--dir", str(d), "--all", "toolkit-ready", "--timeout", "10"]).returncode == 0
    assert _run([bins["wait"], "--dir", str(d), "--any", "nope,also-nope", "--timeout", "1"]).returncode == 1
    assert _run([bins["wait"], "--bogus"]).returncode == 2


def test_runtime_shim_clean(bins, tmp_path):
    root = fakesys.make_node(tmp_path / "n", n_gpus=2)
    dev = tmp_path / "dev"
    (dev / "dev/dri").mkdir(parents=True)
    os.symlink("/dev/null", dev / "dev/kfd")
    for i in range(2):
        os.symlink("/dev/null", dev / f"dev/dri/renderD{128 + i}")
    env = dict(ENV, AMD_CONTAINER_RUNTIME_RUNTIMES="/bin/true", AMD_CONTAINER_RUNTIME_SYS_ROOT=str(root),
               AMD_CONTAINER_RUNTIME_DEV_ROOT=str(dev), AMD_CONTAINER_RUNTIME_CDI_SPEC_DIRS=str(tmp_path / "cdi"))
    cases = {
        "ok": {"process": {"env": ["AMD_VISIBLE_DEVICES=all", "X=\"q\\u00e9\\ud83d\\ude00\""]},
               "linux": {"resources": {"memory": {"limit": 1.5e20}}}, "annotations": {"a": "b"}},
        "nested": {"a": [[[[{"b": [1, -2.5e-3, True, False, None, "\\n\\t"]}]]]],
                   "process": {"env": ["AMD_VISIBLE_DEVICES=0"]}},
    }
    for name, spec in cases.items():
        b = tmp_path / name
        b.mkdir()
        (b / "config.json").write_text(json.dumps(spec))
        p = _run([bins["shim"], "--root", "/r", "create", "--bundle", str(b), "c"], env=env)
        assert p.returncode == 0, p.stderr
        json.loads((b / "config.json").read_text())
    for bad in ('{"process": {"env": ["AMD_VISIBLE_DEVICES=0"]', '{"a": "\\uZZZZ"}', "[" * 300 + "]" * 300,
                '{"a": 1,}', ""):
        b = tmp_path / f"bad{abs(hash(bad))}"
        b.mkdir()
        (b / "config.json").write_text(bad)
        p = _run([bins["shim"], "create", "--bundle", str(b), "c"], env=env)
        assert p.returncode in (0, 1)
