"""``amdgpu-driver``: entrypoint of the amdgpu driver container (state-driver DaemonSet).

Counterpart of the reference's external ``nvidia-driver init`` image (SURVEY.md §2.2 row 3,
§2.3): installs the kernel driver on the host from a container. The amdgpu stack is only
kernel modules + firmware (no user-space driver libraries to expose), so:

``init``
  1. host facts: kernel release (``uname -r``) and ``/host-etc/os-release``;
  2. module source, fastest first:
       - precompiled for this exact kernel (``/opt/amdgpu/precompiled/<kernel>/*.ko[.xz]``,
         what the per-kernel DaemonSets of ``driver.usePrecompiled`` ship) -> insmod in
         dependency order — seconds instead of a DKMS build;
       - DKMS (``dkms install amdgpu/<version> -k <kernel>``) -> ``modprobe``;
  3. firmware from the image to the host's ``/lib/firmware/updates/amdgpu``;
  4. module parameters from the ``kernelModuleConfig`` ConfigMap (``/drivers/amdgpu.conf``);
  5. wait, event-driven and bounded, for ``initstate=live``, ``/dev/kfd`` and one KFD agent
     per amdgpu-bound GPU — then write the ``.driver-ctr`` marker (read by the driver manager
     and the startup probe) and block; SIGTERM unloads the modules again if unused.

``probe``  exit 0 iff the driver is live with all GPUs enumerated (the startupProbe; it
           touches ``.driver-ctr-ready`` on success, which the validator waits on).

Reload on request: a memory-partition (NPS) change only takes effect once amdgpu reloads, and
only this container has the module tree that loaded it (precompiled ``.ko`` files under
``/opt/amdgpu`` or its DKMS build). While ``init`` blocks it serves a node-local request file,
``/run/amd/driver/reload-request`` (JSON ``{"id", "ts", "deadline"}``, written by the partition
manager): it unloads the modules, loads them again -- insmod of the precompiled ``.ko`` files, or
``modprobe`` of the module DKMS built at init (a reload never rebuilds) -- within the requester's
deadline, waits for readiness, rewrites the ``.driver-ctr`` marker and answers in ``reload-result``
with the same id, whatever happens. A request older than this container, or past its deadline (its
requester gave up), is answered ``stale`` and never unloads the driver.
"""

from __future__ import annotations

import argparse
import glob
import json
import logging
import os
import shutil
import signal
import subprocess
import sys
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

from .. import devices
from ..utils import mounts

log = logging.getLogger("amdgpu-driver")

LOAD_ORDER = ["amdkcl", "amdttm", "amddrm_ttm_helper", "amddrm_buddy", "amdxcp", "amdgpu"]
RELOAD_REQUEST = "reload-request"
RELOAD_RESULT = "reload-result"


class DriverError(Exception):
    pass


def os_release(path: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    try:
        with open(path) as f:
            for line in f:
                if "=" in line:
                    k, v = line.rstrip("\n").split("=", 1)
                    out[k] = v.strip().strip('"')
    except OSError:
        pass
    return out


def module_params(path: str) -> List[str]:
    """``options amdgpu a=1 b=2`` lines (modprobe.d syntax) or bare ``a=1`` lines."""
    out: List[str] = []
    try:
        with open(path) as f:
            for line in f:
                line = line.split("#", 1)[0].strip()
                if not line:
                    continue
                parts = line.split()
                if parts[0] == "options":
                    if len(parts) >= 2 and parts[1] == "amdgpu":
                        out += parts[2:]
                else:
                    out += parts
    except OSError:
        pass
    return out


def _mod_name(path: str) -> str:
    base = os.path.basename(path)
    for ext in (".ko.xz", ".ko.zst", ".ko.gz", ".ko"):
        if base.endswith(ext):
            return base[: -len(ext)]
    return base


class DriverContainer:
    def __init__(self, sys_root: str = "/", dev_root: str = "/", image_root: str = "/",
                 host_etc: str = "/host-etc", run_dir: str = "/run/amd", firmware_dir: str = "/lib/firmware",
                 params_file: str = "/drivers/amdgpu.conf", kernel: Optional[str] = None,
                 driver_version: str = "", run: Callable = subprocess.run, ready_timeout: float = 300.0,
                 poll: float = 0.05):
        self.sys_root = sys_root
        self.dev_root = dev_root
        self.image_root = image_root
        self.host_etc = host_etc
        self.run_dir = run_dir
        self.firmware_dir = firmware_dir
        self.params_file = params_file
        self.kernel = kernel or os.uname().release
        self.driver_version = driver_version or os.environ.get("DRIVER_VERSION", "")
        self.run = run
        self.ready_timeout = ready_timeout
        self.poll = poll
        self.started = time.time()          # reload requests written before this are stale

    @property
    def marker(self) -> str:
        return os.path.join(self.run_dir, "driver", ".driver-ctr")

    @property
    def driver_dir(self) -> str:
        return os.path.join(self.run_dir, "driver")

    # -- sources -------------------------------------------------------------------------------
    def precompiled_modules(self) -> List[str]:
        d = mounts.path(os.path.join(self.image_root, "opt/amdgpu/precompiled", self.kernel))
        mods = {_mod_name(p): p for p in glob.glob(os.path.join(d, "*.ko*"))}
        if "amdgpu" not in mods:
            return []
        ordered = [mods.pop(m) for m in LOAD_ORDER if m in mods]
        return sorted(mods.values()) + ordered       # unknown helpers first, amdgpu last

    def install_firmware(self) -> int:
        src = mounts.path(os.path.join(self.image_root, "opt/amdgpu/firmware"))
        if not os.path.isdir(src):
            return 0
        dst = os.path.join(self.firmware_dir, "updates", "amdgpu")
        os.makedirs(dst, exist_ok=True)
        n = 0
        for f in sorted(os.listdir(src)):
            s, d = os.path.join(src, f), os.path.join(dst, f)
            if os.path.exists(d) and os.path.getsize(d) == os.path.getsize(s):
                continue
            shutil.copy2(s, d + ".tmp")
            os.replace(d + ".tmp", d)
            n += 1
        return n

    def _run(self, argv: List[str], what: str, timeout: float = 1800.0) -> None:
        if timeout <= 0:
            raise DriverError(f"{what}: no time left before the reload deadline")
        try:
            p = self.run(argv, capture_output=True, text=True, timeout=timeout)
        except subprocess.TimeoutExpired:
            raise DriverError(f"{what} did not finish within {timeout:.0f}s")
        except OSError as e:
            raise DriverError(f"{what}: {e}")
        if p.returncode != 0:
            raise DriverError(f"{what} failed ({p.returncode}): {(p.stderr or '').strip()[-2000:]}")

    def load(self) -> Tuple[str, List[str]]:
        params = module_params(self.params_file)
        mods = self.precompiled_modules()
        if mods:
            for m in mods:
                args = ["insmod", m] + (params if _mod_name(m) == "amdgpu" else [])
                self._run(args, f"insmod {_mod_name(m)}")
            return "precompiled", [_mod_name(m) for m in mods]
        if not self.driver_version:
            raise DriverError(f"no precompiled modules for kernel {self.kernel} and DRIVER_VERSION unset")
        self._run(["dkms", "install", f"amdgpu/{self.driver_version}", "-k", self.kernel], "dkms install")
        self._run(["modprobe", "amdgpu"] + params, "modprobe amdgpu")
        return "dkms", ["amdgpu"]

    def load_built(self, deadline: float) -> Tuple[str, List[str]]:
        """``load`` without building: what a reload needs (init built or found the modules).
        Every step is bounded by ``deadline`` (time.monotonic())."""
        params = module_params(self.params_file)
        mods = self.precompiled_modules()
        if mods:
            for m in mods:
                self._run(["insmod", m] + (params if _mod_name(m) == "amdgpu" else []), f"insmod {_mod_name(m)}",
                          deadline - time.monotonic())
            return "precompiled", [_mod_name(m) for m in mods]
        self._run(["modprobe", "amdgpu"] + params, "modprobe amdgpu", deadline - time.monotonic())
        return "dkms", ["amdgpu"]

    def unload(self, deadline: Optional[float] = None) -> List[str]:
        """Remove what ``load`` inserted: precompiled modules in reverse load order (amdgpu
        first), else ``modprobe -r amdgpu`` (DKMS). The GPU clients are gone by now (the partition
        manager paused them); a module still in use fails the unload."""
        left = (lambda: deadline - time.monotonic()) if deadline is not None else (lambda: 1800.0)
        mods = [_mod_name(m) for m in self.precompiled_modules()]
        if mods:
            loaded = [m for m in reversed(mods) if os.path.isdir(os.path.join(self.sys_root, "sys/module", m))]
            for m in loaded:
                self._run(["rmmod", m], f"rmmod {m}", left())
            return loaded
        self._run(["modprobe", "-r", "amdgpu"], "modprobe -r amdgpu", left())
        return ["amdgpu"]

    def _write_marker(self, info: Dict) -> None:
        os.makedirs(os.path.dirname(self.marker), exist_ok=True)
        with open(self.marker + ".tmp", "w") as f:
            json.dump(info, f)
        os.replace(self.marker + ".tmp", self.marker)

    def reload(self, budget_s: Optional[float] = None) -> Dict:
        """Unload and load again (no DKMS build), all within ``budget_s`` (the requester's deadline;
        default ``ready_timeout``), then wait for readiness inside what is left."""
        t0 = time.monotonic()
        deadline = t0 + (self.ready_timeout if budget_s is None else budget_s)
        removed = self.unload(deadline)
        mode, mods = self.load_built(deadline)
        why = self.wait_ready(deadline)
        info = {"kernel": self.kernel, "mode": mode, "modules": mods, "unloaded": removed,
                "version": self.driver_version, "reload_s": round(time.monotonic() - t0, 3), "ts": time.time(),
                "state": why}
        self._write_marker(info)
        log.info("amdgpu reloaded: %s", info)
        return info

    def _answer(self, res: Dict) -> None:
        res["ts"] = time.time()
        out = os.path.join(self.driver_dir, RELOAD_RESULT)
        with open(out + ".tmp", "w") as f:
            json.dump(res, f)
        os.replace(out + ".tmp", out)

    def serve_reloads(self, stop: threading.Event, period: float = 1.0) -> None:
        """Answer reload requests until ``stop`` (event-driven: inotify on the driver dir). Every
        request gets a result, also when the reload raises something unexpected; a stale request
        (older than this container, or past the requester's deadline) never touches the driver."""
        os.makedirs(self.driver_dir, exist_ok=True)
        req = os.path.join(self.driver_dir, RELOAD_REQUEST)
        while not stop.is_set():
            if not os.path.exists(req):
                try:
                    devices.wait_files(self.driver_dir, [RELOAD_REQUEST], timeout=period)
                except Exception:  # noqa: BLE001 - no inotify (no native library): poll
                    stop.wait(period)
                continue
            try:
                with open(req) as f:
                    body = json.load(f) or {}
            except (OSError, ValueError):
                body = {}
            try:
                os.unlink(req)
            except FileNotFoundError:
                pass
            rid = body.get("id", "")
            now = time.time()
            ts, deadline = float(body.get("ts") or 0.0), float(body.get("deadline") or 0.0)
            if ts < self.started or (deadline and deadline <= now):
                why = "written before this driver container started" if ts < self.started else \
                    "past the requester's deadline"
                log.warning("ignoring stale reload request %s (%s)", rid, why)
                self._answer({"id": rid, "ok": False, "stale": True, "error": f"stale request ignored: {why}"})
                continue
            try:
                res = {"id": rid, "ok": True, "info": self.reload(deadline - now if deadline else None)}
            except Exception as e:  # noqa: BLE001 - the requester waits for an answer either way
                log.error("reload failed: %s", e)
                res = {"id": rid, "ok": False, "error": f"{type(e).__name__}: {e}"}
            try:
                self._answer(res)
            except OSError as e:
                log.error("could not write the reload result: %s", e)

    # -- readiness -----------------------------------------------------------------------------
    def ready(self) -> Tuple[bool, str]:
        st = devices.driver_state(self.sys_root, self.dev_root)
        if not st["module_loaded"]:
            return False, "amdgpu not loaded"
        if not st["live"]:
            return False, "initstate not live"
        if not st["kfd_present"]:
            return False, "/dev/kfd missing"
        bound = {f["bdf"] for f in devices.scan_pci(self.sys_root) if f["driver"] == "amdgpu" and not f["is_virtfn"]}
        agents = {g["pci_bdf"] for g in devices.enumerate_gpus(self.sys_root)}
        if not bound or not bound <= agents:
            return False, f"{len(bound & agents)}/{len(bound)} GPUs enumerated by KFD"
        return True, f"{len(bound)} GPU(s), {st['kfd_gpu_nodes']} KFD agent(s)"

    def wait_ready(self, deadline: Optional[float] = None) -> str:
        deadline = time.monotonic() + self.ready_timeout if deadline is None else deadline
        while True:
            ok, why = self.ready()
            if ok:
                return why
            if time.monotonic() > deadline:
                raise DriverError(f"driver did not become ready: {why}")
            time.sleep(self.poll)

    # -- commands ------------------------------------------------------------------------------
    def init(self) -> Dict:
        t0 = time.monotonic()
        st = devices.driver_state(self.sys_root, self.dev_root)
        if st["module_loaded"] and not os.path.exists(self.marker):
            raise DriverError("amdgpu is already loaded by the host; the driver container must not "
                              "run on nodes with a pre-installed driver")
        osr = os_release(os.path.join(self.host_etc, "os-release"))
        fw = self.install_firmware()
        if st["module_loaded"]:
            mode, mods = "reused", []
        else:
            mode, mods = self.load()
        why = self.wait_ready()
        info = {"kernel": self.kernel, "os": f"{osr.get('ID', '')}{osr.get('VERSION_ID', '')}",
                "mode": mode, "modules": mods, "firmware_files": fw, "version": self.driver_version,
                "load_s": round(time.monotonic() - t0, 3), "ts": time.time(), "state": why}
        self._write_marker(info)
        log.info("amdgpu ready: %s", info)
        return info

    def shutdown(self) -> None:
        try:
            with open(os.path.join(self.sys_root, "sys/module/amdgpu/refcnt")) as f:
                users = int(f.read().strip() or 0)
        except (OSError, ValueError):
            users = 0
        if users == 0:
            p = self.run(["modprobe", "-r", "amdgpu"], capture_output=True, text=True, timeout=120)
            if p.returncode != 0:
                log.warning("could not unload amdgpu: %s", (p.stderr or "").strip())
        else:
            log.warning("amdgpu in use (refcnt %d): leaving it loaded", users)
        try:
            os.unlink(self.marker)
        except FileNotFoundError:
            pass


def main(argv=None, stop: Optional[threading.Event] = None, dc: Optional[DriverContainer] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amdgpu-driver")
    ap.add_argument("command", choices=["init", "probe", "load-only"])
    a = ap.parse_args(argv)
    dc = dc or DriverContainer(sys_root=os.environ.get("AMD_SYSFS_ROOT", "/"),
                               dev_root=os.environ.get("AMD_DEV_ROOT", "/"),
                               host_etc=mounts.path("/host-etc"), run_dir=mounts.path("/run/amd"),
                               firmware_dir=mounts.path("/lib/firmware"),
                               params_file=mounts.path(os.environ.get("KERNEL_MODULE_PARAMS", "/drivers/amdgpu.conf")))
    if a.command == "probe":
        ok, why = dc.ready()
        print(why)
        return 0 if ok else 1
    try:
        dc.init()
    except DriverError as e:
        log.error("%s", e)
        return 1
    if a.command == "load-only":
        return 0
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
    dc.serve_reloads(stop)
    dc.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
