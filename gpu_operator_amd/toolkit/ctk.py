"""``amd-ctk``: AMD container toolkit CLI (reference counterpart: the container-toolkit operand
image and its ``nvidia-ctk`` / ``nvidia-toolkit`` commands).

    amd-ctk cdi generate [--output DIR] [--device-name-strategy index,uuid]
    amd-ctk cdi list [--spec-dir DIR]
    amd-ctk runtime configure --runtime containerd|docker|crio [--config F] [--set-as-default] [--cdi]
    amd-ctk runtime revert --runtime ... [--config F]
    amd-ctk system create-dev-char-symlinks [--dev-char-path /dev/char]
    amd-ctk install [--daemon]     # the toolkit DaemonSet entrypoint

``install`` copies the native runtime shim into ``$ROOT/toolkit`` (the host install dir),
writes its config, generates the CDI spec, registers the runtime handlers, restarts or signals
the runtime and waits until its socket answers again (event-driven readiness instead of the
reference's fixed ``sleep 5``). With ``--daemon`` it then blocks; SIGTERM
undoes every change (config reverted, CDI spec and binaries removed, runtime reloaded).
"""

from __future__ import annotations

import argparse
import logging
import os
import shutil
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Callable, Dict, List, Optional

from ..utils import mounts
from . import cdi, runtime_config

log = logging.getLogger("amd-ctk")

NATIVE_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native", "bin")
DEFAULT_CONFIGS = {"containerd": "/etc/containerd/config.toml", "docker": "/etc/docker/daemon.json",
                   "crio": "/etc/crio/crio.conf.d/99-amd.conf"}
DEFAULT_SOCKETS = {"containerd": "/run/containerd/containerd.sock", "docker": "/var/run/docker.sock",
                   "crio": "/var/run/crio/crio.sock"}
SERVICES = {"containerd": "containerd", "docker": "docker", "crio": "crio"}


def _env_bool(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    return default if v is None else v.lower() in ("1", "true", "yes", "on")


# ---------------------------------------------------------------------------------------------
# install
# ---------------------------------------------------------------------------------------------
class Installer:
    def __init__(self, root: str, runtime: str, runtime_config: str, runtime_socket: str,
                 handler: str = "amd", set_default: bool = False, cdi_enabled: bool = False,
                 mode: str = "auto", cdi_dir: str = "/var/run/cdi", sys_root: str = "/",
                 dev_root: str = "/", annotation_prefixes: str = "amd.cdi.k8s.io/",
                 restart_mode: str = "", host_root: str = "/host", shim: Optional[str] = None,
                 run: Callable = subprocess.run, socket_timeout: float = 60.0,
                 log_file: str = "/var/log/amd-container-runtime.log"):
        self.root = root
        self.dest = os.path.join(root, "toolkit")
        self.runtime = runtime
        self.runtime_config = runtime_config
        self.runtime_socket = runtime_socket
        self.handler = handler
        self.set_default = set_default
        self.cdi_enabled = cdi_enabled
        self.mode = mode
        self.cdi_dir = cdi_dir
        self.sys_root = sys_root
        self.dev_root = dev_root
        self.annotation_prefixes = annotation_prefixes
        self.restart_mode = restart_mode or ("signal" if runtime == "docker" else "systemd")
        self.host_root = host_root
        self.shim = shim or os.path.join(NATIVE_BIN, "amd-container-runtime")
        self.run = run
        self.socket_timeout = socket_timeout
        self.log_file = log_file

    @classmethod
    def from_env(cls, **kw) -> "Installer":
        runtime = os.environ.get("RUNTIME", "containerd")
        return cls(root=os.environ.get("ROOT", mounts.path("/usr/local/amd")), runtime=runtime,
                   runtime_config=os.environ.get("RUNTIME_CONFIG", mounts.path(DEFAULT_CONFIGS[runtime])),
                   runtime_socket=os.environ.get("RUNTIME_SOCKET", mounts.path(DEFAULT_SOCKETS[runtime])),
                   handler=os.environ.get("RUNTIME_CLASS", "amd"),
                   set_default=_env_bool("CONTAINERD_SET_AS_DEFAULT") or _env_bool("SET_AS_DEFAULT"),
                   cdi_enabled=_env_bool("CDI_ENABLED"), mode=os.environ.get("AMD_RUNTIME_MODE", "auto"),
                   cdi_dir=os.environ.get("CDI_SPEC_DIR", mounts.path("/var/run/cdi")),
                   sys_root=os.environ.get("AMD_SYSFS_ROOT", "/"),
                   dev_root=os.environ.get("AMD_DEV_ROOT", mounts.path("/host")),   # devtmpfs is the host's
                   annotation_prefixes=os.environ.get("AMD_CONTAINER_RUNTIME_MODES_CDI_ANNOTATION_PREFIXES",
                                                      "amd.cdi.k8s.io/"),
                   restart_mode=os.environ.get("RESTART_MODE", ""), **kw)

    # -- steps -----------------------------------------------------------------------------
    def install_binaries(self) -> List[str]:
        os.makedirs(self.dest, exist_ok=True)
        target = os.path.join(self.dest, "amd-container-runtime")
        tmp = target + ".tmp"
        shutil.copy2(self.shim, tmp)
        os.chmod(tmp, 0o755)
        os.replace(tmp, target)
        made = [target]
        for suffix in (".cdi", ".legacy"):
            link = target + suffix
            if os.path.lexists(link):
                os.unlink(link)
            os.symlink("amd-container-runtime", link)
            made.append(link)
        with open(os.path.join(self.dest, "amd-container-runtime.conf"), "w") as f:
            f.write("# written by amd-ctk install\n")
            f.write(f"mode = {self.mode}\n")
            f.write(f"cdi-spec-dirs = /etc/cdi:{self.cdi_dir}\n")
            f.write(f"annotation-prefixes = {self.annotation_prefixes}\n")
            f.write(f"log-file = {self.log_file}\n")
        return made

    def host_binaries(self) -> Dict[str, str]:
        # paths as the host sees them (the install dir is bind-mounted at the same path)
        return runtime_config.handler_binaries(self.dest, self.handler, self.cdi_enabled)

    def generate_cdi(self) -> Optional[str]:
        if not self.cdi_enabled:
            return None
        spec = cdi.generate(self.sys_root, self.dev_root)
        return cdi.write(spec, self.cdi_dir)

    def configure_runtime(self) -> None:
        runtime_config.configure(self.runtime, self.runtime_config, self.host_binaries(),
                                 default=self.handler if self.set_default else None,
                                 cdi=self.cdi_enabled, cdi_dirs=["/etc/cdi", self.cdi_dir])

    def reload_runtime(self) -> None:
        if self.restart_mode == "none":
            return
        if self.restart_mode == "systemd":
            self.run(["chroot", self.host_root, "systemctl", "restart", SERVICES[self.runtime]],
                     check=False, capture_output=True, timeout=120)
        elif self.restart_mode == "signal":
            pid = self._runtime_pid()
            if pid:
                os.kill(pid, signal.SIGHUP)
        self.wait_socket()

    def _runtime_pid(self) -> Optional[int]:
        want = {"containerd": "containerd", "docker": "dockerd", "crio": "crio"}[self.runtime]
        for d in os.listdir("/proc"):
            if not d.isdigit():
                continue
            try:
                with open(f"/proc/{d}/comm") as f:
                    if f.read().strip() == want:
                        return int(d)
            except OSError:
                continue
        return None

    def wait_socket(self) -> bool:
        """Poll-connect the runtime socket until it accepts (the runtime is serving again)."""
        deadline = time.monotonic() + self.socket_timeout
        delay = 0.05
        while time.monotonic() < deadline:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            try:
                s.connect(self.runtime_socket)
                return True
            except OSError:
                time.sleep(delay)
                delay = min(1.0, delay * 2)
            finally:
                s.close()
        log.warning("runtime socket %s did not come back within %.0fs", self.runtime_socket, self.socket_timeout)
        return False

    def install(self) -> Dict[str, object]:
        t0 = time.monotonic()
        self.install_binaries()
        spec = self.generate_cdi()
        self.configure_runtime()
        self.reload_runtime()
        out = {"install_s": round(time.monotonic() - t0, 3), "cdi_spec": spec,
               "handlers": sorted(self.host_binaries())}
        log.info("toolkit installed: %s", out)
        return out

    def uninstall(self) -> None:
        runtime_config.revert(self.runtime, self.runtime_config)
        if self.cdi_enabled:
            p = os.path.join(self.cdi_dir, cdi.SPEC_NAME)
            if os.path.exists(p):
                os.unlink(p)
        shutil.rmtree(self.dest, ignore_errors=True)
        self.reload_runtime()
        log.info("toolkit uninstalled")


# ---------------------------------------------------------------------------------------------
# CLI
# ---------------------------------------------------------------------------------------------
def main(argv=None, stop: Optional[threading.Event] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    ap = argparse.ArgumentParser(prog="amd-ctk")
    sub = ap.add_subparsers(dest="cmd", required=True)

    c = sub.add_parser("cdi").add_subparsers(dest="action", required=True)
    g = c.add_parser("generate")
    g.add_argument("--output", default="/var/run/cdi")
    g.add_argument("--device-name-strategy", default="index,uuid")
    g.add_argument("--sys-root", default=os.environ.get("AMD_SYSFS_ROOT", "/"))
    g.add_argument("--dev-root", default="/")
    g.add_argument("--stdout", action="store_true")
    li = c.add_parser("list")
    li.add_argument("--spec-dir", default="/var/run/cdi")

    r = sub.add_parser("runtime").add_subparsers(dest="action", required=True)
    for name in ("configure", "revert"):
        p = r.add_parser(name)
        p.add_argument("--runtime", required=True, choices=sorted(DEFAULT_CONFIGS))
        p.add_argument("--config", default=None)
        if name == "configure":
            p.add_argument("--root", default="/usr/local/amd/toolkit")
            p.add_argument("--handler", default="amd")
            p.add_argument("--set-as-default", action="store_true")
            p.add_argument("--cdi", action="store_true")

    s = sub.add_parser("system").add_subparsers(dest="action", required=True)
    d = s.add_parser("create-dev-char-symlinks")
    d.add_argument("--dev-root", default="/")
    d.add_argument("--dev-char-path", default="/dev/char")

    inst = sub.add_parser("install")
    inst.add_argument("--daemon", action="store_true")
    a = ap.parse_args(argv)

    if a.cmd == "cdi" and a.action == "generate":
        import json
        spec = cdi.generate(a.sys_root, a.dev_root, a.device_name_strategy)
        if a.stdout:
            print(json.dumps(spec, indent=2))
        else:
            print(cdi.write(spec, a.output))
        return 0
    if a.cmd == "cdi" and a.action == "list":
        for n in cdi.list_devices(a.spec_dir):
            print(n)
        return 0
    if a.cmd == "runtime":
        cfg = a.config or mounts.path(DEFAULT_CONFIGS[a.runtime])
        if a.action == "configure":
            runtime_config.configure(a.runtime, cfg, runtime_config.handler_binaries(a.root, a.handler, a.cdi),
                                     default=a.handler if a.set_as_default else None, cdi=a.cdi)
        else:
            runtime_config.revert(a.runtime, cfg)
        return 0
    if a.cmd == "system":
        for link in cdi.create_dev_char_symlinks(a.dev_root, a.dev_char_path):
            print(link)
        return 0
    if a.cmd == "install":
        inst_ = Installer.from_env()
        inst_.install()
        if not a.daemon:
            return 0
        stop = stop or threading.Event()
        if threading.current_thread() is threading.main_thread():
            signal.signal(signal.SIGTERM, lambda *_: stop.set())
            signal.signal(signal.SIGINT, lambda *_: stop.set())
        stop.wait()
        if not _env_bool("NO_CLEANUP"):
            inst_.uninstall()
        return 0
    return 2


if __name__ == "__main__":
    sys.exit(main())
