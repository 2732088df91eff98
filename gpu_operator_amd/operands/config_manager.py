"""``amd-config-manager``: per-node config selection sidecar (device plugin, partition manager).

Counterpart of the reference's config-manager init container + sidecar
(``handleDevicePluginConfig``, object_controls.go:2184-2289). The
ConfigMap named in ``devicePlugin.config.name`` is mounted at ``CONFIG_FILE_SRCDIR`` with one
key per named config; the node label ``NODE_LABEL`` (``amd.com/device-plugin.config``) picks
one, falling back per ``FALLBACK_STRATEGIES``:

* ``named``  -> ``DEFAULT_CONFIG``;
* ``single`` -> the only config present, if there is exactly one;
* ``empty``  -> an empty config.

The selection is written atomically to ``CONFIG_FILE_DST``; on change the sidecar sends
``SIGNAL`` to ``PROCESS_TO_SIGNAL`` (shared PID namespace) so the plugin reloads without a
restart. ``ONESHOT=true`` (init container) selects once and exits. Event-driven: a Node watch
wakes the sidecar on label changes; the ConfigMap volume is re-read on each wake-up and on a
slow resync (kubelet updates projected volumes asynchronously).
"""

from __future__ import annotations

import logging
import os
import signal
import sys
import threading
from typing import Callable, List, Optional, Tuple

from ..k8s import objects as o

log = logging.getLogger("amd-config-manager")


class ConfigError(Exception):
    pass


def available(src_dir: str) -> List[str]:
    if not os.path.isdir(src_dir):
        return []
    return sorted(f for f in os.listdir(src_dir) if not f.startswith(".") and
                  os.path.isfile(os.path.join(src_dir, f)))


def select(label_value: Optional[str], src_dir: str, default: str, strategies: List[str]) -> Tuple[str, str]:
    """Return (config name, content)."""
    names = available(src_dir)
    want = label_value or ""
    if want:
        if want not in names:
            raise ConfigError(f"config {want!r} selected by node label not in {names}")
        return want, _read(src_dir, want)
    for s in strategies:
        if s == "named" and default:
            if default not in names:
                raise ConfigError(f"default config {default!r} not in {names}")
            return default, _read(src_dir, default)
        if s == "single" and len(names) == 1:
            return names[0], _read(src_dir, names[0])
        if s == "empty":
            return "", ""
    raise ConfigError(f"no config selected and no fallback applies (available: {names})")


def _read(src_dir: str, name: str) -> str:
    with open(os.path.join(src_dir, name)) as f:
        return f.read()


def write_if_changed(dst: str, content: str) -> bool:
    try:
        with open(dst) as f:
            if f.read() == content:
                return False
    except FileNotFoundError:
        pass
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    tmp = dst + ".tmp"
    with open(tmp, "w") as f:
        f.write(content)
    os.replace(tmp, dst)
    return True


def find_pids(name: str, proc: str = "/proc") -> List[int]:
    out = []
    for d in os.listdir(proc):
        if not d.isdigit() or int(d) == os.getpid():
            continue
        try:
            with open(os.path.join(proc, d, "cmdline"), "rb") as f:
                argv = f.read().split(b"\0")
        except OSError:
            continue
        if not argv or not argv[0]:
            continue
        args = [a.decode(errors="replace") for a in argv if a]
        exe = os.path.basename(args[0])
        # python console scripts: "python /usr/local/bin/<name> ..."
        second = os.path.basename(args[1]) if len(args) > 1 else ""
        # the package's own runner: "python -m gpu_operator_amd.cmd.entry <name> ..."
        runner = len(args) > 3 and args[1] == "-m" and args[2] == "gpu_operator_amd.cmd.entry" and args[3] == name
        if exe == name or second == name or runner:
            out.append(int(d))
    return out


class ConfigManager:
    def __init__(self, client, node: str, label: str, src_dir: str, dst: str, default: str = "",
                 strategies: Optional[List[str]] = None, process: str = "", sig: int = signal.SIGHUP,
                 send_signal: bool = True, kill: Callable[[int, int], None] = os.kill,
                 pids: Callable[[str], List[int]] = find_pids, resync: float = 60.0):
        self.client = client
        self.node = node
        self.label = label
        self.src_dir = src_dir
        self.dst = dst
        self.default = default
        self.strategies = strategies or ["named", "single"]
        self.process = process
        self.sig = sig
        self.send_signal = send_signal
        self.kill = kill
        self.pids = pids
        self.resync = resync
        self.current: Optional[str] = None

    @classmethod
    def from_env(cls, client, **kw) -> "ConfigManager":
        e = os.environ
        return cls(client, e.get("NODE_NAME", ""), e.get("NODE_LABEL", "amd.com/device-plugin.config"),
                   e.get("CONFIG_FILE_SRCDIR", "/available-configs"), e.get("CONFIG_FILE_DST", "/config/config.yaml"),
                   default=e.get("DEFAULT_CONFIG", ""),
                   strategies=[s.strip() for s in e.get("FALLBACK_STRATEGIES", "named,single").split(",") if s.strip()],
                   process=e.get("PROCESS_TO_SIGNAL", ""), sig=int(e.get("SIGNAL", str(int(signal.SIGHUP)))),
                   send_signal=e.get("SEND_SIGNAL", "true") == "true", **kw)

    def label_value(self) -> Optional[str]:
        return o.get_labels(self.client.get("v1", "Node", self.node)).get(self.label)

    def sync(self) -> bool:
        """Select + write; signal the consumer when the content changed. True if changed."""
        name, content = select(self.label_value(), self.src_dir, self.default, self.strategies)
        changed = write_if_changed(self.dst, content)
        if changed:
            log.info("config %r written to %s", name or "<empty>", self.dst)
            if self.current is not None and self.send_signal and self.process:
                for pid in self.pids(self.process):
                    log.info("signalling %s (pid %d) with %d", self.process, pid, self.sig)
                    self.kill(pid, self.sig)
        self.current = name
        return changed

    def run(self, stop: threading.Event) -> None:
        wake = threading.Event()

        def on_node(ev):
            if o.name(ev.obj) != self.node:
                return
            old = o.get_labels(ev.old).get(self.label) if ev.old else None
            if ev.old is None or old != o.get_labels(ev.obj).get(self.label):
                wake.set()
        cancel = self.client.watch("v1", "Node", on_node, field_selector=f"metadata.name={self.node}")
        try:
            while not stop.is_set():
                try:
                    self.sync()
                except ConfigError as e:
                    log.error("%s", e)
                wake.wait(self.resync)
                wake.clear()
        finally:
            if callable(cancel):
                cancel()


def main(argv=None, client=None, stop: Optional[threading.Event] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    if client is None:
        from ..k8s.rest import RestClient
        client = RestClient()
    cm = ConfigManager.from_env(client)
    if os.environ.get("ONESHOT", "false") == "true":
        try:
            cm.sync()
            return 0
        except ConfigError as e:
            log.error("%s", e)
            return 1
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
    cm.run(stop)
    return 0


if __name__ == "__main__":
    sys.exit(main())
