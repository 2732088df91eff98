"""``amd-mxgpu-driver``: MxGPU host driver (GIM) container for vm-mxgpu nodes.

Counterpart of the reference's vGPU manager container (``nvidia-driver init`` in the
vgpu-manager image). The GIM kernel module turns each MI-series PF into
an SR-IOV parent; VF creation itself is the MxGPU device manager's job. Shares the load path
of :mod:`.driver_container` (precompiled per-kernel module first, DKMS otherwise, module
parameters from ``/drivers/gim.conf``) and differs in what "ready" means: ``gim`` loaded and
every AMD GPU PF advertising SR-IOV capacity.

    amd-mxgpu-driver init    # load + marker + block (SIGTERM unloads)
    amd-mxgpu-driver probe   # startupProbe: exit 0 iff GIM is ready
"""

from __future__ import annotations

import glob
import os
import sys
from typing import Dict, List, Tuple

from .. import devices
from . import driver_container as dc


class MxGPUDriver(dc.DriverContainer):
    MODULE = "gim"

    @property
    def marker(self) -> str:
        return os.path.join(self.run_dir, "driver", ".mxgpu-ctr")

    def precompiled_modules(self) -> List[str]:
        d = os.path.join(self.image_root, "opt/gim/precompiled", self.kernel)
        mods = sorted(glob.glob(os.path.join(d, "*.ko*")))
        return mods if any(dc._mod_name(m) == "gim" for m in mods) else []

    def load(self) -> Tuple[str, List[str]]:
        params = dc.module_params(self.params_file.replace("amdgpu.conf", "gim.conf"))
        mods = self.precompiled_modules()
        if mods:
            for m in mods:
                self._run(["insmod", m] + (params if dc._mod_name(m) == "gim" else []), f"insmod {dc._mod_name(m)}")
            return "precompiled", [dc._mod_name(m) for m in mods]
        if not self.driver_version:
            raise dc.DriverError(f"no precompiled gim for kernel {self.kernel} and DRIVER_VERSION unset")
        self._run(["dkms", "install", f"gim/{self.driver_version}", "-k", self.kernel], "dkms install gim")
        self._run(["modprobe", "gim"] + params, "modprobe gim")
        return "dkms", ["gim"]

    def ready(self) -> Tuple[bool, str]:
        if not os.path.isdir(os.path.join(self.sys_root, "sys/module/gim")):
            return False, "gim not loaded"
        pfs = [f for f in devices.scan_pci(self.sys_root) if not f["is_virtfn"]]
        if not pfs:
            return False, "no AMD GPU PF found"
        missing = [f["bdf"] for f in pfs if f["sriov_totalvfs"] <= 0]
        if missing:
            return False, f"PFs without SR-IOV capacity: {missing}"
        return True, f"{len(pfs)} SR-IOV PF(s), up to {sum(f['sriov_totalvfs'] for f in pfs)} VFs"

    def init(self) -> Dict:
        # GIM replaces amdgpu on the host: refuse if amdgpu owns the devices
        if devices.driver_state(self.sys_root, self.dev_root)["module_loaded"] and \
                any(f["driver"] == "amdgpu" for f in devices.scan_pci(self.sys_root)):
            raise dc.DriverError("amdgpu is bound to the GPUs; vm-mxgpu nodes need it unloaded")
        return super().init() if not os.path.isdir(os.path.join(self.sys_root, "sys/module/gim")) else \
            self._reuse()

    def _reuse(self) -> Dict:
        why = self.wait_ready()
        os.makedirs(os.path.dirname(self.marker), exist_ok=True)
        with open(self.marker, "w") as f:
            f.write('{"mode": "reused"}')
        return {"mode": "reused", "state": why}

    def shutdown(self) -> None:
        self.run(["modprobe", "-r", "gim"], capture_output=True, text=True, timeout=120)
        try:
            os.unlink(self.marker)
        except FileNotFoundError:
            pass


def main(argv=None, stop=None, drv=None) -> int:
    drv = drv or MxGPUDriver(sys_root=os.environ.get("AMD_SYSFS_ROOT", "/"), params_file="/drivers/gim.conf")
    return dc.main(argv, stop=stop, dc=drv)


if __name__ == "__main__":
    sys.exit(main())
