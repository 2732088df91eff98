#!/usr/bin/env python3
"""Dump every GPU's raw sysfs ``gpu_metrics`` blob next to amd-smi's decoding of it.

Used to pin the byte layout the native parser (native/node/amdnode.cpp, ``parse_gpu_metrics``)
reads the xGMI accumulators from: run on the GPU box, the blob and amd-smi's dict become a test
fixture (tests/fixtures/gpu_metrics/). Read-only.

    python3 tools/gpu_metrics_probe.py --out gpurun_out/gm
"""

import argparse
import base64
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    blobs = {}
    for p in sorted(glob.glob("/sys/class/drm/card*/device/gpu_metrics")):
        dev = os.path.realpath(os.path.dirname(p))
        bdf = os.path.basename(dev)
        try:
            with open(p, "rb") as f:
                raw = f.read()
        except OSError as e:
            print(json.dumps({"path": p, "error": str(e)}))
            continue
        blobs[bdf] = raw
        with open(os.path.join(a.out, f"gpu_metrics_{bdf.replace(':', '_')}.bin"), "wb") as f:
            f.write(raw)
        print(json.dumps({"path": p, "bdf": bdf, "size": len(raw), "structure_size": int.from_bytes(raw[0:2], "little"),
                          "format_revision": raw[2], "content_revision": raw[3]}))
    out = {"blobs": {k: base64.b64encode(v).decode() for k, v in blobs.items()}}
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        smi = {}
        for h in amdsmi.amdsmi_get_processor_handles():
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            smi[bdf] = {k: (v if isinstance(v, (int, float, str, list)) else str(v)) for k, v in m.items()}
            try:
                smi[bdf]["_header"] = {k: v for k, v in amdsmi.amdsmi_get_gpu_metrics_header_info(h).items()}
            except Exception as e:  # noqa: BLE001
                smi[bdf]["_header_error"] = str(e)
        out["amdsmi"] = smi
        amdsmi.amdsmi_shut_down()
    except Exception as e:  # noqa: BLE001
        out["amdsmi_error"] = repr(e)
    with open(os.path.join(a.out, "probe.json"), "w") as f:
        json.dump(out, f, indent=1, default=str)
    print(json.dumps({"n_blobs": len(blobs), "amdsmi": "amdsmi" in out}))


if __name__ == "__main__":
    main()
