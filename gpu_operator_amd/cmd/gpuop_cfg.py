"""``amd-gpuop-cfg``: offline validation and migration of operator configuration.

Counterpart of the reference's ``gpuop-cfg`` (cmd/gpuop-cfg):

``validate clusterpolicy``  a ClusterPolicy file, or the Helm chart rendered with its values
                            (+ ``--values`` overrides) exactly as ``helm template`` would: the CR
                            must parse strictly against the API and every enabled operand's
                            image must resolve (CR -> ``*_IMAGE`` env of the rendered operator
                            Deployment). ``--check-registry`` additionally HEADs each manifest
                            on its registry (the reference always does; needs network).
``validate csv``            an OLM ClusterServiceVersion: operator image + every ``*_IMAGE`` env
                            listed in relatedImages, alm-examples parse as ClusterPolicies.
``convert``                 an ``nvidia.com/v1`` ClusterPolicy to ``amd.com/v1``: renamed
                            sections (dcgmExporter -> metricsExporter, gfd -> nodeLabeller,
                            mig/migManager -> partition/partitionManager, vgpu* -> mxgpu*),
                            label keys re-homed to ``amd.com/``, CUDA-only fields dropped with
                            a note each.
"""

from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import urllib.request
from dataclasses import fields as dc_fields
from typing import Dict, List, Optional, Tuple

import yaml

from ..api.schema import ValidationError
from ..api.v1 import clusterpolicy as cp

CHART_DEFAULT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                             "deployments", "amd-gpu-operator")


class ConfigError(Exception):
    pass


# ---------------------------------------------------------------------------------------------
# image resolution
# ---------------------------------------------------------------------------------------------
def operand_images(spec: cp.ClusterPolicySpec, env: Dict[str, str]) -> Dict[str, str]:
    """component -> image for every enabled operand (and their helper images)."""
    out: Dict[str, str] = {}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        for f in dc_fields(spec):
            v = getattr(spec, f.name)
            if isinstance(v, cp.ComponentSpec) and type(v).IMAGE_ENV:
                if not v.is_enabled():
                    continue
                if isinstance(v, cp.GDSSpec):
                    continue          # accepted for migration only, never deployed
                out[f.name] = cp.image_path(v)
                for sub in ("manager", "driverManager"):
                    s = getattr(v, sub, None)
                    if isinstance(s, cp.ImageSpec) and (s.image or os.environ.get(type(s).IMAGE_ENV)):
                        out[f"{f.name}.{sub}"] = cp.image_path(s)
        ic = spec.operator.initContainer
        if ic is not None and (ic.image or os.environ.get(type(ic).IMAGE_ENV)):
            out["operator.initContainer"] = cp.image_path(ic)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return out


def check_registry(image: str, timeout: float = 10.0) -> Tuple[bool, str]:
    """HEAD the image manifest on its registry (anonymous; 401 counts as 'exists')."""
    ref = image
    if "/" not in ref.split(":")[0] or "." not in ref.split("/")[0]:
        ref = "registry-1.docker.io/" + (ref if "/" in ref else "library/" + ref)
    host, _, path = ref.partition("/")
    if "@" in path:
        repo, tag = path.split("@", 1)
    else:
        repo, _, tag = path.rpartition(":") if ":" in path else (path, "", "latest")
    url = f"https://{host}/v2/{repo}/manifests/{tag}"
    req = urllib.request.Request(url, method="HEAD", headers={
        "Accept": "application/vnd.oci.image.index.v1+json, application/vnd.docker.distribution.manifest.v2+json"})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status == 200, f"HTTP {r.status}"
    except urllib.error.HTTPError as e:
        return e.code == 401, f"HTTP {e.code}"
    except OSError as e:
        return False, str(e)


# ---------------------------------------------------------------------------------------------
# validate clusterpolicy
# ---------------------------------------------------------------------------------------------
def _deployment_env(objs: List[Dict]) -> Dict[str, str]:
    for o in objs:
        if o.get("kind") == "Deployment":
            for c in o["spec"]["template"]["spec"]["containers"]:
                if c["name"] == "amd-gpu-operator":
                    return {e["name"]: e["value"] for e in c.get("env", []) if "value" in e}
    return {}


def load_clusterpolicy(path: Optional[str], chart: Optional[str], values: Optional[str]) -> Tuple[Dict, Dict[str, str]]:
    if path:
        with open(path) as f:
            docs = [d for d in yaml.safe_load_all(f) if d]
        objs = docs
    else:
        from ..utils.gotemplate import render_objects
        over = {}
        if values:
            with open(values) as f:
                over = yaml.safe_load(f) or {}
        objs = render_objects(chart or CHART_DEFAULT, over)
    cps = [o for o in objs if o.get("kind") == "ClusterPolicy"]
    if len(cps) != 1:
        raise ConfigError(f"expected exactly one ClusterPolicy, found {len(cps)}")
    return cps[0], _deployment_env(objs)


def validate_clusterpolicy(obj: Dict, env: Dict[str, str], registry: bool = False) -> Dict:
    try:
        pol = cp.ClusterPolicy(obj, strict=True)
    except ValidationError as e:
        raise ConfigError(f"invalid ClusterPolicy: {e}") from e
    try:
        images = operand_images(pol.spec, env)
    except ValueError as e:
        raise ConfigError(str(e)) from e
    report = {"images": images}
    if registry:
        bad = {}
        for comp, img in images.items():
            ok, why = check_registry(img)
            if not ok:
                bad[comp] = f"{img}: {why}"
        if bad:
            raise ConfigError(f"unresolvable images: {bad}")
        report["registry"] = "ok"
    return report


# ---------------------------------------------------------------------------------------------
# validate csv
# ---------------------------------------------------------------------------------------------
def validate_csv(csv: Dict, registry: bool = False) -> Dict:
    spec = csv.get("spec") or {}
    related = {r["image"] for r in spec.get("relatedImages") or []}
    deps = ((spec.get("install") or {}).get("spec") or {}).get("deployments") or []
    if not deps:
        raise ConfigError("CSV has no install deployments")
    problems = []
    images = []
    for d in deps:
        for c in d["spec"]["template"]["spec"]["containers"]:
            images.append(c["image"])
            if c["image"] not in related:
                problems.append(f"operator image {c['image']} not in relatedImages")
            for e in c.get("env") or []:
                if e["name"].endswith("_IMAGE") and "value" in e:
                    images.append(e["value"])
                    if e["value"] not in related:
                        problems.append(f"{e['name']}={e['value']} not in relatedImages")
    try:
        examples = json.loads((csv.get("metadata") or {}).get("annotations", {}).get("alm-examples", "[]"))
    except ValueError as e:
        raise ConfigError(f"alm-examples is not JSON: {e}") from e
    n_cp = 0
    for ex in examples:
        if ex.get("kind") == cp.KIND:
            try:
                cp.ClusterPolicy(ex, strict=True)
            except ValidationError as e:
                problems.append(f"alm-example {ex.get('metadata', {}).get('name')}: {e}")
            n_cp += 1
    if n_cp == 0:
        problems.append("no ClusterPolicy in alm-examples")
    if registry:
        for img in sorted(set(images)):
            ok, why = check_registry(img)
            if not ok:
                problems.append(f"{img}: {why}")
    if problems:
        raise ConfigError("; ".join(problems))
    return {"images": sorted(set(images)), "alm_examples": n_cp}


# ---------------------------------------------------------------------------------------------
# convert nvidia.com/v1 -> amd.com/v1
# ---------------------------------------------------------------------------------------------
SECTION_RENAMES = {"dcgmExporter": "metricsExporter", "dcgm": "rdc", "gfd": "nodeLabeller", "mig": "partition",
                   "migManager": "partitionManager", "vgpuManager": "mxgpuManager",
                   "vgpuDeviceManager": "mxgpuDeviceManager"}
DROPPED = {
    ("driver", "licensingConfig"): "vGPU licensing has no MxGPU equivalent",
    ("driver", "virtualTopology"): "vGPU virtual topology has no MxGPU equivalent",
    ("driver", "useOpenKernelModules"): "NVIDIA open kernel modules",
    ("driver", "kernelModuleType"): "NVIDIA open kernel modules",
    ("driver", "useNvidiaDriverCRD"): "NVIDIADriver CRD",
    ("driver", "gpuDirectRDMA"): "use driver.rdma",
    ("toolkit", "cudaVersion"): "CUDA only",
    ("validator", "cuda"): "renamed to validator.hip",
    ("gds", "*"): "GPUDirect Storage has no ROCm equivalent (field accepted, never deployed)",
}


def _rehome(v):
    if isinstance(v, str):
        return v.replace("nvidia.com/", "amd.com/").replace("NVIDIA_", "AMD_")
    if isinstance(v, list):
        return [_rehome(x) for x in v]
    if isinstance(v, dict):
        return {_rehome(k): _rehome(x) for k, x in v.items()}
    return v


def convert(obj: Dict) -> Tuple[Dict, List[str]]:
    if obj.get("kind") != cp.KIND:
        raise ConfigError(f"not a ClusterPolicy: {obj.get('kind')}")
    notes: List[str] = []
    spec = copy.deepcopy(obj.get("spec") or {})
    out_spec: Dict = {}
    for k, v in spec.items():
        nk = SECTION_RENAMES.get(k, k)
        if nk != k:
            notes.append(f"spec.{k} -> spec.{nk}")
        out_spec[nk] = v
    for (sec, key), why in DROPPED.items():
        s = out_spec.get(sec)
        if not isinstance(s, dict):
            continue
        if key == "*":
            if s.get("enabled"):
                notes.append(f"spec.{sec}: {why}")
            continue
        if key in s:
            val = s.pop(key)
            if (sec, key) == ("validator", "cuda"):
                s["hip"] = val
            notes.append(f"spec.{sec}.{key}: {why}")
    # images point at NVIDIA registries: drop them so the operator's *_IMAGE defaults apply
    for sec, s in out_spec.items():
        if isinstance(s, dict) and "repository" in s and "nvidia" in str(s.get("repository", "")):
            for k in ("repository", "image", "version"):
                s.pop(k, None)
            notes.append(f"spec.{sec}: NVIDIA image removed (operator default applies)")
    if isinstance(out_spec.get("operator"), dict) and out_spec["operator"].get("runtimeClass") == "nvidia":
        out_spec["operator"]["runtimeClass"] = "amd"
    out = {"apiVersion": cp.API_VERSION, "kind": cp.KIND,
           "metadata": {"name": (obj.get("metadata") or {}).get("name", "cluster-policy")},
           "spec": _rehome(out_spec)}
    try:
        cp.ClusterPolicy(out, strict=False)
    except ValidationError as e:
        raise ConfigError(f"converted policy does not validate: {e}") from e
    return out, notes


# ---------------------------------------------------------------------------------------------
def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="amd-gpuop-cfg")
    sub = ap.add_subparsers(dest="cmd", required=True)
    v = sub.add_parser("validate").add_subparsers(dest="what", required=True)
    vc = v.add_parser("clusterpolicy")
    vc.add_argument("--input", help="ClusterPolicy YAML (default: render the Helm chart)")
    vc.add_argument("--chart", default=None)
    vc.add_argument("--values", default=None)
    vc.add_argument("--check-registry", action="store_true")
    vv = v.add_parser("csv")
    vv.add_argument("--input", required=True)
    vv.add_argument("--check-registry", action="store_true")
    cv = sub.add_parser("convert")
    cv.add_argument("--input", required=True)
    a = ap.parse_args(argv)
    try:
        if a.cmd == "validate" and a.what == "clusterpolicy":
            obj, env = load_clusterpolicy(a.input, a.chart, a.values)
            rep = validate_clusterpolicy(obj, env, a.check_registry)
            print(json.dumps(rep, indent=2))
        elif a.cmd == "validate":
            with open(a.input) as f:
                csv = yaml.safe_load(f)
            print(json.dumps(validate_csv(csv, a.check_registry), indent=2))
        else:
            with open(a.input) as f:
                obj = yaml.safe_load(f)
            out, notes = convert(obj)
            for n in notes:
                print(f"# {n}", file=sys.stderr)
            print(yaml.safe_dump(out, sort_keys=False))
    except (ConfigError, OSError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
