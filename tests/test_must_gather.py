"""hack/must-gather.sh against a stub kubectl on PATH that records its argv (VERDICT r2 item 6;
reference: hack/must-gather.sh:38-43,84-116,247)."""

import os
import subprocess

from gpu_operator_amd.controllers import upgrade as U

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "hack", "must-gather.sh")

STUB = r'''#!/bin/bash
echo "$*" >> "$KUBECTL_LOG"
case "$*" in
  *"get clusterversion/version --ignore-not-found -o name"*) echo "clusterversion.config.openshift.io/version" ;;
  *"get clusterversion/version -o yaml"*) echo "kind: ClusterVersion" ;;
  *"get pods -A -l app=amd-gpu-operator"*) printf 'amd-gpu-operator/amd-gpu-operator-7d9f' ;;
  *"get clusterpolicies.amd.com -o name"*) echo "clusterpolicy.amd.com/cluster-policy" ;;
  *"get nodes -l feature.node.kubernetes.io/pci-1002.present -o name"*) printf 'node/gpu-a\nnode/gpu-b\n' ;;
  *"get nodes -l feature.node.kubernetes.io/pci-1200_1002.present -o name"*) printf 'node/gpu-b\n' ;;
  *"get nodes -l amd.com/gpu.present=true -o name"*) echo "node/gpu-a" ;;
  *"get node/gpu-b -o jsonpath"*) printf '{"feature.node.kubernetes.io/pci-1002.present":"true"}' ;;
  *"get pods -l amd.com/precompiled -o name"*) echo "pod/amdgpu-driver-daemonset-6.8.0-45-generic-x1" ;;
  *"get pods -l openshift.driver-toolkit -o name"*) echo "pod/amdgpu-driver-daemonset-rhcos-9.4-y2" ;;
esac
exit 0
'''


def test_must_gather_collects_parity_items(tmp_path):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    (bindir / "kubectl").write_text(STUB)
    (bindir / "kubectl").chmod(0o755)
    log = tmp_path / "kubectl.argv"
    out = tmp_path / "bundle"
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", KUBECTL_LOG=str(log), ARTIFACT_DIR=str(out))
    p = subprocess.run(["bash", SCRIPT], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    calls = log.read_text().splitlines()
    # the upgrade events: the same reason the FSM emits
    ev = [c for c in calls if "get events -A --field-selector" in c]
    assert ev == [f"get events -A --field-selector reason={U.EVENT_REASON}"]
    # OpenShift: cluster version + machines
    assert (out / "openshift_version.yaml").read_text().strip() == "kind: ClusterVersion"
    assert "get machines -A" in calls
    # nodes with the vendor PCI label, adopted or not (gpu-b has no amd.com/gpu.present)
    labels = (out / "gpu_pci_nodes.labels").read_text()
    assert "gpu-a" in labels and "gpu-b" in labels and "pci-1002.present" in labels
    # precompiled and driver-toolkit driver pods get node reports too
    execs = [c for c in calls if " exec " in f" {c} "]
    assert any("amdgpu-driver-daemonset-6.8.0-45-generic-x1" in c for c in execs)
    assert any("amdgpu-driver-daemonset-rhcos-9.4-y2" in c for c in execs)
    assert (out / "clusterpolicy.yaml").exists()
