#!/usr/bin/env bash
# Debug bundle for the AMD GPU operator (reference counterpart: hack/must-gather.sh).
# Collects the ClusterPolicy, GPU node labels/status, operator and operand pods (yaml, describe,
# logs incl. previous), DaemonSets, events, and from every driver/validator pod: amd-smi and
# rocm-smi reports, the KFD topology, partition modes and the validation barrier files.
#   ARTIFACT_DIR=/tmp/amd-must-gather hack/must-gather.sh
set -o nounset
set -o pipefail

K=${KUBECTL:-kubectl}
if ! command -v "$K" >/dev/null 2>&1; then
  echo "FATAL: kubectl not found" >&2
  exit 1
fi
ARTIFACT_DIR=${ARTIFACT_DIR:-/tmp/amd-gpu-operator-must-gather_$(date +%Y%m%d_%H%M)}
mkdir -p "$ARTIFACT_DIR"
exec 1> >(tee "$ARTIFACT_DIR/must-gather.log") 2> "$ARTIFACT_DIR/must-gather.stderr.log"

# the upgrade state machine's event reason (gpu_operator_amd/controllers/upgrade.py EVENT_REASON;
# tests/test_must_gather.py checks the two agree)
UPGRADE_EVENT_REASON=${UPGRADE_EVENT_REASON:-AMDGPUDriverUpgrade}
# NFD labels that mark a node with an AMD GPU, adopted or not (controllers/consts.py GPU_NODE_LABELS)
GPU_PCI_LABELS=(feature.node.kubernetes.io/pci-1002.present feature.node.kubernetes.io/pci-0300_1002.present
                feature.node.kubernetes.io/pci-0380_1002.present feature.node.kubernetes.io/pci-1200_1002.present)

echo "# collecting into $ARTIFACT_DIR"
if [ "$0" = "/usr/bin/gather" ]; then
  printf 'AMD GPU Operator\n%s\n' "${VERSION:-N/A}" > "$ARTIFACT_DIR/version"
fi
$K version -o yaml > "$ARTIFACT_DIR/kubectl_version.yaml" 2>&1

OCP=$($K get clusterversion/version --ignore-not-found -o name 2>/dev/null || true)
if [ -n "$OCP" ]; then
  echo "# OpenShift: cluster version and machines"
  $K get clusterversion/version -o yaml > "$ARTIFACT_DIR/openshift_version.yaml"
  $K get machines -A > "$ARTIFACT_DIR/all_machines.list" 2>&1 || true
fi

OPERATOR_POD=$($K get pods -A -l app=amd-gpu-operator -o jsonpath='{.items[0].metadata.namespace}/{.items[0].metadata.name}' 2>/dev/null)
NS=${OPERATOR_NAMESPACE:-${OPERATOR_POD%%/*}}
if [ -z "$NS" ]; then
  echo "WARNING: operator pod not found; using namespace amd-gpu-operator"
  NS=amd-gpu-operator
fi
echo "# operator namespace: $NS"

echo "# ClusterPolicy"
if [ -n "$($K get clusterpolicies.amd.com -o name 2>/dev/null)" ]; then
  $K get clusterpolicies.amd.com -o yaml > "$ARTIFACT_DIR/clusterpolicy.yaml"
else
  touch "$ARTIFACT_DIR/clusterpolicy.missing"
fi

# every node NFD reports with an AMD GPU -- including the ones the operator did not adopt
# (no amd.com/gpu.present label), which is usually what is being debugged
echo "# nodes with AMD PCI labels"
pci_nodes=""
for label in "${GPU_PCI_LABELS[@]}"; do
  pci_nodes="$pci_nodes $($K get nodes -l "$label" -o name 2>/dev/null)"
done
: > "$ARTIFACT_DIR/gpu_pci_nodes.labels"
for node in $(echo "$pci_nodes" | tr ' ' '\n' | sort -u); do
  echo "${node#node/}" >> "$ARTIFACT_DIR/gpu_pci_nodes.labels"
  $K get "$node" -o jsonpath='{.metadata.labels}' | tr ',' '\n' >> "$ARTIFACT_DIR/gpu_pci_nodes.labels"
  echo >> "$ARTIFACT_DIR/gpu_pci_nodes.labels"
done

echo "# GPU nodes"
$K get nodes -l amd.com/gpu.present=true -o wide > "$ARTIFACT_DIR/gpu_nodes.txt"
$K get nodes -l amd.com/gpu.present=true -o yaml > "$ARTIFACT_DIR/gpu_nodes.yaml"
for node in $($K get nodes -l amd.com/gpu.present=true -o name); do
  n=${node#node/}
  $K describe node "$n" > "$ARTIFACT_DIR/node_${n}.describe"
  $K get node "$n" -o jsonpath='{.metadata.labels}' | tr ',' '\n' | grep 'amd.com' > "$ARTIFACT_DIR/node_${n}.amd_labels" || true
done

echo "# operator"
if [ -n "${OPERATOR_POD:-}" ]; then
  p=${OPERATOR_POD#*/}
  $K -n "$NS" get pod "$p" -o yaml > "$ARTIFACT_DIR/operator_pod.yaml"
  $K -n "$NS" logs "$p" --all-containers > "$ARTIFACT_DIR/operator_pod.log"
  $K -n "$NS" logs "$p" --all-containers --previous > "$ARTIFACT_DIR/operator_pod.previous.log" 2>/dev/null || true
fi

echo "# operands"
$K -n "$NS" get all -o wide > "$ARTIFACT_DIR/namespace_all.txt"
$K -n "$NS" get ds -o yaml > "$ARTIFACT_DIR/daemonsets.yaml"
$K -n "$NS" get events --sort-by=.lastTimestamp > "$ARTIFACT_DIR/events.txt"
$K get events -A --field-selector "reason=$UPGRADE_EVENT_REASON" > "$ARTIFACT_DIR/upgrade_events.txt" 2>/dev/null || true
for pod in $($K -n "$NS" get pods -o name); do
  p=${pod#pod/}
  $K -n "$NS" get pod "$p" -o yaml > "$ARTIFACT_DIR/pod_${p}.yaml"
  $K -n "$NS" describe pod "$p" > "$ARTIFACT_DIR/pod_${p}.describe"
  $K -n "$NS" logs "$p" --all-containers --prefix > "$ARTIFACT_DIR/pod_${p}.log" 2>&1
  $K -n "$NS" logs "$p" --all-containers --prefix --previous > "$ARTIFACT_DIR/pod_${p}.previous.log" 2>/dev/null || true
done

echo "# node reports (amd-smi / rocm-smi / KFD topology / barriers)"
# driver pods of every flavour (DKMS, precompiled per kernel, OpenShift driver-toolkit) and validators
node_pods=$( { $K -n "$NS" get pods -l 'app in (amdgpu-driver-daemonset,amd-operator-validator)' -o name;
               $K -n "$NS" get pods -l amd.com/precompiled -o name;
               $K -n "$NS" get pods -l openshift.driver-toolkit -o name; } 2>/dev/null | sort -u)
for pod in $node_pods; do
  p=${pod#pod/}
  out="$ARTIFACT_DIR/node_report_${p}.txt"
  {
    echo "== amd-smi static/metric"
    $K -n "$NS" exec "$p" -- sh -c 'amd-smi static 2>&1; amd-smi metric 2>&1; amd-smi xgmi 2>&1' || true
    echo "== rocm-smi"
    $K -n "$NS" exec "$p" -- sh -c 'rocm-smi --showallinfo 2>&1' || true
    echo "== amd-node-probe (KFD topology, partitions, driver state)"
    $K -n "$NS" exec "$p" -- sh -c 'amd-node-probe --root /host 2>&1 || amd-node-probe 2>&1' || true
    echo "== barriers"
    $K -n "$NS" exec "$p" -- sh -c 'for f in /run/amd/validations/*; do echo "$f: $(cat $f)"; done' || true
    echo "== dmesg (amdgpu)"
    $K -n "$NS" exec "$p" -- sh -c 'dmesg 2>/dev/null | grep -i -E "amdgpu|kfd|gim" | tail -200' || true
  } > "$out" 2>&1
done

echo "# done: $ARTIFACT_DIR"
