#!/usr/bin/env bash
# Reusable assertions (reference counterpart: tests/scripts/checks.sh).
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"

wait_ds_ready() {           # wait_ds_ready <app label>
  local app=$1
  echo "waiting for DaemonSet app=$app"
  for _ in $(seq 1 90); do
    if $K -n "$NAMESPACE" get ds -l app="$app" -o name | grep -q .; then break; fi
    sleep 2
  done
  $K -n "$NAMESPACE" rollout status ds -l app="$app" --timeout="$READY_TIMEOUT"
}

check_pod_ready() {         # check_pod_ready <app label>
  $K -n "$NAMESPACE" wait pod -l app="$1" --for=condition=Ready --timeout="$READY_TIMEOUT"
}

check_clusterpolicy_ready() {
  $K wait clusterpolicies.amd.com/cluster-policy --for=jsonpath='{.status.state}'=ready --timeout="$READY_TIMEOUT"
}

check_no_restarts() {       # operand restart count <= 1 (reference: verify-operand-restarts.sh)
  local bad
  bad=$($K -n "$NAMESPACE" get pods -o jsonpath='{range .items[*]}{.metadata.name}{" "}{range .status.containerStatuses[*]}{.restartCount}{" "}{end}{"\n"}{end}' \
        | awk '{for(i=2;i<=NF;i++) if ($i>1) print $1}')
  if [ -n "$bad" ]; then echo "pods restarted more than once: $bad"; return 1; fi
}

check_gpu_capacity() {      # amd.com/gpu capacity on the node >= $1
  local node want have
  want=${1:-8}
  node=$($K get nodes -l amd.com/gpu.present=true -o jsonpath='{.items[0].metadata.name}')
  have=$($K get node "$node" -o jsonpath='{.status.capacity.amd\.com/gpu}')
  echo "node $node amd.com/gpu=$have (want >= $want)"
  [ "${have:-0}" -ge "$want" ]
}

run_gpu_pod() {             # a HIP GEMM workload pod on N GPUs must succeed
  local n=${1:-1}
  $K -n "$NAMESPACE" delete pod e2e-gemm --ignore-not-found --wait
  cat <<YAML | $K -n "$NAMESPACE" apply -f -
apiVersion: v1
kind: Pod
metadata:
  name: e2e-gemm
spec:
  restartPolicy: Never
  tolerations: [{key: amd.com/gpu, operator: Exists, effect: NoSchedule}]
  containers:
  - name: gemm
    image: $REGISTRY/amd-gpu-operator-node:$VERSION
    command: [amd-gemm-validate, --shapes, "8192", --iters, "20"]
    resources: {limits: {amd.com/gpu: $n}}
YAML
  $K -n "$NAMESPACE" wait pod/e2e-gemm --for=jsonpath='{.status.phase}'=Succeeded --timeout=600s
  $K -n "$NAMESPACE" logs e2e-gemm | tail -3
}

test_operator_restart() {   # kill the operator; it must be Running again within 100 s
  local pod
  pod=$($K -n "$NAMESPACE" get pods -l app=amd-gpu-operator -o jsonpath='{.items[0].metadata.name}')
  $K -n "$NAMESPACE" delete pod "$pod" --wait=false
  for _ in $(seq 1 20); do
    sleep 5
    if $K -n "$NAMESPACE" get pods -l app=amd-gpu-operator -o jsonpath='{.items[0].status.phase}' | grep -q Running; then
      echo "operator recovered"; return 0
    fi
  done
  echo "operator did not recover within 100 s"; return 1
}

node_time_to_ready() {      # validator-exported time-to-ready of the GPU node
  local pod
  pod=$($K -n "$NAMESPACE" get pods -l app=amd-operator-validator -o jsonpath='{.items[0].metadata.name}')
  $K -n "$NAMESPACE" exec "$pod" -c amd-operator-validator -- sh -c \
    'wget -qO- localhost:${METRICS_PORT:-8000}/metrics 2>/dev/null | grep -E "time_to_ready|gemm_tflops|allreduce"' || true
}
