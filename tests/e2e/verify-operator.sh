#!/usr/bin/env bash
# Every operand ready, ClusterPolicy ready, GPUs advertised (reference: verify-operator.sh).
source "$(dirname "${BASH_SOURCE[0]}")/checks.sh"
check_pod_ready amd-gpu-operator
for app in amdgpu-driver-daemonset amd-container-toolkit-daemonset amd-device-plugin-daemonset \
           amd-node-labeller amd-metrics-exporter amd-operator-validator; do
  if $K get clusterpolicies.amd.com cluster-policy -o yaml | grep -q "driver:" && [ "$app" = amdgpu-driver-daemonset ] \
     && [ "$($K get clusterpolicies.amd.com cluster-policy -o jsonpath='{.spec.driver.enabled}')" = false ]; then
    continue
  fi
  wait_ds_ready "$app"
done
check_clusterpolicy_ready
check_gpu_capacity 8
node_time_to_ready
