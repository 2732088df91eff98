#!/usr/bin/env bash
# Full single-node flow on an 8x MI355X node (reference: tests/scripts/end-to-end.sh).
source "$(dirname "${BASH_SOURCE[0]}")/checks.sh"
here=$(dirname "${BASH_SOURCE[0]}")
t0=$(date +%s)
"$here/install-operator.sh" --set driver.enabled="${DRIVER_ENABLED:-false}"
"$here/verify-operator.sh"
echo "install -> ready: $(( $(date +%s) - t0 )) s"
check_no_restarts
run_gpu_pod 1
run_gpu_pod 8
"$here/update-clusterpolicy.sh"
test_operator_restart
echo "== disable all operands on the node, then re-enable"
node=$($K get nodes -l amd.com/gpu.present=true -o jsonpath='{.items[0].metadata.name}')
$K label node "$node" amd.com/gpu.deploy.operands=false --overwrite
sleep 30
$K label node "$node" amd.com/gpu.deploy.operands-
"$here/verify-operator.sh"
echo "== uninstall / reinstall with sandbox workloads enabled"
$HELM uninstall amd-gpu-operator -n "$NAMESPACE" --wait
"$here/install-operator.sh" --set sandboxWorkloads.enabled=true --set sandboxWorkloads.defaultWorkload=container
"$here/verify-operator.sh"
run_gpu_pod 1
$HELM uninstall amd-gpu-operator -n "$NAMESPACE" --wait
echo "e2e passed in $(( $(date +%s) - t0 )) s"
