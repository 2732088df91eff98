#!/usr/bin/env bash
# Day-2 changes (reference: tests/scripts/update-clusterpolicy.sh): env injection, time-slicing,
# partition mode change, operand disable/enable, custom DaemonSet labels.
source "$(dirname "${BASH_SOURCE[0]}")/checks.sh"
node=$($K get nodes -l amd.com/gpu.present=true -o jsonpath='{.items[0].metadata.name}')

echo "== env injection into the device plugin"
$K patch clusterpolicies.amd.com cluster-policy --type=json \
  -p='[{"op":"add","path":"/spec/devicePlugin/env/-","value":{"name":"E2E_MARKER","value":"1"}}]'
wait_ds_ready amd-device-plugin-daemonset
$K -n "$NAMESPACE" get ds amd-device-plugin-daemonset -o yaml | grep -q E2E_MARKER

echo "== time-slicing: 4 replicas per GPU"
cat <<YAML | $K -n "$NAMESPACE" apply -f -
apiVersion: v1
kind: ConfigMap
metadata: {name: e2e-plugin-config}
data:
  ts4: |
    version: v1
    sharing:
      timeSlicing:
        resources:
        - {name: amd.com/gpu, replicas: 4}
YAML
$K patch clusterpolicies.amd.com cluster-policy --type=merge \
  -p '{"spec":{"devicePlugin":{"config":{"name":"e2e-plugin-config","default":"ts4"}}}}'
wait_ds_ready amd-device-plugin-daemonset
sleep 10
check_gpu_capacity 32

echo "== compute partition change SPX -> CPX -> SPX"
$K label node "$node" amd.com/gpu.partition.config=all-cpx --overwrite
$K wait node "$node" --for=jsonpath='{.metadata.labels.amd\.com/gpu\.partition\.state}'=success --timeout=900s
check_gpu_capacity 64
$K label node "$node" amd.com/gpu.partition.config=spx-nps1 --overwrite
$K wait node "$node" --for=jsonpath='{.metadata.labels.amd\.com/gpu\.partition\.state}'=success --timeout=900s

echo "== disable / re-enable the metrics exporter"
$K patch clusterpolicies.amd.com cluster-policy --type=merge -p '{"spec":{"metricsExporter":{"enabled":false}}}'
$K -n "$NAMESPACE" wait ds -l app=amd-metrics-exporter --for=delete --timeout=300s || true
$K patch clusterpolicies.amd.com cluster-policy --type=merge -p '{"spec":{"metricsExporter":{"enabled":true}}}'
wait_ds_ready amd-metrics-exporter

echo "== custom DaemonSet labels"
$K patch clusterpolicies.amd.com cluster-policy --type=merge -p '{"spec":{"daemonsets":{"labels":{"e2e":"yes"}}}}'
sleep 10
$K -n "$NAMESPACE" get ds -l e2e=yes -o name | grep -q .
