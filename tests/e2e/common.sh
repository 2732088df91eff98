#!/usr/bin/env bash
# Shared settings for the single-node (8x MI355X) end-to-end flow.
set -euo pipefail
export NAMESPACE=${NAMESPACE:-amd-gpu-operator}
export CHART=${CHART:-$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)/deployments/amd-gpu-operator}
export HELM=${HELM:-helm}
export K=${KUBECTL:-kubectl}
export REGISTRY=${REGISTRY:-registry.example.com/amd}
export VERSION=${VERSION:-v0.1.0}
# event-driven waits with generous ceilings (the reference waits 45 min per operand)
export READY_TIMEOUT=${READY_TIMEOUT:-900s}
