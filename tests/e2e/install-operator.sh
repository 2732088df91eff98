#!/usr/bin/env bash
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
$HELM upgrade --install amd-gpu-operator "$CHART" -n "$NAMESPACE" --create-namespace --wait \
  --set operator.repository="$REGISTRY" --set operator.version="$VERSION" "$@"
