#!/bin/bash
# Where the validator's HIP step spends its time on this box: interpreter start, the GEMM probe
# binary (with / without clock stabilisation), the whole `amd-validator --component hip` (local).
# Usage (repo root, on the box): bash tools/ttr_breakdown.sh > gpurun_out/<dir>/breakdown.txt
set -eo pipefail
B=gpu_operator_amd/_native/bin
TIMEFORMAT='%R s'
for i in 1 2 3; do echo -n "python -c pass: "; { time python -c pass; } 2>&1; done
for i in 1 2 3; do echo -n "import validator.main + k8s.rest: "; { time python -c "import gpu_operator_amd.validator.main, gpu_operator_amd.k8s.rest"; } 2>&1; done
for i in 1 2; do echo -n "amd-hip-smoke: "; { time timeout -k 5 60 $B/amd-hip-smoke > /dev/null; } 2>&1; done
for i in 1 2; do echo -n "gemm-validate --smoke 8192 (stabilised, 50 iters): "; { time timeout -k 5 60 $B/amd-gemm-validate --smoke --shapes 8192 > /dev/null; } 2>&1; done
for i in 1 2; do echo -n "gemm-validate 8192 --no-stabilise --iters 5: "; { time timeout -k 5 60 $B/amd-gemm-validate --shapes 8192 --no-stabilise --iters 5 --warmup 1 > /dev/null; } 2>&1; done
for i in 1 2; do echo -n "gemm-validate 1024 --no-stabilise --iters 1: "; { time timeout -k 5 60 $B/amd-gemm-validate --shapes 1024 --no-stabilise --iters 1 --warmup 0 > /dev/null; } 2>&1; done
mkdir -p /tmp/ttrb
for i in 1 2; do echo -n "amd-validator --component hip (local, 8192): "; { time HIP_VALIDATION_MODE=local GEMM_SHAPES=8192 OUTPUT_DIR=/tmp/ttrb timeout -k 5 120 python -m gpu_operator_amd.cmd.entry amd-validator --component hip > /tmp/ttrb/hip.log 2>&1; } 2>&1; done
grep -o '"seconds": [0-9.]*' /tmp/ttrb/hip.log || true
