#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/tune_kernel.py run ${1:-64} ${2:-resnet} ${3:-float32} ${4:-0} > gpurun_out/tune_${2:-resnet}.log 2>&1 || { echo "tune failed"; tail -30 gpurun_out/tune_${2:-resnet}.log; exit 1; }
cat gpurun_out/tune_${2:-resnet}.log
