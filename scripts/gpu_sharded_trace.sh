#!/bin/bash
# Kernel timeline of the sharded path on one GPU (forced 1-rank RCCL reduce), for gap analysis.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
C=${1:-4}
M=${2:-native}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/strace_c${C}_${M} -o trace -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe --force-collective --chunks $C --comm $M \
  > gpurun_out/strace_c${C}_${M}.log 2>&1
