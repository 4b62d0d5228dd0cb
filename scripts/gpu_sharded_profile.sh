#!/bin/bash
# rocprof kernel stats + timeline of the sharded path on one GPU (forced 1-rank RCCL, native round).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
C=${1:-4}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof_c${C} -o run -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --force-collective --chunks $C \
  > gpurun_out/sprof_c${C}.log 2>&1
