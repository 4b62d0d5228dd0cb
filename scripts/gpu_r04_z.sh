#!/bin/bash
# Round 4 end: the ring as its own kernel instantiation (split) vs one kernel with both paths
# (joint), then the whole GPU suite, smoke and the default bench line on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
VARIANTS="split joint" REPS=3 bash scripts/gpu_ab_pers.sh > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
cat $O/ab.txt
bash scripts/gpu_r04_u.sh || exit 1
