#!/bin/bash
# Interleaved A/B of this tree against another checkout in the tree (e.g. ab_r02/, a worktree of an
# earlier round with its own built library) on one box: the same bench.py command in each.
#   TREES=". ab_r02" ARGS="--layout gpt2s --total-clients 128 --in-dtype float16" REPS=3 bash scripts/gpu_ab_tree.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abtree
for rep in $(seq 1 ${REPS:-3}); do
  for t in ${TREES:-. ab_r02}; do
    tag=$(echo "$t" | tr -c 'a-zA-Z0-9' '_')
    (cd "$t" && timeout -k 10 300 python bench.py --no-cpu-baseline --no-probe --steps ${STEPS:-10} --warmup 3 ${ARGS:-}) \
      > gpurun_out/abtree/${tag}_$rep.log 2>&1 || { echo "$t failed rc=$?"; tail -20 gpurun_out/abtree/${tag}_$rep.log; exit 1; }
    echo "$t $rep $(grep '^{' gpurun_out/abtree/${tag}_$rep.log | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r.get("mean_launch_ms"), r.get("achieved"), r.get("frac"))')"
  done
done
