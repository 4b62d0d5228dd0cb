#!/bin/bash
# Same-box interleaved A/B of the round-1 tree (ab_r01/: `git archive 600809e`, built in place)
# against HEAD on the headline workload (64 x ResNet-18 fp32 -> fp32). Each side runs its own
# bench.py with its own library; REPS alternations, kernel ms from each side's HIP events.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_r01
REPS=${REPS:-4}
ARGS=${ARGS:---steps 50 --warmup 10 --no-cpu-baseline --no-probe}
for rep in $(seq 1 $REPS); do
  for side in r01 head; do
    if [ $side = r01 ]; then dir=ab_r01; else dir=.; fi
    (cd $dir && timeout -k 10 180 python bench.py $ARGS) > gpurun_out/ab_r01/${side}_$rep.log 2>&1 || { echo "$side failed rc=$?"; tail -20 gpurun_out/ab_r01/${side}_$rep.log; exit 1; }
    echo "$side $rep $(grep '^{' gpurun_out/ab_r01/${side}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r["achieved"], r["frac"])')"
  done
done
