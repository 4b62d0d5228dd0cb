#!/bin/bash
# Interleaved A/B of an environment knob on one box: ENVS="A=1;A=2" ARGS="bench args" REPS=2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abenv
IFS=';' read -ra E <<< "$ENVS"
for rep in $(seq 1 ${REPS:-2}); do
  for e in "${E[@]}"; do
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-probe $ARGS > gpurun_out/abenv/run.log 2>&1 || { echo "$e failed"; tail -20 gpurun_out/abenv/run.log; exit 1; }
    echo "$e rep $rep: $(grep '^{' gpurun_out/abenv/run.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r["achieved"], r["frac"])')"
  done
done
