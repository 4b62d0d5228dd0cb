#!/bin/bash
# A/B of library variants on one box: VARIANTS="a b" CMD="python scripts/bench_personalized.py ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
for v in $VARIANTS; do
FEDAVG_ALLOW_ABLATED=1 FEDAVG_HIP_LIB=distributed_learning_simulation_lib_amd/_lib/variants/lib_$v.so timeout -k 10 300 $CMD > gpurun_out/ab/${v}_$rep.log 2>&1 || { echo "$v failed rc=$?"; tail -20 gpurun_out/ab/${v}_$rep.log; exit 1; }
echo "$v $rep $(tail -1 gpurun_out/ab/${v}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; print(d.get("ms_per_step"), d.get("kernel_ms_per_step", r.get("kernel_ms_per_step")), r.get("achieved", ""), d.get("weights",""))')"
done
done
