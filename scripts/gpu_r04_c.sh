#!/bin/bash
# Round 4: PersonalizedFedAVG split-weight pipeline A/B (ps1 = shipped build, ps0 = PERS_SPLIT=0)
# and the PMC passes of both builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
cp distributed_learning_simulation_lib_amd/_lib/libfedavg_hip.so distributed_learning_simulation_lib_amd/_lib/variants/lib_ps1.so
for w in int float; do
  echo "== personalized $w" >> $O/pers_ab.txt
  VARIANTS="ps1 ps0" REPS=2 CMD="python scripts/bench_personalized.py --steps 10 --warmup 3 --no-probe --weights $w" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { echo "pers ab failed"; cat $O/pers_ab.txt; exit 1; }
done
cat $O/pers_ab.txt
TAG=ps1 bash scripts/gpu_pers_pmc.sh > $O/pers_pmc_ps1.log 2>&1 || { echo "pers pmc ps1 failed"; tail -20 $O/pers_pmc_ps1.log; exit 1; }
TAG=ps0 FEDAVG_HIP_LIB=distributed_learning_simulation_lib_amd/_lib/variants/lib_ps0.so bash scripts/gpu_pers_pmc.sh > $O/pers_pmc_ps0.log 2>&1 || { echo "pers pmc ps0 failed"; tail -20 $O/pers_pmc_ps0.log; exit 1; }
echo done
