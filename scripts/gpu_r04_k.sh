#!/bin/bash
# Round 4: float-weight A/B of the register pipeline's incremental weight rows (pold / pnew) and
# the plugin's per-update host profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
cp distributed_learning_simulation_lib_amd/_lib/libfedavg_hip.so distributed_learning_simulation_lib_amd/_lib/variants/lib_pnew.so
B="python scripts/bench_personalized.py --steps 10 --warmup 3 --no-probe"
echo "== float" > $O/pers_ab.txt
VARIANTS="pold pnew" REPS=3 CMD="$B --weights float" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
cat $O/pers_ab.txt
timeout -k 10 300 python scripts/plugin_host_profile.py > $O/host_profile.txt 2>&1 || { echo "host profile failed"; tail -20 $O/host_profile.txt; exit 1; }
head -40 $O/host_profile.txt
echo done
