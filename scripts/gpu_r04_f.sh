#!/bin/bash
# Round 4: PersonalizedFedAVG ring-loop A/B for integer weights (pr0: one wait per client, pr1 =
# shipped: halves, pr2: next client ahead), then the plugin early-wave exploration.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
cp distributed_learning_simulation_lib_amd/_lib/libfedavg_hip.so distributed_learning_simulation_lib_amd/_lib/variants/lib_pr1.so
B="python scripts/bench_personalized.py --steps 10 --warmup 3 --no-probe"
echo "== int (ring)" > $O/pers_ab.txt
VARIANTS="pr0 pr1 pr2" REPS=2 CMD="$B --weights int" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
echo "== float" >> $O/pers_ab.txt
VARIANTS="pr1" REPS=2 CMD="$B --weights float" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
cat $O/pers_ab.txt
bash scripts/gpu_r04_plugin.sh
