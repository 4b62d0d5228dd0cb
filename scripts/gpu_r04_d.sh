#!/bin/bash
# Round 4: headline traffic refresh (profile.sh r04) and the QSGD XCD placement A/B + PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
bash scripts/profile.sh r04 > $O/profile.log 2>&1 || { echo "profile failed"; tail -20 $O/profile.log; exit 1; }
tail -3 $O/profile.log
cp distributed_learning_simulation_lib_amd/_lib/libfedavg_hip.so distributed_learning_simulation_lib_amd/_lib/variants/lib_qxs1.so
VARIANTS="qxs1 qxs0" REPS=3 CMD="python bench.py --workload qsgd --steps 20 --warmup 5 --no-probe --no-cpu-baseline" bash scripts/gpu_ab.sh > $O/qsgd_ab.txt 2>&1 || { echo "qsgd ab failed"; cat $O/qsgd_ab.txt; exit 1; }
cat $O/qsgd_ab.txt
bash scripts/gpu_qsgd_pmc.sh > $O/qsgd_pmc.log 2>&1 || { echo "qsgd pmc failed"; tail -20 $O/qsgd_pmc.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-include-regex qsgd --pmc FETCH_SIZE -d $O/qfetch -o run --output-format csv -- python3 bench.py --workload qsgd --steps 3 --warmup 1 --no-probe --no-cpu-baseline > $O/qfetch.log 2>&1 || { echo "qsgd fetch failed"; tail -20 $O/qfetch.log; exit 1; }
echo done
