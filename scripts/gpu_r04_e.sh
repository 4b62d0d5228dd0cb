#!/bin/bash
# Round 4: PersonalizedFedAVG A/B — ps1 (split weights, round-4 first cut) vs psn (shipped: products
# before sums, ring compiled out of the separately rounded fold, 3 waves/SIMD), int weights with the
# LDS ring and with the register pipeline (FEDAVG_PERS_RING=0); then the profile/QSGD pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
cp distributed_learning_simulation_lib_amd/_lib/libfedavg_hip.so distributed_learning_simulation_lib_amd/_lib/variants/lib_psn.so
B="python scripts/bench_personalized.py --steps 10 --warmup 3 --no-probe"
echo "== int (ring)" > $O/pers_ab.txt
VARIANTS="ps1 psn" REPS=2 CMD="$B --weights int" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
echo "== int (register pipeline)" >> $O/pers_ab.txt
VARIANTS="ps1 psn" REPS=2 CMD="env FEDAVG_PERS_RING=0 $B --weights int" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
echo "== float" >> $O/pers_ab.txt
VARIANTS="ps1 psn" REPS=2 CMD="$B --weights float" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
cat $O/pers_ab.txt
bash scripts/gpu_r04_d.sh
