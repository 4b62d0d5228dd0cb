#!/bin/bash
# Round 4: fused own-window peer exchange validation (scripts/gpu_r04_i.sh) + PersonalizedFedAVG
# ring addressing A/B (pold: per-client index arithmetic, pnew = shipped: incremental).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_r04_i.sh || exit 1
O=gpurun_out/r04j
mkdir -p $O
cp distributed_learning_simulation_lib_amd/_lib/libfedavg_hip.so distributed_learning_simulation_lib_amd/_lib/variants/lib_pnew.so
B="python scripts/bench_personalized.py --steps 10 --warmup 3 --no-probe"
echo "== int (ring)" > $O/pers_ab.txt
VARIANTS="pold pnew" REPS=3 CMD="$B --weights int" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
cat $O/pers_ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_personalized.py "tests/test_gpu_geometry.py::test_personalized_kernel_edges_bit_identical" > $O/pytest_pers.log 2>&1 || { echo "pers tests failed"; tail -30 $O/pytest_pers.log; exit 1; }
tail -1 $O/pytest_pers.log
echo done
