#!/bin/bash
# Round 4: PersonalizedFedAVG epilogue reciprocals from the host (prcp = shipped) against the
# previous build (pinc) and 8-client ring stages (psc8), integer and float weights; then the
# personalized parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
cp distributed_learning_simulation_lib_amd/_lib/libfedavg_hip.so distributed_learning_simulation_lib_amd/_lib/variants/lib_prcp.so
B="python scripts/bench_personalized.py --steps 10 --warmup 3 --no-probe"
: > $O/pers_ab.txt
for w in int float; do
  echo "== $w" >> $O/pers_ab.txt
  VARIANTS="pinc prcp psc8" REPS=3 CMD="$B --weights $w" bash scripts/gpu_ab.sh >> $O/pers_ab.txt 2>&1 || { cat $O/pers_ab.txt; exit 1; }
done
cat $O/pers_ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_personalized.py "tests/test_gpu_geometry.py::test_personalized_kernel_edges_bit_identical" > $O/pytest_pers.log 2>&1 || { echo "pers tests failed"; tail -30 $O/pytest_pers.log; exit 1; }
tail -1 $O/pytest_pers.log
echo done
