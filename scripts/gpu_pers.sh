#!/bin/bash
# PersonalizedFedAVG on the GPU box: parity tests, then the bench (float and int weights).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_personalized.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pers.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_pers.log; exit 1; }
tail -3 gpurun_out/pytest_pers.log
for w in float int; do
timeout -k 10 300 python scripts/bench_personalized.py --weights $w ${PERS_ARGS:-} > gpurun_out/pers_$w.log 2>&1 || { echo "bench $w failed rc=$?"; tail -20 gpurun_out/pers_$w.log; exit 1; }
tail -1 gpurun_out/pers_$w.log
done
