#!/bin/bash
# Round 4, first GPU pass: the new multi-device tests + the staging regression test, then the
# headline traffic refresh (profile.sh r04) and the PersonalizedFedAVG PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multi_device.py "tests/test_gpu_staging.py::test_delta_first_round_then_reordered_full_update" > $O/pytest_multi.log 2>&1 || { echo "multi tests failed rc=$?"; tail -60 $O/pytest_multi.log; exit 1; }
tail -3 $O/pytest_multi.log
bash scripts/profile.sh r04 > $O/profile.log 2>&1 || { echo "profile failed"; tail -20 $O/profile.log; exit 1; }
tail -5 $O/profile.log
bash scripts/gpu_pers_pmc.sh > $O/pers_pmc.log 2>&1 || { echo "pers pmc failed"; tail -20 $O/pers_pmc.log; exit 1; }
echo done
