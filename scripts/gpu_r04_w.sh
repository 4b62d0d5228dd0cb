#!/bin/bash
# Round 4: PersonalizedFedAVG plugin after the flat-output launch / result-buffer reuse —
# personalized parity, then the plugin round timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_personalized.py tests/test_gpu_division_edges.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pers.log 2>&1 || { tail -40 $O/pytest_pers.log; exit 1; }
tail -1 $O/pytest_pers.log
timeout -k 10 300 python scripts/plugin_pers_bench.py > $O/plugin_pers.txt 2>&1 || { tail -30 $O/plugin_pers.txt; exit 1; }
head -30 $O/plugin_pers.txt
