#!/bin/bash
# Round 4: PersonalizedFedAVG plugin host overhead (round vs kernel, cProfile of one round).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04v}
mkdir -p $O
timeout -k 10 300 python scripts/plugin_pers_bench.py > $O/plugin_pers.txt 2>&1 || { tail -30 $O/plugin_pers.txt; exit 1; }
head -40 $O/plugin_pers.txt
