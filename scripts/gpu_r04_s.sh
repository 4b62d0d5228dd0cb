#!/bin/bash
# Round 4: PersonalizedFedAVG after the immediate vmcnt waits — parity, bench lines (int / float
# weights, 64 x 64 x ResNet-18) and a rocprofv3 kernel-trace summary of the integer-weight round.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_personalized.py tests/test_gpu_division_edges.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pers.log 2>&1 || { tail -40 $O/pytest_pers.log; exit 1; }
tail -1 $O/pytest_pers.log
: > $O/bench.jsonl
for w in int float int float; do
  timeout -k 10 300 python bench.py --workload personalized --pers-weights $w --steps 10 --warmup 3 --no-cpu-baseline --no-probe >> $O/bench.jsonl 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o pers --output-format csv -- python bench.py --workload personalized --pers-weights int --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
echo done
