#!/bin/bash
# Round 4: personalized static-vmcnt A/B (parity of both variants + interleaved timing), and the
# host breakdown of FedAvgContext.aggregate on 8- and 64-client tables.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 120 python scripts/plugin_call_breakdown.py > $O/call_breakdown.jsonl 2> $O/call_breakdown.err || { tail -20 $O/call_breakdown.err; exit 1; }
cat $O/call_breakdown.jsonl
VARIANTS="new old" REPS=4 bash scripts/gpu_ab_pers.sh > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
cat $O/ab.txt
echo done
if [ -n "$WITH_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o pers --output-format csv -- python bench.py --workload personalized --pers-weights int --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  find $O/prof -name "*kernel_stats.csv"
fi
