#!/bin/bash
# PersonalizedFedAVG: bench lines (float and int weights) and a rocprofv3 kernel-stats summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pers_prof
for w in float int; do
timeout -k 10 300 python bench.py --workload personalized --pers-weights $w --steps 10 --warmup 2 > gpurun_out/pers_prof/bench_$w.log 2>&1 || { echo "bench $w failed rc=$?"; tail -20 gpurun_out/pers_prof/bench_$w.log; exit 1; }
tail -1 gpurun_out/pers_prof/bench_$w.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pers_prof/trace -o run --output-format csv -- python bench.py --workload personalized --pers-weights float --steps 10 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/pers_prof/prof.log 2>&1 || { echo "rocprof failed rc=$?"; tail -20 gpurun_out/pers_prof/prof.log; exit 1; }
find gpurun_out/pers_prof/trace -name "*kernel_stats.csv" -exec cat {} \;
