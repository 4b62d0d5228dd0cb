#!/bin/bash
# rocprofv3 kernel stats + the bench line for config 2 with fp64 inputs and fp64 output
# (what AggregationWorker sends, aggregation_worker.py:152); run on the GPU box from the repo root.
# (profiles/ written on the box does not come back: copy gpurun_out/prof_<tag>_f64/{trace/run_kernel_stats.csv,bench_trace.log} into profiles/ locally)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}_f64
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --in-dtype float64 --out-dtype float64 > $OUT/bench_trace.log 2>&1 || { echo "f64 trace pass failed"; tail -20 $OUT/bench_trace.log; exit 1; }
cp $OUT/trace/run_kernel_stats.csv profiles/${TAG}_f64_kernel_stats.csv
grep -h "^{\"metric\"" $OUT/bench_trace.log > profiles/${TAG}_f64_bench.json
head -3 profiles/${TAG}_f64_kernel_stats.csv
