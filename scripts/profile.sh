#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box from the repo root).
#   pass 1: kernel trace + stats (per-kernel durations)
#   pass 2/3: PMC FETCH_SIZE and WRITE_SIZE in separate passes (TCC slot limits; never combined
#             with any other trace domain)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/bench_trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/bench_trace.log; exit 1; }
echo trace ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- python3 $BENCH > $OUT/bench_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/bench_fetch.log; exit 1; }
echo fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- python3 $BENCH > $OUT/bench_write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/bench_write.log; exit 1; }
echo write ok
python3 scripts/summarize_profile.py $OUT $TAG
