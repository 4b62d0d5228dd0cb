#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/tl
mkdir -p $OUT
for c in 1 8; do
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/c$c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --force-collective --chunks $c > $OUT/bench_c$c.log 2>&1 || { echo "trace c$c failed"; tail -5 $OUT/bench_c$c.log; exit 1; }
echo "chunks=$c: $(tail -1 $OUT/bench_c$c.log | cut -c1-200)"
python3 scripts/timeline.py $(find $OUT/c$c -name "*kernel_trace.csv" | head -1)
done
