#!/bin/bash
# Headline bench repeated (run-to-run spread of ms_per_step and kernel time).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in ${1:-1 2 3}; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-probe ${BENCH_ARGS:-} > gpurun_out/rep_$i.log 2>&1 || { echo "run $i failed"; tail -5 gpurun_out/rep_$i.log; exit 1; }
grep '"metric"' gpurun_out/rep_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('run', $i, d['ms_per_step'], r['kernel_ms_per_step'], d['value'])"
done
