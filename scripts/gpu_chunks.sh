#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 1 2 4 8; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --force-collective --chunks $c > gpurun_out/chunks_$c.log 2>&1 || { echo "c$c failed"; tail -5 gpurun_out/chunks_$c.log; exit 1; }
grep '"metric"' gpurun_out/chunks_$c.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('chunks', $c, d['ms_per_step'], r['kernel_ms_per_step'])"
done
