#!/bin/bash
# A/B: root finalize per chunk on the comm stream (1) vs one finalize at the end (0), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
# (the FEDAVG_CHUNK_FINALIZE switch was removed after this A/B; kept for the record)
for r in 1 2 3; do for v in 0 1; do for c in ${1:-2 4}; do
FEDAVG_CHUNK_FINALIZE=$v timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-probe --force-collective --chunks $c > gpurun_out/abf.log 2>&1 || exit 1
grep '"metric"' gpurun_out/abf.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('rep $r chunkfin $v chunks $c', d['ms_per_step'])"
done; done; done
