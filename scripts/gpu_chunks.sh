#!/bin/bash
# Cost of the sharded path's chunking on one GPU (RCCL reduce over 1 rank forced through):
# chunks x partial streams. Usage: bash scripts/gpu_chunks.sh "1 2 4 8" "1 2"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in ${2:-1 2}; do
for c in ${1:-1 2 4 8}; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --force-collective --chunks $c --partial-streams $s > gpurun_out/chunks_${c}_s${s}.log 2>&1 || { echo "c$c s$s failed"; tail -5 gpurun_out/chunks_${c}_s${s}.log; exit 1; }
grep '"metric"' gpurun_out/chunks_${c}_s${s}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('chunks', $c, 'streams', $s, d['ms_per_step'], r['kernel_ms_per_step'])"
done
done
