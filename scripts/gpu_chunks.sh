#!/bin/bash
# Cost of the sharded path's chunking on one GPU (RCCL reduce over 1 rank forced through),
# for both exchange implementations. Usage: bash scripts/gpu_chunks.sh "1 2 4 8" "torch native"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${2:-torch native}; do
for c in ${1:-1 2 4 8}; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --force-collective --chunks $c --comm $m > gpurun_out/chunks_${c}_${m}.log 2>&1 || { echo "c$c $m failed"; tail -5 gpurun_out/chunks_${c}_${m}.log; exit 1; }
grep '"metric"' gpurun_out/chunks_${c}_${m}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('chunks', $c, '$m', d['ms_per_step'], r['kernel_ms_per_step'], 'host', d['host_enqueue_ms_per_step'])"
done
done
