#!/bin/bash
# Timing perturbation of the per-launch profiling events: headline (fused) and native sharded
# round (1 rank forced), with and without events.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "fused, events"; bash scripts/gpu_bench_repeat.sh "1 2" || exit 1
echo "fused, no events"; BENCH_ARGS=--no-kernel-events bash scripts/gpu_bench_repeat.sh "3 4" || exit 1
for e in "" "--no-kernel-events"; do
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probe --force-collective --chunks 4 $e > gpurun_out/c4ev.log 2>&1 || exit 1
grep '"metric"' gpurun_out/c4ev.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('native c4 $e', d['ms_per_step'], r['mean_launch_ms'], r['achieved'], r['kernel'])"
done
