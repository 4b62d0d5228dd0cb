#!/bin/bash
# Round 4: plugin host costs after the staging extension's reference / shape-cache change —
# staging parity tests, per-piece breakdown, round timelines, plugin and gradient bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04n}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_staging.py tests/test_gpu_multi_device.py tests/test_gpu_parity.py tests/test_gpu_gradient.py tests/test_gpu_personalized.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 180 python scripts/plugin_host_breakdown.py > $O/breakdown.jsonl 2> $O/breakdown.err || { tail -20 $O/breakdown.err; exit 1; }
cat $O/breakdown.jsonl
: > $O/timeline.jsonl
for cfg in "64 64 0" "64 32 0" "8 8 0"; do
  timeout -k 10 120 python scripts/plugin_round_timeline.py $cfg >> $O/timeline.jsonl 2>> $O/timeline.err || { echo "timeline $cfg failed"; tail -20 $O/timeline.err; exit 1; }
done
cat $O/timeline.jsonl
: > $O/bench.jsonl
for a in "--workload plugin" "--workload plugin --wave 64" "--workload gradient"; do
  timeout -k 10 180 python bench.py $a --no-cpu-baseline --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || { echo "bench $a failed"; tail -20 $O/bench.err; exit 1; }
done
echo done
