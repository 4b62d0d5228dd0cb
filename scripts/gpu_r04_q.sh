#!/bin/bash
# Round 4: the whole GPU suite + smoke on the staging / result-buffer / default-wave changes, then
# the plugin and gradient lines and round timelines that go into profiles/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
: > $O/timeline.jsonl
for cfg in "64 64 0" "64 32 0" "8 8 0"; do
  timeout -k 10 120 python scripts/plugin_round_timeline.py $cfg >> $O/timeline.jsonl 2>> $O/timeline.err || { echo "timeline $cfg failed"; tail -20 $O/timeline.err; exit 1; }
done
: > $O/bench.jsonl
for a in "--workload plugin" "--workload plugin --wave 32" "--workload gradient"; do
  timeout -k 10 180 python bench.py $a --no-cpu-baseline --steps 30 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || { echo "bench $a failed"; tail -20 $O/bench.err; exit 1; }
done
echo done
