#!/bin/bash
# Round 4: parity of the rebuilt kernels (personalized, staging) + multi-device rehearsal + smoke,
# then the plugin timelines / bench lines after the host-cost cuts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_r04_g.sh || exit 1
O=gpurun_out/r04h
mkdir -p $O
: > $O/timeline.jsonl
for cfg in "64 64 0" "64 32 0" "64 64 8" "8 8 0" "8 8 2"; do
  timeout -k 10 120 python scripts/plugin_round_timeline.py $cfg >> $O/timeline.jsonl 2>> $O/timeline.err || { echo "timeline $cfg failed"; tail -20 $O/timeline.err; exit 1; }
done
cat $O/timeline.jsonl
: > $O/bench.jsonl
for a in "--workload plugin" "--workload plugin --wave 64" "--workload gradient"; do
  timeout -k 10 180 python bench.py $a --no-cpu-baseline --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || { echo "bench $a failed"; tail -20 $O/bench.err; exit 1; }
done
echo done
