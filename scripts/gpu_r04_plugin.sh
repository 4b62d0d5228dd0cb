#!/bin/bash
# Round 4: plugin early waves (wave_min) — round timelines and bench lines per setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_plugin
mkdir -p $O
: > $O/timeline.jsonl
for cfg in "64 64 0" "64 32 0" "64 64 4" "64 64 8" "64 64 16" "8 8 0" "8 8 1" "8 8 2"; do
  timeout -k 10 120 python scripts/plugin_round_timeline.py $cfg >> $O/timeline.jsonl 2>> $O/timeline.err || { echo "timeline $cfg failed"; tail -20 $O/timeline.err; exit 1; }
done
: > $O/bench.jsonl
for wm in 0 4 8 16; do
  timeout -k 10 180 python bench.py --workload plugin --wave 64 --wave-min $wm --no-cpu-baseline --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || { echo "plugin $wm failed"; tail -20 $O/bench.err; exit 1; }
done
timeout -k 10 180 python bench.py --workload plugin --wave-min 0 --no-cpu-baseline --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || exit 1
for wm in 0 1 2; do
  timeout -k 10 180 python bench.py --workload gradient --clients-per-gpu 8 --wave 8 --wave-min $wm --no-cpu-baseline --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || { echo "gradient $wm failed"; tail -20 $O/bench.err; exit 1; }
done
echo done
