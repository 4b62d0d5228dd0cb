#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
for wm in 0 8 12 16 24; do
  for rep in 1 2; do
    timeout -k 10 200 python -u bench.py --workload plugin --no-cpu-baseline --wave-min $wm --steps 30 --warmup 5 > $O/plugin_wm${wm}_$rep.log 2>&1 || { echo "wm $wm failed"; tail -20 $O/plugin_wm${wm}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/plugin_wm${wm}_$rep.log').read().strip().splitlines()[-1]); c=d['config']; print('wm', $wm, d['ms_per_step'], c['waves_per_round'], c['process_worker_data_ms_per_round'], d['roofline']['kernel_ms_per_step'])"
  done
done
timeout -k 10 200 python -u bench.py --workload gradient --no-cpu-baseline --steps 50 --warmup 5 > $O/gradient.log 2>&1 && tail -1 $O/gradient.log | cut -c1-400
