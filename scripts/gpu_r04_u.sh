#!/bin/bash
# Round 4 end: the driver's checks on the final tree — the whole GPU suite, smoke, and the default
# bench line — plus the plugin / gradient / personalized lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.jsonl 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
: > $O/lines.jsonl
for a in "--workload plugin" "--workload gradient" "--workload personalized --pers-weights int" "--workload personalized --pers-weights float"; do
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-probe --steps 20 --warmup 5 >> $O/lines.jsonl 2>> $O/lines.err || { echo "bench $a failed"; tail -20 $O/lines.err; exit 1; }
done

timeout -k 10 300 python scripts/plugin_pers_bench.py > $O/plugin_pers.txt 2>&1 || { tail -30 $O/plugin_pers.txt; exit 1; }
sed -n 2p $O/plugin_pers.txt
echo done
