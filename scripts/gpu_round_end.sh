#!/bin/bash
# Round-end evidence on one MI355X: smoke, the whole -m gpu suite, the headline bench line, its
# rocprofv3 kernel stats, and one line per secondary workload -> gpurun_out/final/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest_gpu.log; exit 1; }
  echo "pytest: $(tail -1 $O/pytest_gpu.log)"
fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-probe > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1) || { echo "rocprof rc=$?"; tail -20 $O/prof.log; exit 1; }
find $O/prof -type f ! -name "*kernel_stats.csv" -delete
i=0
IFS=';' read -ra RUNS <<< "${EXTRA_BENCH:---workload plugin;--workload plugin --wave 32;--workload gradient;--workload qsgd;--workload nnadq;--workload personalized;--workload personalized --pers-weights int}"
for args in "${RUNS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $args --steps 20 --warmup 5 > $O/extra_$i.json 2> $O/extra_$i.err || { echo "bench $args failed rc=$?"; tail -20 $O/extra_$i.err; exit 1; }
  echo "== $args: $(head -c 400 $O/extra_$i.json)"
done
