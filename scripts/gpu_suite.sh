#!/bin/bash
# GPU box: smoke + the whole -m gpu suite + the headline bench + extra bench lines (EXTRA_BENCH:
# ';'-separated argument lists, each one bench.py run) -> gpurun_out/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
echo smoke ok
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
echo pytest ok
tail -3 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
i=0
IFS=';' read -ra RUNS <<< "${EXTRA_BENCH:-}"
for args in "${RUNS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $args > gpurun_out/bench_extra_$i.log 2>&1 || { echo "bench $args failed rc=$?"; tail -30 gpurun_out/bench_extra_$i.log; exit 1; }
  echo "== $args"; grep '^{' gpurun_out/bench_extra_$i.log
done
