#!/bin/bash
# Quantised-update paths on one MI355X (QSGD + NNADQ): parity tests, a bench line and a
# rocprofv3 kernel-stats summary per codec -> gpurun_out/quant/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/quant
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_nnadq.py tests/test_gpu_qsgd.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/quant/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/quant/pytest.log; exit 1; }
tail -2 gpurun_out/quant/pytest.log
for w in ${WORKLOADS:-nnadq qsgd}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/quant/bench_$w.json 2> gpurun_out/quant/bench_$w.err || { echo "bench $w rc=$?"; tail -20 gpurun_out/quant/bench_$w.err; exit 1; }
  cat gpurun_out/quant/bench_$w.json
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/quant/prof_$w" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-probe > "$GRAFT_REPO_ROOT/gpurun_out/quant/prof_$w.log" 2>&1) || { echo "rocprof $w rc=$?"; tail -20 "gpurun_out/quant/prof_$w.log"; exit 1; }
  find "gpurun_out/quant/prof_$w" -name "*kernel_stats.csv" -exec head -6 {} \;
  find "gpurun_out/quant/prof_$w" -type f ! -name "*kernel_stats.csv" -delete
done
