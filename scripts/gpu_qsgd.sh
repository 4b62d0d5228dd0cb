# QSGD fused-dequant path on one MI355X: parity tests, bench line, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/qsgd
timeout -k 10 300 python -u -m pytest tests/test_gpu_qsgd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qsgd/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/qsgd/pytest.log; exit 1; }
tail -2 gpurun_out/qsgd/pytest.log
timeout -k 10 300 python bench.py --workload qsgd --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/qsgd/bench.json 2> gpurun_out/qsgd/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/qsgd/bench.err; exit 1; }
cat gpurun_out/qsgd/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex qsgd -d "$GRAFT_REPO_ROOT/gpurun_out/qsgd/prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --workload qsgd --steps 20 --warmup 5 --no-cpu-baseline --no-probe > "$GRAFT_REPO_ROOT/gpurun_out/qsgd/prof.log" 2>&1 || { echo "rocprof rc=$?"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/qsgd/prof.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/qsgd/prof" -name "*kernel_stats.csv" -exec cat {} \;
find "$GRAFT_REPO_ROOT/gpurun_out/qsgd/prof" -type f ! -name "*kernel_stats.csv" -delete
