#!/bin/bash
# round 3: QSGD prefetch-depth rewrite — parity (QSGD + NNADQ + QSGD geometry edges) on the
# shipped library, then an interleaved A/B of library variants on the QSGD bench, then the
# NNADQ bench line + rocprof stats. -> gpurun_out/r03q/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03q
timeout -k 10 600 python -u -m pytest tests/test_gpu_qsgd.py tests/test_gpu_nnadq.py "tests/test_gpu_geometry.py::test_qsgd_kernel_edges_bit_identical" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r03q/pytest.log; exit 1; }
tail -2 gpurun_out/r03q/pytest.log
for rep in 1 2; do
for v in ${VARIANTS:-old d1 d2 d3}; do
FEDAVG_HIP_LIB=distributed_learning_simulation_lib_amd/_lib/variants/lib_$v.so timeout -k 10 300 python bench.py --workload qsgd --steps 30 --warmup 5 --no-cpu-baseline --no-probe > gpurun_out/r03q/ab_${v}_$rep.log 2>&1 || { echo "$v failed rc=$?"; tail -20 gpurun_out/r03q/ab_${v}_$rep.log; exit 1; }
echo "$v $rep $(tail -1 gpurun_out/r03q/ab_${v}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["mean_launch_ms"], r["achieved"], r["frac"])')"
done
done
timeout -k 10 300 python bench.py --workload nnadq --steps 20 --warmup 5 > gpurun_out/r03q/bench_nnadq.json 2> gpurun_out/r03q/bench_nnadq.err || { echo "nnadq bench rc=$?"; tail -20 gpurun_out/r03q/bench_nnadq.err; exit 1; }
cat gpurun_out/r03q/bench_nnadq.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r03q/prof_nnadq" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --workload nnadq --steps 20 --warmup 5 --no-cpu-baseline --no-probe > "$GRAFT_REPO_ROOT/gpurun_out/r03q/prof_nnadq.log" 2>&1) || { echo "rocprof rc=$?"; tail -20 gpurun_out/r03q/prof_nnadq.log; exit 1; }
find gpurun_out/r03q/prof_nnadq -name "*kernel_stats.csv" -exec head -5 {} \;
find gpurun_out/r03q/prof_nnadq -type f ! -name "*kernel_stats.csv" -delete
