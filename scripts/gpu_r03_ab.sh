#!/bin/bash
# Round-3 A/B call: headline kernel (round-1 tree vs HEAD vs variants), PersonalizedFedAVG ring
# weights, a rocprofv3 kernel trace of the QSGD workload (table kernel vs tile kernel), and the
# plugin's host breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_qsgd
REPS=4 VARIANTS="${HEAD_VARIANTS:-r01like r01k nbp}" bash scripts/gpu_ab_matrix.sh || exit 1
echo "== personalized int"
REPS=2 VARIANTS="prw1 prw0" CMD="python bench.py --workload personalized --pers-weights int --no-cpu-baseline --no-probe --steps 10 --warmup 3" bash scripts/gpu_ab.sh || exit 1
echo "== personalized float"
REPS=2 VARIANTS="prw1 prw1m" CMD="python bench.py --workload personalized --pers-weights float --no-cpu-baseline --no-probe --steps 10 --warmup 3" bash scripts/gpu_ab.sh || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_qsgd -o q -- python bench.py --workload qsgd --no-cpu-baseline --no-probe --steps 20 > gpurun_out/prof_qsgd/bench.log 2>&1 || { echo "rocprof qsgd failed"; tail -20 gpurun_out/prof_qsgd/bench.log; exit 1; }
grep '^{' gpurun_out/prof_qsgd/bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("qsgd", d["roofline"]["mean_launch_ms"], d["roofline"]["achieved"])'
timeout -k 10 200 python scripts/plugin_host_breakdown.py > gpurun_out/host_breakdown.json && cat gpurun_out/host_breakdown.json
