#!/bin/bash
# QSGD table build through the level reciprocal (FEDAVG_FAST_DIV): parity on the variant + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
FEDAVG_HIP_LIB=distributed_learning_simulation_lib_amd/_lib/variants/lib_qf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_qsgd.py -x -q --timeout 240 --timeout-method thread > gpurun_out/qsgd_parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/qsgd_parity.log; exit 1; }
echo "qf parity: $(tail -n 1 gpurun_out/qsgd_parity.log)"
export VARIANTS="qf qi"
for r in 1 2; do
CMD="python bench.py --workload qsgd --steps 30 --warmup 5 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh || exit 1
done
