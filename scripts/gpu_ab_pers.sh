#!/bin/bash
# Personalized kernel variants: parity (the personalized GPU tests on each variant) + interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  FEDAVG_HIP_LIB=distributed_learning_simulation_lib_amd/_lib/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_personalized.py tests/test_gpu_division_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pers_$v.log 2>&1 || { echo "$v parity failed"; tail -30 gpurun_out/pers_$v.log; exit 1; }
  echo "$v parity: $(tail -n 1 gpurun_out/pers_$v.log)"
done
CMD="python bench.py --workload personalized --pers-weights int --steps 10 --warmup 3 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh || exit 1
CMD="python bench.py --workload personalized --pers-weights float --steps 10 --warmup 3 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh || exit 1
