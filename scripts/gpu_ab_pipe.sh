#!/bin/bash
# FEDAVG_PIPE_CONTIG A/B: parity on the new variant, then interleaved bench A/B on 2-byte inputs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
FEDAVG_HIP_LIB=distributed_learning_simulation_lib_amd/_lib/variants/lib_c1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_property.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pipe_parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/pipe_parity.log; exit 1; }
echo "c1 parity: $(tail -n 1 gpurun_out/pipe_parity.log)"
export VARIANTS="c1 c0"
CMD="python bench.py --in-dtype float16 --steps 30 --warmup 5 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh || exit 1
CMD="python bench.py --layout gpt2s --in-dtype float16 --clients-per-gpu 128 --steps 10 --warmup 3 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh || exit 1
CMD="python bench.py --layout gpt2s --in-dtype float16 --clients-per-gpu 128 --wave 32 --steps 10 --warmup 3 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh || exit 1
CMD="python bench.py --in-dtype bfloat16 --wave 16 --steps 30 --warmup 5 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh || exit 1
