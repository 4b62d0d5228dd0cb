#!/bin/bash
# Round-3 validation + measurement call: smoke, the GPU suite, the headline bench, the plugin /
# output-dtype lines, the headline A/B against the round-1 tree, QSGD PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
EXTRA_BENCH="--out-dtype float64 --no-cpu-baseline --no-probe;--workload plugin --no-cpu-baseline --steps 20;--workload plugin --out-dtype float32 --no-cpu-baseline --steps 20;--workload plugin --wave 32 --no-cpu-baseline --steps 20;--workload gradient --no-cpu-baseline --steps 50" bash scripts/gpu_suite.sh || exit 1
REPS=3 VARIANTS="nbp" bash scripts/gpu_ab_matrix.sh || exit 1
bash scripts/gpu_qsgd_pmc.sh || exit 1
