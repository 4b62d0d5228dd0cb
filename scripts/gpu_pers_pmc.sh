#!/bin/bash
# PMC pass over the personalized bench: where do the waves' cycles go?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pers_pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/pers_pmc -o pmc1 -- python scripts/bench_personalized.py --steps 2 --warmup 1 --no-probe ${PERS_ARGS:-} > gpurun_out/pers_pmc/run1.log 2>&1 || { echo "pmc1 failed rc=$?"; tail -20 gpurun_out/pers_pmc/run1.log; exit 1; }
find gpurun_out/pers_pmc -name "*counter_collection.csv" | head
