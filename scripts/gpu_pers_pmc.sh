#!/bin/bash
# PMC pass over the personalized bench (FEDAVG_HIP_LIB may select a tuning build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pers_pmc
rm -f gpurun_out/pers_pmc/*.db
for w in ${WEIGHTS:-float int}; do
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/pers_pmc -o pmc_$w -- python scripts/bench_personalized.py --steps 2 --warmup 1 --no-probe --weights $w > gpurun_out/pers_pmc/run_$w.log 2>&1 || { echo "pmc $w failed rc=$?"; tail -20 gpurun_out/pers_pmc/run_$w.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH -d gpurun_out/pers_pmc -o pmc2_$w -- python scripts/bench_personalized.py --steps 2 --warmup 1 --no-probe --weights $w > gpurun_out/pers_pmc/run2_$w.log 2>&1 || { echo "pmc2 $w failed rc=$?"; tail -20 gpurun_out/pers_pmc/run2_$w.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pers_pmc -o pmc3_$w -- python scripts/bench_personalized.py --steps 2 --warmup 1 --no-probe --weights $w > gpurun_out/pers_pmc/run3_$w.log 2>&1 || { echo "pmc3 $w failed rc=$?"; tail -20 gpurun_out/pers_pmc/run3_$w.log; exit 1; }
done
for f in $(find gpurun_out/pers_pmc -name "*results.db"); do python3 scripts/pmc_summary.py personalized $f; done > gpurun_out/pers_pmc/summary.txt 2>&1 || true
ls gpurun_out/pers_pmc
