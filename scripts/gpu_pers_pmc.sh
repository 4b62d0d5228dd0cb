#!/bin/bash
# PMC passes over the personalized bench. FEDAVG_HIP_LIB may select a tuning build; TAG names the
# output directory (gpurun_out/pers_pmc_$TAG).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pers_pmc_${TAG:-head}
mkdir -p $O
rm -f $O/*.db
B="scripts/bench_personalized.py --steps 2 --warmup 1 --no-probe"
for w in ${WEIGHTS:-float int}; do
timeout -s KILL 120 rocprofv3 --kernel-include-regex personalized --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES -d $O -o pmc1_$w -- python $B --weights $w > $O/run1_$w.log 2>&1 || { echo "pmc1 $w failed rc=$?"; tail -20 $O/run1_$w.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-include-regex personalized --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH -d $O -o pmc2_$w -- python $B --weights $w > $O/run2_$w.log 2>&1 || { echo "pmc2 $w failed rc=$?"; tail -20 $O/run2_$w.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-include-regex personalized --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O -o pmc3_$w -- python $B --weights $w > $O/run3_$w.log 2>&1 || { echo "pmc3 $w failed rc=$?"; tail -20 $O/run3_$w.log; exit 1; }
done
for f in $(find $O -name "*results.db"); do echo "== $f"; python3 scripts/pmc_summary.py personalized $f; done > $O/summary.txt 2>&1 || true
find $O -name "*.db" -delete
ls $O
