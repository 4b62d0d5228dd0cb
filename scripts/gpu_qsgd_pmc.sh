#!/bin/bash
# PMC passes over the QSGD fused-dequant kernel (bench --workload qsgd): wave-cycle breakdown,
# LDS bank conflicts, instruction mix. One pass per counter set, kernel filter on qsgd.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/qsgd_pmc
mkdir -p $OUT
rm -f $OUT/*.db
B="bench.py --workload qsgd --steps 3 --warmup 1 --no-probe --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -s KILL 150 rocprofv3 --kernel-include-regex qsgd --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $OUT -o p1 -- python3 $B > $OUT/p1.log 2>&1 || { echo "p1 failed rc=$?"; tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-include-regex qsgd --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS -d $OUT -o p2 -- python3 $B > $OUT/p2.log 2>&1 || { echo "p2 failed rc=$?"; tail -20 $OUT/p2.log; exit 1; }
for f in $(find $OUT -name "*results.db"); do python3 scripts/pmc_summary.py qsgd $f; done | tee $OUT/summary.txt
find $OUT -name "*.db" -delete
