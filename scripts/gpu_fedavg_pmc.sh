#!/bin/bash
# PMC pass over the FedAvg bench for two input dtypes (wave-cycle breakdown, instruction mix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fa_pmc
rm -f gpurun_out/fa_pmc/*.db
# CFGS: ';'-separated "name:bench args" (default: GPT-2 fp32 / fp16 one launch)
IFS=';' read -ra CFG_LIST <<< "${CFGS:-fp32:--layout gpt2s --clients-per-gpu 64;fp16:--layout gpt2s --clients-per-gpu 128 --in-dtype float16}"
for cfg in "${CFG_LIST[@]}"; do
name=${cfg%%:*}; args=${cfg#*:}
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES -d gpurun_out/fa_pmc -o pmc_$name -- python bench.py --steps 3 --warmup 1 --no-probe --no-cpu-baseline $args > gpurun_out/fa_pmc/run_$name.log 2>&1 || { echo "pmc $name failed rc=$?"; tail -20 gpurun_out/fa_pmc/run_$name.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc TA_BUSY_avr TA_TA_BUSY_sum SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM -d gpurun_out/fa_pmc -o pmc2_$name -- python bench.py --steps 3 --warmup 1 --no-probe --no-cpu-baseline $args > gpurun_out/fa_pmc/run2_$name.log 2>&1 || { echo "pmc2 $name failed rc=$?"; tail -20 gpurun_out/fa_pmc/run2_$name.log; exit 1; }
done
ls gpurun_out/fa_pmc
