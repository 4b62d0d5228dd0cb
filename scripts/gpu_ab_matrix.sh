#!/bin/bash
# Same-box interleaved A/B matrix for the headline kernel (64 x ResNet-18 fp32 -> fp32):
#   r01      the round-1 tree (ab_r01/, `git archive 600809e`) with its own library
#   head     HEAD's bench and library
# (the round-1 host code cannot drive HEAD's library: the accumulator padding changed)
#   head+V   HEAD's bench with the variant library _lib/variants/lib_V.so (VARIANTS="...")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abm
REPS=${REPS:-3}
ARGS=${ARGS:---steps 50 --warmup 10 --no-cpu-baseline --no-probe}
line() { grep '^{' "$1" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_ms_per_step"], r["achieved"])'; }
for rep in $(seq 1 $REPS); do
  for side in r01 head $VARIANTS; do
    log=gpurun_out/abm/${side}_$rep.log
    case $side in
      r01) (cd ab_r01 && timeout -k 10 180 python bench.py $ARGS) > $log 2>&1 ;;
      head) timeout -k 10 180 python bench.py $ARGS > $log 2>&1 ;;
      *) FEDAVG_ALLOW_ABLATED=1 FEDAVG_HIP_LIB=distributed_learning_simulation_lib_amd/_lib/variants/lib_$side.so timeout -k 10 180 python bench.py $ARGS > $log 2>&1 ;;
    esac || { echo "$side failed rc=$?"; tail -20 $log; exit 1; }
    echo "$side $rep $(line $log)"
  done
done
