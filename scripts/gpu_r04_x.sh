#!/bin/bash
# Round 4: per-dispatch durations of the PersonalizedFedAVG kernel (integer and float weights) in
# launch order, to see whether the integer-weight round's spread follows the launch sequence.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
for w in int float; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$w -o pers --output-format csv -- python bench.py --workload personalized --pers-weights $w --steps 30 --warmup 3 --no-cpu-baseline --no-probe > $O/trace_$w.log 2>&1 || { tail -20 $O/trace_$w.log; exit 1; }
done
find $O -name "*kernel_trace.csv"
echo done
