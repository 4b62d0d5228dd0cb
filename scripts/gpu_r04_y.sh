#!/bin/bash
# Round 4: integer weights on the LDS-DMA ring (default) vs the register pipeline
# (FEDAVG_PERS_RING=0), interleaved, with per-dispatch durations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
for rep in 1 2 3; do
  for ring in 1 0; do
    FEDAVG_PERS_RING=$ring timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_${ring}_$rep -o pers --output-format csv -- python bench.py --workload personalized --pers-weights int --steps 20 --warmup 3 --no-cpu-baseline --no-probe > $O/t_${ring}_$rep.log 2>&1 || { tail -20 $O/t_${ring}_$rep.log; exit 1; }
  done
done
echo done
