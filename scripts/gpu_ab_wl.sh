#!/bin/bash
# Interleaved A/B of library variants per workload on one box:
#   AB="nnadq:main,n_g8pk0 qsgd:main,old" REPS=2 [TESTS="tests/..."] bash scripts/gpu_ab_wl.sh
# variant "main" = the in-tree library; others = _lib/variants/lib_<name>.so -> gpurun_out/abwl/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abwl
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/abwl/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/abwl/pytest.log; exit 1; }
  tail -2 gpurun_out/abwl/pytest.log
fi
for rep in $(seq 1 ${REPS:-2}); do
for spec in $AB; do
  wl=${spec%%:*}; vs=${spec#*:}
  for v in ${vs//,/ }; do
    lib=""; [ "$v" != main ] && lib=distributed_learning_simulation_lib_amd/_lib/variants/lib_$v.so
    case $wl in
      pers_int) wargs="--workload personalized --pers-weights int";;
      pers_float) wargs="--workload personalized --pers-weights float";;
      *) wargs="--workload $wl";;
    esac
    FEDAVG_HIP_LIB=$lib timeout -k 10 300 python bench.py $wargs --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-probe ${BENCH_ARGS:-} > gpurun_out/abwl/${wl}_${v}_$rep.log 2>&1 || { echo "$wl $v failed rc=$?"; tail -20 gpurun_out/abwl/${wl}_${v}_$rep.log; exit 1; }
    echo "$wl $v $rep $(tail -1 gpurun_out/abwl/${wl}_${v}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; print(d["ms_per_step"], r.get("mean_launch_ms", r.get("kernel_ms_per_step", d.get("kernel_ms_per_step"))), r.get("achieved"), r.get("frac"))')"
  done
done
done
