#!/bin/bash
# One parametrised GPU-box runner (replaces the per-call one-off scripts of rounds 3-4).
#   bash scripts/gpu_run.sh <out-tag> <step> [<step> ...]
# Steps (each under its own time limit, chained: the first failure ends the call):
#   smoke                 __graft_entry__.smoke()
#   tests[=<pytest args>] pytest -m gpu (default: the whole GPU suite; e.g. tests=tests/test_gpu_multi_device.py)
#   bench                 the headline N=1 line (bench.py, default flags)
#   alias<G>              the single-process peer round rehearsed with G aliased entries on cuda:0
#   plugin / gradient     bench.py --workload plugin / gradient
#   plugin_static / gradient_static   the same with the dynamic wave off (FEDAVG_DYN=0)
#   bursts / bursts_static / bursts_spin   plugin rounds in 4 bursts 2 ms apart (the reference server's
#                         poll-then-sleep cadence): default wave / wave off / wave that never idles out
#   idle=<us>             plugin + gradient lines with FEDAVG_DYN_IDLE_US=<us>
#   cpu                   the headline line with its CPU baseline (pinned child process)
#   pers_int / pers_float bench.py --workload personalized (integer / float weights)
#   profile               scripts/profile.sh <out-tag> (kernel trace + FETCH/WRITE PMC passes)
#   pers_pmc              scripts/gpu_pers_pmc.sh
# Output goes to gpurun_out/<out-tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
run() {  # run <name> <seconds> <command...>: output to $O/<name>.log, a failure ends the call
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $name failed rc=$rc"
    tail -40 "$O/$name.log"
    exit 1
  fi
  echo "step $name ok"
  grep -h '^{' "$O/$name.log" | tail -1 | cut -c1-600
}
for step in "$@"; do
  case "$step" in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
           tail -3 "$O/tests.log" ;;
    tests=*) run tests 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${step#tests=}
             tail -3 "$O/tests.log" ;;
    bench) run bench 400 python -u bench.py ;;
    alias*) G=${step#alias}
            run alias$G 400 python -u bench.py --procs 1 --gpus "$G" --alias --no-probe --stage-timeout 200 ;;
    plugin) run plugin 300 python -u bench.py --workload plugin --no-cpu-baseline ;;
    gradient) run gradient 300 python -u bench.py --workload gradient --no-cpu-baseline ;;
    plugin_static) FEDAVG_DYN=0 run plugin_static 300 python -u bench.py --workload plugin --no-cpu-baseline ;;
    bursts) run bursts 300 python -u bench.py --workload plugin --no-cpu-baseline --arrival bursts:4:2 ;;
    bursts_static) FEDAVG_DYN=0 run bursts_static 300 python -u bench.py --workload plugin --no-cpu-baseline --arrival bursts:4:2 ;;
    bursts_spin) FEDAVG_DYN_IDLE_US=1000000 run bursts_spin 300 python -u bench.py --workload plugin --no-cpu-baseline --arrival bursts:4:2 ;;
    idle=*) I=${step#idle=}
            FEDAVG_DYN_IDLE_US=$I run plugin_idle$I 300 python -u bench.py --workload plugin --no-cpu-baseline
            FEDAVG_DYN_IDLE_US=$I run gradient_idle$I 300 python -u bench.py --workload gradient --no-cpu-baseline ;;
    cpu) run cpu 400 python -u bench.py --no-probe --steps 5 --warmup 2 ;;
    gradient_static) FEDAVG_DYN=0 run gradient_static 300 python -u bench.py --workload gradient --no-cpu-baseline ;;
    pers_int) run pers_int 300 python -u bench.py --workload personalized --pers-weights int --no-cpu-baseline --no-probe ;;
    pers_float) run pers_float 300 python -u bench.py --workload personalized --pers-weights float --no-cpu-baseline --no-probe ;;
    profile) run profile 900 bash scripts/profile.sh "$TAG" ;;
    pers_pmc) run pers_pmc 600 bash scripts/gpu_pers_pmc.sh ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
