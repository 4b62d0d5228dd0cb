#!/bin/bash
# rocprofv3 evidence for the dynamic wave (dyn_wave_kernel) of the plugin workloads: per workload a
# kernel-trace pass and FETCH_SIZE / WRITE_SIZE PMC passes (separate runs; never combined with
# another trace domain). The bench line's HBM probes in the same process calibrate the counters.
#   WORKLOADS="plugin:--workload plugin;gradient:--workload gradient" bash scripts/dyn_traffic.sh
# Summaries: python scripts/dyn_traffic_summary.py gpurun_out/dynprof <name> <tag> (on the build host).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/dynprof
mkdir -p $OUT
IFS=';' read -ra WLS <<< "${WORKLOADS:-plugin:--workload plugin;gradient:--workload gradient}"
for wl in "${WLS[@]}"; do
  name=${wl%%:*}; args=${wl#*:}
  B="bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 3 $args"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/${name}_trace -o run --output-format csv -- python3 $B > $OUT/${name}_trace.log 2>&1 || { echo "$name trace failed"; tail -20 $OUT/${name}_trace.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/${name}_fetch -o run --output-format csv -- python3 $B > $OUT/${name}_fetch.log 2>&1 || { echo "$name fetch failed"; tail -20 $OUT/${name}_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/${name}_write -o run --output-format csv -- python3 $B > $OUT/${name}_write.log 2>&1 || { echo "$name write failed"; tail -20 $OUT/${name}_write.log; exit 1; }
  python3 - "$OUT" "$name" <<'PY'
import csv, sys
from pathlib import Path
out, name = Path(sys.argv[1]), sys.argv[2]
keep = ("dyn_wave_kernel", "fedavg_tile_kernel", "bw_read_kernel", "bw_copy_kernel")
for sub in ("trace", "fetch", "write"):
    d = out / f"{name}_{sub}"
    for f in list(d.rglob("*")):
        if not f.is_file():
            continue
        if f.name == "run_kernel_stats.csv":
            continue
        if f.name in ("run_counter_collection.csv", "run_kernel_trace.csv"):
            rows = list(csv.DictReader(open(f)))
            fields = rows[0].keys() if rows else []
            rows = [r for r in rows if any(k in r.get("Kernel_Name", "") for k in keep)]
            with open(f, "w", newline="") as fh:
                w = csv.DictWriter(fh, fieldnames=list(fields))
                w.writeheader()
                w.writerows(rows)
            continue
        f.unlink()
PY
  echo "$name ok: $(grep '^{' $OUT/${name}_trace.log | head -c 300)"
done
