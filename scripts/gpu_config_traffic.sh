#!/bin/bash
# Per-config rocprofv3 evidence (kernel stats + PMC traffic) for BASELINE configs on one GPU.
# CONFIGS: ';'-separated "name:bench args" entries. Three passes each (trace, FETCH_SIZE,
# WRITE_SIZE), never combined with other trace domains; summaries via scripts/traffic_summary.py
# are made afterwards from gpurun_out/cfgprof/ on the build host.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/cfgprof
mkdir -p $OUT
IFS=';' read -ra CFGS <<< "$CONFIGS"
for cfg in "${CFGS[@]}"; do
  name=${cfg%%:*}; args=${cfg#*:}
  B="bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 $args"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/${name}_trace -o run --output-format csv -- python3 $B > $OUT/${name}_trace.log 2>&1 || { echo "$name trace failed"; tail -20 $OUT/${name}_trace.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/${name}_fetch -o run --output-format csv -- python3 $B > $OUT/${name}_fetch.log 2>&1 || { echo "$name fetch failed"; tail -20 $OUT/${name}_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/${name}_write -o run --output-format csv -- python3 $B > $OUT/${name}_write.log 2>&1 || { echo "$name write failed"; tail -20 $OUT/${name}_write.log; exit 1; }
  # keep only the rows of the kernels the summary reads (gpurun_out/ must stay under 64 MiB)
  python3 - "$OUT" "$name" <<'PY'
import csv, sys
from pathlib import Path
out, name = Path(sys.argv[1]), sys.argv[2]
keep = ("fedavg_tile_kernel", "qsgd_tile_kernel", "qsgd_table_kernel", "nnadq_tile_kernel", "bw_read_kernel", "bw_copy_kernel")
for sub in ("trace", "fetch", "write"):
    d = out / f"{name}_{sub}"
    for f in list(d.rglob("*")):
        if not f.is_file():
            continue
        if f.name == "run_kernel_stats.csv":
            continue
        if f.name == "run_counter_collection.csv":
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
