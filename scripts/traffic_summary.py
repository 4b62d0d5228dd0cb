"""HBM traffic of a bench line's FedAvg kernels from a scripts/gpu_config_traffic.sh pass set.

Usage: python scripts/traffic_summary.py OUT_DIR NAME TAG [KERNEL]   (KERNEL: fedavg_tile_kernel by
default; qsgd_tile_kernel / nnadq_tile_kernel for the quantised lines)
  OUT_DIR/NAME_trace  rocprofv3 --kernel-trace --stats   (+ the bench JSON line in NAME_trace.log)
  OUT_DIR/NAME_fetch  rocprofv3 --pmc FETCH_SIZE          (separate passes: TCC slot limits)
  OUT_DIR/NAME_write  rocprofv3 --pmc WRITE_SIZE
FETCH_SIZE / WRITE_SIZE (KB) are corrected the way MI355X_MICROARCH.md prescribes for gfx950:
calibrated on bench.py's HBM probes in the same pass (bw_read_kernel streams exactly 4 GiB,
bw_copy_kernel reads + writes 4 GiB with the same 16-B non-temporal access pattern). Traffic per
step = mean per dispatch x the line's launches per step; it is compared with the line's
algorithmic bytes per step (roofline.bytes_per_step_this_rank). Writes profiles/TAG_traffic_NAME.json
and appends the line, with roofline.traffic filled in, to profiles/TAG_configs.jsonl.
"""
import csv
import json
import statistics
import sys
from pathlib import Path

out_dir, name, tag = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
repo = Path(__file__).resolve().parent.parent
prof = repo / "profiles"
PROBE_BYTES = 4 << 30
KERNEL = sys.argv[4] if len(sys.argv) > 4 else "fedavg_tile_kernel"


def counter(pass_dir, kernel_substr):
    rows = list(csv.DictReader(open(out_dir / pass_dir / "run_counter_collection.csv")))
    return [float(r["Counter_Value"]) for r in rows if kernel_substr in r["Kernel_Name"]]


line = next(json.loads(x) for x in open(out_dir / f"{name}_trace.log") if x.startswith("{"))
stats = {r["Name"]: r for r in csv.DictReader(open(out_dir / f"{name}_trace" / "run_kernel_stats.csv"))}
avg_ns = float(stats[KERNEL]["AverageNs"]) if KERNEL in stats else None
read_corr = PROBE_BYTES / (statistics.median(counter(f"{name}_fetch", "bw_read_kernel")) * 1024)
write_corr = PROBE_BYTES / (statistics.median(counter(f"{name}_write", "bw_copy_kernel")) * 1024)
fetch = statistics.mean(counter(f"{name}_fetch", KERNEL)) * 1024 * read_corr
write = statistics.mean(counter(f"{name}_write", KERNEL)) * 1024 * write_corr
r = line["roofline"]
per_step_launches = r["launches"] / line["steps"]
traffic_step = (fetch + write) * per_step_launches
alg_step = (r.get("bytes_per_step_this_rank") or r.get("bytes_per_timed_launch")
            or (r.get("bytes_per_launch", 0) * per_step_launches or None))
out = {
    "tag": tag,
    "workload": line["config"]["workload"],
    "kernel": KERNEL,
    "launches_per_step": per_step_launches,
    "kernel_avg_ms_rocprof": None if avg_ns is None else avg_ns / 1e6,
    "kernel_ms_per_step_hip_events": r.get("kernel_ms_per_step", r.get("mean_launch_ms")),
    "fetch_bytes_per_launch": fetch,
    "write_bytes_per_launch": write,
    "hbm_traffic_bytes_per_step": traffic_step,
    "algorithmic_bytes_per_step": alg_step,
    "traffic_over_algorithmic": traffic_step / alg_step if alg_step else None,
    "calibration": {"read_correction": read_corr, "write_correction": write_corr, "probe_bytes": PROBE_BYTES},
    "source": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE (separate passes), "
              "scripts/gpu_config_traffic.sh",
}
(prof / f"{tag}_traffic_{name}.json").write_text(json.dumps(out, indent=1) + "\n")
r["traffic"] = traffic_step
r["traffic_unit"] = "bytes per step (all launches of the step, PMC-corrected)"
r["traffic_source"] = f"profiles/{tag}_traffic_{name}.json"
with open(prof / f"{tag}_configs.jsonl", "a") as f:
    f.write(json.dumps(line) + "\n")
print(json.dumps(out, indent=1))
