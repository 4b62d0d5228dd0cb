"""HBM traffic of the dynamic wave (dyn_wave_kernel) per round, from a scripts/dyn_traffic.sh pass set.

Usage: python scripts/dyn_traffic_summary.py OUT_DIR NAME TAG
  OUT_DIR/NAME_trace  rocprofv3 --kernel-trace --stats   (+ the plugin / gradient bench line in NAME_trace.log)
  OUT_DIR/NAME_fetch  rocprofv3 --pmc FETCH_SIZE
  OUT_DIR/NAME_write  rocprofv3 --pmc WRITE_SIZE
FETCH_SIZE / WRITE_SIZE (KB) are corrected as MI355X_MICROARCH.md prescribes for gfx950, calibrated on
the line's HBM probes in the same pass (bw_read_kernel streams exactly 4 GiB; bw_copy_kernel reads +
writes 4 GiB). A round's wave is one body launch + one edge launch (more when it was continued);
traffic per round = the summed counters of every dyn_wave_kernel dispatch / the rounds. Algorithmic
bytes per round = N clients x P x s_in + P x s_out (the fused aggregate's: the accumulators never
leave the registers). Writes profiles/TAG_dyn_traffic_NAME.json.
"""
import csv
import json
import statistics
import sys
from pathlib import Path

out_dir, name, tag = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
repo = Path(__file__).resolve().parent.parent
PROBE = 4 << 30


def rows(pass_dir: str, fname: str = "run_counter_collection.csv") -> list[dict]:
    return list(csv.DictReader(open(out_dir / pass_dir / fname)))


def counter(pass_dir: str, substr: str) -> list[float]:
    return [float(r["Counter_Value"]) for r in rows(pass_dir) if substr in r["Kernel_Name"]]


line = next(json.loads(x) for x in open(out_dir / f"{name}_trace.log") if x.startswith("{"))
cfg = line["config"]
N, P = cfg["clients"], cfg["params_per_client"]
s_in = {"float32": 4, "float16": 2, "bfloat16": 2, "float64": 8}[cfg["in_dtype"]]
s_out = {"float32": 4, "float64": 8}[cfg["out_dtype"]]
algorithmic = N * P * s_in + P * s_out
read_corr = PROBE / (statistics.median(counter(f"{name}_fetch", "bw_read_kernel")) * 1024)
write_corr = PROBE / (statistics.median(counter(f"{name}_write", "bw_copy_kernel")) * 1024)


def per_kind(pass_dir: str) -> dict[str, list[float]]:
    out: dict[str, list[float]] = {"body": [], "edge": []}
    for r in rows(pass_dir):
        k = r["Kernel_Name"]
        if "dyn_wave_kernel" in k:
            out["edge" if "true" in k.split("dyn_wave_kernel", 1)[1][:40] else "body"].append(float(r["Counter_Value"]))
    return out


fetch, write = per_kind(f"{name}_fetch"), per_kind(f"{name}_write")
rounds = len(fetch["body"])  # one body launch per round (continued waves would add launches: see waves_per_round)
fetch_b = (sum(fetch["body"]) + sum(fetch["edge"])) * 1024 * read_corr
write_b = (sum(write["body"]) + sum(write["edge"])) * 1024 * write_corr
waves_per_round = line["config"].get("dynamic_wave", {}).get("waves", 1) or 1
n_rounds = rounds / max(1.0, 1.0 + line["config"].get("dynamic_wave", {}).get("reopens", 0))
traffic = (fetch_b + write_b) / n_rounds if n_rounds else None
# kernel-trace durations of the body launches (enqueue-independent: GPU start -> end)
durs = []
try:
    for r in rows(f"{name}_trace", "run_kernel_trace.csv"):
        if "dyn_wave_kernel" in r["Kernel_Name"] and "false" in r["Kernel_Name"].split("dyn_wave_kernel", 1)[1][:40]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
except (FileNotFoundError, KeyError):
    pass
dyn = line["config"].get("dynamic_wave", {})
res = {
    "tag": tag, "workload": cfg["workload"], "kernel": "dyn_wave_kernel (body + edge launches)",
    "rounds_profiled": n_rounds, "dispatches": {"body": len(fetch["body"]), "edge": len(fetch["edge"])},
    "fetch_bytes_per_round": fetch_b / n_rounds if n_rounds else None,
    "write_bytes_per_round": write_b / n_rounds if n_rounds else None,
    "hbm_traffic_bytes_per_round": traffic, "algorithmic_bytes_per_round": algorithmic,
    "traffic_over_algorithmic": traffic / algorithmic if traffic else None,
    "body_launch_ms_median_kernel_trace": round(statistics.median(durs), 4) if durs else None,
    "fold_after_last_rows_ms_median": dyn.get("rows_to_end_ms_median"),
    "fold_after_close_seen_ms_median": dyn.get("close_to_end_ms_median"),
    "calibration": {"read_correction": read_corr, "write_correction": write_corr, "probe_bytes": PROBE},
    "bench_line": {k: line[k] for k in ("value", "unit", "ms_per_step")},
    "source": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE (separate passes), "
              "scripts/dyn_traffic.sh",
}
(repo / "profiles" / f"{tag}_dyn_traffic_{name}.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
