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


def per_kind(pass_dir: str, fname: str = "run_counter_collection.csv", value=lambda r: float(r["Counter_Value"])):
    """The dyn_wave_kernel dispatches split into body / edge launches (names are truncated by -T:
    the body launch is the one with the larger grid — a workgroup per 6,144-element body tile)."""
    dyn = [r for r in rows(pass_dir, fname) if "dyn_wave_kernel" in r["Kernel_Name"]]
    body_grid = max((int(r.get("Grid_Size") or r["Grid_Size_X"]) for r in dyn), default=0)
    out: dict[str, list[float]] = {"body": [], "edge": []}
    for r in dyn:
        out["body" if int(r.get("Grid_Size") or r["Grid_Size_X"]) == body_grid else "edge"].append(value(r))
    return out


fetch, write = per_kind(f"{name}_fetch"), per_kind(f"{name}_write")
# one body launch per wave; a round's wave is continued (another launch pair) reopens times
n_rounds = len(fetch["body"]) / (1.0 + (line["config"].get("dynamic_wave", {}).get("reopens", 0) or 0))
fetch_b = (sum(fetch["body"]) + sum(fetch["edge"])) * 1024 * read_corr
write_b = (sum(write["body"]) + sum(write["edge"])) * 1024 * write_corr
traffic = (fetch_b + write_b) / n_rounds if n_rounds else None
# kernel-trace durations of the body launches (GPU start -> end: the arrival phase included)
durs = per_kind(f"{name}_trace", "run_kernel_trace.csv",
                lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)["body"]
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
