"""Per-kernel summary of a rocprofv3 kernel trace (its rocpd SQLite database or kernel_trace.csv):
calls, mean / min / max duration in microseconds, and the launch geometry.

    python scripts/rocpd_summary.py gpurun_out/<tag>/<dir> [--json out.json]
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sqlite3
import statistics


def _rows(path: str) -> list[dict]:
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) else [path]
    dbs = [d for d in dbs if d.endswith(".db")]
    if dbs:
        c = sqlite3.connect(dbs[0])
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        return [dict(zip(cols, r)) for r in c.execute("select * from kernels order by start")]
    csvs = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    out = []
    with open(csvs[0]) as f:
        for r in csv.DictReader(f):
            out.append({"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                        "grid_x": int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
                        "workgroup_x": int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)})
    return out


def summary(path: str) -> list[dict]:
    by: dict[str, list] = {}
    for r in _rows(path):
        by.setdefault(r["name"], []).append(r)
    out = []
    for name, rs in by.items():
        d = [(r["end"] - r["start"]) / 1e3 for r in rs]
        out.append({"kernel": name[:120], "calls": len(rs), "mean_us": round(statistics.mean(d), 2),
                    "min_us": round(min(d), 2), "max_us": round(max(d), 2),
                    "grid": rs[0].get("grid_x"), "workgroup": rs[0].get("workgroup_x")})
    return sorted(out, key=lambda x: -x["mean_us"] * x["calls"])


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--json")
    a = ap.parse_args()
    s = summary(a.path)
    for r in s:
        print(f"{r['calls']:5d} {r['mean_us']:10.2f} {r['min_us']:10.2f} {r['max_us']:10.2f}  {r['kernel']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(s, f, indent=1)


if __name__ == "__main__":
    main()
