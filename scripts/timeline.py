"""Summarise a rocprofv3 kernel trace: per-step GPU busy time and the gaps between kernels."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = 20 if len(sys.argv) < 3 else int(sys.argv[2])
rows = rows[-400:]
prev_end = None
gaps = []
per_kernel = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"][:60]
    per_kernel[name].append((e - s) / 1e3)
    if prev_end is not None:
        gaps.append((s - prev_end) / 1e3)
    prev_end = e
for k, v in per_kernel.items():
    print(f"{k:60s} n={len(v):4d} mean={sum(v)/len(v):9.2f} us total={sum(v):10.1f} us")
gaps_sorted = sorted(gaps)
print(f"gaps: n={len(gaps)} total={sum(gaps):.1f} us median={gaps_sorted[len(gaps)//2]:.2f} max={gaps_sorted[-1]:.1f}")
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"span of last {len(rows)} kernels: {span:.1f} us")
