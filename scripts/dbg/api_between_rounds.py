"""Debug: the HIP API calls of the last plugin round (from a rocprofv3 --hip-trace csv directory):
names in call order from the second-to-last dynamic-wave launch, repeated names collapsed."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*hip_api_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Function"] for r in rows]
launches = [i for i, n in enumerate(names) if n in ("hipLaunchKernel", "hipExtLaunchKernel", "hipModuleLaunchKernel")]
start = launches[-6] if len(launches) >= 6 else 0
out, prev, cnt = [], None, 0
for n in names[start:]:
    if n == prev:
        cnt += 1
        continue
    if prev is not None:
        out.append(f"{prev}x{cnt}" if cnt > 1 else prev)
    prev, cnt = n, 1
out.append(f"{prev}x{cnt}")
print(" ".join(out))
