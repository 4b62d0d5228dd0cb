"""Print the last kernels of a rocprofv3 --kernel-trace CSV as a timeline (µs from the first
shown kernel), with the gap before each kernel: where a step's time goes between launches.

    python scripts/trace_timeline.py gpurun_out/strace_c4/trace_kernel_trace.csv [count]
"""

import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sel = rows[-int(sys.argv[2]) if len(sys.argv) > 2 else -24:]
    t0 = int(sel[0]["Start_Timestamp"])
    prev = None
    for r in sel:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        gap = "" if prev is None else f"gap {s - prev:6.1f}"
        print(f"{s:9.1f} {e:9.1f} {e - s:7.1f} {gap:11s} q{r['Queue_Id']} s{r['Stream_Id']} {r['Kernel_Name'][:64]}")
        prev = e


if __name__ == "__main__":
    main()
