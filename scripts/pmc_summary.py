"""Print per-counter means for kernels matching a substring from rocprofv3 *_results.db files."""
import collections
import sqlite3
import sys

sub = sys.argv[1]
for path in sys.argv[2:]:
    db = sqlite3.connect(path)
    agg = collections.defaultdict(list)
    for name, counter, value in db.execute("select kernel_name, counter_name, value from counters_collection"):
        if sub in name:
            agg[counter].append(value)
    print(path)
    for k, v in sorted(agg.items()):
        print(f"  {k:24s} n={len(v):3d} mean={sum(v) / len(v):.4g}")
