"""Debug: which HIP API call enqueued each fill kernel in a rocprofv3 --hip-trace database
(prints the last rounds' kernels with the API call that launched them)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print([t for t in tabs if not t.startswith("rocpd_") or "region" in t][:30])
kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
kern = [dict(zip(kcols, r)) for r in c.execute("select * from kernels order by start")]
rtab = "regions" if "regions" in tabs else None
api = {}
if rtab:
    rcols = [r[1] for r in c.execute(f"pragma table_info({rtab})")]
    print(rcols)
    for r in c.execute(f"select * from {rtab}"):
        d = dict(zip(rcols, r))
        api[d.get("corr_id") or d.get("id")] = d
t0 = kern[-12]["start"]
for k in kern[-12:]:
    a = api.get(k.get("corr_id"))
    print(k["name"][:40], round((k["start"] - t0) / 1e3, 1), round((k["end"] - k["start"]) / 1e3, 1),
          a and a.get("name"), a and round((a["start"] - t0) / 1e3, 1))
