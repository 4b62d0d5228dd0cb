"""Per-dispatch wave-cycle breakdown of the FedAvg tile kernel from rocprofv3 PMC databases
(scripts/gpu_fedavg_pmc.sh): share of wave cycles parked on s_waitcnt (SQ_WAIT_ANY), stalled at
issue (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY) — disjoint, they sum to
SQ_WAVE_CYCLES (MI355X_MICROARCH.md, SQ counters) — plus VALU instructions and duration.

    python scripts/pmc_dispatch_summary.py gpurun_out/fa_pmc/pmc_<name>_results.db ...
"""
import collections
import re
import sqlite3
import sys

for path in sys.argv[1:]:
    db = sqlite3.connect(path)
    ctr = collections.defaultdict(dict)
    meta = {}
    q = ("select dispatch_id, kernel_name, counter_name, value, start, end, vgpr_count "
         "from counters_collection where kernel_name like '%fedavg_tile_kernel%'")
    for disp, name, c, v, st, en, vg in db.execute(q):
        ctr[disp][c] = v
        m = re.search(r"fedavg_tile_kernel<([^>]*)>", name)
        meta[disp] = (m.group(1) if m else name[:60], (en - st) / 1e6, vg)
    print(path)
    print("  dispatch  kernel<T, OUT, SPLIT, VEC, FOLD, TILEN>           ms    vgpr  waitcnt  issue-stall  issuing  VALU insts")
    for d in sorted(ctr):
        c = ctr[d]
        wc = c["SQ_WAVE_CYCLES"]
        k, ms, vg = meta[d]
        print(f"  {d:8d}  {k:45s} {ms:6.3f}  {vg:4d}  {c['SQ_WAIT_ANY'] / wc:7.2f}  {c['SQ_WAIT_INST_ANY'] / wc:11.2f}"
              f"  {c['SQ_ACTIVE_INST_ANY'] / wc:7.2f}  {c['SQ_INSTS_VALU']:.3g}")
