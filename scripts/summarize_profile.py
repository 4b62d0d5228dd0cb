"""Turn a scripts/profile.sh output directory into the committed profiles/<tag>_*.json/csv.

HBM traffic per launch of the main kernel is FETCH_SIZE/WRITE_SIZE (KB) corrected the way
MI355X_MICROARCH.md prescribes for gfx950: calibrated on a known byte count in the same access
pattern. bench.py's probes run in the same pass: bw_read_kernel streams exactly 4 GiB with
16-B/lane non-temporal loads (like the main kernel) and bw_copy_kernel reads + writes 4 GiB; the
ratio known-bytes / counter-bytes of the probes is the correction applied to the main kernel.
"""
import csv
import json
import shutil
import statistics
import sys
from pathlib import Path

out_dir = Path(sys.argv[1])
tag = sys.argv[2]
repo = Path(__file__).resolve().parent.parent
prof = repo / "profiles"
prof.mkdir(exist_ok=True)
PROBE_BYTES = 4 << 30


def counter(pass_name, kernel_substr):
    rows = list(csv.DictReader(open(out_dir / pass_name / "run_counter_collection.csv")))
    return [float(r["Counter_Value"]) for r in rows if kernel_substr in r["Kernel_Name"]]


stats_src = out_dir / "trace" / "run_kernel_stats.csv"
shutil.copy(stats_src, prof / f"{tag}_kernel_stats.csv")
stats = {r["Name"]: r for r in csv.DictReader(open(stats_src))}
main_avg_ns = float(stats["fedavg_tile_kernel"]["AverageNs"])

fetch_main = statistics.mean(counter("fetch", "fedavg_tile_kernel"))
write_main = statistics.mean(counter("write", "fedavg_tile_kernel"))
fetch_read_probe = statistics.median(counter("fetch", "bw_read_kernel"))
fetch_copy_probe = statistics.median(counter("fetch", "bw_copy_kernel"))
write_copy_probe = statistics.median(counter("write", "bw_copy_kernel"))
read_corr = PROBE_BYTES / (fetch_read_probe * 1024)
write_corr = PROBE_BYTES / (write_copy_probe * 1024)
P, K = 11_689_512, 64
alg = K * P * 4 + P * 4
traffic = fetch_main * 1024 * read_corr + write_main * 1024 * write_corr
out = {
    "tag": tag,
    "kernel": "fedavg_tile_kernel<float, OUT_F32, 1, true, fma>",
    "workload": "64 clients x ResNet-18 (62 tensors, 11,689,512 params) fp32 -> fp32, fp64 accumulation",
    "kernel_avg_ms_rocprof": main_avg_ns / 1e6,
    "algorithmic_bytes_per_launch": alg,
    "achieved_GBps_rocprof": alg / main_avg_ns,
    "FETCH_SIZE_KB_per_launch": fetch_main,
    "WRITE_SIZE_KB_per_launch": write_main,
    "calibration": {
        "read_probe_FETCH_SIZE_KB": fetch_read_probe,
        "copy_probe_FETCH_SIZE_KB": fetch_copy_probe,
        "copy_probe_WRITE_SIZE_KB": write_copy_probe,
        "probe_bytes": PROBE_BYTES,
        "read_correction": read_corr,
        "write_correction": write_corr,
    },
    "hbm_traffic_bytes_per_launch": traffic,
    "traffic_over_algorithmic": traffic / alg,
    "source": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE (separate passes), scripts/profile.sh",
}
(prof / f"{tag}_traffic.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out, indent=1))
