"""cProfile of the plugin path with device-resident updates (scripts/plugin_device_bench.py's
round): where the host time of process_worker_data goes."""
import cProfile
import pstats
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.argv = [sys.argv[0]]
import plugin_device_bench as b  # noqa: E402  (runs its own measurement first)

pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    b.plugin_round(64)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
