"""bench.py helpers that run without a GPU: the pinned CPU baseline child, the committed-traffic
lookups, the speed-up block (CPU)."""

from __future__ import annotations

import importlib.util
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_helpers_mod", REPO / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    argv = sys.argv
    sys.argv = ["bench.py"]
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.argv = argv
    return mod


def test_cpu_baseline_runs_pinned_in_a_child(bench, monkeypatch):
    # a tiny sample: 2 clients of the flat 1M layout, 3 repeats; the child pins itself to the CPUs
    # it was given and reports the spread and the host's load beside the best round
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    layout = bench.LAYOUTS["flat1m"]()
    cb = bench.cpu_baseline(layout, n_clients=2, repeats=3, budget_s=5.0)
    assert cb["kind"] == "port" and cb["cores"] == 2 and cb["value"] > 0
    rep = cb["repeats"]
    assert rep["n"] == 3 and rep["min_s"] <= rep["median_s"] <= rep["max_s"]
    assert cb["seconds_per_round"] == rep["min_s"]
    assert len(cb["pinning"]["cpus"]) == min(2, len(os.sched_getaffinity(0)))
    assert set(cb["pinning"]["cpus"]) <= set(os.sched_getaffinity(0))
    assert cb["pinning"]["threads_seen"] == 2
    assert len(cb["host_load"]["loadavg_1_5_15_before"]) == 3


def test_gpu_local_cpus_falls_back_to_the_affinity_mask(bench):
    cpus, source = bench.gpu_local_cpus(0)  # no GPU here: the sysfs lookup cannot run
    assert cpus == sorted(os.sched_getaffinity(0)) and "affinity" in source


def test_committed_dyn_traffic_matches_the_workload(bench):
    t, ratio, src = bench.committed_dyn_traffic("plugin_fedavg_resnet18_fp32_64_clients")
    assert t and 0.9 < ratio < 1.2 and src.startswith("profiles/r") and "dyn_traffic_plugin" in src
    assert bench.committed_dyn_traffic("no_such_workload") == (None, None, None)


def test_committed_headline_traffic(bench):
    t, src = bench.committed_traffic(1, 64, "float32", "float32")
    assert t and src.startswith("profiles/r") and src.endswith("_traffic.json")
    assert bench.committed_traffic(2, 64, "float32", "float32") == (None, None)
