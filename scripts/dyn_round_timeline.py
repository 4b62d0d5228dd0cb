"""Where a plugin round's time goes with the dynamic wave (GPU box): K device-resident ResNet-18 fp32
updates through FedAVGAlgorithm, wall-clock marks (microseconds from the round's first
process_worker_data call) at the wave's open, every publication, the last arrival, the close
(entry / return), the NaN readback and the round's end. Prints one JSON line of means over R rounds.

    python scripts/dyn_round_timeline.py [K] [R]
"""
from __future__ import annotations

import json
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
R = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda", 0)
layout = resnet18_layout()
w = dataset_size_weights(K)
_, views = make_clients(layout, 0, K, dev, torch.float32)
params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]

marks: dict[str, float] = {}
pubs: list[tuple[float, int]] = []


def wrap(name, fn, record=None):
    def inner(self, *a, **k):
        marks[name + "_in"] = time.perf_counter()
        r = fn(self, *a, **k)
        marks[name + "_out"] = time.perf_counter()
        if record is not None:
            record(r)
        return r
    return inner


FedAvgContext.dyn_open = wrap("open", FedAvgContext.dyn_open)
_pub = FedAvgContext.dyn_publish


def pub(self, table):
    t = time.perf_counter()
    n = _pub(self, table)
    pubs.append((time.perf_counter() - t, n))
    return n


FedAvgContext.dyn_publish = pub
FedAvgContext.dyn_close = wrap("close", FedAvgContext.dyn_close)
FedAvgContext.raise_on_nan = wrap("nan", FedAvgContext.raise_on_nan)
FedAvgContext.reset = wrap("reset", FedAvgContext.reset)

algo = FedAVGAlgorithm(device=dev, result_dtype=torch.float64)
rows: list[dict] = []
for r in range(R + 5):
    marks.clear()
    pubs.clear()
    msgs = [ParameterMessage(parameter=dict(p), aggregation_weight=x) for p, x in zip(params, w)]
    t0 = time.perf_counter()
    for i, m in enumerate(msgs):
        algo.process_worker_data(i, m)
    t_arr = time.perf_counter()
    algo.aggregate_worker_data()
    t_agg = time.perf_counter()
    algo.clear_worker_data()
    t_end = time.perf_counter()
    if r < 5:
        continue
    us = lambda t: (t - t0) * 1e6  # noqa: E731
    rows.append({"open_in": us(marks["open_in"]), "open_out": us(marks["open_out"]), "arrivals_done": us(t_arr),
                 "close_in": us(marks["close_in"]), "close_out": us(marks["close_out"]),
                 "nan_in": us(marks["nan_in"]), "nan_out": us(marks["nan_out"]), "aggregate_out": us(t_agg),
                 "round_end": us(t_end), "publications": len(pubs),
                 "published_rows_before_close": sum(n for _, n in pubs[:-1]),
                 "publish_us_total": sum(d for d, _ in pubs) * 1e6})
out = {k: round(statistics.mean(x[k] for x in rows), 1) for k in rows[0]}
out["round_ms_median"] = round(statistics.median(x["round_end"] for x in rows) / 1e3, 4)
out.update(clients=K, rounds=R, dyn_stats=algo.dyn_stats)
print(json.dumps(out), flush=True)
