"""Where the plugin's host time per update goes (GPU box): 64 device-resident ResNet-18 fp32
updates through FedAVGAlgorithm, each piece of process_worker_data timed on its own over many
rounds (perf_counter around loops, no profiler overhead)."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage, _staging  # noqa: E402
from distributed_learning_simulation_lib_amd.algorithm.aggregation_algorithm import AggregationAlgorithm  # noqa: E402
from distributed_learning_simulation_lib_amd.message import is_delta_message, is_parameter_message  # noqa: E402

K, R = 64, 30
dev = torch.device("cuda", 0)
layout = resnet18_layout()
w = dataset_size_weights(K)
_, views = make_clients(layout, 0, K, dev, torch.float32)
params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]


def msgs():
    return [ParameterMessage(parameter=dict(p), aggregation_weight=x) for p, x in zip(params, w)]


out = {}
t0 = time.perf_counter()
for _ in range(R):
    msgs()
out["build_messages_us"] = (time.perf_counter() - t0) / (R * K) * 1e6

algo = FedAVGAlgorithm(device=dev, wave_size=K)
for _ in range(3):  # steady state
    for k, m in enumerate(msgs()):
        algo.process_worker_data(k, m)
    algo.aggregate_worker_data()
    algo.clear_worker_data()
torch.cuda.synchronize()

pw, agg, clr = 0.0, 0.0, 0.0
for _ in range(R):
    ms = msgs()
    a = time.perf_counter()
    for k, m in enumerate(ms):
        algo.process_worker_data(k, m)
    b = time.perf_counter()
    algo.aggregate_worker_data()
    torch.cuda.synchronize()
    c = time.perf_counter()
    algo.clear_worker_data()
    d = time.perf_counter()
    pw, agg, clr = pw + b - a, agg + c - b, clr + d - c
out["process_worker_data_us"] = pw / (R * K) * 1e6
out["aggregate_worker_data_ms"] = agg / R * 1e3
out["clear_worker_data_ms"] = clr / R * 1e3

base = type("Base", (AggregationAlgorithm,), {"aggregate_worker_data": lambda self: None})()
ms = msgs()
t0 = time.perf_counter()
for _ in range(R):
    for k, m in enumerate(ms):
        AggregationAlgorithm.process_worker_data(base, k, m)
out["base_process_worker_data_us"] = (time.perf_counter() - t0) / (R * K) * 1e6
t0 = time.perf_counter()
for _ in range(R):
    for m in ms:
        is_delta_message(m)
        is_parameter_message(m)
out["recognition_us"] = (time.perf_counter() - t0) / (R * K) * 1e6

index = {n: i for i, n in enumerate(layout.names)}
shapes = [tuple(s) for s in layout.shapes]
t0 = time.perf_counter()
for _ in range(R):
    tab = _staging.NativeClientTable(layout.num_segments, 0)
    for p, x in zip(params, w):
        tab.rows.append(p, index, shapes, x, -1)
out["native_rows_append_us"] = (time.perf_counter() - t0) / (R * K) * 1e6
print(json.dumps({k: round(v, 3) for k, v in out.items()}))

# aggregate_worker_data's pieces on the same 64-client table (the plugin's common path, by hand)
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext, OutputTable  # noqa: E402

ctx = FedAvgContext(layout, dev)
offs, total = layout.padded_offsets(8)
tab = _staging.NativeClientTable(layout.num_segments, 0)
for p, x in zip(params, w):
    tab.rows.append(p, index, shapes, x, -1)
ext = _staging.module()
t_alloc = t_enq = t_sync = t_flags = t_views = 0.0
for _ in range(R + 3):
    torch.cuda.synchronize()
    a = time.perf_counter()
    flat = torch.empty(total, dtype=torch.float64, device=dev)
    ot = OutputTable.from_flat(flat, offs, layout)
    b = time.perf_counter()
    ctx.aggregate(tab, torch.float32, ot, torch.float64)
    c = time.perf_counter()
    torch.cuda.synchronize()
    d = time.perf_counter()
    ctx.raise_on_nan([])
    e = time.perf_counter()
    ext.views(flat, offs, shapes)
    f = time.perf_counter()
    ctx.reset()
    if _ >= 3:
        t_alloc, t_enq, t_sync, t_flags, t_views = (t_alloc + b - a, t_enq + c - b, t_sync + d - c, t_flags + e - d,
                                                     t_views + f - e)
out2 = {"alloc_outputs_us": t_alloc / R * 1e6, "aggregate_enqueue_us": t_enq / R * 1e6,
        "kernel_wait_us": t_sync / R * 1e6, "flags_us": t_flags / R * 1e6, "views_us": t_views / R * 1e6}
print(json.dumps({k: round(v, 2) for k, v in out2.items()}))
