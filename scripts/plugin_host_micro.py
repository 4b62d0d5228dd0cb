"""Per-update host costs of the plugin path on the GPU box (µs per update, medians of R rounds):
building the ParameterMessage, the native row append alone (staging_ext Rows.append over the
update's 62 tensors), and the whole FedAVGAlgorithm.process_worker_data; then the pieces of one
aggregate_worker_data (scripts/plugin_round_timeline.py has the full timeline). argv: clients."""
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
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage, _staging  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
R = 30
dev = torch.device("cuda", 0)
layout = resnet18_layout()
w = dataset_size_weights(K)
_, views = make_clients(layout, 0, K, dev, torch.float32)
params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
ext = _staging.module()
index = {n: i for i, n in enumerate(layout.names)}
shapes = [tuple(s) for s in layout.shapes]

res: dict[str, list[float]] = {"message": [], "rows_append": [], "process_worker_data": [], "round": []}
algo = FedAVGAlgorithm(device=dev)
for r in range(R + 3):
    t0 = time.perf_counter()
    msgs = [ParameterMessage(parameter=dict(p), aggregation_weight=x) for p, x in zip(params, w)]
    t1 = time.perf_counter()
    rows = ext.Rows(len(layout.names), 0)
    for p, x in zip(params, w):
        rows.append(p, index, shapes, x, 0)
    t2 = time.perf_counter()
    for i, m in enumerate(msgs):
        algo.process_worker_data(i, m)
    t3 = time.perf_counter()
    algo.aggregate_worker_data()
    algo.clear_worker_data()
    t4 = time.perf_counter()
    del rows
    if r >= 3:
        res["message"].append((t1 - t0) / K * 1e6)
        res["rows_append"].append((t2 - t1) / K * 1e6)
        res["process_worker_data"].append((t3 - t2) / K * 1e6)
        res["round"].append((t4 - t2) * 1e6)
print(json.dumps({k + ("_us" if k == "round" else "_us_per_update"): round(statistics.median(v), 3)
                  for k, v in res.items()} | {"clients": K, "tensors": layout.num_segments}))
