"""Host cost of FedAVGAlgorithm.process_worker_data per device-resident update (GPU box): wall time
per call, and a cProfile of 20 rounds x 64 ResNet-18 updates (tottime per function)."""
from __future__ import annotations

import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage  # noqa: E402

K, R = 64, 20
dev = torch.device("cuda", 0)
layout = resnet18_layout()
w = dataset_size_weights(K)
_, views = make_clients(layout, 0, K, dev, torch.float32)
params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
algo = FedAVGAlgorithm(device=dev, wave_size=K)


def msgs():
    return [ParameterMessage(parameter=dict(p), aggregation_weight=x) for p, x in zip(params, w)]


for _ in range(3):
    for i, m in enumerate(msgs()):
        algo.process_worker_data(i, m)
    algo.aggregate_worker_data()
    algo.clear_worker_data()
torch.cuda.synchronize()
tot = 0.0
pr = cProfile.Profile()
for r in range(R):
    ms = msgs()
    t0 = time.perf_counter()
    for i, m in enumerate(ms):
        algo.process_worker_data(i, m)
    tot += time.perf_counter() - t0
    algo.aggregate_worker_data()
    algo.clear_worker_data()
print(f"process_worker_data: {tot / (R * K) * 1e6:.2f} us per update")
ms = msgs()
pr.enable()
for _ in range(5):
    for i, m in enumerate(ms):
        algo.process_worker_data(i, m)
    algo.aggregate_worker_data()
    algo.clear_worker_data()
    ms = msgs()
pr.disable()
buf = io.StringIO()
pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
print(buf.getvalue())
