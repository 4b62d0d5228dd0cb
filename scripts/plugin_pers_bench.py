"""Host overhead of the PersonalizedFedAVG plugin with device-resident updates (GPU box).

64 workers x ResNet-18 fp32 already in HBM, every worker a receiver (float weights), driven
through PersonalizedFedAVGAlgorithm (set_worker_weights once): process_worker_data x 64,
aggregate_worker_data (results left on the device), one algorithm object across rounds (cleared
after each, as the server does). Reports the round, the kernel alone (the context's own launch on
the same staged table, HIP events) and a breakdown of the host side.
"""

from __future__ import annotations

import cProfile
import json
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import ParameterMessage, PersonalizedFedAVGAlgorithm  # noqa: E402

K = 64
dev = torch.device("cuda", 0)
layout = resnet18_layout()
buckets, views = make_clients(layout, 0, K, dev, torch.float32)
params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
rng = np.random.default_rng(3)
ww = {j: {i: float(rng.uniform(0.01, 3.0)) for i in range(K) if i != j} for j in range(K)}


def plugin_round(algo):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        algo.process_worker_data(k, ParameterMessage(parameter=dict(params[k])))
    t1 = time.perf_counter()
    res = algo.aggregate_worker_data()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    algo.clear_worker_data()
    assert len(res.worker_data) == K
    return t2 - t0, t1 - t0


algo = PersonalizedFedAVGAlgorithm(device=dev)
algo.set_worker_weights(ww)  # once (the reference asserts it is set once)
plugin_round(algo)
runs = [plugin_round(algo) for _ in range(5)]
best = min(runs)
pr = cProfile.Profile()
pr.enable()
plugin_round(algo)
pr.disable()
print(json.dumps({"workload": "PersonalizedFedAVG plugin, 64 workers x 64 receivers x ResNet-18 fp32, device-resident",
                  "round_ms": round(best[0] * 1e3, 3), "process_worker_data_ms": round(best[1] * 1e3, 3)}))
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
