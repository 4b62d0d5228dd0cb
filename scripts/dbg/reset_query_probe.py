"""Debug: the caller's stream state (hipStreamQuery) at each FedAvgContext.reset of plugin rounds."""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage  # noqa: E402
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
layout = resnet18_layout()
K = 64
w = dataset_size_weights(K)
_, views = make_clients(layout, 0, K, dev, torch.float32)
params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
log = []
_reset, _nan, _close = FedAvgContext.reset, FedAvgContext.raise_on_nan, FedAvgContext.dyn_close


def reset(self, *a, **k):
    log.append(("reset", hip.hipStreamQuery(self.stream)))
    return _reset(self, *a, **k)


def nan(self, *a, **k):
    r = _nan(self, *a, **k)
    log.append(("after_nan", hip.hipStreamQuery(self.stream)))
    return r


def close(self, *a, **k):
    r = _close(self, *a, **k)
    log.append(("after_close", hip.hipStreamQuery(self.stream)))
    return r


FedAvgContext.reset, FedAvgContext.raise_on_nan, FedAvgContext.dyn_close = reset, nan, close
algo = FedAVGAlgorithm(device=dev, result_dtype=torch.float64)
for r in range(4):
    for i, (p, x) in enumerate(zip(params, w)):
        algo.process_worker_data(i, ParameterMessage(parameter=dict(p), aggregation_weight=x))
    log.append(("round", r))
    algo.aggregate_worker_data()
    log.append(("aggregated", hip.hipStreamQuery(dev and FedAvgContext.stream.fget(algo._context()))))
    algo.clear_worker_data()
print(log)
