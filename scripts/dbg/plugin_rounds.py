"""Debug: N plugin rounds of 64 ResNet-18 updates through FedAVGAlgorithm, nothing else."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from bench import dataset_size_weights, make_clients, resnet18_layout  # noqa: E402
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage  # noqa: E402

dev = torch.device("cuda", 0)
layout = resnet18_layout()
K = 64
w = dataset_size_weights(K)
_, views = make_clients(layout, 0, K, dev, torch.float32)
params = [{n: v.view(s) for n, s, v in zip(layout.names, layout.shapes, row)} for row in views]
algo = FedAVGAlgorithm(device=dev, result_dtype=torch.float64)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for i, (p, x) in enumerate(zip(params, w)):
        algo.process_worker_data(i, ParameterMessage(parameter=dict(p), aggregation_weight=x))
    algo.aggregate_worker_data()
    algo.clear_worker_data()
print("done")
