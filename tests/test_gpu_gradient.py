"""GradientWorker-style rounds on the MI355X (gradient_worker.py:83-93): every training step each
worker sends its native-dtype gradient dict with ``in_round=True`` and its dataset size as the
weight, and blocks for the average. Many short rounds on one long-lived FedAVGAlgorithm (the
server's steady state, aggregation_server.py:111-172) must each be bit-identical to the oracle and
carry ``in_round`` through."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu

# a small conv net's named gradients (weights + biases + a BN scale, ragged sizes)
SHAPES = {"conv1.weight": (16, 3, 3, 3), "conv1.bias": (16,), "bn.weight": (16,), "conv2.weight": (32, 16, 3, 3),
          "fc.weight": (10, 1152), "fc.bias": (10,)}


def _np(t: torch.Tensor) -> np.ndarray:
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("workers", [4, 16])
def test_in_round_gradient_rounds_bit_identical(hip_device, dtype, workers):
    rng = np.random.default_rng(workers)
    sizes = [int(x) for x in rng.integers(100, 5001, size=workers)]  # trainer.dataset_size per worker
    algo = FedAVGAlgorithm(device=hip_device)
    g = torch.Generator().manual_seed(3)
    for step in range(5):
        oracle = OracleFedAvg()
        for wid in rng.permutation(workers):  # arrival order changes every step
            wid = int(wid)
            grads = {n: (torch.randn(s, generator=g) * 1e-2).to(dtype) for n, s in SHAPES.items()}
            algo.process_worker_data(wid, ParameterMessage(parameter={n: t.to(hip_device) for n, t in grads.items()},
                                                           in_round=True, aggregation_weight=sizes[wid]))
            oracle.process_worker_data(wid, OracleMessage(parameter={n: _np(t) for n, t in grads.items()},
                                                          in_round=True, aggregation_weight=sizes[wid],
                                                          dtype="bfloat16" if dtype == torch.bfloat16 else None))
        res = algo.aggregate_worker_data()
        want = oracle.aggregate_worker_data()
        assert res.in_round and want.in_round
        assert list(res.parameter) == list(want.parameter)
        for n, w in want.parameter.items():
            assert bits_equal(res.parameter[n].cpu().numpy(), w), (step, n)
        algo.clear_worker_data()
