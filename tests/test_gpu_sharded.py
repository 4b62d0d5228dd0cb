"""The sharded (multi-GPU) path's HIP + RCCL pieces on one GPU: a one-rank nccl group forced
through partial -> chunked RCCL reduce -> chunked finalize, against the fused kernel."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
from distributed_learning_simulation_lib_amd.sharded import HipLocalReducer, sharded_reduce

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def nccl_group(hip_device):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=hip_device)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("chunks", [1, 3, 8])
def test_forced_collective_matches_fused(chunks, hip_device, nccl_group):
    rng = np.random.default_rng(chunks)
    layout = ModelLayout(names=("a", "b", "c"), shapes=((70001,), (33, 65), (9000,)))
    g = torch.Generator().manual_seed(chunks)
    rows = [[torch.randn(n, generator=g).to(hip_device) for n in layout.numels] for _ in range(12)]
    weights = [float(rng.integers(100, 5000)) for _ in range(12)]
    table = ClientTable(3)
    for r, w in zip(rows, weights):
        table.add_client(r, [w] * 3)
    totals = [sum(weights)] * 3

    ctx_a = FedAvgContext(layout, hip_device)
    out_a = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in layout.numels]
    sharded_reduce(HipLocalReducer(ctx_a, table, torch.float32, out_a, torch.float64), totals, chunks=chunks)

    ctx_b = FedAvgContext(layout, hip_device)
    out_b = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in layout.numels]
    got = sharded_reduce(HipLocalReducer(ctx_b, table, torch.float32, out_b, torch.float64), totals,
                         chunks=chunks, force_collective=True)
    assert got == totals
    ctx_b.raise_on_nan()
    for a, b in zip(out_a, out_b):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))
