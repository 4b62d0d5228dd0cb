"""BASELINE config 1: 4 worker processes x 1M fp32 over pipes -> one server process.

The reference's own CPU-runnable case (configs[0]): its simulator cannot run here (unvendored
`cyy_*` dependencies), so this is the build's own loopback with the server's
per-message contract (aggregation_server.py:111-175) and the poll loop (server.py:122-152).
CPU test: the server's algorithm is the oracle (checker for the IPC / sequencing logic).
GPU test: the same loopback with the HIP FedAVGAlgorithm, bit-identical to the oracle.
"""

from __future__ import annotations

import multiprocessing as mp
import time

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd.server import AggregationServer, PipeServerEndpoint, run_pipe_worker
from oracle.fedavg_oracle import fedavg_flat
from tests.helpers import OracleAlgorithm, config1_update

WORKERS, ROUNDS, NUMEL = 4, 2, 1_000_000


def _worker(conn, wid):
    run_pipe_worker(conn, lambda r: config1_update(wid, r, NUMEL), ROUNDS)


def run_loopback(algorithm):
    ctx = mp.get_context("spawn")
    pipes = [ctx.Pipe() for _ in range(WORKERS)]
    procs = [ctx.Process(target=_worker, args=(pipes[i][1], i)) for i in range(WORKERS)]
    for p in procs:
        p.start()
    srv = AggregationServer(algorithm=algorithm, worker_number=WORKERS,
                            endpoint=PipeServerEndpoint([p[0] for p in pipes]), round_number=ROUNDS)
    t0 = time.perf_counter()
    srv.start()
    elapsed = time.perf_counter() - t0
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return srv, elapsed


def expected(round_idx, order):
    """The oracle in the server's actual arrival order (the fp64 sum is order-sensitive)."""
    ups = [config1_update(w, round_idx, NUMEL) for w in order]
    return fedavg_flat([u.parameter["model"].numpy() for u in ups], [u.aggregation_weight for u in ups])


def test_config1_loopback_cpu_oracle():
    srv, elapsed = run_loopback(OracleAlgorithm())
    assert len(srv.results) == ROUNDS
    for r in range(ROUNDS):
        got = srv.results[r].parameter["model"].numpy()
        assert np.array_equal(got.view(np.uint64), expected(r, srv.arrivals[r]).view(np.uint64))
    print(f"config 1 loopback (oracle): {ROUNDS} rounds in {elapsed:.2f} s, per round {srv.round_seconds}")


@pytest.mark.gpu
def test_config1_loopback_hip(hip_device):
    from distributed_learning_simulation_lib_amd import FedAVGAlgorithm

    srv, elapsed = run_loopback(FedAVGAlgorithm(device=hip_device))
    for r in range(ROUNDS):
        got = srv.results[r].parameter["model"].numpy()
        assert got.dtype == np.float64
        assert np.array_equal(got.view(np.uint64), expected(r, srv.arrivals[r]).view(np.uint64))
    print(f"config 1 loopback (HIP): {ROUNDS} rounds in {elapsed:.2f} s, per round {srv.round_seconds}")


@pytest.mark.gpu
def test_server_delta_rounds_hip_vs_oracle(hip_device):
    """Round 1 full updates, round 2 delta updates: the HIP algorithm gets the deltas unrestored
    (fused restore, fedavg_*_delta); the oracle server restores on the host. Bit-identical."""
    from distributed_learning_simulation_lib_amd import DeltaParameterMessage, FedAVGAlgorithm
    from distributed_learning_simulation_lib_amd.message import ParameterMessage

    def rounds(srv):
        g = torch.Generator().manual_seed(3)
        shapes = {"w": (4099,), "b": (33,)}
        for wid in range(3):
            srv._process_worker_data(wid, ParameterMessage(
                parameter={k: torch.randn(s, generator=g) for k, s in shapes.items()}, aggregation_weight=10 + wid))
        for wid in range(3):
            delta = {k: torch.randn(s, generator=g, dtype=torch.float64) * 1e-3 for k, s in shapes.items()}
            srv._process_worker_data(wid, DeltaParameterMessage(delta_parameter=delta, aggregation_weight=7 * wid + 1))
        return srv.results

    hip = rounds(AggregationServer(algorithm=FedAVGAlgorithm(device=hip_device), worker_number=3, round_number=2))
    ref = rounds(AggregationServer(algorithm=OracleAlgorithm(), worker_number=3, round_number=2))
    for rh, rr in zip(hip, ref):
        for k in rr.parameter:
            assert torch.equal(rh.parameter[k].view(torch.int64), rr.parameter[k].view(torch.int64)), k
