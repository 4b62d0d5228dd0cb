"""The multi-rank round with the real HIP kernels: two processes on the one GPU.

RCCL refuses two ranks on one device, so the exchange runs over a ``gloo`` process group, which
``sharded_reduce`` stages through host memory; everything else is the product path — each rank
folds its shard with the HIP partial kernels (``HipLocalReducer``: prepared plans, tile chunks),
the root finalizes (reduce exchange) or every rank divides its window and the root copies the
gathered result out (scatter exchange, ``fedavg_plan_finalize_window`` / ``fedavg_plan_copy_out``).

Parity: each rank's partial is the exact arrival-order fp64 chain of its shard; with two ranks
the cross-rank sum S0 + S1 is one correctly rounded fp64 addition whatever the order, so the
result equals the oracle's (S0 + S1) / W bit for bit, and the reference's single chain
(fed_avg_algorithm.py:43-99) within |Δ| <= 1e-12 * sum|w x| / W (DESIGN.md §5 tolerance).
"""

from __future__ import annotations


import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.fedavg_oracle import fedavg_flat
from tests.helpers import rendezvous_url

pytestmark = pytest.mark.gpu

SHAPES = ((70001,), (33, 65), (4096 * 3,), (7,))
N_CLIENTS = 9


def _clients():
    g = torch.Generator().manual_seed(11)
    clients = [[torch.randn(int(np.prod(s)), generator=g) for s in SHAPES] for _ in range(N_CLIENTS)]
    weights = [float(w) for w in np.random.default_rng(12).integers(100, 5000, size=N_CLIENTS)]
    return clients, weights


def _rank_main(rank, world, port, exchange, pass_totals, nan_client, q):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
        from distributed_learning_simulation_lib_amd.sharded import HipLocalReducer, sharded_reduce

        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
        layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(SHAPES))), shapes=SHAPES)
        clients, weights = _clients()
        if nan_client is not None:
            clients[nan_client][0][1234] = float("nan")
        lo, hi = rank * N_CLIENTS // world, (rank + 1) * N_CLIENTS // world
        table = ClientTable(layout.num_segments)
        for c, w in zip(clients[lo:hi], weights[lo:hi]):
            table.add_client([t.to(device) for t in c], [w] * layout.num_segments)
        ctx = FedAvgContext(layout, device)
        outs = None
        if rank == 0:
            outs = [torch.full((n,), -1.0, dtype=torch.float64, device=device) for n in layout.numels]
        red = HipLocalReducer(ctx, table, torch.float32, outs, torch.float64)
        local = [sum(weights[lo:hi])] * layout.num_segments
        glob = [sum(weights)] * layout.num_segments if pass_totals else None
        for _ in range(2 if nan_client is None else 1):  # a second round on the same plans
            try:
                totals = sharded_reduce(red, local, chunks=3, global_total_weights=glob, exchange=exchange)
            except AssertionError as e:
                q.put((rank, "AssertionError", str(e)))
                return
        if rank == 0:
            q.put((rank, "ok", ([o.cpu().numpy() for o in outs], totals)))
        else:
            q.put((rank, "ok", None))
    except Exception as e:  # surfaced by the parent
        q.put((rank, "err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _port():
    # a file rendezvous: no TCP port to collide with another test\'s store
    return rendezvous_url()


def _run(exchange, pass_totals, nan_client=None, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, exchange, pass_totals, nan_client, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, status, payload = q.get(timeout=100)
            got[rank] = (status, payload)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return got


@pytest.mark.parametrize("exchange,pass_totals", [("reduce", True), ("scatter", False), ("scatter", True),
                                                  ("reduce", False)])
def test_two_ranks_hip_kernels_match_the_oracle(exchange, pass_totals):
    got = _run(exchange, pass_totals)
    assert all(s == "ok" for s, _ in got.values()), got
    outs, totals = got[0][1]
    clients, weights = _clients()
    W = sum(weights)
    assert totals == [W] * len(SHAPES)  # the all-reduced totals when not passed in
    lo = N_CLIENTS // 2
    for s in range(len(SHAPES)):
        xs = [c[s].numpy() for c in clients]
        # each rank's exact arrival-order partial, then the one cross-rank addition
        parts = []
        for a, b in ((0, lo), (lo, N_CLIENTS)):
            acc = xs[a].astype(np.float64) * weights[a]
            for x, w in zip(xs[a + 1 : b], weights[a + 1 : b]):
                acc = acc + x.astype(np.float64) * w
            parts.append(acc)
        want = (parts[0] + parts[1]) / W
        assert np.array_equal(outs[s].view(np.uint64), want.view(np.uint64)), s
        chain = fedavg_flat(xs, weights)
        mag = sum(np.abs(x.astype(np.float64)) * w for x, w in zip(xs, weights)) / W
        assert np.all(np.abs(outs[s] - chain) <= 1e-12 * mag)


@pytest.mark.parametrize("exchange", ["reduce", "scatter"])
def test_a_nan_in_the_other_shard_fails_every_rank(exchange):
    got = _run(exchange, True, nan_client=N_CLIENTS - 1)  # the client lives on rank 1
    # the flag words are OR-ed across ranks before anyone raises (no rank left in a collective)
    assert got[0][0] == "AssertionError" and got[1][0] == "AssertionError", got
