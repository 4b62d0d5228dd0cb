"""Element-range sharding with the real HIP kernels: two / three processes on the one GPU over a
gloo group (RCCL refuses two ranks on one device). Each rank folds its element range of every
client with the fused kernel; the gathered model is bit-identical to the one-GPU fused result
and to the oracle — every element keeps its single arrival-order chain — and a NaN in one rank's
range fails every rank (fed_avg_algorithm.py:35,93,97)."""

from __future__ import annotations


import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.fedavg_oracle import fedavg_flat
from tests.helpers import rendezvous_url

pytestmark = pytest.mark.gpu

SHAPES = ((70001,), (33, 65), (4096 * 3,), (7,), (20000,))
N_CLIENTS = 7


def _clients():
    g = torch.Generator().manual_seed(21)
    clients = [[torch.randn(int(np.prod(s)), generator=g) for s in SHAPES] for _ in range(N_CLIENTS)]
    weights = [float(w) for w in np.random.default_rng(22).integers(100, 5000, size=N_CLIENTS)]
    return clients, weights


def _rank_main(rank, world, port, nan_at, out_dtype_name, q):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        from distributed_learning_simulation_lib_amd.fedavg import ClientTable, ModelLayout
        from distributed_learning_simulation_lib_amd.range_sharded import RangeShard, range_sharded_reduce

        out_dtype = getattr(torch, out_dtype_name)
        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
        layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(SHAPES))), shapes=SHAPES)
        clients, weights = _clients()
        if nan_at is not None:
            clients[nan_at[0]][nan_at[1]][nan_at[2]] = float("nan")
        shard = RangeShard(layout, world, rank, device)
        table = ClientTable(len(shard.pieces))
        for c, w in zip(clients, weights):
            full = [t.to(device) for t in c]
            table.add_client(shard.views(full), [w] * len(shard.pieces))
        out = torch.empty(layout.total_numel, dtype=out_dtype, device=device) if rank == 0 else None
        for _ in range(2):  # a second round on the same shard
            try:
                range_sharded_reduce(shard, table, torch.float32, out, out_dtype)
            except AssertionError as e:
                q.put((rank, "AssertionError", str(e)))
                return
        q.put((rank, "ok", out.cpu().numpy() if rank == 0 else None))
    except Exception as e:  # surfaced by the parent
        q.put((rank, "err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _port():
    # a file rendezvous: no TCP port to collide with another test\'s store
    return rendezvous_url()


def _run(world, nan_at=None, out_dtype="float64"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, nan_at, out_dtype, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, st, v = q.get(timeout=150)
        got[r] = (st, v)
    for p in procs:
        p.join(timeout=60)
    return got


@pytest.mark.parametrize("world,out_dtype", [(2, "float64"), (3, "float32")])
def test_range_sharded_matches_the_oracle_bitwise(world, out_dtype):
    got = _run(world, out_dtype=out_dtype)
    assert all(st == "ok" for st, _ in got.values()), got
    clients, weights = _clients()
    want = np.concatenate([fedavg_flat([c[s].numpy() for c in clients], weights) for s in range(len(SHAPES))])
    if out_dtype == "float32":
        want = want.astype(np.float32)
    have = got[0][1]
    assert have.dtype == want.dtype and np.array_equal(have.view(np.uint8), want.view(np.uint8))


def test_range_sharded_nan_fails_every_rank():
    got = _run(2, nan_at=(3, 4, 19999))  # the last tensor: the second rank's range
    assert all(st == "AssertionError" for st, _ in got.values()), got
