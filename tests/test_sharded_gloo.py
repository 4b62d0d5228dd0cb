"""Multi-rank FedAvg (clients sharded over ranks + chunked reduce) on CPU with gloo.

Covers ``sharded.sharded_reduce`` — chunking, both exchanges (the reduce of fp64 partials to
the root; the reduce-scatter + window finalize + gather), the weight totals, the root's NaN
check, sub-groups — with world_size 2 and 3 on the CPU. The per-rank
compute is a plain torch stand-in for the HIP reducer (same tile geometry as the native
library: 2048-element tiles that never cross a tensor, 16-byte aligned accumulator
segments); the GPU parity tests cover the HIP reducer itself.
"""

from __future__ import annotations


import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_learning_simulation_lib_amd.fedavg import ModelLayout
from distributed_learning_simulation_lib_amd.sharded import chunk_bounds, exchange_candidates, sharded_reduce
from oracle.fedavg_oracle import fedavg_flat
from tests.helpers import rendezvous_url

TILE = 2048


class TorchCPUReducer:
    def __init__(self, layout: ModelLayout, clients, weights, outs):
        self.layout = layout
        self.clients = clients  # list of list[tensor] (per segment)
        self.weights = weights  # list of list[float]
        self.outs = outs
        offs, total = layout.padded_offsets(8)
        self.acc_off = offs
        self.accumulator = torch.zeros(total, dtype=torch.float64)
        self.tiles = [(s, st, min(TILE, n - st)) for s, n in enumerate(layout.numels) for st in range(0, n, TILE)]
        self.totals = None

    @property
    def num_tiles(self):
        return len(self.tiles)

    def tile_range(self, tb, te):
        s0, st0, _ = self.tiles[tb]
        s1, st1, c1 = self.tiles[te - 1]
        end = self.acc_off[s1] + st1 + c1
        if st1 + c1 == self.layout.numels[s1]:
            end = self.acc_off[s1 + 1] if s1 + 1 < self.layout.num_segments else self.accumulator.numel()
        return self.acc_off[s0] + st0, end

    def partial(self, tb, te):
        for s, st, c in self.tiles[tb:te]:
            dst = self.accumulator[self.acc_off[s] + st : self.acc_off[s] + st + c]
            dst.zero_()
            for row, w in zip(self.clients, self.weights):
                dst += row[s][st : st + c].double() * w[s]

    def set_accumulated(self, totals):
        self.totals = list(totals)

    def finalize_range(self, tb, te):
        for s, st, c in self.tiles[tb:te]:
            src = self.accumulator[self.acc_off[s] + st : self.acc_off[s] + st + c]
            self.outs[s][st : st + c] = src / self.totals[s]

    def prefold(self):
        pass

    # scatter exchange pieces: a window of accumulator positions, padding skipped
    def _seg_of(self):
        seg = torch.full((self.accumulator.numel(),), -1, dtype=torch.int64)
        for s_, (o, n) in enumerate(zip(self.acc_off, self.layout.numels)):
            seg[o : o + n] = s_
        return seg

    def result_buffer(self):
        return torch.full((self.accumulator.numel(),), float("nan"), dtype=torch.float64)

    def finalize_window(self, src, lo, hi, res):
        seg = self._seg_of()[lo:hi]
        keep = seg >= 0
        tot = torch.tensor(self.totals, dtype=torch.float64)
        res[lo:hi][keep] = src[: hi - lo][keep] / tot[seg[keep]]

    def copy_out(self, res):
        for s_, (o, n) in enumerate(zip(self.acc_off, self.layout.numels)):
            self.outs[s_][:] = res[o : o + n]

    def nan_flags(self):
        if self.outs is not None and any(bool(o.isnan().any()) for o in self.outs):
            return 0x1  # FLAG_ACC_NAN: an input NaN leaves the sum NaN
        return 0

    def raise_on_nan(self):
        if self.outs is not None:
            assert not any(bool(o.isnan().any()) for o in self.outs), "NaN in the aggregate"

    def fused(self):
        self.partial(0, self.num_tiles)
        self.set_accumulated([sum(w[s] for w in self.weights) for s in range(self.layout.num_segments)])
        self.finalize_range(0, self.num_tiles)


LAYOUT = ModelLayout(names=("a", "b", "c", "d"), shapes=((5000,), (3, 7), (4096,), (2049,)))


def make_all_clients(n):
    g = torch.Generator().manual_seed(5)
    clients = [[torch.randn(m, generator=g) for m in LAYOUT.numels] for _ in range(n)]
    rng = np.random.default_rng(6)
    weights = [[float(rng.integers(100, 5000))] * LAYOUT.num_segments for _ in range(n)]
    return clients, weights


def _worker(rank, world, port, n_clients, chunks, pass_totals, q, exchange="reduce", subgroup=False, shape="even"):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        group = None
        if subgroup:  # the shard ranks are global ranks 1..world-1; group rank 0 = global rank 1
            group = dist.new_group(list(range(1, world)))
            if rank == 0:
                return
        g_world, g_rank = dist.get_world_size(group), dist.get_rank(group)
        clients, weights = make_all_clients(n_clients)
        mine = [i for i in range(n_clients) if i % g_world == g_rank]
        outs = [torch.empty(m, dtype=torch.float64) for m in LAYOUT.numels] if g_rank == 0 else None
        red = TorchCPUReducer(LAYOUT, [clients[i] for i in mine], [weights[i] for i in mine], outs)
        local = [sum(weights[i][s] for i in mine) for s in range(LAYOUT.num_segments)]
        glob = [sum(w[s] for w in weights) for s in range(LAYOUT.num_segments)] if pass_totals else None
        totals = sharded_reduce(red, local, chunks=chunks, global_total_weights=glob, group=group,
                                exchange=exchange, shape=shape)
        if g_rank == 0:
            q.put(("ok", [o.numpy() for o in outs], totals))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put(("err", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    # a file rendezvous: no TCP port to collide with another test\'s store
    return rendezvous_url()


@pytest.mark.parametrize("exchange", ["reduce", "scatter"])
@pytest.mark.parametrize("world,chunks,pass_totals,subgroup,shape", [
    (2, 4, True, False, "even"), (2, 1, False, False, "even"), (3, 3, False, False, "even"),
    (3, 2, True, True, "even"), (2, 3, True, False, "taper"), (3, 4, False, False, "ramp")])
def test_sharded_reduce_gloo(world, chunks, pass_totals, subgroup, shape, exchange):
    n_clients = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, n_clients, chunks, pass_totals, q, exchange, subgroup, shape))
             for r in range(world)]
    for p in procs:
        p.start()
    status, outs, totals = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert status == "ok", outs
    clients, weights = make_all_clients(n_clients)
    for s in range(LAYOUT.num_segments):
        want = fedavg_flat([c[s].numpy() for c in clients], [w[s] for w in weights])
        mag = sum(np.abs(c[s].numpy().astype(np.float64)) * w[s] for c, w in zip(clients, weights)) / totals[s]
        assert np.all(np.abs(outs[s] - want) <= 1e-12 * mag)
        assert np.array_equal(outs[s].astype(np.float32), want.astype(np.float32)) or np.all(
            np.abs(outs[s].astype(np.float32) - want.astype(np.float32)) <= np.spacing(np.abs(want.astype(np.float32)))
        )


def test_single_rank_uses_the_fused_path():
    clients, weights = make_all_clients(3)
    outs = [torch.empty(m, dtype=torch.float64) for m in LAYOUT.numels]
    red = TorchCPUReducer(LAYOUT, clients, weights, outs)
    totals = sharded_reduce(red, [sum(w[s] for w in weights) for s in range(4)])
    assert len(totals) == 4
    for s in range(4):
        want = fedavg_flat([c[s].numpy() for c in clients], [w[s] for w in weights])
        np.testing.assert_allclose(outs[s].numpy(), want, rtol=1e-14)


def _nan_worker(rank, world, port, exchange, q, tune=False):
    from distributed_learning_simulation_lib_amd.sharded import exchange_candidates, tune_exchange

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        clients, weights = make_all_clients(4)
        if rank == world - 1:
            clients[rank][2][100] = float("nan")  # the last rank's shard holds a NaN
        mine = [i for i in range(4) if i % world == rank]
        outs = [torch.empty(m, dtype=torch.float64) for m in LAYOUT.numels] if rank == 0 else None
        red = TorchCPUReducer(LAYOUT, [clients[i] for i in mine], [weights[i] for i in mine], outs)
        local = [sum(weights[i][s] for i in mine) for s in range(LAYOUT.num_segments)]
        try:
            if tune:
                tune_exchange(red, local, exchange_candidates(2), rounds=1)
            else:
                sharded_reduce(red, local, chunks=2, exchange=exchange)
            q.put((rank, "no error"))
        except AssertionError:
            q.put((rank, "AssertionError"))
        # a round after the error still completes on every rank (no rank is left in a collective)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("exchange, tune", [("reduce", False), ("scatter", False), ("auto", True)])
def test_every_rank_raises_on_a_nan_in_another_shard(exchange, tune):
    # only the root used to raise; the other ranks went on into the next round's
    # collectives and waited there forever (tune_exchange checks NaN on every round)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nan_worker, args=(r, world, port, exchange, q, tune)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: "AssertionError", 1: "AssertionError"}  # fed_avg_algorithm.py:35/93/97


def _union_worker(rank, world, port, q):
    from distributed_learning_simulation_lib_amd.sharded import union_flags

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        q.put((rank, union_flags([0x1, 0x2, 0x100][rank])))
    finally:
        dist.destroy_process_group()


def test_union_flags_is_a_bitwise_or():
    # MAX of bitmasks turned {ACC, RESULT} into RESULT on every rank
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_union_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert got == {0: 0x103, 1: 0x103, 2: 0x103}


def _tune_worker(rank, world, port, q):
    from distributed_learning_simulation_lib_amd.sharded import exchange_candidates, tune_exchange

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        clients, weights = make_all_clients(5)
        mine = [i for i in range(5) if i % world == rank]
        outs = [torch.empty(m, dtype=torch.float64) for m in LAYOUT.numels] if rank == 0 else None
        red = TorchCPUReducer(LAYOUT, [clients[i] for i in mine], [weights[i] for i in mine], outs)
        local = [sum(weights[i][s] for i in mine) for s in range(LAYOUT.num_segments)]
        (ex, ch, sh), times = tune_exchange(red, local, exchange_candidates(), rounds=2)
        sharded_reduce(red, local, chunks=ch, exchange=ex, shape=sh)  # the tuned round still aggregates
        q.put((rank, (ex, ch, sh), sorted(times), [o.numpy() for o in outs] if rank == 0 else None))
    finally:
        dist.destroy_process_group()


def test_tune_exchange_agrees_across_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tune_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: (choice, timed, outs) for r, choice, timed, outs in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    assert got[0][0] == got[1][0]  # max-over-ranks times: one answer everywhere
    assert got[0][1] == sorted(exchange_candidates()) and got[0][0] in exchange_candidates()
    clients, weights = make_all_clients(5)
    for s in range(LAYOUT.num_segments):
        want = fedavg_flat([c[s].numpy() for c in clients], [w[s] for w in weights])
        mag = sum(np.abs(c[s].numpy().astype(np.float64)) * w[s] for c, w in zip(clients, weights)) / sum(
            w[s] for w in weights)
        assert np.all(np.abs(got[0][2][s] - want) <= 1e-12 * mag)


def test_exchange_candidates():

    assert exchange_candidates(4) == [("reduce", 4, "even"), ("reduce", 4, "taper"), ("reduce", 4, "ramp"),
                                      ("reduce", 4, "tail"), ("scatter", 4, "even"), ("scatter", 4, "taper"),
                                      ("scatter", 4, "ramp"), ("scatter", 4, "tail")]
    assert exchange_candidates(1) == [("reduce", 1, "even"), ("scatter", 1, "even")]
    assert len(exchange_candidates()) == 32


def test_resolve_exchange():
    from distributed_learning_simulation_lib_amd.sharded import resolve_exchange, scatter_windows

    assert resolve_exchange("auto", 2) == "scatter" and resolve_exchange("auto", 4) == "reduce"
    assert resolve_exchange("reduce", 2) == "reduce"
    with pytest.raises(ValueError):
        resolve_exchange("allreduce", 2)
    assert scatter_windows(64, 64 + 4096 * 3, 8) == (4096 * 3 // 8, 0)
    assert scatter_windows(0, 10, 3) == (3, 1)


@pytest.mark.parametrize("shape", ["even", "taper", "ramp"])
def test_chunk_bounds_partition_tiles(shape):
    for n in (1, 2, 7, 100, 5709):
        for c in (1, 2, 3, 4, 8, 1000):
            b = chunk_bounds(n, c, shape)
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
            assert all(x[1] > x[0] for x in b)


def test_chunk_shapes():
    from distributed_learning_simulation_lib_amd.sharded import chunk_edges

    assert chunk_edges(1427, 4) == [0, 357, 714, 1070, 1427]
    taper, ramp = chunk_edges(1400, 4, "taper"), chunk_edges(1400, 4, "ramp")
    assert taper == [0, 400, 800, 1200, 1400] and ramp == [0, 200, 600, 1000, 1400]
    assert chunk_edges(1300, 4, "tail") == [0, 400, 800, 1200, 1300]
    assert chunk_edges(10, 1, "taper") == [0, 10]
    with pytest.raises(ValueError):
        chunk_edges(10, 2, "zigzag")


class _FakeCommLib:
    """Stands in for the HIP library: rank 0's id bytes, and what each rank joined with."""

    ID = bytes(range(7, 7 + 128))

    def __init__(self):
        self.joined = None

    def fedavg_comm_unique_id(self, ptr):
        import ctypes

        ctypes.memmove(ptr.value, self.ID, len(self.ID))
        return 0

    def fedavg_comm_create(self, out, id_ptr, world, rank, device):
        import ctypes

        self.joined = (ctypes.string_at(id_ptr.value, 128), world, rank)
        return 0

    def fedavg_comm_destroy(self, h):
        return 0


def _comm_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        from distributed_learning_simulation_lib_amd import _native, sharded

        fake = _FakeCommLib()
        _native.load = lambda path=None: fake  # the id exchange only: no RCCL on the CPU
        comm = sharded.RcclComm(torch.device("cpu"))
        q.put((rank, fake.joined, comm.world, comm.rank))
    finally:
        dist.destroy_process_group()


def test_rccl_comm_ships_rank0_id_to_every_rank():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, joined, w, r in got:
        assert joined == (_FakeCommLib.ID, world, rank) and (w, r) == (world, rank)


def test_exchange_model_terms():
    """DESIGN.md §5 cost model: the anchor, the pipeline and the choice it makes for config 3."""
    from distributed_learning_simulation_lib_amd.sharded import ExchangeModel, chunk_edges

    m = ExchangeModel()
    P, tiles = 11_689_512, 2854  # ResNet-18, 4096-element tiles
    assert abs(m.one_gpu_ms(P, 256, 4, 4) - 1.863) < 0.01  # the measured 1.864 ms anchor
    for G in (2, 4, 8):
        (ex, ch, sh), r = m.best(G, P, 256, 4, 4, tiles)
        assert (ex, ch, sh) in exchange_candidates()
        assert r["step_ms"] >= r["fold_ms"] > 0 and r["speedup"] < G
        # nothing beats the fold: the even 4-chunk reduce costs at least as much as the choice
        even = m.round_ms(G, P, 256, 4, 4, chunk_edges(tiles, 4, "even"), "reduce")
        assert even["step_ms"] >= r["step_ms"]
    # a faster link shortens the exposed tail, a slower one lengthens it
    fast, slow = ExchangeModel(link_eff=1.0), ExchangeModel(link_eff=0.4)
    e = chunk_edges(tiles, 4, "taper")
    assert fast.round_ms(4, P, 256, 4, 4, e, "reduce")["step_ms"] < slow.round_ms(4, P, 256, 4, 4, e, "reduce")["step_ms"]


def _tune_budget_worker(rank, world, port, q):
    from distributed_learning_simulation_lib_amd.sharded import exchange_candidates, tune_exchange

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        clients, weights = make_all_clients(4)
        mine = [i for i in range(4) if i % world == rank]
        outs = [torch.empty(m, dtype=torch.float64) for m in LAYOUT.numels] if rank == 0 else None
        red = TorchCPUReducer(LAYOUT, [clients[i] for i in mine], [weights[i] for i in mine], outs)
        local = [sum(weights[i][s] for i in mine) for s in range(LAYOUT.num_segments)]
        choice, times = tune_exchange(red, local, exchange_candidates(), rounds=1, budget_s=0.0)
        q.put((rank, choice, sorted(times)))
    finally:
        dist.destroy_process_group()


def test_tune_budget_stops_every_rank_after_the_same_candidate():
    # bench.py --tune-budget: the max-over-ranks elapsed time decides, so no rank is left timing a
    # candidate the others skipped
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tune_budget_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (c, t)) for r, c, t in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    first = exchange_candidates()[0]
    assert got[0] == got[1] == (first, [first])


def test_exchange_model_prices_the_peer_window_exchange():
    """the single-process peer exchange writes no whole fp64 partial and has no
    collective kernel; on the same assumptions it beats the RCCL schedules at every G."""
    from distributed_learning_simulation_lib_amd.sharded import ExchangeModel

    m = ExchangeModel()
    P, tiles = 11_689_512, 2854
    for G in (2, 4, 8):
        (ex, ch, sh), peer = m.best(G, P, 256, 4, 4, tiles, exchange_candidates(exchanges=("peer",)))
        _, rccl = m.best(G, P, 256, 4, 4, tiles)
        assert ex == "peer" and peer["speedup"] > rccl["speedup"] and peer["speedup"] < G
        assert peer["step_ms"] >= peer["fold_ms"] > 0
    (_, _, _), p4 = m.best(4, P, 256, 4, 4, tiles, exchange_candidates(exchanges=("peer",)))
    assert p4["speedup"] >= 3.6  # the own window folded with the received partials (no own-slot pass)
    # no link at all on one device: the fold alone plus the combine
    one = m.round_ms(1, P, 256, 4, 4, [0, tiles], "peer")
    assert one["last_chunk_exchange_ms"] == 0.0
