"""Element-range sharding (range_sharded.py) on CPU: the range geometry, and world 2 / 3 over
gloo with the fold replaced by the oracle restricted to each rank's range — the gathered model is
bit-identical to the oracle over the whole model (each element keeps its single arrival-order
chain, fed_avg_algorithm.py:43-99), and a NaN in one rank's range fails every rank."""

from __future__ import annotations


import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_learning_simulation_lib_amd.fedavg import ModelLayout
from distributed_learning_simulation_lib_amd.range_sharded import (
    RangeShard,
    element_ranges,
    layout_ranges,
    range_pieces,
    range_sharded_reduce,
    segment_views,
)
from oracle.fedavg_oracle import fedavg_flat
from tests.helpers import rendezvous_url

LAYOUT = ModelLayout(names=("a", "b", "c", "d"), shapes=((5000,), (3, 7), (9000,), (2049,)))


def test_element_ranges_cover_the_model():
    for total in (1, 4095, 4096, 16117, 11_689_512):
        for world in (1, 2, 3, 4, 8):
            r = element_ranges(total, world)
            assert r[0][0] == 0 and r[-1][1] == total and len(r) == world
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert all(lo % 4096 == 0 or lo == total for lo, _ in r)
            sizes = [hi - lo for lo, hi in r]
            assert max(sizes) - min(sizes) <= 2 * 4096 or total < world * 4096


def test_layout_ranges_keep_pieces_segment_aligned():
    import bench

    for layout in (LAYOUT, bench.resnet18_layout()):
        offs = np.cumsum([0] + layout.numels[:-1])
        for world in (1, 2, 3, 4, 8):
            r = layout_ranges(layout, world)
            assert r[0][0] == 0 and r[-1][1] == layout.total_numel
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            for lo, _ in r:
                for p in range_pieces(layout, lo, layout.total_numel)[:1]:
                    assert p.lo % 4096 == 0, (world, lo, p)
            if layout is not LAYOUT:
                sizes = [hi - lo for lo, hi in r]
                assert max(sizes) - min(sizes) <= 2 * 4096  # ResNet-18: cuts close to even
    del offs


def test_range_pieces_and_views():
    pieces = range_pieces(LAYOUT, 4096, 8192)  # ends in segment c
    assert [(p.seg, p.lo, p.hi) for p in pieces] == [(0, 4096, 5000), (1, 0, 21), (2, 0, 3171)]
    shard = RangeShard(LAYOUT, 4, 1, None)
    assert (shard.lo, shard.hi) == (4096, 9117)  # cut at c's first 4096-element boundary
    full = [torch.arange(n, dtype=torch.float32) for n in LAYOUT.numels]
    v = shard.views(full)
    assert [t.numel() for t in v] == [904, 21, 4096] and float(v[0][0]) == 4096.0
    flat = torch.arange(LAYOUT.total_numel, dtype=torch.float64)
    sv = segment_views(flat, LAYOUT)
    assert sv["b"].shape == (3, 7) and float(sv["c"][0]) == 5021.0


class OracleRangeShard(RangeShard):
    """RangeShard whose fold is the oracle over this rank's pieces (no GPU)."""

    def __init__(self, *a, clients, weights, **kw):
        super().__init__(*a, **kw)
        self.clients, self.weights = clients, weights
        self._flags = 0

    def fold(self, table, in_dtype, out_dtype):
        flat, _ = self.local_output(out_dtype)
        pos = 0
        for p in self.pieces:
            arrs = [c[p.seg].reshape(-1)[p.lo:p.hi].numpy() for c in self.clients]
            r = fedavg_flat(arrs, [w[p.seg] for w in self.weights])
            if np.isnan(r).any():
                self._flags |= 1
            flat[pos : pos + p.hi - p.lo] = torch.from_numpy(r).to(out_dtype)
            pos += p.hi - p.lo
        return flat

    def flags(self):
        return self._flags

    def raise_local(self, tables):
        raise AssertionError("NaN in this rank's range")


class FailingRangeShard(OracleRangeShard):
    """Rank 1's fold fails (as a rank with elements but no clients does)."""

    def fold(self, table, in_dtype, out_dtype):
        if self.rank == 1:
            raise RuntimeError("nothing to aggregate in this rank's range")
        return super().fold(table, in_dtype, out_dtype)


def _clients(n, nan=None):
    g = torch.Generator().manual_seed(3)
    clients = [[torch.randn(s, generator=g) for s in LAYOUT.shapes] for _ in range(n)]
    rng = np.random.default_rng(4)
    weights = [[float(rng.integers(100, 5000))] * LAYOUT.num_segments for _ in range(n)]
    if nan is not None:
        clients[nan[0]][nan[1]].view(-1)[nan[2]] = float("nan")
    return clients, weights


def _worker(rank, world, port, nan, q, failing=False, bad_out=False):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        clients, weights = _clients(6, nan)
        cls = FailingRangeShard if failing else OracleRangeShard
        shard = cls(LAYOUT, world, rank, None, clients=clients, weights=weights)
        out = torch.empty(LAYOUT.total_numel, dtype=torch.float64) if rank == 0 else None
        if bad_out and rank == 0:
            out = torch.empty(LAYOUT.total_numel - 1, dtype=torch.float64)  # the root's output is too short
        try:
            range_sharded_reduce(shard, None, torch.float32, out, torch.float64)
        except AssertionError:
            q.put((rank, "AssertionError", None))
            return
        except ValueError:
            q.put((rank, "ValueError", None))
            return
        except RuntimeError:
            q.put((rank, "RuntimeError", None))
            return
        q.put((rank, "ok", out.numpy() if rank == 0 else None))
    finally:
        dist.destroy_process_group()


def _port():
    # a file rendezvous: no TCP port to collide with another test\'s store
    return rendezvous_url()


def _run(world, nan=None, failing=False, bad_out=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nan, q, failing, bad_out)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: (st, v) for r, st, v in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world", [2, 3])
def test_range_sharded_gloo_bitwise(world):
    got = _run(world)
    clients, weights = _clients(6)
    want = np.concatenate([fedavg_flat([c[s].reshape(-1).numpy() for c in clients], [w[s] for w in weights])
                           for s in range(LAYOUT.num_segments)])
    assert got[0][0] == "ok"
    assert np.array_equal(got[0][1].view(np.uint64), want.view(np.uint64))


def test_a_failed_fold_fails_every_rank_without_a_hang():
    got = _run(3, failing=True)
    assert all(st == "RuntimeError" for st, _ in got.values())


def test_a_bad_root_output_fails_every_rank_without_a_hang():
    # the root's output check used to raise before the flag reduction, leaving the
    # other ranks blocked in it; now the root raises its ValueError after it, the others a RuntimeError
    got = _run(2, bad_out=True)
    assert got[0][0] == "ValueError" and got[1][0] == "RuntimeError"


def test_range_sharded_nan_fails_every_rank():
    got = _run(3, nan=(2, 3, 2000))  # segment d, in the last rank's range
    assert all(st == "AssertionError" for st, _ in got.values())


from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=60, deadline=None)
@given(sizes=st.lists(st.integers(min_value=1, max_value=30000), min_size=1, max_size=12),
       world=st.integers(min_value=1, max_value=9))
def test_pieces_cover_every_element_once(sizes, world):
    """Any layout, any world: the ranks' pieces tile every tensor exactly once, each piece
    starts on a multiple of 4096 elements of its tensor (or at its start)."""
    layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(sizes))), shapes=tuple((n,) for n in sizes))
    seen = [np.zeros(n, dtype=np.int32) for n in sizes]
    for rank in range(world):
        shard = RangeShard(layout, world, rank, None)
        for p in shard.pieces:
            assert p.lo % 4096 == 0 or p.lo == 0 or (p.seg, p.lo) == (shard.pieces[0].seg, shard.pieces[0].lo)
            seen[p.seg][p.lo:p.hi] += 1
        if shard.pieces:
            first = shard.pieces[0]
            assert first.lo % 4096 == 0
    assert all((s == 1).all() for s in seen)
