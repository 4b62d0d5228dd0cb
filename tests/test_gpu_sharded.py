"""The sharded (multi-GPU) path's HIP + RCCL pieces on one GPU: a one-rank nccl group forced
through partial -> chunked RCCL reduce -> chunked finalize, against the fused kernel."""

from __future__ import annotations


import numpy as np
import pytest
import torch
import torch.distributed as dist

from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
from distributed_learning_simulation_lib_amd.sharded import HipLocalReducer, RcclComm, sharded_reduce

pytestmark = pytest.mark.gpu


@pytest.fixture
def nccl_group(hip_device):
    # one rank: an in-process store, no TCP port to race for
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=hip_device)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["reduce", "scatter"])
@pytest.mark.parametrize("native", [False, True])
@pytest.mark.parametrize("chunks,shape", [(1, "even"), (3, "even"), (8, "even"), (3, "taper"), (4, "ramp")])
def test_forced_collective_matches_fused(chunks, shape, native, exchange, hip_device, nccl_group):
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
    comm = RcclComm(hip_device) if native else None
    red = HipLocalReducer(ctx_b, table, torch.float32, out_b, torch.float64)
    for _ in range(2):  # a second round reuses the plans and the communicator's events
        for o in out_b:
            o.fill_(float("nan"))
        got = sharded_reduce(red, totals, chunks=chunks, force_collective=True, comm=comm, exchange=exchange,
                             shape=shape)
        assert got == totals
        ctx_b.raise_on_nan()
        for a, b in zip(out_a, out_b):
            assert torch.equal(a.view(torch.int64), b.view(torch.int64))
    if comm is not None:
        torch.cuda.synchronize(hip_device)
        comm.close()


def test_native_comm_rejects_bad_arguments(hip_device, nccl_group):
    from distributed_learning_simulation_lib_amd import _native

    comm = RcclComm(hip_device)
    lib = _native.load()
    # root out of range, and a root without a finalize plan
    assert lib.fedavg_sharded_round(comm.handle, None, None, None, 1, 0, None) == _native.ERR_INVALID
    layout = ModelLayout(names=("a",), shapes=((1000,),))
    ctx = FedAvgContext(layout, hip_device)
    table = ClientTable(1)
    table.add_client([torch.ones(1000, device=hip_device)], [1.0])
    plan = ctx.plan_partial(table, torch.float32, zero_init=True)
    assert lib.fedavg_sharded_round(comm.handle, ctx._h, plan._h, None, 1, 5, None) == _native.ERR_INVALID
    assert lib.fedavg_sharded_round(comm.handle, ctx._h, plan._h, None, 1, 0, None) == _native.ERR_INVALID
    # the scatter round needs a finalize plan on every rank
    assert lib.fedavg_sharded_round_scatter(comm.handle, ctx._h, plan._h, None, 1, 0, None) == _native.ERR_INVALID
    assert lib.fedavg_sharded_round_scatter(comm.handle, ctx._h, plan._h, plan._h, 1, 0, None) == _native.ERR_INVALID
    # explicit chunk edges must run from 0 to the tile count, strictly increasing
    import ctypes

    n = ctx.num_tiles
    for edges in ([0, n + 1], [1, n], [0, 0, n], [0]):
        arr = (ctypes.c_int32 * len(edges))(*edges)
        assert lib.fedavg_sharded_round_edges(comm.handle, ctx._h, plan._h, None, arr, len(edges),
                                              _native.EXCHANGE_REDUCE, 0, None) == _native.ERR_INVALID
    arr = (ctypes.c_int32 * 2)(0, n)
    assert lib.fedavg_sharded_round_edges(comm.handle, ctx._h, plan._h, None, arr, 2, 7, 0, None) == _native.ERR_INVALID
    comm.close()


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.float64])
def test_window_finalize_and_copy_out_match_finalize(out_dtype, hip_device):
    """The scatter exchange's pieces on one GPU: windows that cut segments (and their padding)
    anywhere, divided into a result buffer in accumulator coordinates, then copied out == the
    tile finalize, bit for bit; a NaN in the result buffer reaches the flags."""
    layout = ModelLayout(names=("a", "b", "c"), shapes=((4097,), (3, 5), (20000,)))
    g = torch.Generator().manual_seed(2)
    table = ClientTable(3)
    weights = [float(w) for w in np.random.default_rng(3).integers(100, 5000, size=5)]
    for w in weights:
        table.add_client([torch.randn(n, generator=g).to(hip_device) for n in layout.numels], [w] * 3)
    totals = [sum(weights)] * 3
    ctx = FedAvgContext(layout, hip_device)
    assert all(ctx.segment_offset(t) % 32 == 0 for t in range(3))  # FEDAVG_ACC_ALIGN
    want = [torch.empty(n, dtype=out_dtype, device=hip_device) for n in layout.numels]
    ctx.aggregate(table, torch.float32, want, out_dtype)
    ctx.raise_on_nan()
    ctx.partial(table, torch.float32, zero_init=True)
    got = [torch.full((n,), -1.0, dtype=out_dtype, device=hip_device) for n in layout.numels]
    fin = ctx.plan_finalize(totals, got, out_dtype)
    res = torch.full((ctx.acc_numel,), float("nan"), dtype=out_dtype, device=hip_device)
    acc = ctx.accumulator
    edges = [0, 1, 4095, 4100, 4133, 4160, 9000, ctx.acc_numel]
    for lo, hi in zip(edges[:-1], edges[1:]):
        fin.finalize_window(acc[lo:hi].clone(), lo, hi, res)
    fin.copy_out(res)
    ctx.raise_on_nan()
    for a, b in zip(want, got):
        assert torch.equal(a, b)
    res[ctx.segment_offset(2) + 7] = float("nan")
    fin.copy_out(res)
    with pytest.raises(AssertionError):
        ctx.raise_on_nan()


@pytest.mark.parametrize("exchange", ["reduce", "scatter"])
@pytest.mark.parametrize("native", [False, True])
def test_forced_collective_with_quantised_records(native, exchange, hip_device, nccl_group):
    """The sharded round over QSGD records (dequantisation fused into the shard partials) equals
    the fused single-launch quantised aggregate bit for bit on a one-rank world."""
    from distributed_learning_simulation_lib_amd.quantized import QSGD_F32, quantize_tensor

    layout = ModelLayout(names=("a", "b"), shapes=((50001,), (4096 * 3,)))
    g = torch.Generator(device=hip_device).manual_seed(3)
    table = ClientTable(2)
    weights = [float(w) for w in np.random.default_rng(4).integers(100, 5000, size=9)]
    for w in weights:
        recs = [quantize_tensor(torch.randn(n, device=hip_device, generator=g), generator=g).record
                for n in layout.numels]
        table.add_client(recs, [w] * 2)
    totals = [sum(weights)] * 2
    ctx_a = FedAvgContext(layout, hip_device)
    out_a = [torch.empty(n, dtype=torch.float32, device=hip_device) for n in layout.numels]
    ctx_a.aggregate(table, QSGD_F32, out_a, torch.float32)
    ctx_a.raise_on_nan()
    ctx_b = FedAvgContext(layout, hip_device)
    out_b = [torch.empty(n, dtype=torch.float32, device=hip_device) for n in layout.numels]
    comm = RcclComm(hip_device) if native else None
    red = HipLocalReducer(ctx_b, table, QSGD_F32, out_b, torch.float32)
    sharded_reduce(red, totals, chunks=3, force_collective=True, comm=comm, exchange=exchange)
    ctx_b.raise_on_nan()
    for a, b in zip(out_a, out_b):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    if comm is not None:
        torch.cuda.synchronize(hip_device)
        comm.close()
