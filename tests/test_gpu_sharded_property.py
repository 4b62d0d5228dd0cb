"""Property test (hypothesis) of the whole multi-GPU round through the library's own RCCL
communicator (``fedavg_sharded_round``) on a one-rank world, against the oracle, BIT-FOR-BIT:
random layouts (odd segment sizes, tiny and multi-tile segments), input dtypes, integer and
fractional weights, chunk counts (including more chunks than tiles) and fp32 / fp64 outputs.
On one rank the RCCL sum is the identity, so the round must reproduce the reference exactly;
the cross-rank reorder at N > 1 is covered by tests/test_sharded_gloo.py."""

from __future__ import annotations


import numpy as np
import pytest
import torch
import torch.distributed as dist
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
from distributed_learning_simulation_lib_amd.sharded import HipLocalReducer, RcclComm, sharded_reduce
from oracle.fedavg_oracle import fedavg_flat

pytestmark = pytest.mark.gpu
TORCH_DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16, "float64": torch.float64}


@pytest.fixture(scope="module")
def native_comm(hip_device):
    # one rank: an in-process store, no TCP port to race for
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=hip_device)
    comm = RcclComm(hip_device)
    yield comm
    torch.cuda.synchronize(hip_device)
    comm.close()
    dist.destroy_process_group()


@settings(max_examples=40, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(n=st.integers(1, 20), sizes=st.lists(st.integers(1, 20000), min_size=1, max_size=5),
       dtype=st.sampled_from(list(TORCH_DT)), int_weights=st.booleans(), chunks=st.integers(1, 12),
       out64=st.booleans(), seed=st.integers(0, 2**31 - 1))
def test_native_round_is_bit_identical_to_the_oracle(hip_device, native_comm, n, sizes, dtype, int_weights,
                                                     chunks, out64, seed):
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(sizes))), shapes=tuple((s,) for s in sizes))
    tdt = TORCH_DT[dtype]
    rows = [[torch.randn(s, generator=g).to(tdt) for s in sizes] for _ in range(n)]
    weights = ([float(x) for x in rng.integers(1, 5000, size=n)] if int_weights
               else [float(x) for x in rng.uniform(1e-3, 10.0, size=n)])
    table = ClientTable(len(sizes))
    for r, w in zip(rows, weights):
        table.add_client([t.to(hip_device) for t in r], [w] * len(sizes))
    out_dt = torch.float64 if out64 else torch.float32
    ctx = FedAvgContext(layout, hip_device)
    outs = [torch.full((s,), float("nan"), dtype=out_dt, device=hip_device) for s in sizes]
    total = -0.0  # arrival-order fp64 sum, like the reference's total weight
    for w in weights:
        total += w
    sharded_reduce(HipLocalReducer(ctx, table, tdt, outs, out_dt), [total] * len(sizes), chunks=chunks,
                   force_collective=True, comm=native_comm)
    ctx.raise_on_nan()
    for s, (size, o) in enumerate(zip(sizes, outs)):
        xs = [(r[s].float() if tdt == torch.bfloat16 else r[s]).numpy() for r in rows]  # bf16 -> f32 is exact
        want = fedavg_flat(xs, weights).astype(np.float64 if out64 else np.float32)
        got = o.cpu().numpy()
        assert np.array_equal(got.view(np.uint64 if out64 else np.uint32), want.view(np.uint64 if out64 else np.uint32)), (
            f"segment {s} (size {size}) differs")
    ctx.close()
