"""Every geometry edge of the kernels, derived from the build, against the oracle (MI355X).

The round-1 PersonalizedFedAVG ring bug (a 4-client stage split 1/1/1 over 3 waves, client 3 of
every stage never loaded) passed every golden and property test: none of them crossed a
wave-count boundary. Here the sizes are placed around each edge the kernels have — read from the
library itself (``fedavg_kernel_constant``), not copied into the tests — and every result must be
BIT-IDENTICAL to the oracle (itself pinned to the reference's own outputs):

* FedAvg: segment lengths around one lane vector (16 B), a lane-vector row of a tile (the PARTV
  pieces of the balanced orders), the 4096- and 8192-element tiles; client counts around the load
  group and the 2-byte pipeline stage (one, two and three stages / groups, a short tail); every
  fold kind (MULADD: fractional weights; FMA: integer weights, exact products; DELTA: restore
  fused) and input dtype; one launch, and streaming waves that cut the groups unevenly; a layout
  long enough for the balanced orders' head of whole waves (fp32 and fp64);
* QSGD: segment lengths around the 16-element lane and the 4096-element tile, client counts
  around one and two groups of the record pipeline;
* PersonalizedFedAVG: receivers at every multiple of the per-wave block (16) ± 1 up to two
  launches of 128 (1-8 waves per workgroup, a second launch), clients around the LDS-DMA ring
  stage (4) and its depth, integer (ring) and float (register pipeline) weights, chunks ± 1.
"""

from __future__ import annotations

import zlib

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import ParameterMessage, PersonalizedFedAVGAlgorithm
from distributed_learning_simulation_lib_amd._native import kernel_constant as K
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
from distributed_learning_simulation_lib_amd.quantized import QSGD_F32, QuantizedTensor
from oracle import qsgd_oracle as qo
from oracle.fedavg_oracle import OracleMessage, as_f64, fedavg_flat
from oracle.personalized_oracle import OraclePersonalizedFedAvg
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu

DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16, "f64": torch.float64}


def around(*centers: int, lo: int = 1) -> list[int]:
    return sorted({c + d for c in centers for d in (-1, 0, 1) if c + d >= lo})


def fedavg_lengths(d: str) -> list[int]:
    n = 16 // DT[d].itemsize  # elements per 16-B lane vector
    lv = K(f"lanes_{d}") * n  # a lane-vector row of a whole-layout tile
    lv4 = K(f"lanes4096_{d}") * n
    return around(n, lv4, lv, 3 * lv4, K("tile"), K("tile_wide"), 2 * K("tile_wide"))


def fedavg_clients(d: str) -> list[int]:
    g, p = K(f"group_{d}"), K(f"pipe_{d}")
    cs = around(g, 2 * g) + (around(p, 2 * p, 3 * p) if p else [])
    return sorted(set(cs) | {1})


def _np(t: torch.Tensor) -> np.ndarray:
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


def _clients(gen, lengths, n, dt):
    return [[torch.randn(m, generator=gen).to(dt) for m in lengths] for _ in range(n)]


def _oracle(host, weights, dt, base=None):
    out = []
    for s in range(len(host[0])):
        xs = [as_f64(_np(c[s]), "bfloat16" if dt == torch.bfloat16 else None) for c in host]
        if base is not None:
            xs = [base[s] + x for x in xs]  # DeltaParameterMessage.restore (message.py:40-61)
        out.append(fedavg_flat(xs, weights))
    return out


def _tables(host, weights, device, waves):
    tabs = []
    for a, b in waves:
        t = ClientTable(len(host[0]))
        for c, w in zip(host[a:b], weights[a:b]):
            t.add_client([x.to(device) for x in c], [w] * len(c))
        tabs.append(t)
    return tabs


def _run(ctx, tabs, dt, out_dtype, device, base_dev=None):
    outs = [torch.empty(n, dtype=out_dtype, device=device) for n in ctx.layout.numels]
    for t in tabs[:-1]:
        if base_dev is None:
            ctx.accumulate(t, dt)
        else:
            ctx.accumulate_delta(t, dt, base_dev)
    if base_dev is None:
        ctx.aggregate(tabs[-1], dt, outs, out_dtype)
    else:
        ctx.aggregate_delta(tabs[-1], dt, base_dev, outs, out_dtype)
    ctx.raise_on_nan([(t, dt) for t in tabs])
    ctx.reset()
    return [o.cpu().numpy() for o in outs]


@pytest.mark.parametrize("d", list(DT))
@pytest.mark.parametrize("fold", ["float", "int", "delta"])
@pytest.mark.parametrize("balance", ["auto", "always"])
def test_fedavg_kernel_edges_bit_identical(hip_device, d, fold, balance, monkeypatch):
    # "always": the balanced whole-layout orders (pieces of whole lane-vectors, the PV kernels)
    # for every layout, not only where the last wave of workgroups is thin
    if balance == "always":
        monkeypatch.setenv("FEDAVG_BALANCE_ALWAYS", "1")
    dt = DT[d]
    lengths = fedavg_lengths(d)
    layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(lengths))), shapes=tuple((m,) for m in lengths))
    ctx = FedAvgContext(layout, hip_device)
    seed = zlib.crc32(f"{d}/{fold}".encode())
    gen = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed)
    base = [rng.standard_normal(m) for m in lengths] if fold == "delta" else None
    base_dev = [torch.from_numpy(b).to(hip_device) for b in base] if base is not None else None
    g = K(f"group_{d}")
    for n in fedavg_clients(d):
        host = _clients(gen, lengths, n, dt)
        weights = ([int(x) for x in rng.integers(1, 5000, n)] if fold == "int"
                   else [float(x) for x in rng.uniform(1e-3, 9.0, n)])
        want = _oracle(host, weights, dt, base)
        # one launch, and waves of g + 1 (every wave's groups end in a short tail)
        for waves in ([(0, n)], [(a, min(n, a + g + 1)) for a in range(0, n, g + 1)]):
            got = _run(ctx, _tables(host, weights, hip_device, waves), dt, torch.float64, hip_device, base_dev)
            for s, (a, b) in enumerate(zip(got, want)):
                assert bits_equal(a, b), (d, fold, n, len(waves), lengths[s])


@pytest.mark.parametrize("d", ["f32", "f64"])
def test_fedavg_balanced_head_bit_identical(hip_device, d, monkeypatch):
    """A layout of many whole tiles: the balanced order's head of whole waves, then the pieces."""
    monkeypatch.setenv("FEDAVG_BALANCE_ALWAYS", "1")
    dt = DT[d]
    tile = K("tile_wide") if d == "f32" else K("tile")
    lengths = [700 * tile + 777, 3 * tile, 1]
    layout = ModelLayout(names=("a", "b", "c"), shapes=tuple((m,) for m in lengths))
    ctx = FedAvgContext(layout, hip_device)
    gen = torch.Generator().manual_seed(11)
    host = _clients(gen, lengths, 3, dt)
    weights = [17, 4999, 1234]
    want = _oracle(host, weights, dt)
    got = _run(ctx, _tables(host, weights, hip_device, [(0, 3)]), dt, torch.float32, hip_device)
    for a, b in zip(got, want):
        assert bits_equal(a, b.astype(np.float32))


def test_qsgd_kernel_edges_bit_identical(hip_device):
    # every client count around the library's group size (read at run time, not collection)
    for n in around(K("qsgd_group"), 2 * K("qsgd_group")):
        _qsgd_edges_case(hip_device, n)


def _qsgd_edges_case(hip_device, n):
    lengths = around(K("qsgd_ae"), K("qsgd_tile"), 2 * K("qsgd_tile"))
    rng = np.random.default_rng(n)
    recs = [[qo.quantize(rng.standard_normal(m).astype(np.float32), rng) for m in lengths] for _ in range(n)]
    weights = [float(rng.uniform(0.01, 5.0)) for _ in range(n)]
    want = [fedavg_flat([qo.dequantize(recs[k][s], m, np.float32) for k in range(n)], weights)
            for s, m in enumerate(lengths)]
    layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(lengths))), shapes=tuple((m,) for m in lengths))
    ctx = FedAvgContext(layout, hip_device)
    for waves in ([(0, n)], [(a, min(n, a + 3)) for a in range(0, n, 3)]):
        tabs = []
        for a, b in waves:
            t = ClientTable(len(lengths))
            for k in range(a, b):
                qts = [QuantizedTensor(torch.from_numpy(r).to(hip_device), (m,), QSGD_F32)
                       for r, m in zip(recs[k], lengths)]
                t.add_client([q.record for q in qts], [weights[k]] * len(lengths))
            tabs.append(t)
        got = _run(ctx, tabs, QSGD_F32, torch.float64, hip_device)
        for s, (a, b) in enumerate(zip(got, want)):
            assert bits_equal(a, b), (n, len(waves), lengths[s])


def pers_receivers() -> list[int]:
    jb, grp = K("pers_jb"), K("pers_group")
    return sorted({r for m in range(jb, 2 * grp + 1, jb) for r in (m - 1, m, m + 1) if 1 <= r <= 2 * grp} | {1})


@pytest.mark.parametrize("kind", ["int", "float"])
def test_personalized_kernel_edges_bit_identical(hip_device, kind):
    stage, depth = K("pers_ring_stage"), K("pers_ring_depth")
    chunk, ve = K("pers_chunk"), 4
    lengths = around(ve, chunk, 3 * chunk)
    receivers = pers_receivers()
    workers = max(receivers)
    # clients per receiver around one ring stage, the ring depth and beyond; the receiver set
    # cycles through them
    client_counts = around(stage, 2 * stage, (depth + 1) * stage, lo=2)
    rng = np.random.default_rng(7 if kind == "int" else 8)
    gen = torch.Generator().manual_seed(9)
    updates = {i: {f"t{s}": torch.randn(m, generator=gen) for s, m in enumerate(lengths)} for i in range(workers)}
    for r_i, n_recv in enumerate(receivers):
        n_send = client_counts[r_i % len(client_counts)]
        ww = {}
        for j in range(n_recv):
            senders = [int(x) for x in rng.choice(workers, size=min(workers, n_send + 1), replace=False) if x != j]
            ww[j] = {i: (int(rng.integers(1, 500)) if kind == "int" else float(rng.uniform(0.01, 3.0)))
                     for i in senders[:n_send]}
        active = sorted({i for row in ww.values() for i in row} | set(range(n_recv)))
        algo = PersonalizedFedAVGAlgorithm(device=hip_device)
        oracle = OraclePersonalizedFedAvg()
        algo.set_worker_weights({j: dict(v) for j, v in ww.items()})
        oracle.set_worker_weights({j: dict(v) for j, v in ww.items()})
        for i in active:
            p = updates[i]
            algo.process_worker_data(i, ParameterMessage(parameter={a: b.to(hip_device) for a, b in p.items()}))
            oracle.process_worker_data(i, OracleMessage(parameter={a: b.numpy() for a, b in p.items()}))
        want = oracle.aggregate_worker_data()
        got = algo.aggregate_worker_data()
        for j, r in want.worker_data.items():
            for name, w in r.parameter.items():
                assert bits_equal(got.worker_data[j].parameter[name].cpu().numpy(), w), (kind, n_recv, n_send, j, name)
        for name, w in want.centralized_parameter.items():
            assert bits_equal(got.other_data["centralized_parameter"][name].cpu().numpy(), w), (kind, n_recv, name)
