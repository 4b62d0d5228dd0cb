"""Server-side QSGD dequantisation fused into the FedAvg fold, on the MI355X.

Bar: BIT-IDENTICAL to "dequantise every record with oracle/qsgd_oracle.py, then the pinned
FedAvg oracle" (fp64 arrival-order fold, IEEE division) — for fp32 and fp64 codecs, fp32 and
fp64 outputs, ragged segments, streaming waves, plans, shard partials, the plugin and the ratio
path. The codec restatement itself is "parity unpinned" (cyy_torch_algorithm is not vendored;
see the oracle's header).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, NaNAggregationError, ParameterMessage
from distributed_learning_simulation_lib_amd._native import NativeError
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
from distributed_learning_simulation_lib_amd.quantized import (
    QSGD_F32,
    QSGD_F64,
    QuantizedTensor,
    quantize_tensor,
)
from oracle import qsgd_oracle as qo
from oracle.fedavg_oracle import fedavg_flat
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu

CODECS = {"float32": QSGD_F32, "float64": QSGD_F64}


def make_round(rng, numels, n_clients, codec, scale=1.0):
    """Host records [client][segment] (numpy) + device QuantizedTensors."""
    recs = []
    for _ in range(n_clients):
        row = []
        for n in numels:
            x = (rng.standard_normal(n) * scale * rng.choice([1e-3, 1.0, 50.0])).astype(codec)
            row.append(qo.quantize(x, rng, level=int(rng.choice([255, 255, 7]))))
        recs.append(row)
    return recs


def oracle_result(recs, numels, codec, weights):
    out = []
    for t, n in enumerate(numels):
        dense = [qo.dequantize(recs[k][t], n, codec) for k in range(len(recs))]
        out.append(fedavg_flat(dense, [weights[k] for k in range(len(recs))]))
    return out


def device_table(recs, numels, codec, weights, device):
    table = ClientTable(len(numels))
    for k, row in enumerate(recs):
        qts = [QuantizedTensor(torch.from_numpy(r).to(device), (n,), CODECS[codec]) for r, n in zip(row, numels)]
        table.add_client([q.record for q in qts], [weights[k]] * len(numels))
    return table


LAYOUTS = [[1], [7, 4096], [4095, 4097, 33], [10_000, 1, 8192, 300], [65_536]]


@pytest.mark.parametrize("codec", ["float32", "float64"])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("li", range(len(LAYOUTS)))
def test_fused_aggregate_bit_identical(hip_device, codec, out_dtype, li):
    numels = LAYOUTS[li]
    rng = np.random.default_rng(100 + li)
    n_clients = int(rng.integers(1, 11))
    recs = make_round(rng, numels, n_clients, codec)
    weights = [float(rng.integers(1, 5000)) if li % 2 else float(rng.random() + 0.01) for _ in range(n_clients)]
    want = oracle_result(recs, numels, codec, weights)
    ctx = FedAvgContext(ModelLayout(names=tuple(f"t{i}" for i in range(len(numels))),
                                    shapes=tuple((n,) for n in numels)), hip_device)
    table = device_table(recs, numels, codec, weights, hip_device)
    outs = [torch.empty(n, dtype=out_dtype, device=hip_device) for n in numels]
    ctx.aggregate(table, CODECS[codec], outs, out_dtype)
    ctx.raise_on_nan([(table, CODECS[codec])])
    np_out = np.float32 if out_dtype == torch.float32 else np.float64
    for o, w in zip(outs, want):
        assert bits_equal(o.cpu().numpy(), w.astype(np_out))
    ctx.close()


@pytest.mark.parametrize("codec", ["float32", "float64"])
def test_streaming_waves_plans_and_partial(hip_device, codec):
    numels = [5000, 4096, 12]
    rng = np.random.default_rng(7)
    recs = make_round(rng, numels, 13, codec)
    weights = [float(rng.integers(1, 100)) for _ in range(13)]
    want = oracle_result(recs, numels, codec, weights)
    layout = ModelLayout(names=("a", "b", "c"), shapes=tuple((n,) for n in numels))
    ctx = FedAvgContext(layout, hip_device)
    fmt = CODECS[codec]
    # waves of 5 + 5 + 3 through the fp64 accumulator
    for lo, hi in [(0, 5), (5, 10)]:
        ctx.accumulate(device_table(recs[lo:hi], numels, codec, weights[lo:hi], hip_device), fmt)
    outs = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in numels]
    ctx.aggregate(device_table(recs[10:], numels, codec, weights[10:], hip_device), fmt, outs, torch.float64)
    ctx.raise_on_nan()
    for o, w in zip(outs, want):
        assert bits_equal(o.cpu().numpy(), w)
    # prepared plan, run twice
    table = device_table(recs, numels, codec, weights, hip_device)
    outs2 = [torch.empty(n, dtype=torch.float32, device=hip_device) for n in numels]
    plan = ctx.plan(table, fmt, outs2, torch.float32)
    for _ in range(2):
        plan.run()
        ctx.raise_on_nan()
        for o, w in zip(outs2, want):
            assert bits_equal(o.cpu().numpy(), w.astype(np.float32))
    plan.close()
    # shard partial in two tile ranges, then finalize: same as the fused call
    nt = ctx.num_tiles
    ctx.partial(table, fmt, zero_init=True, tile_begin=0, tile_end=nt // 2)
    ctx.partial(table, fmt, zero_init=True, tile_begin=nt // 2, tile_end=nt)
    ctx.set_accumulated([sum(weights)] * 3)
    outs3 = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in numels]
    ctx.finalize_range(outs3, torch.float64)
    ctx.raise_on_nan()
    for o, w in zip(outs3, want):
        assert bits_equal(o.cpu().numpy(), w)
    ctx.close()


def test_quantised_then_dense_waves_keep_arrival_order(hip_device):
    numels = [4100]
    rng = np.random.default_rng(3)
    recs = make_round(rng, numels, 4, "float32")
    dense = [rng.standard_normal(4100).astype(np.float32) for _ in range(3)]
    weights = [3.0, 1.5, 2.0, 7.0, 0.25, 9.0, 1.0]
    want = fedavg_flat([qo.dequantize(r[0], 4100, "float32") for r in recs] + dense, weights)
    ctx = FedAvgContext(ModelLayout.flat(4100), hip_device)
    ctx.accumulate(device_table(recs, numels, "float32", weights[:4], hip_device), QSGD_F32)
    t2 = ClientTable(1)
    for x, w in zip(dense, weights[4:]):
        t2.add_client([torch.from_numpy(x).to(hip_device)], [w])
    out = torch.empty(4100, dtype=torch.float64, device=hip_device)
    ctx.aggregate(t2, torch.float32, [out], torch.float64)
    ctx.raise_on_nan()
    assert bits_equal(out.cpu().numpy(), want)


def test_nan_norm_names_the_client(hip_device):
    numels = [3000, 50]
    rng = np.random.default_rng(9)
    recs = make_round(rng, numels, 5, "float32")
    recs[3][1][0:8] = np.frombuffer(np.float64(np.nan).tobytes(), np.uint8)
    ctx = FedAvgContext(ModelLayout(names=("a", "b"), shapes=((3000,), (50,))), hip_device)
    table = device_table(recs, numels, "float32", [1.0] * 5, hip_device)
    outs = [torch.empty(n, dtype=torch.float32, device=hip_device) for n in numels]
    ctx.aggregate(table, QSGD_F32, outs, torch.float32)
    with pytest.raises(NaNAggregationError) as ei:
        ctx.raise_on_nan([(table, QSGD_F32)])
    assert ei.value.stage == "input" and ei.value.bad_clients == [3]


def test_unaligned_record_and_delta_rejected(hip_device):
    ctx = FedAvgContext(ModelLayout.flat(100), hip_device)
    buf = torch.zeros(qo.record_bytes(100) + 16, dtype=torch.uint8, device=hip_device)
    t = ClientTable(1)
    t.add_client([buf[8 : 8 + qo.record_bytes(100)]], [1.0])
    with pytest.raises(NativeError):
        ctx.accumulate(t, QSGD_F32)
    t2 = ClientTable(1)
    t2.add_client([buf[: qo.record_bytes(100)]], [1.0])
    base = [torch.zeros(100, dtype=torch.float64, device=hip_device)]
    with pytest.raises(NativeError):
        ctx.accumulate_delta(t2, QSGD_F32, base)


@pytest.mark.parametrize("from_host", [False, True])
@pytest.mark.parametrize("accumulate", [True, False])
def test_plugin_with_quantised_messages(hip_device, from_host, accumulate):
    shapes = {"conv.weight": (16, 3, 3, 3), "conv.bias": (16,), "fc.weight": (10, 4096), "fc.bias": (10,)}
    rng = np.random.default_rng(21)
    g = torch.Generator(device="cpu").manual_seed(4)
    algo = FedAVGAlgorithm(device=hip_device, wave_size=3, result_dtype=torch.float64)
    algo.accumulate = accumulate
    n = 7
    weights = [int(x) for x in rng.integers(100, 5000, size=n)]
    msgs, dense = [], []
    for k in range(n):
        p = {name: torch.randn(s, generator=g) for name, s in shapes.items()}
        q = {name: quantize_tensor(t, generator=g) for name, t in p.items()}
        dense.append({name: qo.dequantize(q[name].record.numpy(), q[name].numel, "float32") for name in shapes})
        if not from_host:
            q = {name: v.to(hip_device) for name, v in q.items()}
        msgs.append(ParameterMessage(parameter=q, aggregation_weight=weights[k]))
    for k, m in enumerate(msgs):
        algo.process_worker_data(k, m)
    res = algo.aggregate_worker_data().parameter
    if accumulate:
        want = {name: fedavg_flat([d[name] for d in dense], weights) for name in shapes}
    else:
        tot = sum(weights)
        ratios = [float(w) / float(tot) for w in weights]  # get_ratios, aggregation_algorithm.py:42-49
        want = {}
        for name in shapes:
            acc = dense[0][name].astype(np.float64) * ratios[0]
            for d, r in zip(dense[1:], ratios[1:]):
                acc = acc + d[name].astype(np.float64) * r
            want[name] = acc
    for name, s in shapes.items():
        assert tuple(res[name].shape) == s
        assert bits_equal(res[name].reshape(-1).cpu().numpy(), want[name])


# ---- property test: random quantised rounds through the plugin ------------------------------
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from oracle.fedavg_oracle import OracleFedAvg, OracleMessage  # noqa: E402


@settings(max_examples=40, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(n=st.integers(1, 20), sizes=st.lists(st.integers(1, 9000), min_size=1, max_size=4),
       codec=st.sampled_from(["float32", "float64"]), level=st.sampled_from([1, 7, 100, 255]),
       int_weights=st.booleans(), wave=st.integers(1, 25), seed=st.integers(0, 2**31 - 1),
       skip_every=st.integers(0, 4), neg_weight=st.booleans())
def test_random_quantised_rounds_bit_identical(hip_device, n, sizes, codec, level, int_weights, wave, seed,
                                               skip_every, neg_weight):
    """Random layouts / client counts / levels / wave sizes / skipped clients / weight signs:
    the plugin's fused fold equals the oracle dequantisation + the pinned FedAvg oracle."""
    rng = np.random.default_rng(seed)
    weights = ([float(x) for x in rng.integers(1, 5000, size=n)] if int_weights
               else [float(x) for x in rng.uniform(1e-3, 10.0, size=n)])
    if neg_weight and n > 1:
        weights[1] = -weights[1] * 0.25  # a negative weight flips the product signs (table sign logic)
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave, result_dtype=torch.float64)
    oracle = OracleFedAvg()
    for k in range(n):
        if skip_every and k % skip_every == skip_every - 1 and k != 0:
            algo.process_worker_data(k, None)
            oracle.process_worker_data(k, None)
            continue
        params, dense = {}, {}
        for i, s in enumerate(sizes):
            x = (rng.standard_normal(s) * rng.choice([1e-30, 1e-3, 1.0, 1e30])).astype(codec)
            rec = qo.quantize(x, rng, level=level)
            params[f"t{i}"] = QuantizedTensor(torch.from_numpy(rec).to(hip_device), (s,), CODECS[codec])
            dense[f"t{i}"] = qo.dequantize(rec, s, codec)
        algo.process_worker_data(k, ParameterMessage(parameter=params, aggregation_weight=weights[k]))
        oracle.process_worker_data(k, OracleMessage(parameter=dense, aggregation_weight=weights[k]))
    try:
        want = oracle.aggregate_worker_data().parameter
    except AssertionError:
        with pytest.raises(AssertionError):
            algo.aggregate_worker_data()
        return
    got = algo.aggregate_worker_data().parameter
    for name, w in want.items():
        assert bits_equal(got[name].reshape(-1).cpu().numpy(), w.reshape(-1)), name


@pytest.mark.parametrize("cap", [1, 3 * 2048 * 2, 1 << 30])
def test_table_cap_splits_launches_bit_identically(hip_device, monkeypatch, cap):
    # FEDAVG_QSGD_TABLE_CAP: a launch whose |p| tables would pass the cap runs over
    # segment runs of at most cap / (clients x 2 KiB) segments (at least one), each building its own
    # tables into one buffer; partial plans over tile ranges take the same path
    monkeypatch.setenv("FEDAVG_QSGD_TABLE_CAP", str(cap))
    numels = [4095, 4097, 33, 10_000, 1, 8192, 300]
    rng = np.random.default_rng(7)
    n_clients = 3
    recs = make_round(rng, numels, n_clients, "float32")
    weights = [float(rng.integers(1, 5000)) for _ in range(n_clients)]
    want = oracle_result(recs, numels, "float32", weights)
    layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(numels))), shapes=tuple((n,) for n in numels))
    ctx = FedAvgContext(layout, hip_device)
    table = device_table(recs, numels, "float32", weights, hip_device)
    outs = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in numels]
    ctx.aggregate(table, QSGD_F32, outs, torch.float64)
    ctx.raise_on_nan([(table, QSGD_F32)])
    for o, w in zip(outs, want):
        assert bits_equal(o.cpu().numpy(), w)
    # a ranged partial + finalize (the sharded path) under the same cap
    W = sum(weights)
    nt = ctx.num_tiles
    for tb, te in ((0, nt // 3), (nt // 3, nt)):
        ctx.partial(table, QSGD_F32, zero_init=True, tile_begin=tb, tile_end=te)
    ctx.set_accumulated([W] * len(numels))
    ctx.finalize_range(outs, torch.float64)
    ctx.raise_on_nan()
    for o, w in zip(outs, want):
        assert bits_equal(o.cpu().numpy(), w)
