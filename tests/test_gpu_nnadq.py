"""Server-side NNADQ dequantisation fused into the FedAvg fold (NNADQServerEndpoint,
quantized_endpoint.py:114-142 + QuantServerEndpoint.get :69-77), on the MI355X.

Bar: BIT-IDENTICAL to "dequantise every record with oracle/nnadq_oracle.py, then the pinned
FedAvg oracle" (fp64 arrival-order fold, IEEE division) — fp32 and fp64 codecs, fp32 and fp64
outputs, ragged segments, every geometry edge of nnadq_tile_kernel (read from the library),
streaming waves, plans, shard partials, the plugin (device and host records, both aggregation
paths) and random rounds. The codec restatement itself is "parity unpinned"
(cyy_torch_algorithm is not vendored; see the oracle's header).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, NaNAggregationError, ParameterMessage
from distributed_learning_simulation_lib_amd._native import kernel_constant as K
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout
from distributed_learning_simulation_lib_amd.quantized import (
    NNADQ,
    NNADQ_F32,
    NNADQ_F64,
    QuantizedTensor,
)
from oracle import nnadq_oracle as no
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage, fedavg_flat
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu

CODECS = {"float32": NNADQ_F32, "float64": NNADQ_F64}


def around(*centers: int, lo: int = 1) -> list[int]:
    return sorted({c + d for c in centers for d in (-1, 0, 1) if c + d >= lo})


def make_round(rng, numels, n_clients, codec):
    """Host records [client][segment] (numpy)."""
    recs = []
    for _ in range(n_clients):
        row = []
        for n in numels:
            x = (rng.standard_normal(n) * rng.choice([1e-3, 1.0, 50.0]) + rng.choice([0.0, 3.0])).astype(codec)
            row.append(no.quantize(x, float(rng.choice([0.001, 0.01, 0.3]))))
        recs.append(row)
    return recs


def oracle_result(recs, numels, codec, weights):
    return [fedavg_flat([no.dequantize(recs[k][t], n, codec) for k in range(len(recs))], list(weights))
            for t, n in enumerate(numels)]


def device_table(recs, numels, codec, weights, device):
    table = ClientTable(len(numels))
    for k, row in enumerate(recs):
        qts = [QuantizedTensor(torch.from_numpy(r).to(device), (n,), CODECS[codec]) for r, n in zip(row, numels)]
        table.add_client([q.record for q in qts], [weights[k]] * len(numels))
    return table


def _layout(numels):
    return ModelLayout(names=tuple(f"t{i}" for i in range(len(numels))), shapes=tuple((n,) for n in numels))


LAYOUTS = [[1], [7, 4096], [4095, 4097, 33], [10_000, 1, 8192, 300], [65_536]]


@pytest.mark.parametrize("codec", ["float32", "float64"])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("li", range(len(LAYOUTS)))
def test_fused_aggregate_bit_identical(hip_device, codec, out_dtype, li):
    numels = LAYOUTS[li]
    rng = np.random.default_rng(200 + li)
    n_clients = int(rng.integers(1, 11))
    recs = make_round(rng, numels, n_clients, codec)
    # odd layouts: integer weights (the FMA fold when every product is exact); even: fractional
    weights = [float(rng.integers(1, 5000)) if li % 2 else float(rng.random() + 0.01) for _ in range(n_clients)]
    want = oracle_result(recs, numels, codec, weights)
    ctx = FedAvgContext(_layout(numels), hip_device)
    table = device_table(recs, numels, codec, weights, hip_device)
    outs = [torch.empty(n, dtype=out_dtype, device=hip_device) for n in numels]
    ctx.aggregate(table, CODECS[codec], outs, out_dtype)
    ctx.raise_on_nan([(table, CODECS[codec])])
    np_out = np.float32 if out_dtype == torch.float32 else np.float64
    for o, w in zip(outs, want):
        assert bits_equal(o.cpu().numpy(), w.astype(np_out))
    ctx.close()


@pytest.mark.parametrize("codec", ["float32", "float64"])
@pytest.mark.parametrize("weights_kind", ["float", "int"])
def test_kernel_edges_bit_identical(hip_device, codec, weights_kind):
    """Client counts around one and two load groups; segment lengths around the 16-element lane
    and the 4096-element tile (constants read from the library)."""
    g = K("nnadq_group")
    lengths = around(K("nnadq_ae"), K("nnadq_tile"), 2 * K("nnadq_tile"))
    ctx = FedAvgContext(_layout(lengths), hip_device)
    fmt = CODECS[codec]
    for n in sorted(set(around(g, 2 * g)) | {1}):
        rng = np.random.default_rng(n * 7 + (weights_kind == "int"))
        recs = make_round(rng, lengths, n, codec)
        weights = ([float(x) for x in rng.integers(1, 5000, n)] if weights_kind == "int"
                   else [float(x) for x in rng.uniform(0.01, 5.0, n)])
        want = oracle_result(recs, lengths, codec, weights)
        for waves in ([(0, n)], [(a, min(n, a + 3)) for a in range(0, n, 3)]):
            tabs = [device_table(recs[a:b], lengths, codec, weights[a:b], hip_device) for a, b in waves]
            outs = [torch.empty(m, dtype=torch.float64, device=hip_device) for m in lengths]
            for t in tabs[:-1]:
                ctx.accumulate(t, fmt)
            ctx.aggregate(tabs[-1], fmt, outs, torch.float64)
            ctx.raise_on_nan([(t, fmt) for t in tabs])
            ctx.reset()
            for s, (o, w) in enumerate(zip(outs, want)):
                assert bits_equal(o.cpu().numpy(), w), (codec, weights_kind, n, len(waves), lengths[s])
    ctx.close()


@pytest.mark.parametrize("codec", ["float32", "float64"])
def test_streaming_waves_plans_and_partial(hip_device, codec):
    numels = [5000, 4096, 12]
    rng = np.random.default_rng(17)
    recs = make_round(rng, numels, 13, codec)
    weights = [float(rng.integers(1, 100)) for _ in range(13)]
    want = oracle_result(recs, numels, codec, weights)
    ctx = FedAvgContext(_layout(numels), hip_device)
    fmt = CODECS[codec]
    for lo, hi in [(0, 5), (5, 10)]:
        ctx.accumulate(device_table(recs[lo:hi], numels, codec, weights[lo:hi], hip_device), fmt)
    outs = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in numels]
    ctx.aggregate(device_table(recs[10:], numels, codec, weights[10:], hip_device), fmt, outs, torch.float64)
    ctx.raise_on_nan()
    for o, w in zip(outs, want):
        assert bits_equal(o.cpu().numpy(), w)
    table = device_table(recs, numels, codec, weights, hip_device)
    outs2 = [torch.empty(n, dtype=torch.float32, device=hip_device) for n in numels]
    plan = ctx.plan(table, fmt, outs2, torch.float32)
    for _ in range(2):
        plan.run()
        ctx.raise_on_nan()
        for o, w in zip(outs2, want):
            assert bits_equal(o.cpu().numpy(), w.astype(np.float32))
    plan.close()
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


def test_nnadq_then_dense_waves_keep_arrival_order(hip_device):
    numels = [4100]
    rng = np.random.default_rng(4)
    recs = make_round(rng, numels, 4, "float32")
    dense = [rng.standard_normal(4100).astype(np.float32) for _ in range(3)]
    weights = [3.0, 1.5, 2.0, 7.0, 0.25, 9.0, 1.0]
    want = fedavg_flat([no.dequantize(r[0], 4100, "float32") for r in recs] + dense, weights)
    ctx = FedAvgContext(ModelLayout.flat(4100), hip_device)
    ctx.accumulate(device_table(recs, numels, "float32", weights[:4], hip_device), NNADQ_F32)
    t2 = ClientTable(1)
    for x, w in zip(dense, weights[4:]):
        t2.add_client([torch.from_numpy(x).to(hip_device)], [w])
    out = torch.empty(4100, dtype=torch.float64, device=hip_device)
    ctx.aggregate(t2, torch.float32, [out], torch.float64)
    ctx.raise_on_nan()
    assert bits_equal(out.cpu().numpy(), want)


def test_nan_record_names_the_client(hip_device):
    numels = [3000, 50]
    rng = np.random.default_rng(9)
    recs = make_round(rng, numels, 5, "float32")
    recs[2][1][0:8] = np.frombuffer(np.float64(np.nan).tobytes(), np.uint8)  # lo = NaN
    ctx = FedAvgContext(_layout(numels), hip_device)
    table = device_table(recs, numels, "float32", [1.0] * 5, hip_device)
    outs = [torch.empty(n, dtype=torch.float32, device=hip_device) for n in numels]
    ctx.aggregate(table, NNADQ_F32, outs, torch.float32)
    with pytest.raises(NaNAggregationError) as ei:
        ctx.raise_on_nan([(table, NNADQ_F32)])
    assert ei.value.stage == "input" and ei.value.bad_clients == [2]


@pytest.mark.parametrize("from_host", [False, True])
@pytest.mark.parametrize("accumulate", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_plugin_with_nnadq_messages(hip_device, from_host, accumulate, dtype):
    """NNADQClientEndpoint-quantised updates through FedAVGAlgorithm (both paths)."""
    shapes = {"conv.weight": (16, 3, 3, 3), "conv.bias": (16,), "fc.weight": (10, 4096), "fc.bias": (10,)}
    rng = np.random.default_rng(31)
    g = torch.Generator(device="cpu").manual_seed(5)
    quant, _ = NNADQ(weight=0.01)
    algo = FedAVGAlgorithm(device=hip_device, wave_size=3, result_dtype=torch.float64)
    algo.accumulate = accumulate
    n = 7
    weights = [int(x) for x in rng.integers(100, 5000, size=n)]
    codec = "float64" if dtype == torch.float64 else "float32"
    msgs, dense = [], []
    for k in range(n):
        p = {name: torch.randn(s, generator=g, dtype=dtype) for name, s in shapes.items()}
        q = quant(p)
        dense.append({name: no.dequantize(q[name].record.numpy(), q[name].numel, codec) for name in shapes})
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
        assert bits_equal(res[name].reshape(-1).cpu().numpy(), want[name].reshape(-1))


# ---- property test: random NNADQ rounds through the plugin ----------------------------------
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=40, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(n=st.integers(1, 20), sizes=st.lists(st.integers(1, 9000), min_size=1, max_size=4),
       codec=st.sampled_from(["float32", "float64"]), qweight=st.sampled_from([1e-4, 0.01, 0.2, 3.0]),
       int_weights=st.booleans(), wave=st.integers(1, 25), seed=st.integers(0, 2**31 - 1),
       skip_every=st.integers(0, 4), neg_weight=st.booleans())
def test_random_nnadq_rounds_bit_identical(hip_device, n, sizes, codec, qweight, int_weights, wave, seed,
                                           skip_every, neg_weight):
    rng = np.random.default_rng(seed)
    weights = ([float(x) for x in rng.integers(1, 5000, size=n)] if int_weights
               else [float(x) for x in rng.uniform(1e-3, 10.0, size=n)])
    if neg_weight and n > 1:
        weights[1] = -weights[1] * 0.25
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave, result_dtype=torch.float64)
    oracle = OracleFedAvg()
    for k in range(n):
        if skip_every and k % skip_every == skip_every - 1 and k != 0:
            algo.process_worker_data(k, None)
            oracle.process_worker_data(k, None)
            continue
        params, dense = {}, {}
        for i, s in enumerate(sizes):
            x = (rng.standard_normal(s) * rng.choice([1e-30, 1e-3, 1.0, 1e30]) + rng.choice([0.0, 1.0])).astype(codec)
            rec = no.quantize(x, qweight)
            params[f"t{i}"] = QuantizedTensor(torch.from_numpy(rec).to(hip_device), (s,), CODECS[codec])
            dense[f"t{i}"] = no.dequantize(rec, s, codec)
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
