"""HIP FedAvg vs the reference (golden fixtures) and vs the oracle, on the MI355X.

Tolerance statement (BASELINE.json north_star asks for "a stated fp32 tolerance"):
  * single-GPU kernels in the exact client order (the default for every layout large
    enough to fill the chip, and split_policy=1): BIT-IDENTICAL to the reference's float64
    results, including signed zeros — asserted with `bits_equal`;
  * the LDS split-client kernel (split_policy=2, small layouts with many clients) reorders
    the fp64 sum: |Δ| <= 1e-12 * sum_k |w_k x_k| / W per element (float64 output), and
    <= 1 fp32 ulp after the float32 cast (float32 output).
"""

from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

import tests.foreign_messages as foreign
from distributed_learning_simulation_lib_amd import (
    FedAVGAlgorithm,
    NaNAggregationError,
    ParameterMessage,
)
from distributed_learning_simulation_lib_amd import message as _pkg_message
from distributed_learning_simulation_lib_amd.algorithm import AggregationAlgorithm
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, FedAvgContext, ModelLayout, bw_probe
from oracle.fedavg_oracle import as_f64, fedavg_flat
from tests.golden_hooks import make_hooked_class
from tests.golden_io import bits_equal, load_golden

pytestmark = pytest.mark.gpu
CASES = load_golden()
TORCH_DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16, "float64": torch.float64}


def hook_spec(case):
    """The golden case's hooks (tests/golden_hooks.py) with its per-element weights as tensors."""
    elem = None
    if case.weight_mode is not None and case.weight_mode.startswith("elementwise"):
        elem = [{k: torch.from_numpy(v.copy()) for k, v in a.elem_weights.items()} if a.elem_weights else None
                for a in case.arrivals]
    return {"per_tensor_weight": case.per_tensor_weight, "weight_mode": case.weight_mode,
            "total_weight_hook": case.total_weight_hook, "elem_weights": elem}


def run_hip(case, device, wave_size, from_host=False, split_policy=1, wire=None, delta_checks=False, algo_out=None,
            **algo_kw):
    """Drive the plugin like AggregationServer does. ``wire``: the message module (default this
    package's; tests.foreign_messages = another class hierarchy with the same schema, as the
    reference server passes). ``delta_checks``: deltas carry new_parameter (not fusable)."""
    wire = wire or _pkg_message
    algo = make_hooked_class(FedAVGAlgorithm, hook_spec(case))(device=device, wave_size=wave_size,
                                                               split_policy=split_policy, **algo_kw)
    algo.accumulate = case.accumulate
    algo.aggregate_loss = case.aggregate_loss
    kinds = case.kinds or ["full"] * len(case.arrivals)
    old = None
    if case.old is not None:
        old = {k: torch.from_numpy(v.copy()) for k, v in case.old.items()}  # the server's fp64 host cache
        algo.set_old_parameter(old)
    for a, kind in zip(case.arrivals, kinds):
        if a.arrays is None:
            algo.process_worker_data(a.worker_id, None)
            continue
        params = case.torch_params(a, "cpu" if from_host else device)
        if kind == "delta":
            msg = wire.DeltaParameterMessage(delta_parameter=params, aggregation_weight=a.weight,
                                             other_data=dict(a.other_data))
            if delta_checks:
                msg.new_parameter = {k: old[k] + v.double().cpu() for k, v in params.items()}
        else:
            msg = wire.ParameterMessage(parameter=params, aggregation_weight=a.weight, other_data=dict(a.other_data))
            if old is not None:
                msg.complete(old)
        algo.process_worker_data(a.worker_id, msg)
    if algo_out is not None:
        algo_out.append(algo)
    try:
        return algo.aggregate_worker_data()
    finally:
        algo.exit()


@pytest.mark.parametrize("wave_size", [1, 3, 64])
@pytest.mark.parametrize("name", sorted(CASES))
def test_plugin_matches_reference_bitwise(name, wave_size, hip_device):
    case = CASES[name]
    if case.error is not None:
        exc = {"AssertionError": AssertionError, "RuntimeError": RuntimeError}[case.error]
        with pytest.raises(exc):
            run_hip(case, hip_device, wave_size)
        return
    res = run_hip(case, hip_device, wave_size, from_host=(wave_size == 3))
    assert list(res.parameter.keys()) == case.meta["out_keys"]
    for k, want in case.expected.items():
        got = res.parameter[k]
        assert got.dtype == torch.float64 and tuple(got.shape) == want.shape
        assert bits_equal(got.cpu().numpy(), want), f"{name}/{k}"
    assert res.other_data == case.meta["result_other_data"]
    assert res.in_round == case.meta["in_round"] and res.end_training == case.meta["end_training"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_plugin_result_on_the_host_bitwise(name, hip_device):
    """result_device="cpu" (the reference's server caches host fp64 tensors): one pinned D2H copy
    of the flat result, same bits, host tensors."""
    case = CASES[name]
    if case.error is not None or not case.accumulate:
        return
    res = run_hip(case, hip_device, 64, result_device="cpu")
    for k, want in case.expected.items():
        got = res.parameter[k]
        assert got.device.type == "cpu" and got.dtype == torch.float64
        assert bits_equal(got.numpy(), want), f"{name}/{k}"


def test_total_weight_hook_receives_the_reference_totals(hip_device):
    case = CASES["total_weight_hook"]
    algos = []
    run_hip(case, hip_device, 2, algo_out=algos)
    assert algos[0].seen_totals == case.meta["hook_totals"]


def test_eager_nan_check_fails_the_arrival(hip_device):
    """eager_nan_check: fed_avg_algorithm.py:35 fires while the offending update arrives."""
    case = CASES["err_nan_input"]
    algo = FedAVGAlgorithm(device=hip_device, eager_nan_check=True)
    a0, a1 = case.arrivals[0], case.arrivals[1]
    algo.process_worker_data(a0.worker_id, ParameterMessage(parameter=case.torch_params(a0, hip_device),
                                                            aggregation_weight=a0.weight))
    with pytest.raises(NaNAggregationError) as ei:
        algo.process_worker_data(a1.worker_id, ParameterMessage(parameter=case.torch_params(a1, "cpu"),
                                                                aggregation_weight=a1.weight))
    assert ei.value.stage == "input" and ei.value.bad_clients == [a1.worker_id]
    algo.exit()


@pytest.mark.parametrize("name", sorted(CASES))
def test_plugin_with_foreign_messages_bitwise(name, hip_device):
    """Messages of another wire module (the reference server passes simulation_lib.message
    objects): recognised by their fields, answered in their own ParameterMessage class."""
    case = CASES[name]
    if case.error is not None:
        exc = {"AssertionError": AssertionError, "RuntimeError": RuntimeError}[case.error]
        with pytest.raises(exc):
            run_hip(case, hip_device, 3, wire=foreign)
        return
    res = run_hip(case, hip_device, 3, from_host=True, wire=foreign)
    assert type(res) is foreign.ParameterMessage
    assert list(res.parameter.keys()) == case.meta["out_keys"]
    for k, want in case.expected.items():
        assert bits_equal(res.parameter[k].cpu().numpy(), want), f"{name}/{k}"
    assert res.other_data == case.meta["result_other_data"]


@pytest.mark.parametrize("wire", [None, foreign], ids=["pkg", "foreign"])
def test_unfusable_deltas_are_restored_bitwise(wire, hip_device):
    """Deltas carrying new_parameter (restore()'s consistency check) take the host restore, then
    the ordinary fold: still the reference's bits (golden case delta_restore)."""
    case = CASES["delta_restore"]
    res = run_hip(case, hip_device, 2, from_host=True, wire=wire, delta_checks=True)
    for k, want in case.expected.items():
        assert bits_equal(res.parameter[k].cpu().numpy(), want), k


def test_deltas_on_the_ratio_path(hip_device):
    """accumulate=False with delta updates: restored, then weighted_avg (oracle restatement)."""
    from oracle import fedavg_oracle as O

    case = CASES["delta_restore"]
    algo = FedAVGAlgorithm(device=hip_device)
    algo.accumulate = False
    old = {k: torch.from_numpy(v.copy()) for k, v in case.old.items()}
    algo.set_old_parameter(old)
    odata = {}
    for a, kind in zip(case.arrivals, case.kinds):
        params = case.torch_params(a, "cpu")  # workers send host tensors
        host = {k: v.cpu().numpy() for k, v in params.items()}
        if kind == "delta":
            algo.process_worker_data(a.worker_id, _pkg_message.DeltaParameterMessage(
                delta_parameter=params, aggregation_weight=a.weight))
            host = O.restore(host, case.old)
        else:
            msg = ParameterMessage(parameter=params, aggregation_weight=a.weight)
            msg.complete(old)
            algo.process_worker_data(a.worker_id, msg)
            O.complete(host, case.old)
        odata[a.worker_id] = O.OracleMessage(parameter=host, aggregation_weight=a.weight)
    res = algo.aggregate_worker_data()
    want = O.weighted_avg(odata, O.get_ratios(odata))
    for k in want:
        assert bits_equal(res.parameter[k].cpu().numpy(), want[k]), k


def test_nan_input_names_the_client(hip_device):
    case = CASES["err_nan_input"]
    with pytest.raises(NaNAggregationError) as ei:
        run_hip(case, hip_device, wave_size=64)
    assert ei.value.stage == "input" and ei.value.bad_clients == [1]


def test_inf_minus_inf_is_an_accumulator_nan(hip_device):
    with pytest.raises(NaNAggregationError) as ei:
        run_hip(CASES["err_inf_minus_inf"], hip_device, wave_size=64)
    assert ei.value.stage == "accumulator"


def test_zero_total_weight_is_a_result_nan(hip_device):
    with pytest.raises(NaNAggregationError) as ei:
        run_hip(CASES["err_zero_total_weight"], hip_device, wave_size=64)
    assert ei.value.stage == "result"


# ---------------------------------------------------------------------------------------
# context-level sweeps against the oracle
# ---------------------------------------------------------------------------------------
def _random_layout(rng, n_seg, max_numel):
    shapes = [(int(rng.integers(1, max_numel)),) for _ in range(n_seg)]
    return ModelLayout(names=tuple(f"t{i}" for i in range(n_seg)), shapes=tuple(shapes))


def _clients(layout, K, dtype, device, seed, offset=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    rows = []
    for _ in range(K):
        row = []
        for n in layout.numels:
            base = torch.randn(n + offset, generator=g).to(dtype).to(device)
            row.append(base[offset:])  # offset > 0 -> unaligned views (scalar path)
        rows.append(row)
    return rows


def _oracle(rows, weights, layout):
    out = []
    for i in range(layout.num_segments):
        xs = [as_f64(r[i].cpu().view(torch.int16).numpy().view(np.uint16), "bfloat16")
              if r[i].dtype == torch.bfloat16 else r[i].cpu().numpy() for r in rows]
        out.append(fedavg_flat(xs, [w[i] for w in weights]))
    return out


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16", "float64"])
@pytest.mark.parametrize("K", [1, 2, 7, 9, 64, 100])
@pytest.mark.parametrize("out_dtype", ["float64", "float32"])
def test_aggregate_sweep_exact(dtype, K, out_dtype, hip_device):
    rng = np.random.default_rng(K * 7 + len(dtype))
    layout = _random_layout(rng, n_seg=5, max_numel=9000)
    dt, odt = TORCH_DT[dtype], TORCH_DT[out_dtype]
    rows = _clients(layout, K, dt, hip_device, seed=K)
    weights = [[float(rng.integers(100, 5000))] * layout.num_segments for _ in range(K)]
    ctx = FedAvgContext(layout, hip_device, split_policy=1)
    table = ClientTable(layout.num_segments)
    for r, w in zip(rows, weights):
        table.add_client(r, w)
    outs = [torch.empty(n, dtype=odt, device=hip_device) for n in layout.numels]
    ctx.aggregate(table, dt, outs, odt)
    ctx.raise_on_nan()
    want = _oracle(rows, weights, layout)
    for o, w in zip(outs, want):
        w_cast = w.astype(np.float32).astype(np.float64) if odt == torch.float32 else w
        assert bits_equal(o.double().cpu().numpy(), w_cast)


@pytest.mark.parametrize("offset", [1, 3])
def test_unaligned_views_take_the_scalar_path(offset, hip_device):
    rng = np.random.default_rng(offset)
    layout = _random_layout(rng, n_seg=3, max_numel=5000)
    rows = _clients(layout, 11, torch.float32, hip_device, seed=5, offset=offset)
    weights = [[float(rng.integers(1, 50))] * 3 for _ in range(11)]
    ctx = FedAvgContext(layout, hip_device)
    table = ClientTable(3)
    for r, w in zip(rows, weights):
        table.add_client(r, w)
    outs = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in layout.numels]
    ctx.aggregate(table, torch.float32, outs, torch.float64)
    for o, w in zip(outs, _oracle(rows, weights, layout)):
        assert bits_equal(o.cpu().numpy(), w)


def test_streaming_waves_equal_one_shot(hip_device):
    """accumulate(wave 1) + accumulate(wave 2) + aggregate(wave 3) == the oracle's sequence."""
    rng = np.random.default_rng(11)
    layout = _random_layout(rng, n_seg=4, max_numel=20000)
    rows = _clients(layout, 23, torch.float32, hip_device, seed=3)
    weights = [[float(x) for x in rng.uniform(0.01, 3.0, size=4)] for _ in range(23)]
    ctx = FedAvgContext(layout, hip_device)
    for lo, hi in ((0, 8), (8, 15)):
        t = ClientTable(4)
        for r, w in zip(rows[lo:hi], weights[lo:hi]):
            t.add_client(r, w)
        ctx.accumulate(t, torch.float32)
    t = ClientTable(4)
    for r, w in zip(rows[15:], weights[15:]):
        t.add_client(r, w)
    outs = [torch.empty(n, dtype=torch.float64, device=hip_device) for n in layout.numels]
    ctx.aggregate(t, torch.float32, outs, torch.float64)
    for o, w in zip(outs, _oracle(rows, weights, layout)):
        assert bits_equal(o.cpu().numpy(), w)


def test_split_kernel_within_tolerance(hip_device):
    """Small layout, many clients: the LDS split kernel (4 waves x client ranges)."""
    rng = np.random.default_rng(2)
    layout = _random_layout(rng, n_seg=3, max_numel=3000)
    K = 96
    rows = _clients(layout, K, torch.float32, hip_device, seed=9)
    weights = [[float(rng.integers(100, 5000))] * 3 for _ in range(K)]
    want = _oracle(rows, weights, layout)
    for out_dtype in (torch.float64, torch.float32):
        ctx = FedAvgContext(layout, hip_device, split_policy=2)
        table = ClientTable(3)
        for r, w in zip(rows, weights):
            table.add_client(r, w)
        outs = [torch.empty(n, dtype=out_dtype, device=hip_device) for n in layout.numels]
        ctx.aggregate(table, torch.float32, outs, out_dtype)
        for i, (o, w) in enumerate(zip(outs, want)):
            got = o.double().cpu().numpy()
            if out_dtype == torch.float64:
                mag = sum(np.abs(r[i].cpu().numpy().astype(np.float64)) * wt[i] for r, wt in zip(rows, weights))
                W = sum(wt[i] for wt in weights)
                assert np.all(np.abs(got - w) <= 1e-12 * mag / W)
            else:
                w32 = w.astype(np.float32)
                ulp = np.spacing(np.abs(w32)).astype(np.float64)
                assert np.all(np.abs(got - w32.astype(np.float64)) <= ulp)


def test_partial_chunks_and_finalize_match_fused(hip_device):
    """The multi-GPU shard primitives on one rank: chunked partial + finalize == fused."""
    rng = np.random.default_rng(4)
    layout = _random_layout(rng, n_seg=6, max_numel=70000)
    rows = _clients(layout, 10, torch.float32, hip_device, seed=1)
    weights = [[float(rng.integers(100, 5000))] * 6 for _ in range(10)]
    table = ClientTable(6)
    for r, w in zip(rows, weights):
        table.add_client(r, w)
    ctx = FedAvgContext(layout, hip_device)
    n = ctx.num_tiles
    edges = [0, n // 3, n // 2, n]
    for tb, te in zip(edges[:-1], edges[1:]):
        ctx.partial(table, torch.float32, zero_init=True, tile_begin=tb, tile_end=te)
    totals = [sum(w[i] for w in weights) for i in range(6)]
    ctx.set_accumulated(totals)
    outs = [torch.empty(m, dtype=torch.float64, device=hip_device) for m in layout.numels]
    for tb, te in zip(edges[:-1], edges[1:]):
        ctx.finalize_range(outs, torch.float64, tb, te)
    ctx.raise_on_nan()
    for o, w in zip(outs, _oracle(rows, weights, layout)):
        # zero_init starts at +0.0: bitwise equal for non-zero data
        assert bits_equal(o.cpu().numpy(), w)
    # tile ranges tile the accumulator without gaps
    a0, _ = ctx.tile_range(0, 1)
    _, b1 = ctx.tile_range(n - 1, n)
    assert a0 == 0 and b1 == ctx.accumulator.numel()


def test_weighted_avg_classmethod(hip_device):
    case = CASES["ratio_path"]
    data = {}
    for a in case.arrivals:
        data[a.worker_id] = ParameterMessage(parameter=case.torch_params(a, hip_device), aggregation_weight=a.weight)
    res = AggregationAlgorithm.weighted_avg(data, AggregationAlgorithm.get_ratios(data), device=hip_device)
    for k, want in case.expected.items():
        assert bits_equal(res[k].cpu().numpy(), want)


def test_resnet18_64_clients_full_size(hip_device):
    """BASELINE config 2 at full size: every element vs the oracle, fp32 output."""
    from bench import dataset_size_weights, make_clients, resnet18_layout

    layout = resnet18_layout()
    K = 64
    buckets, views = make_clients(layout, 0, K, hip_device, torch.float32)
    w = dataset_size_weights(K)
    table = ClientTable(layout.num_segments)
    for row, wk in zip(views, w):
        table.add_client(row, [wk] * layout.num_segments)
    ctx = FedAvgContext(layout, hip_device)
    offs, padded = layout.padded_offsets(4)
    flat = torch.empty(padded, dtype=torch.float32, device=hip_device)
    outs = [flat[o : o + m] for o, m in zip(offs, layout.numels)]
    ctx.aggregate(table, torch.float32, outs, torch.float32)
    ctx.raise_on_nan()
    host = buckets.cpu().numpy()
    got = flat.cpu().numpy()
    acc = host[0].astype(np.float64) * w[0]
    for k in range(1, K):
        acc += host[k].astype(np.float64) * w[k]
    want = (acc / float(sum(w))).astype(np.float32)
    for o, m in zip(offs, layout.numels):
        assert np.array_equal(got[o : o + m].view(np.uint32), want[o : o + m].view(np.uint32))


def test_bw_probe_and_profiling(hip_device):
    src = torch.ones(1 << 24, dtype=torch.float32, device=hip_device)
    dst = torch.zeros_like(src)
    bw_probe(src, dst, 0)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    bw_probe(src, dst, 1)
    layout = ModelLayout.flat(4096)
    ctx = FedAvgContext(layout, hip_device)
    ctx.prof_enable(True)
    t = ClientTable(1)
    t.add_client([src[:4096]], [2.0])
    out = [torch.empty(4096, dtype=torch.float64, device=hip_device)]
    ctx.aggregate(t, torch.float32, out, torch.float64)
    ms, n = ctx.prof_collect()
    assert n == 1 and ms > 0
    assert torch.equal(out[0], torch.ones(4096, dtype=torch.float64, device=hip_device))


def test_native_rejects_bad_arguments(hip_device):
    from distributed_learning_simulation_lib_amd import _native

    lib = _native.load()
    h = ctypes.c_void_p()
    n = (ctypes.c_int64 * 1)(0)
    assert lib.fedavg_ctx_create(ctypes.byref(h), 0, n, 1, None) == _native.ERR_INVALID
    layout = ModelLayout.flat(100)
    ctx = FedAvgContext(layout, hip_device)
    out = [torch.empty(100, dtype=torch.float64, device=hip_device)]
    with pytest.raises(_native.NativeError):  # nothing accumulated (fed_avg_algorithm.py:88)
        ctx.aggregate(None, torch.float32, out, torch.float64)


def test_plan_equals_aggregate_and_guards_state(hip_device):
    rng = np.random.default_rng(21)
    layout = _random_layout(rng, n_seg=4, max_numel=30000)
    rows = _clients(layout, 13, torch.float32, hip_device, seed=21)
    weights = [[float(rng.integers(100, 5000))] * 4 for _ in range(13)]
    table = ClientTable(4)
    for r, w in zip(rows, weights):
        table.add_client(r, w)
    ctx = FedAvgContext(layout, hip_device)
    outs = [torch.empty(n, dtype=torch.float32, device=hip_device) for n in layout.numels]
    plan = ctx.plan(table, torch.float32, outs, torch.float32)
    for _ in range(3):
        plan.run()
        ctx.raise_on_nan()
        for o, w in zip(outs, _oracle(rows, weights, layout)):
            assert bits_equal(o.double().cpu().numpy(), w.astype(np.float32).astype(np.float64))
    t1 = ClientTable(4)
    t1.add_client(rows[0], weights[0])
    ctx.accumulate(t1, torch.float32)
    from distributed_learning_simulation_lib_amd import _native
    with pytest.raises(_native.NativeError):  # the context holds accumulated data
        plan.run()
    plan.close()
