"""The single-process multi-device mode (include/fedavg_hip.h fedavg_multi_*, multi_device.py) on
one MI355X: the device entries repeat cuda:0 (aliased devices), so the whole exchange — windows,
receive slots, entry-ordered sums, the root's outputs, the events between the entries' streams —
runs on the one GPU the box has.

Expected values: the oracle's sharded composition (oracle/fedavg_oracle.py ``sharded_composition``):
each entry's arrival-order fp64 chain over its clients, the chains summed in entry order, divided by
the arrival-order total weight — what the peer exchange computes, asserted BIT-IDENTICAL. The
reference's single chain differs from it by fp64 reassociation only (asserted within 1e-12 relative
of sum |w x| / W, and the fp32 casts within 1 ulp).
"""

from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage
from distributed_learning_simulation_lib_amd.build import LIB_DIR
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, ModelLayout, NaNAggregationError, OutputTable
from distributed_learning_simulation_lib_amd.multi_device import MultiDeviceContext, window_bounds
from distributed_learning_simulation_lib_amd.sharded import chunk_edges
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage, as_f64, fedavg_flat, sharded_composition
from tests.golden_hooks import make_hooked_class
from tests.golden_io import bits_equal, load_golden
from tests.test_gpu_parity import hook_spec
from tests.multi_tolerance import reference_magnitude, sharded_expectation, ulp32, within_reference_tolerance

pytestmark = pytest.mark.gpu
CASES = load_golden()

LAYOUT = ModelLayout(names=("conv", "bias", "fc", "one", "big", "odd"),
                     shapes=((16, 3, 3, 3), (16,), (10, 257), (1,), (3, 4096), (4096 * 2 + 13,)))


def entry_devices(world: int, placement: str) -> list[int]:
    """``aliased``: every entry on cuda:0 (the whole exchange on one GPU); ``distinct``: entries dealt
    over every visible GPU (peer access, xGMI stores, cross-device events) — skipped on a one-GPU box."""
    if placement == "aliased":
        return [0] * world
    count = torch.cuda.device_count()
    if count < 2:
        pytest.skip("distinct device entries need more than one GPU")
    return [g % count for g in range(world)]


PLACEMENTS = ["aliased", "distinct"]


def _clients(n, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    return [[torch.randn(m, generator=g).to(dtype) for m in LAYOUT.numels] for _ in range(n)]


def _owner(k, n, world, empty=None):
    g = k * world // n
    return 0 if g == empty else g


@pytest.mark.parametrize("placement", PLACEMENTS)
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.float64])
def test_peer_round_is_the_sharded_composition(hip_device, world, dtype, placement):
    n = 11
    rng = np.random.default_rng(world)
    weights = [int(w) for w in rng.integers(1, 5000, n)] if dtype != torch.float64 else \
        [float(w) for w in rng.uniform(0.1, 9.0, n)]
    clients = _clients(n, dtype, 3 + world)
    devices = entry_devices(world, placement)
    m = MultiDeviceContext(LAYOUT, devices)
    try:
        assert m.peer_access and m.world == world
        tables = [ClientTable(LAYOUT.num_segments) for _ in range(world)]
        for k, c in enumerate(clients):
            g = _owner(k, n, world)
            tables[g].add_client([t.to(torch.device("cuda", devices[g])) for t in c], [weights[k]] * LAYOUT.num_segments)
        partials = m.plan_partials(tables, dtype)
        W = -0.0
        for w in weights:
            W += w
        nt = m.num_tiles
        for out_dtype in (torch.float64, torch.float32):
            outs = [torch.empty(s, dtype=out_dtype, device=hip_device) for s in LAYOUT.numels]
            for edges in ([0, nt], chunk_edges(nt, 3), chunk_edges(nt, 4, "taper"), [0, 1, nt]):
                for root in {0, world - 1}:
                    for o in outs:
                        o.fill_(float("nan"))
                    m.round(partials, [W] * LAYOUT.num_segments, outs, out_dtype, root=root, edges=edges)
                    m.raise_on_nan()
                    for s in range(LAYOUT.num_segments):
                        shards = [[clients[k][s].numpy() for k in range(n) if _owner(k, n, world) == g]
                                  for g in range(world)]
                        sw = [[weights[k] for k in range(n) if _owner(k, n, world) == g] for g in range(world)]
                        want = sharded_composition(shards, sw, W)
                        got = outs[s].cpu().numpy()
                        if out_dtype == torch.float64:
                            assert bits_equal(got, want), (edges, root, s)
                        else:
                            assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32)), s
                        # against the reference's single chain: fp64 within 1e-12 of sum |w x| / W,
                        # the fp32 casts at most 1 ulp apart (the device result itself, both dtypes)
                        single = fedavg_flat([clients[k][s].numpy() for k in range(n)], weights)
                        mag = sum(np.abs(as_f64(clients[k][s].numpy())) * abs(weights[k]) for k in range(n)) / W
                        assert np.all(np.abs(want - single) <= 1e-12 * mag)
                        if out_dtype == torch.float64:
                            ok, why = within_reference_tolerance(got, single, mag)
                        else:  # an fp32 result: the 1-ulp form of the bound
                            u = ulp32(got, single)
                            ok, why = bool(u.size == 0 or u.max() <= 1), f"{u.max()} ulp"
                        assert ok, (edges, root, s, why)
    finally:
        m.close()


def test_peer_round_with_an_entry_without_clients(hip_device):
    world, n = 4, 9
    clients = _clients(n, torch.float32, 41)
    weights = list(range(100, 100 + n))
    m = MultiDeviceContext(LAYOUT, [0] * world)
    try:
        tables: list[ClientTable | None] = [ClientTable(LAYOUT.num_segments) for _ in range(world)]
        for k, c in enumerate(clients):
            tables[_owner(k, n, world, empty=2)].add_client([t.to(hip_device) for t in c], [weights[k]] * 6)
        tables[2] = None
        partials = m.plan_partials(tables, torch.float32)
        assert partials[2] is None
        W = float(sum(weights))
        outs = [torch.empty(s, dtype=torch.float64, device=hip_device) for s in LAYOUT.numels]
        for _ in range(2):
            m.round(partials, [W] * 6, outs, torch.float64, root=2, edges=chunk_edges(m.num_tiles, 2))
            m.raise_on_nan()
            for s in range(6):
                shards = [[clients[k][s].numpy() for k in range(n) if _owner(k, n, world, 2) == g] for g in range(world)]
                sw = [[weights[k] for k in range(n) if _owner(k, n, world, 2) == g] for g in range(world)]
                assert bits_equal(outs[s].cpu().numpy(), sharded_composition(shards, sw, W)), s
    finally:
        m.close()


def test_plans_outliving_the_multi_context_leave_no_hip_error(hip_device):
    """Closing the multi-device object closes the plans of its entries first (a native plan reads
    its context); a plan dropped afterwards and the next torch launch see no sticky HIP error, and
    the caller's current device is the one it set."""
    import gc

    dev_before = torch.cuda.current_device()
    m = MultiDeviceContext(LAYOUT, [0, 0])
    t = ClientTable(LAYOUT.num_segments)
    t.add_client([x.to(hip_device) for x in _clients(1, torch.float32, 1)[0]], [3.0] * LAYOUT.num_segments)
    partials = m.plan_partials([t, None], torch.float32)
    outs = [torch.empty(s, dtype=torch.float32, device=hip_device) for s in LAYOUT.numels]
    m.round(partials, [3.0] * LAYOUT.num_segments, outs, torch.float32)
    m.raise_on_nan()
    m.close()
    del partials
    gc.collect()
    assert torch.cuda.current_device() == dev_before
    assert float(torch.ones(8, device=hip_device).sum().item()) == 8.0
    torch.cuda.synchronize(hip_device)


def test_peer_round_nan_input_names_the_client(hip_device):
    world, n = 3, 6
    clients = _clients(n, torch.float32, 5)
    clients[4][2][17] = float("nan")  # entry 2's first client
    m = MultiDeviceContext(LAYOUT, [0] * world)
    try:
        tables = [ClientTable(6) for _ in range(world)]
        for k, c in enumerate(clients):
            tables[_owner(k, n, world)].add_client([t.to(hip_device) for t in c], [1.0] * 6)
        partials = m.plan_partials(tables, torch.float32)
        outs = [torch.empty(s, dtype=torch.float32, device=hip_device) for s in LAYOUT.numels]
        m.round(partials, [float(n)] * 6, outs, torch.float32, edges=chunk_edges(m.num_tiles, 3))
        with pytest.raises(NaNAggregationError) as ei:
            m.raise_on_nan([[(t, torch.float32)] for t in tables])
        assert ei.value.stage == "input" and ei.value.bad_clients == [0]
        # the object is usable after the error (flags cleared)
        clients[4][2][17] = 0.0
        m.raise_on_nan()
    finally:
        m.close()


def test_inf_minus_inf_across_entries_is_the_accumulator_assertion(hip_device):
    # +inf in entry 0's shard, -inf in entry 1's: each chain is finite-or-inf, their sum is NaN —
    # fed_avg_algorithm.py:93 (the reference's single chain hits the same NaN)
    layout = ModelLayout(names=("x",), shapes=((300,),))
    a = torch.zeros(300, device=hip_device)
    b = torch.zeros(300, device=hip_device)
    a[7], b[7] = float("inf"), float("-inf")
    m = MultiDeviceContext(layout, [0, 0])
    try:
        t0, t1 = ClientTable(1), ClientTable(1)
        t0.add_client([a], [1.0])
        t1.add_client([b], [1.0])
        outs = [torch.empty(300, dtype=torch.float64, device=hip_device)]
        m.round(m.plan_partials([t0, t1], torch.float32), [2.0], outs, torch.float64)
        with pytest.raises(NaNAggregationError) as ei:
            m.raise_on_nan([[(t0, torch.float32)], [(t1, torch.float32)]])
        assert ei.value.stage == "accumulator"
    finally:
        m.close()


def test_window_bounds_partition_every_chunk():
    for tb, te in ((0, 1), (0, 7), (5, 1427), (100, 103)):
        for world in (1, 2, 3, 4, 8):
            w = window_bounds(tb, te, world)
            assert w[0][0] == tb and w[-1][1] == te and all(x[1] == y[0] for x, y in zip(w, w[1:]))


# ---- the plugin surface: FedAVGAlgorithm(devices=[...]) ---------------------------------------------
def run_multi(case, device, world, wave_size, from_host=False, devices=None):
    algo = make_hooked_class(FedAVGAlgorithm, hook_spec(case))(devices=devices or [device] * world,
                                                                 wave_size=wave_size)
    algo.accumulate = case.accumulate
    algo.aggregate_loss = case.aggregate_loss
    kinds = case.kinds or ["full"] * len(case.arrivals)
    old = None
    if case.old is not None:
        old = {k: torch.from_numpy(v.copy()) for k, v in case.old.items()}
        algo.set_old_parameter(old)
    from distributed_learning_simulation_lib_amd import message as wire
    for a, kind in zip(case.arrivals, kinds):
        if a.arrays is None:
            algo.process_worker_data(a.worker_id, None)
            continue
        params = case.torch_params(a, "cpu" if from_host else device)
        if kind == "delta":
            msg = wire.DeltaParameterMessage(delta_parameter=params, aggregation_weight=a.weight,
                                             other_data=dict(a.other_data))
        else:
            msg = wire.ParameterMessage(parameter=params, aggregation_weight=a.weight, other_data=dict(a.other_data))
            if old is not None:
                msg.complete(old)
        algo.process_worker_data(a.worker_id, msg)
    try:
        return algo.aggregate_worker_data()
    finally:
        algo.exit()


@pytest.mark.parametrize("world,wave_size", [(2, 1), (3, 64), (4, 3)])
@pytest.mark.parametrize("name", sorted(CASES))
def test_plugin_devices_golden_cases(name, world, wave_size, hip_device):
    case = CASES[name]
    if case.error is not None:
        exc = {"AssertionError": AssertionError, "RuntimeError": RuntimeError}[case.error]
        with pytest.raises(exc):
            run_multi(case, hip_device, world, wave_size)
        return
    res = run_multi(case, hip_device, world, wave_size, from_host=(wave_size == 3))
    assert list(res.parameter.keys()) == case.meta["out_keys"]
    want = case.expected if not case.accumulate else sharded_expectation(case, world)
    mag = reference_magnitude(case) if case.accumulate else None
    for k, v in want.items():
        got = res.parameter[k]
        assert got.dtype == torch.float64 and tuple(got.shape) == v.shape and got.device == hip_device
        assert bits_equal(got.cpu().numpy(), v), f"{name}/{k}"
        if mag is not None:  # and against the reference's single chain at the stated tolerance
            ok, why = within_reference_tolerance(got.cpu().numpy(), case.expected[k], mag[k])
            assert ok, f"{name}/{k}: {why}"
    assert res.other_data == case.meta["result_other_data"]
    assert res.in_round == case.meta["in_round"] and res.end_training == case.meta["end_training"]


@pytest.mark.parametrize("name", sorted(n for n, c in CASES.items() if c.error is None and c.accumulate))
def test_plugin_distinct_devices_golden_cases(name, hip_device):
    """The plugin over every visible GPU (skipped on a one-GPU box): peer loads of the entries'
    accumulators across devices, the result on the first entry's GPU."""
    case = CASES[name]
    devices = [torch.device("cuda", d) for d in entry_devices(torch.cuda.device_count(), "distinct")]
    res = run_multi(case, devices[0], len(devices), 3, devices=devices)
    want = sharded_expectation(case, len(devices))
    mag = reference_magnitude(case)
    for k, v in want.items():
        got = res.parameter[k]
        assert got.device == devices[0] and bits_equal(got.cpu().numpy(), v), f"{name}/{k}"
        ok, why = within_reference_tolerance(got.cpu().numpy(), case.expected[k], mag[k])
        assert ok, f"{name}/{k}: {why}"


@pytest.mark.parametrize("world", [2, 4])
def test_plugin_devices_rounds_and_late_key(hip_device, world):
    # two rounds on one object; a key first seen mid-round grows the layout of every entry; a
    # partial update (a missing key) only folds into its own entry
    algo = FedAVGAlgorithm(devices=[hip_device] * world, wave_size=2)
    shapes = {"a": (40, 33), "b": (7,), "c": (4096 + 9,)}
    g = torch.Generator().manual_seed(3)
    rng = np.random.default_rng(3)
    for rnd in range(2):
        full = OracleFedAvg()
        lanes = [OracleFedAvg() for _ in range(world)]
        for k in range(9):
            sh = dict(shapes)
            if k == 4:
                del sh["b"]
            if k == 6 and rnd == 0:
                sh["late"] = (13,)
            p = {n: torch.randn(s, generator=g) for n, s in sh.items()}
            w = float(rng.uniform(0.1, 3.0))
            algo.process_worker_data(k, ParameterMessage(parameter={n: t.to(hip_device) for n, t in p.items()},
                                                         aggregation_weight=w))
            full.process_worker_data(k, OracleMessage(parameter={n: t.numpy() for n, t in p.items()}, aggregation_weight=w))
            lanes[k % world].process_worker_data(k, OracleMessage(parameter={n: t.numpy() for n, t in p.items()},
                                                                  aggregation_weight=w))
        got = algo.aggregate_worker_data().parameter
        assert list(got) == list(full._acc)
        for name in full._acc:
            parts = [ln._acc[name] for ln in lanes if name in ln._acc]
            s = parts[0]
            for q in parts[1:]:
                s = s + q
            assert bits_equal(got[name].cpu().numpy(), s / full._totals[name]), (rnd, name)
        algo.clear_worker_data()
    algo.exit()


def test_multi_device_c_example_peer(hip_device):
    exe = LIB_DIR / "multi_device_round"
    assert exe.exists(), "run __graft_entry__.build()"
    r = subprocess.run([str(exe), "--devices", "0,0,0,0", "--exchange", "peer"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("fake", ["libfake_rccl.so", "libfake_rccl_nogather.so"])
def test_multi_device_c_example_reduce_in_process_rccl(hip_device, fake):
    # the REDUCE exchange: ncclCommInitAll + grouped ncclReduce from one host thread; real RCCL
    # refuses four ranks on one GPU, so the in-process stand-in sums in rank order (bit-exact)
    exe = LIB_DIR / "multi_device_round"
    env = dict(os.environ, FEDAVG_RCCL_LIB=str(LIB_DIR / fake))
    r = subprocess.run([str(exe), "--devices", "0,0,0", "--exchange", "both"], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("world", [2, 3])
def test_peer_round_with_quantised_and_mixed_entries(hip_device, world):
    """Entries holding QSGD records take the separate-combine form of the peer exchange (every
    window, their own included, into its owner's slot); dense entries fold their own window with
    the received partials. Mixed in one round (entry 0 QSGD, the others fp32), the result is still
    the entry-ordered composition of each entry's chain over its own (dequantised) clients."""
    from distributed_learning_simulation_lib_amd.quantized import QSGD_F32, QuantizedTensor
    from oracle import qsgd_oracle as qo

    n = 7
    rng = np.random.default_rng(40 + world)
    weights = [int(w) for w in rng.integers(1, 3000, n)]
    dense = _clients(n, torch.float32, 11)
    recs = [[qo.quantize(c.numpy(), rng) for c in row] for row in dense]
    deq = [[qo.dequantize(r, m, "float32") for r, m in zip(row, LAYOUT.numels)] for row in recs]
    W = -0.0
    for w in weights:
        W += w
    for mixed in (False, True):
        m = MultiDeviceContext(LAYOUT, [0] * world)
        try:
            plans, rows = [], []
            for g in range(world):
                ks = [k for k in range(n) if _owner(k, n, world) == g]
                t = ClientTable(LAYOUT.num_segments)
                quant = (g == 0) or not mixed
                for k in ks:
                    if quant:
                        qts = [QuantizedTensor(torch.from_numpy(r).to(hip_device), (mm,), QSGD_F32)
                               for r, mm in zip(recs[k], LAYOUT.numels)]
                        t.add_client([q.record for q in qts], [weights[k]] * LAYOUT.num_segments)
                    else:
                        t.add_client([x.to(hip_device) for x in dense[k]], [weights[k]] * LAYOUT.num_segments)
                plans.append(m.contexts[g].plan_partial(t, QSGD_F32 if quant else torch.float32, zero_init=True))
                rows.append([deq[k] if quant else [x.numpy() for x in dense[k]] for k in ks])
            outs = [torch.empty(s, dtype=torch.float64, device=hip_device) for s in LAYOUT.numels]
            for edges in ([0, m.num_tiles], chunk_edges(m.num_tiles, 3)):
                m.round(plans, [W] * LAYOUT.num_segments, outs, torch.float64, root=world - 1, edges=edges)
                m.raise_on_nan()
                for s in range(LAYOUT.num_segments):
                    shards = [[r[s] for r in rows[g]] for g in range(world)]
                    sw = [[weights[k] for k in range(n) if _owner(k, n, world) == g] for g in range(world)]
                    assert bits_equal(outs[s].cpu().numpy(), sharded_composition(shards, sw, W)), (mixed, edges, s)
        finally:
            m.close()
