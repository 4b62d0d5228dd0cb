"""The dynamic wave (include/fedavg_hip.h fedavg_dyn_*): the plugin round's first wave folded while
its clients arrive, on the MI355X.

Every result is asserted BIT-IDENTICAL to the oracle's arrival-order chain (fed_avg_algorithm.py:
43-99): whether the wave divides into the outputs itself, is closed early (a row it cannot take, a
busy stream, its own idle limit) and leaves the ordinary waves the rest, or is abandoned.
"""

from __future__ import annotations

import time

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage, _native
from distributed_learning_simulation_lib_amd._staging import NativeClientTable
from distributed_learning_simulation_lib_amd.fedavg import FedAvgContext, ModelLayout, NaNAggregationError, OutputTable
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu

@pytest.fixture(autouse=True)
def _patient_wave(monkeypatch):
    # these rounds arrive slowly (each builds its tensors and the oracle's): a wave that may idle
    # 1 s between publications folds them all (the idle test sets its own limit)
    monkeypatch.setenv("FEDAVG_DYN_IDLE_US", "1000000")
    monkeypatch.setenv("FEDAVG_DYN_MIN_ROWS", "0")  # every round opens one (the heuristic: its own test)


SHAPES = {"conv": (16, 3, 5, 5), "bias": (16,), "fc": (10, 700), "big": (3, 4096), "tail": (4096 + 37,)}


def _round(algo, dev, n, seed, dtype=torch.float32, weights="int", mutate=None, settle=False):
    """One plugin round against the oracle; ``settle``: the copies of each update are finished
    before it is handed over (every publication then takes its rows at once)."""
    g = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed)
    oracle = OracleFedAvg()
    for k in range(n):
        p = {name: torch.randn(s, generator=g).to(dtype) for name, s in SHAPES.items()}
        if mutate is not None:
            p = mutate(k, p)
        w = int(rng.integers(100, 5000)) if weights == "int" else float(rng.uniform(0.1, 3.0))
        upd = {m: t.to(dev) for m, t in p.items()}
        if settle:
            torch.cuda.current_stream(dev).synchronize()
        algo.process_worker_data(k, ParameterMessage(parameter=upd, aggregation_weight=w))
        arrs = {m: (t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy())
                for m, t in p.items()}
        oracle.process_worker_data(k, OracleMessage(parameter=arrs, aggregation_weight=w,
                                                    dtype="bfloat16" if dtype == torch.bfloat16 else None))
    got = algo.aggregate_worker_data().parameter
    algo.clear_worker_data()
    want = oracle.aggregate_worker_data().parameter
    assert list(got) == list(want)
    for name, v in want.items():
        g_ = got[name]
        if algo.result_dtype == torch.float32:
            assert torch.equal(g_.cpu(), torch.from_numpy(v).to(torch.float32)), name
        else:
            assert bits_equal(g_.cpu().numpy(), v), name


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16, torch.float64])
@pytest.mark.parametrize("n,wave", [(1, 64), (3, 64), (9, 64), (64, 64), (10, 4), (13, 13)])
def test_plugin_rounds_bit_identical(hip_device, dtype, n, wave):
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave, dynamic_wave=True)
    for r in range(2):  # two rounds on one object: the wave reopens every round
        _round(algo, hip_device, n, 10 * n + r, dtype)
    # every round's first wave folded by the dynamic wave; a single-wave round divided by it too
    assert algo.dyn_stats["waves"] == 2 and algo.dyn_stats["rows"] == 2 * min(n, wave), algo.dyn_stats
    assert algo.dyn_stats["finalized"] == (2 if n <= wave else 0), algo.dyn_stats
    algo.exit()


def test_small_rounds_skip_the_wave(hip_device, monkeypatch):
    # FEDAVG_DYN_MIN_ROWS: after a round of fewer updates the next round folds in ordinary waves
    monkeypatch.setenv("FEDAVG_DYN_MIN_ROWS", "16")
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    for r, n in enumerate((8, 8, 20, 20)):
        _round(algo, hip_device, n, 40 + r)
    # round 0 (no history) and round 3 (after a 20-update round) open a wave; rounds 1-2 do not
    assert _core(algo.dyn_stats) == {"waves": 2, "rows": 28, "finalized": 2}, algo.dyn_stats
    algo.exit()


@pytest.mark.parametrize("result_dtype", [torch.float32, torch.float64])
def test_fractional_weights_and_result_dtypes(hip_device, result_dtype):
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True, result_dtype=result_dtype)
    _round(algo, hip_device, 11, 5, weights="float")
    assert _core(algo.dyn_stats) == {"waves": 1, "rows": 11, "finalized": 1}
    algo.exit()


def test_a_row_it_cannot_take_closes_it_early(hip_device):
    # client 4 misses a tensor: the wave keeps clients 0-3, the ordinary waves fold 4-8
    def mutate(k, p):
        if k == 4:
            del p["fc"]
        return p

    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    _round(algo, hip_device, 9, 21, mutate=mutate)
    assert _core(algo.dyn_stats) == {"waves": 1, "rows": 4, "finalized": 0}
    algo.exit()


def test_busy_stream_defers_publication(hip_device):
    # the current stream holds unfinished work at every arrival: nothing is published before the
    # close (which waits for the stream), results unchanged
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)

    def mutate(k, p):
        torch.cuda._sleep(2_000_000)  # ~1 ms of GPU work on the current stream
        return p

    _round(algo, hip_device, 6, 22, mutate=mutate)
    algo.exit()


def _core(st):
    return {k: st[k] for k in ("waves", "rows", "finalized")}


def test_wave_ends_itself_when_arrivals_stop(hip_device, monkeypatch):
    # FEDAVG_DYN_IDLE_US=20000: a 200 ms gap between arrivals ends the wave with the rows it has;
    # the next publication continues the round in a fresh wave that starts from the accumulator,
    # and that wave divides into the result
    monkeypatch.setenv("FEDAVG_DYN_IDLE_US", "20000")
    monkeypatch.setenv("FEDAVG_DYN_BATCH", "1")
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)

    def mutate(k, p):
        if k == 3:
            torch.cuda.synchronize()
            time.sleep(0.2)
        return p

    _round(algo, hip_device, 8, 23, mutate=mutate)
    st = algo.dyn_stats
    assert _core(st) == {"waves": 1, "rows": 8, "finalized": 1} and st["reopens"] == 1, st
    algo.exit()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.float64])
def test_bursts_close_reopen_close_at_the_default_idle_limit(hip_device, monkeypatch, dtype):
    # the reference server's cadence (server.py:133-146: the arrivals of one poll back to back,
    # then a sleep): 3 bursts of 5 with 5 ms gaps, far above the default 200 us idle limit. Each
    # gap ends the wave; the burst after it is folded by a continued wave (from the accumulator);
    # the last one divides. Bit-identical to the single chain.
    monkeypatch.delenv("FEDAVG_DYN_IDLE_US")
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    assert algo.settings.dynamic.idle_us == 200

    def mutate(k, p):
        if k in (5, 10):
            torch.cuda.synchronize()
            time.sleep(0.005)
        return p

    for r in range(2):
        _round(algo, hip_device, 15, 80 + r, dtype, mutate=mutate)
    st = algo.dyn_stats
    assert st["waves"] == 2 and st["rows"] == 30, st
    assert st["reopens"] >= 2, st  # at least one continued wave per round
    # (a wave that ended itself after the round's last publication leaves the division to the
    # ordinary finalize — slow hosts between arrivals: finalized may be 0-2, the bits the same)
    algo.exit()


def test_idle_before_the_aggregate_finalizes_from_the_accumulator(hip_device, monkeypatch):
    # every row folded, then the wave idles out before aggregate_worker_data: the close finds it
    # ended (rows in the accumulator) and the ordinary finalize divides — still bit-identical
    monkeypatch.delenv("FEDAVG_DYN_IDLE_US")
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    orig = algo.aggregate_worker_data

    def late():
        torch.cuda.synchronize()
        time.sleep(0.01)
        return orig()

    algo.aggregate_worker_data = late
    # 5 rows: published at once, then in pairs — every row is out before the sleep (an unpublished
    # last row would instead be handed to a continued wave, which then divides: the other test)
    _round(algo, hip_device, 5, 90, settle=True)
    st = algo.dyn_stats
    # every row folded by waves; the 10 ms sleep ends the last one before the close, which then
    # finalizes from the accumulator (a slow host may also see waves end between arrivals: they
    # are continued, the counts of continued waves vary, the bits do not)
    assert _core(st) == {"waves": 1, "rows": 5, "finalized": 0}, st
    algo.exit()


def test_multi_wave_round_with_bursts(hip_device, monkeypatch):
    # wave_size 6 and 17 updates in bursts: the dynamic wave (continued after a gap) takes the
    # first 6, its flush leaves them in the accumulator, ordinary waves fold the rest
    monkeypatch.delenv("FEDAVG_DYN_IDLE_US")
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True, wave_size=6)

    def mutate(k, p):
        if k in (3, 9):
            torch.cuda.synchronize()
            time.sleep(0.004)
        return p

    _round(algo, hip_device, 17, 91, mutate=mutate)
    st = algo.dyn_stats
    # (the flush publishes what the caller's stream has finished: up to the wave's 6 rows)
    assert st["waves"] == 1 and 1 <= st["rows"] <= 6 and st["finalized"] == 0, st
    algo.exit()


def test_many_small_tensors(hip_device):
    # 1,500 tensors whose sizes are no multiple of the body tile: the edge launch has thousands of
    # workgroups and may hold the GPU first; the mirror is elected from either launch
    rng = np.random.default_rng(5)
    shapes = {f"t{i}": (int(rng.integers(1, 9000)),) for i in range(1500)}
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    g = torch.Generator().manual_seed(12)
    oracle = OracleFedAvg()
    for k in range(5):
        p = {name: torch.randn(s, generator=g) for name, s in shapes.items()}
        w = 10 + 3 * k
        algo.process_worker_data(k, ParameterMessage(parameter={m: t.to(hip_device) for m, t in p.items()},
                                                     aggregation_weight=w))
        oracle.process_worker_data(k, OracleMessage(parameter={m: t.numpy() for m, t in p.items()},
                                                    aggregation_weight=w))
    got = algo.aggregate_worker_data().parameter
    want = oracle.aggregate_worker_data().parameter
    for name, v in want.items():
        assert bits_equal(got[name].cpu().numpy(), v), name
    assert algo.dyn_stats["waves"] == 1 and algo.dyn_stats["rows"] == 5, algo.dyn_stats
    algo.exit()


def test_nan_input_names_the_client(hip_device):
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    g = torch.Generator().manual_seed(3)
    for k in range(5):
        p = {name: torch.randn(s, generator=g) for name, s in SHAPES.items()}
        if k == 2:
            p["fc"][3, 7] = float("nan")
        algo.process_worker_data(k, ParameterMessage(parameter={m: t.to(hip_device) for m, t in p.items()},
                                                     aggregation_weight=10 + k))
    with pytest.raises(NaNAggregationError) as ei:
        algo.aggregate_worker_data()
    assert ei.value.stage == "input" and ei.value.bad_clients == [2]
    algo.clear_worker_data()
    _round(algo, hip_device, 4, 24)  # the object is usable afterwards
    algo.exit()


def test_abandoned_round_and_exit_with_an_open_wave(hip_device):
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    g = torch.Generator().manual_seed(4)
    for k in range(3):
        p = {name: torch.randn(s, generator=g).to(hip_device) for name, s in SHAPES.items()}
        algo.process_worker_data(k, ParameterMessage(parameter=p, aggregation_weight=1 + k))
    algo.clear_worker_data()  # the round is dropped with its wave open
    _round(algo, hip_device, 5, 25)
    for k in range(2):
        p = {name: torch.randn(s, generator=g).to(hip_device) for name, s in SHAPES.items()}
        algo.process_worker_data(k, ParameterMessage(parameter=p, aggregation_weight=1 + k))
    algo.exit()  # the context is destroyed with a wave open
    assert float(torch.ones(4, device=hip_device).sum().item()) == 4.0


def test_c_abi_protocol(hip_device):
    """open / publish / close directly: other launches are refused while the wave is open, an
    accumulator close leaves rows [0, folded) for the ordinary calls, a final close divides."""
    layout = ModelLayout.flat(10_000)
    ctx = FedAvgContext(layout, hip_device)
    g = torch.Generator().manual_seed(6)
    xs = [torch.randn(10_000, generator=g) for _ in range(7)]
    ws = [float(3 + k) for k in range(7)]
    table = NativeClientTable(1, hip_device.index or 0)
    dev = [x.to(hip_device) for x in xs]
    for x, w in zip(dev, ws):
        table.add_client([x], [w])
    want = OracleFedAvg()
    for k, (x, w) in enumerate(zip(xs, ws)):
        want.process_worker_data(k, OracleMessage(parameter={"bucket": x.numpy()}, aggregation_weight=w))
    want = want.aggregate_worker_data().parameter["bucket"]
    out = torch.empty(10_000, dtype=torch.float64, device=hip_device)
    outs = OutputTable([out], layout, hip_device, torch.float64)
    try:
        ctx.dyn_open(torch.float32, 16)
        assert ctx.dyn_state() == (True, 0)
        with pytest.raises(_native.NativeError):
            ctx.accumulate(table, torch.float32)  # refused while the wave is open
        torch.cuda.current_stream(hip_device).synchronize()  # (a device-wide sync waits for the wave)
        assert ctx.dyn_publish(table) == 7
        folded, fin = ctx.dyn_close(outs, torch.float64)
        assert (folded, fin) == (7, True)
        ctx.raise_on_nan()
        assert bits_equal(out.cpu().numpy(), want)
        # accumulator close after 4 rows, the rest by the ordinary call
        from distributed_learning_simulation_lib_amd._staging import TableTail

        head = NativeClientTable(1, hip_device.index or 0)
        for x, w in zip(dev[:4], ws[:4]):
            head.add_client([x], [w])
        ctx.dyn_open(torch.float32, 16)
        torch.cuda.current_stream(hip_device).synchronize()  # (a device-wide sync waits for the wave)
        assert ctx.dyn_publish(head) == 4
        assert ctx.dyn_close(None) == (4, False)
        out.fill_(float("nan"))
        ctx.aggregate(TableTail(table, 4), torch.float32, outs, torch.float64)
        ctx.raise_on_nan()
        assert bits_equal(out.cpu().numpy(), want)
        ctx.reset()
        # join=False: the caller's stream does not wait; the outputs are complete after the check
        ctx.dyn_open(torch.float32, 16)
        torch.cuda.current_stream(hip_device).synchronize()
        assert ctx.dyn_publish(table) == 7
        out.fill_(float("nan"))
        torch.cuda.current_stream(hip_device).synchronize()
        assert ctx.dyn_close(outs, torch.float64, join=False) == (7, True)
        ctx.raise_on_nan()
        assert bits_equal(out.cpu().numpy(), want)
        ctx.reset()
        # a wave that ends itself (1 ms idle limit) is continued by the next publication: rows
        # [0, 3) from the accumulator, rows [3, 7) folded by the fresh launch, which divides
        ctx.dyn_configure(idle_us=1000)
        r0 = ctx.dyn_info()["reopens"]
        ctx.dyn_open(torch.float32, 16)
        torch.cuda.current_stream(hip_device).synchronize()
        head3 = NativeClientTable(1, hip_device.index or 0)
        for x, w in zip(dev[:3], ws[:3]):
            head3.add_client([x], [w])
        assert ctx.dyn_publish(head3) == 3
        time.sleep(0.02)  # the wave ends itself
        assert ctx.dyn_publish(table) == 4
        info = ctx.dyn_info()
        assert info["reopens"] == r0 + 1 and info["base"] == 3 and info["active"] == 1, info
        out.fill_(float("nan"))
        # (the fill runs on the caller's stream, the wave on its own: the fill must be done before
        # the close lets the wave store, or it may run after the wave and overwrite the result)
        torch.cuda.current_stream(hip_device).synchronize()
        assert ctx.dyn_close(outs, torch.float64) == (7, True)
        ctx.raise_on_nan()
        assert bits_equal(out.cpu().numpy(), want)
        # ... and one that ends itself with nothing published is continued zero-initialised
        ctx.dyn_open(torch.float32, 16)
        time.sleep(0.02)
        torch.cuda.current_stream(hip_device).synchronize()
        assert ctx.dyn_publish(table) == 7
        assert ctx.dyn_info()["base"] == 0
        out.fill_(float("nan"))
        # (the fill runs on the caller's stream, the wave on its own: the fill must be done before
        # the close lets the wave store, or it may run after the wave and overwrite the result)
        torch.cuda.current_stream(hip_device).synchronize()
        assert ctx.dyn_close(outs, torch.float64) == (7, True)
        ctx.raise_on_nan()
        assert bits_equal(out.cpu().numpy(), want)
        ctx.reset()
    finally:
        ctx.close()



def test_fresh_contexts_back_to_back(hip_device):
    # each algorithm object has its own context and wave: a mirror allocation recycled from the
    # previous context (same size) must not leak that context's words into the new wave
    for r in range(6):
        algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True, wave_size=64)
        _round(algo, hip_device, 3 + r % 3, 70 + r)
        assert algo.dyn_stats["waves"] == 1
        algo.exit()


def test_last_rows_still_being_copied(hip_device):
    # host updates: every arrival leaves its copy on the stream; the final publication waits for
    # the stream instead of dividing by the rows published so far (a mixed-dtype golden case
    # once returned client 0 alone)
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    g = torch.Generator().manual_seed(9)
    oracle = OracleFedAvg()
    for k in range(6):
        p = {name: torch.randn(s, generator=g) for name, s in SHAPES.items()}
        w = 100 + 17 * k
        algo.process_worker_data(k, ParameterMessage(parameter=dict(p), aggregation_weight=w))  # host tensors
        oracle.process_worker_data(k, OracleMessage(parameter={m: t.numpy() for m, t in p.items()}, aggregation_weight=w))
    got = algo.aggregate_worker_data().parameter
    want = oracle.aggregate_worker_data().parameter
    for name, v in want.items():
        assert bits_equal(got[name].cpu().numpy(), v), name
    algo.exit()


def test_updates_from_another_process_keep_the_wave_off(hip_device):
    # a worker process on the same GPU sends its updates as CUDA tensors (IPC): that process has a
    # context on this GPU, so the round folds in ordinary launches (no wave holding the register
    # file), with the same bits
    import torch.multiprocessing as mp
    from multiprocessing.reduction import ForkingPickler

    from tests.ipc_consumer import produce

    seeds = [31, 32, 33, 34, 35]
    ctx = mp.get_context("spawn")
    parent, child = ctx.Pipe()
    p = ctx.Process(target=produce, args=(child, SHAPES, seeds))
    p.start()
    try:
        algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
        oracle = OracleFedAvg()
        for k, s in enumerate(seeds):
            upd = ForkingPickler.loads(parent.recv_bytes())
            g = torch.Generator().manual_seed(s)
            host = {name: torch.randn(sh, generator=g) for name, sh in SHAPES.items()}
            w = 100 + k
            algo.process_worker_data(k, ParameterMessage(parameter=upd, aggregation_weight=w))
            oracle.process_worker_data(k, OracleMessage(parameter={m: t.numpy() for m, t in host.items()},
                                                        aggregation_weight=w))
            del upd
        got = algo.aggregate_worker_data().parameter
        algo.clear_worker_data()
        want = oracle.aggregate_worker_data().parameter
        for name, v in want.items():
            assert bits_equal(got[name].cpu().numpy(), v), name
        assert algo.dyn_stats["waves"] == 0, algo.dyn_stats
        algo.exit()
        del got
        torch.cuda.synchronize()
    finally:
        parent.send("done")
        p.join(timeout=120)
    assert p.exitcode == 0
    torch.cuda.ipc_collect()


def test_device_round_then_host_rounds(hip_device):
    # a round of device-resident updates (wave), then rounds whose updates arrive in host memory:
    # those fold in ordinary launches and no wave is pre-opened for them (nothing would bind it);
    # a later device round opens one again. Every round bit-identical.
    algo = FedAVGAlgorithm(device=hip_device, dynamic_wave=True)
    _round(algo, hip_device, 6, 60)
    assert algo.dyn_stats["waves"] == 1

    def host_round(seed):
        g = torch.Generator().manual_seed(seed)
        oracle = OracleFedAvg()
        for k in range(5):
            p = {name: torch.randn(s, generator=g) for name, s in SHAPES.items()}
            w = 50 + 7 * k
            algo.process_worker_data(k, ParameterMessage(parameter=dict(p), aggregation_weight=w))
            oracle.process_worker_data(k, OracleMessage(parameter={m: t.numpy() for m, t in p.items()},
                                                        aggregation_weight=w))
        got = algo.aggregate_worker_data().parameter
        algo.clear_worker_data()
        for name, v in oracle.aggregate_worker_data().parameter.items():
            assert bits_equal(got[name].cpu().numpy(), v), name

    launches0 = algo._context().dyn_info()["launches"]
    host_round(61)
    host_round(62)
    assert algo.dyn_stats["waves"] == 1, algo.dyn_stats
    assert algo._context().dyn_info()["launches"] == launches0  # no pre-opened wave either
    _round(algo, hip_device, 6, 63)
    assert algo.dyn_stats["waves"] == 2, algo.dyn_stats
    algo.exit()
