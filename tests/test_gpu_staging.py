"""The native staging of plugin updates (csrc/staging_ext.cpp) against the oracle, on the MI355X.

Device-resident updates with the default hooks go through one native call per update; anything
it does not take (a second dtype in the update, a host tensor, a changed shape, an unknown name)
falls back to the Python staging with nothing changed. Both must give the reference's bits.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage, _staging
from oracle.fedavg_oracle import OracleFedAvg, OracleMessage
from tests.golden_io import bits_equal

pytestmark = pytest.mark.gpu

SHAPES = {"conv": (8, 3, 3, 3), "empty": (0,), "fc": (10, 33), "bias": (10,), "scalar": ()}


def test_extension_is_built_and_loaded():
    assert _staging.module() is not None, "run __graft_entry__.build(): _lib/staging/fedavg_staging.so is missing"


@pytest.mark.parametrize("wave", [1, 3, 64])
def test_native_and_fallback_arrivals_bit_identical(hip_device, wave):
    g = torch.Generator().manual_seed(5)
    rng = np.random.default_rng(5)
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave)
    oracle = OracleFedAvg()
    for k in range(9):
        p = {n: torch.randn(s, generator=g) for n, s in SHAPES.items()}
        dev = {n: t.to(hip_device) for n, t in p.items()}
        if k == 3:  # a second dtype in one update: the Python path unifies it
            dev["fc"] = dev["fc"].double()
            p["fc"] = p["fc"].double()
        if k == 5:  # a host tensor: the pinned ingest path
            dev["bias"] = p["bias"]
        if k == 6:  # a non-contiguous view: the general path makes it contiguous
            dev["fc"] = dev["fc"].t().contiguous().t()
        w = int(rng.integers(100, 5000)) if k % 2 else float(rng.uniform(0.5, 9.0))
        algo.process_worker_data(k, ParameterMessage(parameter=dev, aggregation_weight=w))
        oracle.process_worker_data(k, OracleMessage(parameter={n: t.numpy() for n, t in p.items()},
                                                    aggregation_weight=w))
    got = algo.aggregate_worker_data().parameter
    want = oracle.aggregate_worker_data().parameter
    assert list(got) == list(want)
    for n, v in want.items():
        assert bits_equal(got[n].cpu().numpy(), v), n


def test_changed_shape_still_raises(hip_device):
    algo = FedAVGAlgorithm(device=hip_device)
    algo.process_worker_data(0, ParameterMessage(parameter={"a": torch.ones(4, device=hip_device)},
                                                 aggregation_weight=1.0))
    with pytest.raises(ValueError, match="shape of a changed"):
        algo.process_worker_data(1, ParameterMessage(parameter={"a": torch.ones(5, device=hip_device)},
                                                     aggregation_weight=1.0))


def _delta_round(hip_device):
    from distributed_learning_simulation_lib_amd.message import DeltaParameterMessage

    g = torch.Generator().manual_seed(9)
    old = {n: torch.randn(s, generator=g, dtype=torch.float64) for n, s in SHAPES.items()}
    algo = FedAVGAlgorithm(device=hip_device, wave_size=3)
    algo.set_old_parameter(old)
    for k in range(7):
        d = {n: torch.randn(s, generator=g).to(hip_device) for n, s in SHAPES.items()}
        algo.process_worker_data(k, DeltaParameterMessage(delta_parameter=d, aggregation_weight=100 + 17 * k))
    return {n: t.cpu() for n, t in algo.aggregate_worker_data().parameter.items()}


def test_native_delta_staging_matches_python_staging(hip_device, monkeypatch):
    # fused restore (x = old + delta in the fold) through the native staging and through the Python
    # staging (pinned to the reference by the golden delta cases): the same bits
    native = _delta_round(hip_device)
    monkeypatch.setattr(_staging, "module", lambda: None)
    python = _delta_round(hip_device)
    assert list(native) == list(python)
    for n in native:
        assert bits_equal(native[n].numpy(), python[n].numpy()), n


@pytest.mark.parametrize("wave", [1, 64])
@pytest.mark.parametrize("native", [True, False])
def test_delta_first_round_then_reordered_full_update(hip_device, monkeypatch, wave, native):
    # a round that opens with fused deltas keeps its layout when a later full update arrives with
    # its keys in another order (ParameterMessage.complete appends the missing keys at the end,
    # message.py:28-31): the deltas already staged or folded stay where they are
    from distributed_learning_simulation_lib_amd.message import DeltaParameterMessage
    from oracle.fedavg_oracle import complete, restore

    if not native:
        monkeypatch.setattr(_staging, "module", lambda: None)
    g = torch.Generator().manual_seed(23)
    old = {n: torch.randn(s, generator=g, dtype=torch.float64) for n, s in SHAPES.items()}
    old_np = {n: t.numpy() for n, t in old.items()}
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave)
    algo.set_old_parameter(old)
    oracle = OracleFedAvg()
    for rnd in range(2):  # the second round opens with a delta again, after a reset
        for k in range(5):
            if k in (0, 1, 3):
                d = {n: torch.randn(s, generator=g) for n, s in SHAPES.items()}
                algo.process_worker_data(k, DeltaParameterMessage(
                    delta_parameter={n: t.to(hip_device) for n, t in d.items()}, aggregation_weight=50 + k))
                full = restore({n: t.numpy() for n, t in d.items()}, old_np)
            else:
                part = {n: torch.randn(SHAPES[n], generator=g) for n in ("fc", "scalar", "conv")}
                msg = ParameterMessage(parameter={n: t.to(hip_device) for n, t in part.items()},
                                       aggregation_weight=70 + k)
                msg.complete(old)  # appends "empty" and "bias" after the sent keys
                assert list(msg.parameter)[:3] == ["fc", "scalar", "conv"]
                algo.process_worker_data(k, msg)
                full = {n: t.numpy() for n, t in part.items()}
                complete(full, old_np)
            oracle.process_worker_data(k, OracleMessage(parameter=full, aggregation_weight=(50 if k in (0, 1, 3)
                                                                                              else 70) + k))
        got = algo.aggregate_worker_data().parameter
        want = oracle.aggregate_worker_data().parameter
        assert list(got) == list(want) == list(SHAPES), rnd
        for n, v in want.items():
            assert bits_equal(got[n].cpu().numpy(), v), (rnd, n)
        algo.clear_worker_data()
        oracle = OracleFedAvg()


@pytest.mark.parametrize("wave", [1, 3, 64])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
def test_native_host_staging_bit_identical(hip_device, wave, dtype):
    # whole updates in host memory (what the reference server receives): checked natively,
    # packed into the pinned ring and moved by one DMA per client, folded from the bucket
    g = torch.Generator().manual_seed(11)
    rng = np.random.default_rng(11)
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave)
    oracle = OracleFedAvg()
    for k in range(8):
        p = {n: torch.randn(s, generator=g).to(dtype) for n, s in SHAPES.items()}
        w = int(rng.integers(100, 5000))
        algo.process_worker_data(k, ParameterMessage(parameter=dict(p), aggregation_weight=w))
        oracle.process_worker_data(k, OracleMessage(
            parameter={n: (t.view(torch.int16).numpy().view(np.uint16) if dtype == torch.bfloat16 else t.numpy())
                       for n, t in p.items()},
            aggregation_weight=w, dtype="bfloat16" if dtype == torch.bfloat16 else None))
    got = algo.aggregate_worker_data().parameter
    want = oracle.aggregate_worker_data().parameter
    assert list(got) == list(want)
    for n, v in want.items():
        assert bits_equal(got[n].cpu().numpy(), v), n


@pytest.mark.parametrize("wave", [2, 64])
def test_uniform_totals_then_partial_and_late_updates(hip_device, wave):
    # complete updates keep one running total for every name; a partial update (a missing key)
    # and a late key (a name first seen mid-round) write it out per name first. Float weights make
    # every total order-sensitive; two rounds on one object check that the state is reset.
    algo = FedAVGAlgorithm(device=hip_device, wave_size=wave)
    g = torch.Generator().manual_seed(17)
    rng = np.random.default_rng(17)
    for rnd in range(2):
        oracle = OracleFedAvg()
        for k in range(8):
            shapes = dict(SHAPES)
            if k == 4:
                del shapes["fc"]
            if k == 6 and rnd == 0:
                shapes["late"] = (7,)
            p = {n: torch.randn(s, generator=g) for n, s in shapes.items()}
            w = float(rng.uniform(0.1, 3.0)) if k % 3 else int(rng.integers(1, 9))
            algo.process_worker_data(k, ParameterMessage(parameter={n: t.to(hip_device) for n, t in p.items()},
                                                         aggregation_weight=w))
            oracle.process_worker_data(k, OracleMessage(parameter={n: t.numpy() for n, t in p.items()},
                                                        aggregation_weight=w))
        got = algo.aggregate_worker_data().parameter
        want = oracle.aggregate_worker_data().parameter
        assert list(got) == list(want), rnd
        for n, v in want.items():
            assert bits_equal(got[n].cpu().numpy(), v), (rnd, n)
        algo.clear_worker_data()


def test_common_arrivals_take_the_native_table(hip_device):
    algo = FedAVGAlgorithm(device=hip_device, wave_size=64)
    for k in range(3):
        p = {n: torch.ones(s, device=hip_device) for n, s in SHAPES.items()}
        algo.process_worker_data(k, ParameterMessage(parameter=p, aggregation_weight=k + 1))
    table = algo._FedAVGAlgorithm__table
    assert isinstance(table, _staging.NativeClientTable) and table.num_clients == 3
    # one running total for every name while every update is complete
    assert algo._FedAVGAlgorithm__uniform_count == 3 and algo._FedAVGAlgorithm__host_totals == {}
    out = algo.aggregate_worker_data().parameter
    assert float(out["conv"].flatten()[0]) == 1.0


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_result_buffer_reuse_never_changes_a_kept_result(hip_device, devices):
    """Rounds write into the previous round's result buffer only when the caller let go of every
    result tensor (FedAVGAlgorithm._result_buffer): a kept result keeps its values, a released one
    is reused, and every round matches the oracle bit for bit."""
    g = torch.Generator().manual_seed(11)
    shapes = {"conv": (8, 3, 3, 3), "fc": (10, 33), "bias": (10,)}
    kw = {"devices": [hip_device.index or 0] * 2} if devices else {"device": hip_device}
    algo = FedAVGAlgorithm(wave_size=2, **kw)

    def one_round(seed):
        oracle = OracleFedAvg()
        for k in range(5):
            p = {n: torch.randn(s, generator=g) for n, s in shapes.items()}
            w = float(seed + k + 1)
            algo.process_worker_data(k, ParameterMessage(parameter={n: t.to(hip_device) for n, t in p.items()},
                                                         aggregation_weight=w))
            oracle.process_worker_data(k, OracleMessage(parameter={n: t.numpy() for n, t in p.items()},
                                                        aggregation_weight=w))
        got = algo.aggregate_worker_data().parameter
        algo.clear_worker_data()
        want = oracle.aggregate_worker_data().parameter
        for n, v in want.items():
            assert bits_equal(got[n].cpu().numpy(), v), n
        return got, want

    kept, kept_want = one_round(0)
    kept_ptr = kept["fc"].data_ptr()
    got, _ = one_round(10)  # the kept result's buffer must not be written
    assert got["fc"].data_ptr() != kept_ptr
    for n, v in kept_want.items():
        assert bits_equal(kept[n].cpu().numpy(), v), n
    ptr = got["fc"].data_ptr()
    del got
    again, _ = one_round(20)  # released: its buffer is written again
    assert again["fc"].data_ptr() == ptr
    for n, v in kept_want.items():
        assert bits_equal(kept[n].cpu().numpy(), v), n
    # a result sent to another process (what PipeServerEndpoint.broadcast of the result does with
    # torch.multiprocessing: CUDA IPC, the counts unchanged) is never written again, even after the
    # server dropped every reference to it
    import gc
    from multiprocessing.reduction import ForkingPickler

    import torch.multiprocessing as _torch_mp  # noqa: F401  (registers the tensor reducers)

    sent_ptr = again["fc"].data_ptr()
    sent_sum = float(again["fc"].double().sum().item())
    payload = ForkingPickler.dumps(again["fc"])
    del again
    gc.collect()
    fresh, _ = one_round(30)
    assert fresh["fc"].data_ptr() != sent_ptr
    # the consumer rebuilds and releases it (reads the round-20 result), so the IPC limbo drains
    from tests.ipc_consumer import hand_over

    assert abs(hand_over(bytes(payload)) - sent_sum) <= 1e-9 * (1 + abs(sent_sum))
    del payload
    torch.cuda.ipc_collect()
    algo.exit()
