"""HIP PersonalizedFedAVG vs the reference (golden fixtures) and vs the oracle, on the MI355X.

Tolerance: none — every receiver's model and the centralized model are BIT-IDENTICAL to the
reference's float64 results (asserted with `bits_equal`); float32 outputs equal the reference
result cast to float32.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import (
    MultipleWorkerMessage,
    NaNAggregationError,
    ParameterMessage,
    PersonalizedFedAVGAlgorithm,
)
from oracle.fedavg_oracle import OracleMessage
from oracle.personalized_oracle import OraclePersonalizedFedAvg
from tests.golden_io import bits_equal, load_personalized

pytestmark = pytest.mark.gpu
CASES = load_personalized()


def run_hip(case, device, from_host=False, wire=None):
    algo = PersonalizedFedAVGAlgorithm(device=device)
    algo.set_worker_weights({j: dict(v) for j, v in case.worker_weights.items()})
    msg_cls = ParameterMessage if wire is None else wire.ParameterMessage
    for a in case.arrivals:
        msg = None
        if a.arrays is not None:
            msg = msg_cls(parameter=case.torch_params(a, "cpu" if from_host else device),
                          other_data=dict(a.other_data))
        algo.process_worker_data(a.worker_id, msg)
    return algo.aggregate_worker_data()


@pytest.mark.parametrize("from_host", [False, True])
@pytest.mark.parametrize("name", sorted(CASES))
def test_personalized_matches_reference(hip_device, name, from_host):
    case = CASES[name]
    if case.error is not None:
        exc = {"AssertionError": AssertionError, "RuntimeError": RuntimeError}[case.error]
        with pytest.raises(exc):
            run_hip(case, hip_device, from_host)
        return
    res = run_hip(case, hip_device, from_host)
    assert isinstance(res, MultipleWorkerMessage)
    assert list(res.worker_data) == [r["worker_id"] for r in case.meta["receivers"]]
    for r in case.meta["receivers"]:
        got = res.worker_data[r["worker_id"]]
        assert list(got.parameter) == r["keys"]
        for k, want in case.expected[r["worker_id"]].items():
            assert bits_equal(got.parameter[k].cpu().numpy(), want), f"{name}/{r['worker_id']}/{k}"
        assert got.other_data == r["other_data"]
        assert (got.in_round, got.end_training) == (r["in_round"], r["end_training"])
    central = res.other_data["centralized_parameter"]
    assert list(central) == case.meta["central_keys"]
    for k, want in case.central.items():
        assert bits_equal(central[k].cpu().numpy(), want), f"{name}/central/{k}"


def _random_round(n, receivers, shapes, seed, dtype=torch.float32, weight_kind="float", missing=None):
    g = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed)
    clients = []
    for k in range(n):
        p = {name: torch.randn(s, generator=g).to(dtype) for name, s in shapes.items()}
        if missing and k in missing:
            del p[missing[k]]
        clients.append(p)
    ww = {}
    for j in receivers:
        if weight_kind == "int":
            ww[j] = {i: int(rng.integers(1, 5000)) for i in range(n) if i != j}
        else:
            ww[j] = {i: float(rng.uniform(0.01, 3.0)) for i in range(n) if i != j}
    return clients, ww


def _oracle(clients, ww, dtype_name=None):
    o = OraclePersonalizedFedAvg()
    o.set_worker_weights({j: dict(v) for j, v in ww.items()})
    for k, p in enumerate(clients):
        arrs = {}
        for name, t in p.items():
            arrs[name] = t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()
        o.process_worker_data(k, OracleMessage(parameter=arrs, dtype=dtype_name))
    return o.aggregate_worker_data()


def _hip(clients, ww, device, result_dtype=torch.float64, unaligned=False):
    algo = PersonalizedFedAVGAlgorithm(device=device, result_dtype=result_dtype)
    algo.set_worker_weights({j: dict(v) for j, v in ww.items()})
    for k, p in enumerate(clients):
        dp = {}
        for name, t in p.items():
            if unaligned:  # a view one element into a bigger buffer: the guarded-load path
                buf = torch.empty(t.numel() + 1, dtype=t.dtype, device=device)
                buf[1:].copy_(t.reshape(-1))
                dp[name] = buf[1:].view(t.shape)
            else:
                dp[name] = t.to(device)
        algo.process_worker_data(k, ParameterMessage(parameter=dp))
    return algo.aggregate_worker_data()


def _assert_same(res, want, result_dtype=torch.float64):
    for j, r in want.worker_data.items():
        for k, v in r.parameter.items():
            got = res.worker_data[j].parameter[k].cpu()
            if result_dtype == torch.float64:
                assert bits_equal(got.numpy(), v), f"receiver {j} / {k}"
            else:
                assert torch.equal(got, torch.from_numpy(np.asarray(v)).to(torch.float32)), f"receiver {j} / {k}"
    for k, v in want.centralized_parameter.items():
        assert bits_equal(res.other_data["centralized_parameter"][k].cpu().numpy(), v), f"central / {k}"


SHAPES = {"conv": (32, 16, 3, 3), "bn": (32,), "fc": (10, 300), "odd": (1001,), "s": ()}


def test_weights_changed_in_place_between_rounds_are_used(hip_device):
    """The reference reads ``worker_weights[j][i]`` live on every arrival (:34): a caller that edits
    a receiver's dict in place between rounds (no new set_worker_weights) gets the new weights."""
    n = 6
    clients, ww = _random_round(n, range(n), SHAPES, 17)
    live = {j: dict(v) for j, v in ww.items()}
    algo = PersonalizedFedAVGAlgorithm(device=hip_device)
    algo.set_worker_weights(live)
    for rnd in range(3):
        for k, p in enumerate(clients):
            algo.process_worker_data(k, ParameterMessage(parameter={m: t.to(hip_device) for m, t in p.items()}))
        res = algo.aggregate_worker_data()
        algo.clear_worker_data()
        _assert_same(res, _oracle(clients, live))
        live[2][4] = 0.25 * (rnd + 2)  # in place, seen by the next round
        live[3].pop(1, None)
    algo.exit()


@pytest.mark.parametrize("weight_kind", ["float", "int"])
def test_random_round_matches_oracle(hip_device, weight_kind):
    clients, ww = _random_round(24, range(24), SHAPES, 101, weight_kind=weight_kind)
    _assert_same(_hip(clients, ww, hip_device), _oracle(clients, ww))


@pytest.mark.parametrize("ring", ["1", "0"])
@pytest.mark.parametrize("receivers", [40, 72, 100, 120])
def test_int_weights_ring_with_uneven_wave_counts(hip_device, receivers, ring, monkeypatch):
    # integer weights with FEDAVG_PERS_RING=1 take the LDS-DMA client ring on whole aligned fp32
    # chunks; 3 / 5 / 7 / 8 waves of 16 receivers split a ring stage of 4 clients unevenly (or not
    # at all) between waves; "0" is the default register pipeline
    monkeypatch.setenv("FEDAVG_PERS_RING", ring)  # read when the native context is created
    clients, ww = _random_round(receivers, range(receivers), {"a": (1024,), "b": (300,)}, 110 + receivers,
                                weight_kind="int")
    _assert_same(_hip(clients, ww, hip_device), _oracle(clients, ww))


def test_two_receiver_groups_carry_the_central_chain(hip_device):
    # 130 receivers > 120 per launch: the second launch continues the centralized chain
    clients, ww = _random_round(130, range(130), {"a": (257,), "b": (3, 5)}, 102)
    _assert_same(_hip(clients, ww, hip_device), _oracle(clients, ww))


def test_unaligned_views_and_float32_results(hip_device):
    clients, ww = _random_round(9, range(9), SHAPES, 103)
    want = _oracle(clients, ww)
    _assert_same(_hip(clients, ww, hip_device, unaligned=True), want)
    _assert_same(_hip(clients, ww, hip_device, result_dtype=torch.float32), want, torch.float32)


def test_missing_tensor_in_a_later_update(hip_device):
    clients, ww = _random_round(7, range(7), SHAPES, 104, missing={3: "fc", 5: "bn"})
    _assert_same(_hip(clients, ww, hip_device), _oracle(clients, ww))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float64])
def test_other_input_dtypes(hip_device, dtype):
    clients, ww = _random_round(11, [0, 3, 5, 7, 10], SHAPES, 105, dtype=dtype)
    name = {torch.bfloat16: "bfloat16"}.get(dtype)
    _assert_same(_hip(clients, ww, hip_device), _oracle(clients, ww, name))


def test_nan_input_names_the_worker(hip_device):
    clients, ww = _random_round(5, range(5), {"a": (100,)}, 106)
    clients[3]["a"][7] = float("nan")
    with pytest.raises(NaNAggregationError) as ei:
        _hip(clients, ww, hip_device)
    assert ei.value.stage == "input" and ei.value.bad_clients == [3]


@pytest.mark.parametrize("name", sorted(n for n in CASES if CASES[n].error is None)[:6])
def test_personalized_with_foreign_messages(hip_device, name):
    """Updates of another wire module (the reference server passes simulation_lib.message
    objects): recognised by their fields; the result is that module's MultipleWorkerMessage of
    its ParameterMessages (aggregation_server.py:84-86 dispatches on them), bits unchanged."""
    import tests.foreign_messages as foreign

    case = CASES[name]
    res = run_hip(case, hip_device, wire=foreign)
    assert type(res) is foreign.MultipleWorkerMessage
    for r in case.meta["receivers"]:
        got = res.worker_data[r["worker_id"]]
        assert type(got) is foreign.ParameterMessage
        for k, want in case.expected[r["worker_id"]].items():
            assert bits_equal(got.parameter[k].cpu().numpy(), want), f"{name}/{r['worker_id']}/{k}"



def test_result_buffers_reused_only_when_unobserved(hip_device):
    """One algorithm over three rounds: a receiver's result buffer of an earlier round is written
    again only when the caller kept nothing of it (PersonalizedFedAVGAlgorithm._result_rows):
    kept results keep their values, released buffers are reused, every round matches the oracle."""
    n = 8
    _, ww = _random_round(n, range(n), SHAPES, 7)
    algo = PersonalizedFedAVGAlgorithm(device=hip_device)
    algo.set_worker_weights({j: dict(v) for j, v in ww.items()})

    def one_round(seed):
        clients, _ = _random_round(n, range(n), SHAPES, seed)
        for k, p in enumerate(clients):
            algo.process_worker_data(k, ParameterMessage(parameter={m: t.to(hip_device) for m, t in p.items()}))
        res = algo.aggregate_worker_data()
        algo.clear_worker_data()
        want = _oracle(clients, ww)
        _assert_same(res, want)
        return res, want

    kept, kept_want = one_round(1)
    ptr = kept.worker_data[3].parameter["fc"].data_ptr()
    res2, want2 = one_round(2)  # everything of round 1 is still held: fresh buffers
    assert res2.worker_data[3].parameter["fc"].data_ptr() != ptr
    _assert_same(kept, kept_want)
    ptr2 = res2.worker_data[3].parameter["fc"].data_ptr()
    conv5 = res2.worker_data[5].parameter["conv"]  # one tensor of one receiver kept
    del res2
    res3, _ = one_round(3)
    assert res3.worker_data[3].parameter["fc"].data_ptr() == ptr2  # released: written again
    assert res3.worker_data[5].parameter["conv"].data_ptr() != conv5.data_ptr()
    assert bits_equal(conv5.cpu().numpy(), want2.worker_data[5].parameter["conv"])
    _assert_same(kept, kept_want)
    # receiver 3's model sent to its worker process (PipeServerEndpoint.broadcast of a
    # MultipleWorkerMessage through torch.multiprocessing, aggregation_server.py:202): never written
    # again once the server let go of it
    import gc
    from multiprocessing.reduction import ForkingPickler

    import torch.multiprocessing as _torch_mp  # noqa: F401  (registers the tensor reducers)

    sent = res3.worker_data[3].parameter["fc"].data_ptr()
    sent_sum = sum(float(t.double().sum().item()) for t in res3.worker_data[3].parameter.values())
    payload = ForkingPickler.dumps(res3.worker_data[3].parameter)
    del res3
    gc.collect()
    res4, _ = one_round(4)
    assert res4.worker_data[3].parameter["fc"].data_ptr() != sent
    # the consumer rebuilds and releases it, so the IPC limbo drains before this process ends
    from tests.ipc_consumer import hand_over

    assert abs(hand_over(bytes(payload)) - sent_sum) <= 1e-9 * (1 + abs(sent_sum))
    del payload
    torch.cuda.ipc_collect()
    algo.exit()
