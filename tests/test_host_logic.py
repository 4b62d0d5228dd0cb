"""Host-side logic on the CPU: layouts, tables, messages, registry, server sequencing."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from distributed_learning_simulation_lib_amd import (
    AlgorithmRepository,
    DeltaParameterMessage,
    FedAVGAlgorithm,
    ParameterMessage,
    get_message_size,
)
from distributed_learning_simulation_lib_amd.algorithm import AggregationAlgorithm
from distributed_learning_simulation_lib_amd.algorithm.aggregation_algorithm import split_empty, unify_dtype
from distributed_learning_simulation_lib_amd.fedavg import ClientTable, ModelLayout
from distributed_learning_simulation_lib_amd.server import AggregationServer, ModelCache
from oracle import fedavg_oracle as O
from tests.golden_io import bits_equal, load_golden
from tests.helpers import OracleAlgorithm

CASES = load_golden()


def test_layout_offsets_are_16_byte_aligned():
    lay = ModelLayout(names=("a", "b", "c", "d"), shapes=((3,), (5, 7), (), (0,)))
    assert lay.numels == [3, 35, 1, 0] and lay.total_numel == 39
    for elem in (2, 4, 8):
        offs, total = lay.padded_offsets(elem)
        assert all(o * elem % 16 == 0 for o in offs)
        assert total * elem % 16 == 0 and total >= lay.total_numel
    native, keep = split_empty(lay)
    assert keep == [0, 1, 2] and native.names == ("a", "b", "c")


def test_client_table_rows_and_cache():
    t = ClientTable(3)
    a, b = torch.zeros(4), torch.ones(2)
    t.add_client([a, None, b], [2.0, 9.0, 3.0])
    p, w = t.arrays()
    assert p[1] == 0 and w[1] == 0.0 and p[0] == a.data_ptr() and w.tolist() == [2.0, 0.0, 3.0]
    assert t.arrays()[0] is p  # cached
    t.add_client([a, b, b], [1, 1, 1])
    assert t.arrays()[0] is not p and t.num_clients == 2
    with pytest.raises(ValueError):
        t.add_client([a], [1.0])


def test_unify_dtype_widens_mixed_and_integer_inputs():
    ts, dt = unify_dtype([torch.zeros(2, dtype=torch.float16), torch.zeros(2, dtype=torch.float16)])
    assert dt == torch.float16
    ts, dt = unify_dtype([torch.zeros(2), torch.zeros(2, dtype=torch.float16)])
    assert dt == torch.float64 and all(t.dtype == torch.float64 for t in ts)
    ts, dt = unify_dtype([torch.arange(3)])
    assert dt == torch.float64 and ts[0].tolist() == [0.0, 1.0, 2.0]


def test_complete_and_restore_match_the_oracle():
    g = torch.Generator().manual_seed(3)
    old = {"a": torch.randn(5, generator=g, dtype=torch.float64), "b": torch.randn(3, generator=g, dtype=torch.float64)}
    msg = ParameterMessage(parameter={"b": torch.randn(3, generator=g)})
    msg.complete(old)
    assert list(msg.parameter) == ["b", "a"] and msg.parameter["a"] is old["a"]
    ref = {"b": msg.parameter["b"].numpy().copy()}
    O.complete(ref, {k: v.numpy() for k, v in old.items()})
    assert list(ref) == ["b", "a"]
    delta = {"a": torch.randn(5, generator=g, dtype=torch.float64), "b": torch.randn(3, generator=g, dtype=torch.float64)}
    d = DeltaParameterMessage(delta_parameter=delta, aggregation_weight=7, other_data={"x": 1})
    full = d.restore(old)
    want = O.restore({k: v.numpy() for k, v in delta.items()}, {k: v.numpy() for k, v in old.items()})
    for k in old:
        assert bits_equal(full.parameter[k].numpy(), want[k])
    assert full.aggregation_weight == 7 and full.other_data == {"x": 1}
    assert get_message_size(full) == 8 * 8


def test_scalar_helpers_match_the_oracle():
    case = CASES["ratio_path"]
    data = {a.worker_id: ParameterMessage(parameter={}, aggregation_weight=a.weight) for a in case.arrivals}
    odata = {a.worker_id: O.OracleMessage(parameter={}, aggregation_weight=a.weight) for a in case.arrivals}
    assert AggregationAlgorithm.get_total_weight(data) == O.get_total_weight(odata)
    assert AggregationAlgorithm.get_ratios(data) == O.get_ratios(odata)
    for m in data.values():
        m.other_data["training_loss"] = 0.25
    for m in odata.values():
        m.other_data["training_loss"] = 0.25
    r = AggregationAlgorithm.get_ratios(data)
    assert AggregationAlgorithm.weighted_avg_for_scalar(data, r, "training_loss") == O.weighted_avg_for_scalar(
        odata, O.get_ratios(odata), "training_loss"
    )
    bad = {0: ParameterMessage(parameter={}, aggregation_weight=-1)}
    with pytest.raises(AssertionError):
        AggregationAlgorithm.get_ratios(bad)


def test_registry_api():
    assert AlgorithmRepository.has_algorithm("fed_avg")
    assert AlgorithmRepository.config["fed_avg"]["algorithm_cls"] is FedAVGAlgorithm
    with pytest.raises(AssertionError):
        AlgorithmRepository.register_algorithm("fed_avg", client_cls=object, server_cls=object)

    class Ctx:
        def create_server_endpoint(self, **kw):
            return ("endpoint", kw)

    class Srv:
        def __init__(self, endpoint, **kw):
            self.endpoint, self.kw = endpoint, kw

    AlgorithmRepository.register_algorithm("test_only_alg", client_cls=object, server_cls=Srv, algorithm_cls=dict)
    try:
        s = AlgorithmRepository.create_server("test_only_alg", kwargs={"a": 1}, endpoint_kwargs={}, context=Ctx())
        assert s.kw["a"] == 1 and s.kw["algorithm"] == {} and s.endpoint[0] == "endpoint"
    finally:
        del AlgorithmRepository.config["test_only_alg"]


def test_hip_algorithm_fails_loudly_without_a_gpu():
    algo = FedAVGAlgorithm(device="cpu", wave_size=1)
    with pytest.raises((ValueError, RuntimeError, ImportError)):
        algo.process_worker_data(0, ParameterMessage(parameter={"a": torch.ones(3)}, aggregation_weight=1))
        algo.aggregate_worker_data()


def test_server_sequencing_with_the_oracle_algorithm():
    """aggregation_server.py:111-175: restore/complete, skip, count reporters, cache fp64."""
    srv = AggregationServer(algorithm=OracleAlgorithm(), worker_number=3, round_number=2)
    g = torch.Generator().manual_seed(1)
    p = [{"a": torch.randn(4, generator=g), "b": torch.randn(2, generator=g)} for _ in range(3)]
    srv._process_worker_data(0, ParameterMessage(parameter=dict(p[0]), aggregation_weight=1))
    srv._process_worker_data(1, None)
    assert not srv.results
    srv._process_worker_data(2, ParameterMessage(parameter=dict(p[2]), aggregation_weight=3))
    assert len(srv.results) == 1 and srv.round_index == 2
    r1 = srv.current_aggregated_model.parameter
    assert all(v.dtype == torch.float64 for v in r1.values())
    want = (p[0]["a"].double() * 1 + p[2]["a"].double() * 3) / 4
    assert torch.equal(r1["a"], want)
    # round 2: a delta and an incomplete full update (complete() fills "b" from the cache)
    delta = {"a": torch.full((4,), 0.5, dtype=torch.float64), "b": torch.zeros(2, dtype=torch.float64)}
    srv._process_worker_data(0, DeltaParameterMessage(delta_parameter=delta, aggregation_weight=2))
    srv._process_worker_data(1, ParameterMessage(parameter={"a": torch.ones(4)}, aggregation_weight=2))
    srv._process_worker_data(2, None)
    r2 = srv.results[-1].parameter
    assert torch.equal(r2["b"], r1["b"])
    assert torch.equal(r2["a"], ((r1["a"] + 0.5) * 2 + torch.ones(4, dtype=torch.float64) * 2) / 4)
    assert srv._stopped()


def test_model_cache_copies_to_host_fp64():
    mc = ModelCache()
    assert not mc.has_data
    mc.cache_parameter({"x": torch.ones(3, dtype=torch.float16)})
    assert mc.parameter["x"].dtype == torch.float64
    assert torch.equal(mc.get_parameter_diff({"x": torch.full((3,), 2.0, dtype=torch.float64)})["x"], torch.ones(3, dtype=torch.float64))
    assert np.all(mc.parameter["x"].numpy() == 1.0)


def test_model_cache_add_parameter_diff():
    # model_cache.py:39-43: every cached name += the diff (moved to the host), fp64 kept
    mc = ModelCache()
    mc.cache_parameter({"x": torch.tensor([1.0, -2.0, 0.5]), "y": torch.zeros(2)})
    diff = {"x": torch.tensor([0.25, 0.5, -0.5], dtype=torch.float32), "y": torch.tensor([1.0, 2.0], dtype=torch.float64)}
    mc.add_parameter_diff(diff)
    assert mc.parameter["x"].dtype == torch.float64 and mc.parameter["x"].tolist() == [1.25, -1.5, 0.0]
    assert mc.parameter["y"].tolist() == [1.0, 2.0]
    # get_parameter_diff undoes it
    back = mc.get_parameter_diff({"x": torch.tensor([1.25, -1.5, 0.0], dtype=torch.float64), "y": torch.zeros(2, dtype=torch.float64)})
    assert back["x"].tolist() == [0.0, 0.0, 0.0] and back["y"].tolist() == [-1.0, -2.0]


def test_client_table_rejects_operands_the_kernel_would_misread():
    """A client tensor is read as a flat buffer of the layout's size: non-contiguous views are
    refused when added, wrong sizes / element sizes / devices before any launch (validate)."""
    from distributed_learning_simulation_lib_amd.fedavg import ClientTable

    t = ClientTable(2)
    with pytest.raises(ValueError, match="contiguous"):
        t.add_client([torch.ones(4, 4).t(), torch.ones(3)], [1.0, 1.0])
    t.add_client([torch.ones(4, 4), None], [1.0, 1.0])  # an absent tensor is never checked
    t.add_client([torch.ones(16), torch.ones(3)], [2.0, 2.0])
    t.validate([16, 3], 4, -1, "ok")  # host tensors, fp32: matches
    with pytest.raises(ValueError, match="client 1, tensor 1: 3 elements"):
        t.validate([16, 5], 4, -1, "size")
    with pytest.raises(ValueError, match="of 4 bytes"):
        t.validate([16, 3], 2, -1, "dtype")
    with pytest.raises(ValueError, match="on device -1"):
        t.validate([16, 3], 4, 0, "device")


def test_early_wave_policy():
    """wave_min: a partial wave of >= wave_min staged clients is folded at the next arrival only
    while the GPU has finished the waves flushed so far; a full wave always is; 0 disables it."""
    from distributed_learning_simulation_lib_amd import FedAVGAlgorithm

    class Ev:
        def __init__(self, done: bool) -> None:
            self.done = done

        def query(self) -> bool:
            return self.done

    a = FedAVGAlgorithm(device="cpu", wave_size=8, wave_min=3)
    assert a._wave_due(8) and not a._wave_due(2)
    assert a._wave_due(3)  # nothing flushed yet: the GPU is idle
    a._FedAVGAlgorithm__wave_event = Ev(False)
    assert not a._wave_due(5) and a._wave_due(8)
    a._FedAVGAlgorithm__wave_event = Ev(True)
    assert a._wave_due(3) and not a._wave_due(2)
    b = FedAVGAlgorithm(device="cpu", wave_size=8, wave_min=0)
    assert not b._wave_due(7) and b._wave_due(8)


def test_quick_arrival_leaves_the_general_flows_state(monkeypatch):
    """FedAVGAlgorithm._arrive_quick (the one-pass common arrival) changes exactly what the
    general process_worker_data flow changes: the recorded messages, the rows handed to the
    wave's table, the running totals (uniform while updates are complete, per name after an
    incomplete one) and the released payloads — over full, partial and late-name updates, a
    None message and a full wave."""
    import torch

    import distributed_learning_simulation_lib_amd.algorithm.fed_avg_algorithm as fa
    from distributed_learning_simulation_lib_amd import FedAVGAlgorithm, ParameterMessage

    class Rows:
        def __init__(self, log):
            self.n, self.log = 0, log

        @property
        def num_clients(self):
            return self.n

        def append(self, params, index, shapes, w, want):
            if any(k not in index for k in params):
                return -1  # a name the layout does not know: the general flow grows the layout
            self.n += 1
            self.log.append((tuple(params), w))
            return 0 | (16 if len(params) == len(index) else 0)

    def run(quick: bool):
        log, flushed = [], []

        class Table:
            def __init__(self, T, dev):
                self.rows = Rows(log)

            @property
            def num_clients(self):
                return self.rows.num_clients

        monkeypatch.setattr(fa, "NativeClientTable", Table)
        a = FedAVGAlgorithm(device="cpu", wave_size=3)
        if not quick:
            monkeypatch.setattr(a, "_arrive_quick", lambda *args: False)
        names = ("a", "b", "c")
        lay = {}

        def fast_maps():
            layout = a._FedAVGAlgorithm__layout
            if lay.get("l") is not layout:
                lay["l"] = layout
                lay["m"] = (layout, {n: i for i, n in enumerate(layout.names)}, [(2,)] * len(layout.names), 0)
            return lay["m"]

        monkeypatch.setattr(a, "_fast_maps", fast_maps)
        monkeypatch.setattr(a, "_flush", lambda: (flushed.append(a._FedAVGAlgorithm__table.num_clients),
                                                  setattr(a, "_FedAVGAlgorithm__table", None)))
        msgs = []
        seq = [(names, 2.0), (names, 3), (("a", "b"), 1.5), None, (names, 4.0), (names, 0.5), (names, 7)]
        for k, item in enumerate(seq):
            if item is None:
                a.process_worker_data(k, None)
                continue
            keys, w = item
            m = ParameterMessage(parameter={n: torch.ones(2) for n in keys}, aggregation_weight=w)
            msgs.append(m)
            a.process_worker_data(k, m)
        a._materialize_totals()
        state = (log, flushed, dict(a._FedAVGAlgorithm__host_totals), sorted(a._all_worker_data),
                 [m.parameter for m in msgs], a._FedAVGAlgorithm__has_data)
        return state

    assert run(True) == run(False)
