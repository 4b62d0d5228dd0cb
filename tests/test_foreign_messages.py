"""The plugin boundary with messages of another wire module (CPU; no kernel calls).

The reference's AggregationServer passes ``simulation_lib.message`` objects to the algorithm
(aggregation_server.py:117-130) and dispatches on the returned class (:83-87, :148). These tests
drive the staging logic with such objects — the test-only look-alike module everywhere, and the
reference's own ``message.py`` (loaded through the golden generator's shim) where /root/reference
exists — with the GPU fold replaced by a recorder, so they run without a GPU.
"""

from __future__ import annotations

import importlib.util
from pathlib import Path

import pytest
import torch

import tests.foreign_messages as F
from distributed_learning_simulation_lib_amd import FedAVGAlgorithm
from distributed_learning_simulation_lib_amd import message as M

REF = Path("/root/reference")


class RecordingFedAvg(FedAVGAlgorithm):
    """FedAVGAlgorithm with the GPU wave replaced by a recorder of what would be staged."""

    def __init__(self, **kw) -> None:
        super().__init__(device="cpu", **kw)
        self.staged: list[tuple[dict, bool]] = []

    def _stage_client(self, delta: bool = False, worker_id=None) -> None:
        row = self._FedAVGAlgorithm__row  # the staged (tensor, weight) row of this arrival
        self._FedAVGAlgorithm__row = {}
        self.staged.append((dict(row), delta))

    def _aggregate_parameter(self, chosen_worker_ids=None):
        return {"x": torch.zeros(1, dtype=torch.float64)}


def _reference_message_module():
    if not REF.exists():
        pytest.skip("the reference is only mounted in the build container")
    spec = importlib.util.spec_from_file_location("_gen_golden", Path(__file__).parent / "golden" / "gen_golden.py")
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    message, _agg, _fed = gen._load_reference()
    return message


@pytest.fixture(params=["look_alike", "reference"])
def wire(request):
    return F if request.param == "look_alike" else _reference_message_module()


def test_structural_recognition(wire):
    p = wire.ParameterMessage(parameter={"a": torch.ones(2)}, aggregation_weight=3)
    d = wire.DeltaParameterMessage(delta_parameter={"a": torch.ones(2)}, aggregation_weight=3)
    assert M.is_parameter_message(p) and not M.is_delta_message(p)
    assert M.is_delta_message(d) and not M.is_parameter_message(d)
    assert M.is_parameter_message_base(p) and M.is_parameter_message_base(d)
    assert not M.is_parameter_message(wire.Message()) and not M.is_parameter_message_base(wire.Message())
    assert not M.is_parameter_message({"parameter": 1}) and not M.is_message(None)
    assert M.wire_class(p, "ParameterMessage") is wire.ParameterMessage
    assert M.wire_class(d, "ParameterMessage") is wire.ParameterMessage  # via the message's module
    assert M.wire_class(p, "MultipleWorkerMessage") is wire.MultipleWorkerMessage
    assert M.wire_class(None, "ParameterMessage") is M.ParameterMessage


def test_foreign_updates_are_staged_and_answered_in_their_class(wire):
    algo = RecordingFedAvg()
    for wid, w in enumerate([3, 5]):
        msg = wire.ParameterMessage(parameter={"x": torch.full((4,), float(wid))}, aggregation_weight=w,
                                    other_data={"epoch": 2}, in_round=True)
        assert algo.process_worker_data(wid, msg)
        assert msg.parameter == {}  # payload released (fed_avg_algorithm.py:63-64)
    assert [list(r) for r, _ in algo.staged] == [["x"], ["x"]]
    assert [r["x"][1] for r, _ in algo.staged] == [3, 5]
    res = algo.aggregate_worker_data()
    # the reference server matches `case ParameterMessageBase()` on its own classes
    assert type(res) is wire.ParameterMessage and isinstance(res, wire.ParameterMessageBase)
    assert res.in_round and res.other_data == {"epoch": 2} and res.aggregation_weight is None


def test_fusable_delta_is_staged_as_delta(wire):
    algo = RecordingFedAvg()
    algo.set_old_parameter({"x": torch.zeros(4, dtype=torch.float64)})
    d = wire.DeltaParameterMessage(delta_parameter={"x": torch.ones(4, dtype=torch.float64)}, aggregation_weight=2)
    algo.process_worker_data(0, d)
    assert len(algo.staged) == 1 and algo.staged[0][1] is True


def test_unfusable_delta_is_restored_on_the_host(wire):
    """A delta with the consistency-check fields (message.py:42-59) is restored like the
    reference server does (aggregation_server.py:123-125), then staged as a full update."""
    old = {"x": torch.arange(4, dtype=torch.float64)}
    algo = RecordingFedAvg()
    algo.set_old_parameter(old)
    delta = torch.full((4,), 0.5, dtype=torch.float64)
    d = wire.DeltaParameterMessage(delta_parameter={"x": delta}, aggregation_weight=2,
                                   new_parameter={"x": old["x"] + delta})
    algo.process_worker_data(0, d)
    assert len(algo.staged) == 1 and algo.staged[0][1] is False
    t, w = algo.staged[0][0]["x"]
    assert w == 2 and torch.equal(t, old["x"] + delta)
    assert M.is_parameter_message(algo._all_worker_data[0])


def test_delta_on_the_ratio_path_is_restored(wire):
    """accumulate=False keeps whole updates for weighted_avg: a delta must be restored first."""
    old = {"x": torch.arange(4, dtype=torch.float64)}
    algo = RecordingFedAvg()
    algo.accumulate = False
    algo.set_old_parameter(old)
    d = wire.DeltaParameterMessage(delta_parameter={"x": torch.ones(4, dtype=torch.float64)}, aggregation_weight=2)
    algo.process_worker_data(0, d)
    kept = algo._all_worker_data[0]
    assert M.is_parameter_message(kept) and torch.equal(kept.parameter["x"], old["x"] + 1)
    assert algo.staged == []  # the ratio path reads _all_worker_data at aggregate time


def test_server_drives_foreign_messages():
    """This package's server takes look-alike messages too (delta restore / complete / cache)."""
    from distributed_learning_simulation_lib_amd.server import AggregationServer
    from tests.helpers import OracleAlgorithm

    srv = AggregationServer(algorithm=OracleAlgorithm(), worker_number=2, round_number=2)
    srv._process_worker_data(0, F.ParameterMessage(parameter={"a": torch.ones(3)}, aggregation_weight=1))
    srv._process_worker_data(1, F.ParameterMessage(parameter={"a": torch.zeros(3)}, aggregation_weight=1))
    r1 = srv.current_aggregated_model.parameter["a"]
    assert torch.equal(r1, torch.full((3,), 0.5, dtype=torch.float64))
    srv._process_worker_data(0, F.DeltaParameterMessage(delta_parameter={"a": torch.ones(3, dtype=torch.float64)},
                                                        aggregation_weight=1))
    srv._process_worker_data(1, F.ParameterMessage(parameter={}, aggregation_weight=1))  # complete()d from cache
    assert torch.equal(srv.results[-1].parameter["a"], torch.full((3,), 1.0, dtype=torch.float64))
