"""Wire / data model of client updates (the input and output format of the hot path).

Same classes, fields and semantics as the reference's ``simulation_lib/message.py``:
``Message`` (:11-16), ``ParameterMessageBase`` (:19-21), ``ParameterMessage`` (:24-31) with
``complete`` (:28-31), ``DeltaParameterMessage`` (:34-61) with ``restore`` (:40-61),
``FeatureMessage`` (:64-66), ``MultipleWorkerMessage`` (:69-71) and ``get_message_size``
(:74-84). ``ModelParameter`` is a ``dict[str, torch.Tensor]`` (the reference imports that alias
from ``cyy_torch_toolbox``).
"""

from __future__ import annotations

import copy
from collections.abc import Mapping
from dataclasses import dataclass, field, fields
from typing import Any

import torch

ModelParameter = dict[str, torch.Tensor]


@dataclass(kw_only=True, slots=True)
class Message:
    other_data: dict[str, Any] = field(default_factory=dict)
    in_round: bool = False
    end_training: bool = False
    aggregation_weight: float | None = None


@dataclass(kw_only=True, slots=True)
class ParameterMessageBase(Message):
    is_initial: bool = False


@dataclass(kw_only=True, slots=True)
class ParameterMessage(ParameterMessageBase):
    parameter: ModelParameter

    def complete(self, other_parameter: ModelParameter) -> None:
        """Fill the keys this client did not send from the old global model (message.py:28-31).

        Missing keys are appended in the old model's key order, as the reference does.
        """
        self.parameter.update(
            {name: value for name, value in other_parameter.items() if name not in self.parameter}
        )


@dataclass(kw_only=True, slots=True)
class DeltaParameterMessage(ParameterMessageBase):
    delta_parameter: ModelParameter
    old_parameter: ModelParameter | None = None
    new_parameter: ModelParameter | None = None

    def restore(self, parameter: ModelParameter) -> ParameterMessage:
        """Rebuild the full update: ``old.to(float64) + delta`` per tensor (message.py:40-61).

        ``parameter`` is the server's cached global model. It is deep-copied, never mutated.
        The optional ``old_parameter`` / ``new_parameter`` of the message are consistency
        checks, exactly as in the reference.
        """
        model = copy.deepcopy(parameter)
        if self.old_parameter is not None:
            assert len(self.old_parameter) == len(model)
            assert all((t.cpu() == model[name]).all().item() for name, t in self.old_parameter.items())
        assert len(self.delta_parameter) == len(parameter)
        for name, delta in self.delta_parameter.items():
            full = model[name].to(dtype=torch.float64) + delta
            model[name] = full
            if self.new_parameter is None:
                continue
            expected = self.new_parameter[name].to(dtype=torch.float64, device="cpu")
            assert torch.allclose(expected, full), (
                f"Restoration mismatch for key {name}: delta={delta}, result={full}, expected={expected}"
            )
        out = ParameterMessage(parameter=model)
        for f in fields(out):
            if f.name == "parameter" or not hasattr(self, f.name):
                continue
            setattr(out, f.name, getattr(self, f.name))
        return out


@dataclass(kw_only=True, slots=True)
class FeatureMessage(Message):
    feature: torch.Tensor | None


@dataclass(kw_only=True, slots=True)
class MultipleWorkerMessage(Message):
    worker_data: Mapping[int, Message]


def _count_tensor_bytes(obj: Any) -> int:
    if isinstance(obj, torch.Tensor):
        return obj.element_size() * obj.numel()
    if isinstance(obj, Mapping):
        return sum(_count_tensor_bytes(v) for v in obj.values())
    if isinstance(obj, (list, tuple, set)):
        return sum(_count_tensor_bytes(v) for v in obj)
    if hasattr(obj, "__slots__") or hasattr(obj, "__dataclass_fields__"):
        return sum(_count_tensor_bytes(getattr(obj, f.name)) for f in fields(obj))
    return 0


def get_message_size(msg: Message) -> int:
    """Bytes of every tensor reachable from the message (message.py:74-84)."""
    cnt = _count_tensor_bytes(msg)
    assert cnt > 0
    return cnt
