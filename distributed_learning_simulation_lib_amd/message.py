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
import sys
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


# ---- structural recognition --------------------------------------------------------------
# The algorithms are handed messages by whichever server hosts them: this package's
# AggregationServer, or the reference's own (simulation_lib/server/aggregation_server.py:117-130),
# which passes simulation_lib.message objects. Those are a different class hierarchy with the same
# dataclass schema, so the plugins recognise a message by its fields, never by class identity,
# and answer with the ParameterMessage / MultipleWorkerMessage class of the caller's module (the
# reference server dispatches on `case ParameterMessageBase()` / `case MultipleWorkerMessage()`,
# aggregation_server.py:83-87, and `isinstance(result, ParameterMessageBase)`, :148).
_FIELD_CACHE: dict[type, frozenset[str]] = {}


def _field_names(obj: Any) -> frozenset[str]:
    cls = type(obj)
    names = _FIELD_CACHE.get(cls)
    if names is None:
        dc = getattr(cls, "__dataclass_fields__", None)
        names = frozenset(dc) if dc is not None else frozenset()
        _FIELD_CACHE[cls] = names
    return names


def is_message(obj: Any) -> bool:
    """A Message of any wire module (message.py:11-16 fields)."""
    return {"other_data", "in_round", "end_training", "aggregation_weight"} <= _field_names(obj)


def is_parameter_message_base(obj: Any) -> bool:
    """ParameterMessageBase (message.py:19-21): a Message with ``is_initial``."""
    return is_message(obj) and "is_initial" in _field_names(obj)


def is_parameter_message(obj: Any) -> bool:
    """ParameterMessage (message.py:24-31): a full update, ``parameter`` dict of tensors."""
    names = _field_names(obj)
    return "parameter" in names and "delta_parameter" not in names and is_parameter_message_base(obj)


def is_delta_message(obj: Any) -> bool:
    """DeltaParameterMessage (message.py:34-61): ``delta_parameter`` against the cached model."""
    return "delta_parameter" in _field_names(obj) and is_parameter_message_base(obj)


KIND_OTHER, KIND_PARAMETER, KIND_DELTA = 0, 1, 2
_KIND_CACHE: dict[type, int] = {}


def message_kind(obj: Any) -> int:
    """KIND_PARAMETER / KIND_DELTA / KIND_OTHER of ``obj`` (is_parameter_message /
    is_delta_message in one class-keyed lookup: the plugins ask once per arrival)."""
    cls = type(obj)
    kind = _KIND_CACHE.get(cls)
    if kind is None:
        kind = KIND_PARAMETER if is_parameter_message(obj) else KIND_DELTA if is_delta_message(obj) else KIND_OTHER
        _KIND_CACHE[cls] = kind
    return kind


_WIRE_CACHE: dict[tuple[type, str], type] = {}


def wire_class(like: Any, name: str) -> type:
    """The class ``name`` ("ParameterMessage", "MultipleWorkerMessage", ...) of the wire module
    ``like`` comes from; this package's class when ``like`` is None or its module has none
    (looked up once per message class: the plugins answer every round)."""
    key = (type(like), name)
    cls = _WIRE_CACHE.get(key)
    if cls is None:
        cls = _WIRE_CACHE[key] = _find_wire_class(like, name)
    return cls


def _find_wire_class(like: Any, name: str) -> type:
    if like is not None:
        for cls in type(like).__mro__:
            if cls.__name__ == name and hasattr(cls, "__dataclass_fields__"):
                return cls
        mod = sys.modules.get(type(like).__module__)
        cls = getattr(mod, name, None) if mod is not None else None
        if isinstance(cls, type) and hasattr(cls, "__dataclass_fields__"):
            return cls
    return globals()[name]


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
