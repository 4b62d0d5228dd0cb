"""A second wire module with the reference's message schema but its own classes (test-only).

The reference server hands the algorithm objects of ``simulation_lib.message``
(``simulation_lib/server/aggregation_server.py:117-130``), a class hierarchy this package does not
share. These look-alikes stand in for it on the GPU box (where the reference does not exist):
same dataclass fields as ``simulation_lib/message.py:11-71``, unrelated to
``distributed_learning_simulation_lib_amd.message``. The plugins must recognise them by their
fields and answer with *these* classes.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any

import torch


@dataclass(kw_only=True)
class Message:
    other_data: dict[str, Any] = field(default_factory=dict)
    in_round: bool = False
    end_training: bool = False
    aggregation_weight: float | None = None


@dataclass(kw_only=True)
class ParameterMessageBase(Message):
    is_initial: bool = False


@dataclass(kw_only=True)
class ParameterMessage(ParameterMessageBase):
    parameter: dict[str, torch.Tensor]

    def complete(self, other_parameter: dict[str, torch.Tensor]) -> None:
        for name, value in other_parameter.items():
            self.parameter.setdefault(name, value)


@dataclass(kw_only=True)
class DeltaParameterMessage(ParameterMessageBase):
    delta_parameter: dict[str, torch.Tensor]
    old_parameter: dict[str, torch.Tensor] | None = None
    new_parameter: dict[str, torch.Tensor] | None = None

    def restore(self, parameter: dict[str, torch.Tensor]) -> ParameterMessage:
        full = copy.deepcopy(parameter)
        assert len(self.delta_parameter) == len(full)
        for name, delta in self.delta_parameter.items():
            full[name] = full[name].to(dtype=torch.float64) + delta
            if self.new_parameter is not None:
                assert torch.allclose(self.new_parameter[name].to(torch.float64).cpu(), full[name].cpu())
        return ParameterMessage(parameter=full, other_data=self.other_data, in_round=self.in_round,
                                end_training=self.end_training, aggregation_weight=self.aggregation_weight,
                                is_initial=self.is_initial)


@dataclass(kw_only=True)
class MultipleWorkerMessage(Message):
    worker_data: dict[int, Message]
