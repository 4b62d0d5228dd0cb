"""The server-side aggregation plugin interface, with the ratio reduce on the GPU.

Mirrors the reference's ``AggregationAlgorithm`` ABC
(``simulation_lib/algorithm/aggregation_algorithm.py:12-112``): same methods, same argument
meaning, same assertions. The one tensor operation of the class, ``weighted_avg``
(:51-76), runs in the HIP kernel (``fedavg_weighted_avg`` of ``include/fedavg_hip.h``)
instead of torch CPU ops; the scalar helpers (total weight, ratios, scalar averages) are
host logic and stay in Python.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from collections import OrderedDict
from collections.abc import Mapping, MutableMapping
from typing import Any

import torch

from ..fedavg import ClientTable, FedAvgContext, ModelLayout
from ..message import Message, ModelParameter, is_parameter_message
from ..quantized import QuantizedTensor, dequantize_tensor

# (device index, layout, split policy) -> context, for the class-level weighted_avg
_CTX_CACHE: OrderedDict[tuple[int, ModelLayout, int], FedAvgContext] = OrderedDict()
_CTX_CACHE_SIZE = 4


def context_for(layout: ModelLayout, device: torch.device, split_policy: int = 1) -> FedAvgContext:
    """A cached native context for (device, layout)."""
    key = (device.index, layout, split_policy)
    ctx = _CTX_CACHE.get(key)
    if ctx is None:
        ctx = FedAvgContext(layout, device, split_policy=split_policy)
        _CTX_CACHE[key] = ctx
        while len(_CTX_CACHE) > _CTX_CACHE_SIZE:
            _CTX_CACHE.popitem(last=False)[1].close()
    else:
        _CTX_CACHE.move_to_end(key)
    return ctx


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("the MI355X FedAvg path needs a visible GPU (HIP device)")
    return torch.device("cuda", torch.cuda.current_device())


def to_device_operand(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    """A contiguous copy/view of ``t`` on ``device`` (data movement only, no arithmetic)."""
    if t.device != device:
        t = t.to(device)
    return t.contiguous()


def unify_dtype(tensors: list[torch.Tensor]) -> tuple[list[torch.Tensor], torch.dtype]:
    """One kernel input dtype per call. Mixed or non-float inputs are widened to float64,
    which is exact: the reference converts every tensor to float64 before the product."""
    dtypes = {t.dtype for t in tensors}
    if len(dtypes) == 1:
        (dt,) = dtypes
        if dt in (torch.float32, torch.float16, torch.bfloat16, torch.float64):
            return tensors, dt
    return [t.to(torch.float64) for t in tensors], torch.float64


def split_empty(layout: ModelLayout) -> tuple[ModelLayout | None, list[int]]:
    """The native layout holds the non-empty tensors only; returns it and their indices."""
    keep = [i for i, n in enumerate(layout.numels) if n > 0]
    if not keep:
        return None, []
    return ModelLayout(
        names=tuple(layout.names[i] for i in keep), shapes=tuple(layout.shapes[i] for i in keep)
    ), keep


class AggregationAlgorithm(ABC):
    def __init__(self) -> None:
        self._all_worker_data: MutableMapping[int, Message] = {}
        self.__skipped_workers: set[int] = set()
        self._old_parameter: ModelParameter | None = None
        self._config: Any = None

    def set_old_parameter(self, old_parameter: ModelParameter) -> None:
        self._old_parameter = old_parameter

    @property
    def config(self) -> Any:
        assert self._config is not None
        return self._config

    def set_config(self, config: Any) -> None:
        self._config = config

    @property
    def skipped_workers(self) -> set[int]:
        return set(self.__skipped_workers)

    # ---- scalar host logic (aggregation_algorithm.py:30-49, 78-91) --------------------------
    @classmethod
    def get_total_weight(cls, data_dict: Mapping[int, Message]) -> float:
        """Sum of the clients' aggregation weights; every weight must be set and >= 0."""
        weights = [msg.aggregation_weight for msg in data_dict.values()]
        assert all(w is not None and w >= 0 for w in weights)
        total: float = sum(w for w in weights if w is not None)
        assert total >= 0
        return total

    @classmethod
    def get_ratios(cls, data_dict: Mapping[int, Message]) -> dict[int, float]:
        """weight / total weight per client, computed in Python floats like the reference."""
        total = float(cls.get_total_weight(data_dict=data_dict))
        out: dict[int, float] = {}
        for worker_id, msg in data_dict.items():
            assert msg.aggregation_weight is not None and msg.aggregation_weight >= 0
            out[worker_id] = float(msg.aggregation_weight) / total
        return out

    @classmethod
    def weighted_avg_for_scalar(
        cls,
        data_dict: MutableMapping[int, Message],
        weights: dict[int, float] | float,
        scalar_key: str,
    ) -> float:
        assert data_dict
        acc: float = 0
        for worker_id, msg in data_dict.items():
            r = weights[worker_id] if isinstance(weights, dict) else weights
            assert 0 <= r <= 1
            acc += msg.other_data[scalar_key] * r
        return acc

    # ---- the tensor reduce, on the GPU (aggregation_algorithm.py:51-76) ---------------------
    @classmethod
    def weighted_avg(
        cls,
        data_dict: Mapping[int, Message],
        weights: dict[int, float] | float,
        device: torch.device | None = None,
    ) -> ModelParameter:
        """sum_k ratio_k * x_k in float64, clients in dict order, keys of the first client.

        Returns float64 tensors on the GPU. Raises ``AssertionError`` where the reference
        does: empty input, a ratio outside [0, 1], a non-parameter message, NaN in the result.
        """
        assert data_dict
        device = device or default_device()
        messages = list(data_dict.items())
        first = messages[0][1]
        assert is_parameter_message(first)
        assert first.parameter
        layout = ModelLayout.from_parameters(first.parameter)
        native, keep = split_empty(layout)
        rows: list[list[torch.Tensor]] = []
        ratios: list[float] = []
        for worker_id, msg in messages:
            r = weights[worker_id] if isinstance(weights, dict) else weights
            assert 0 <= r <= 1
            assert is_parameter_message(msg)
            assert msg.parameter
            rows.append([msg.parameter[name] for name in layout.names])
            ratios.append(float(r))
        result: ModelParameter = {}
        if native is not None:
            flat = [rows[k][i] for k in range(len(rows)) for i in keep]
            codecs = {t.codec for t in flat if isinstance(t, QuantizedTensor)}
            if len(codecs) == 1 and all(isinstance(t, QuantizedTensor) for t in flat):
                # QSGD records: dequantised inside the kernel (quantized.py)
                dt = codecs.pop()
                flat = [t.record.to(device) for t in flat]
            else:
                flat = [to_device_operand(dequantize_tensor(t) if isinstance(t, QuantizedTensor) else t, device)
                        for t in flat]
                flat, dt = unify_dtype(flat)
            T = len(keep)
            table = ClientTable(T)
            for k in range(len(rows)):
                table.add_client(flat[k * T : (k + 1) * T], [ratios[k]] * T)
            ctx = context_for(native, device)
            outs = [torch.empty(n, dtype=torch.float64, device=device) for n in native.numels]
            ctx.weighted_avg(table, dt, outs, torch.float64)
            ctx.raise_on_nan([(table, dt)])
            for j, i in enumerate(keep):
                result[layout.names[i]] = outs[j].view(layout.shapes[i])
        for i, name in enumerate(layout.names):
            if i not in keep:
                result[name] = torch.empty(layout.shapes[i], dtype=torch.float64, device=device)
        return {name: result[name] for name in layout.names}

    # ---- plugin protocol (aggregation_algorithm.py:93-112) ----------------------------------
    def process_worker_data(
        self,
        worker_id: int,
        worker_data: Message | None,
    ) -> bool:
        if worker_data is None:
            self.__skipped_workers.add(worker_id)
            return True
        self._all_worker_data[worker_id] = worker_data
        return True

    @abstractmethod
    def aggregate_worker_data(self) -> Any: ...

    def clear_worker_data(self) -> None:
        self._all_worker_data.clear()
        self.__skipped_workers.clear()

    def exit(self) -> None:  # noqa: B027
        pass
