"""FedAvg on MI355X: the reference's streaming weighted average, folded in waves on the GPU.

Same plugin surface as ``FedAVGAlgorithm`` in the reference
(``simulation_lib/algorithm/fed_avg_algorithm.py:12-149``): ``accumulate`` /
``aggregate_loss`` flags, the ``_accumulate_parameter`` / ``_get_weight`` /
``_apply_total_weight`` / ``_aggregate_parameter`` hooks, ``process_worker_data`` /
``aggregate_worker_data`` with the same message semantics.

What differs is where the arithmetic happens. ``_accumulate_parameter`` stages each client
tensor (a client that arrived in host memory is packed into pinned memory and DMA'd to HBM in
one transfer, ``ingest.py``) instead of doing
``acc += x.to(float64) * w`` on the CPU. Every ``wave_size`` clients the wave is folded into a
device-resident fp64 accumulator by one HIP kernel launch, in arrival order, with separately
rounded products and sums — bit-identical to the reference's fp64 sequence. The last wave is
folded and divided by the total weight in the same launch (``fedavg_aggregate``), with the
reference's NaN assertions fused into the kernel.

Differences a caller can observe, all documented in DESIGN.md:
  * the NaN assertions fire at the wave flush / aggregate, not at the offending arrival;
  * ``aggregate_worker_data`` returns float64 tensors on the GPU (``result_device`` moves
    them, e.g. to ``"cpu"`` as the reference's server does on caching);
  * a key that first appears in a later client than the first one raises
    ``NotImplementedError`` (the reference server always calls ``complete()`` first).
"""

from __future__ import annotations

import os
from collections.abc import MutableMapping
from typing import Any

import torch

from ..fedavg import ClientTable, FedAvgContext, ModelLayout, NaNAggregationError, OutputTable
from ..ingest import HostIngest
from ..message import (
    DeltaParameterMessage,
    Message,
    ModelParameter,
    ParameterMessage,
    is_delta_message,
    is_parameter_message,
    wire_class,
)
from ..quantized import QuantizedTensor, dequantize_tensor, record_layout
from .aggregation_algorithm import (
    AggregationAlgorithm,
    default_device,
    split_empty,
    to_device_operand,
    unify_dtype,
)


class FedAVGAlgorithm(AggregationAlgorithm):
    def __init__(
        self,
        device: torch.device | str | None = None,
        wave_size: int | None = None,
        result_dtype: torch.dtype = torch.float64,
        result_device: torch.device | str | None = None,
        split_policy: int = 1,
    ) -> None:
        super().__init__()
        self.accumulate: bool = True
        self.aggregate_loss: bool = False
        self._device = torch.device(device) if device is not None else None
        self.wave_size = int(wave_size or os.environ.get("FEDAVG_WAVE_SIZE", 64))
        assert self.wave_size >= 1
        self.result_dtype = result_dtype
        self.result_device = torch.device(result_device) if result_device is not None else None
        self.split_policy = split_policy
        self.__layout: ModelLayout | None = None
        self.__native_layout: ModelLayout | None = None
        self.__keep: list[int] = []
        self.__ctx: FedAvgContext | None = None
        self.__ctx_key: tuple | None = None
        self.__table: ClientTable | None = None
        self.__table_dtype: torch.dtype | None = None
        self.__table_delta = False
        self.__base: OutputTable | None = None
        self.__row: dict[str, tuple[torch.Tensor, Any]] = {}
        self.__has_data = False
        self.__ingest: HostIngest | None = None
        self.__result_flat: torch.Tensor | None = None
        self.__record_layouts: dict[tuple[int, ...], ModelLayout] = {}

    # ---- setup -------------------------------------------------------------------------
    @property
    def device(self) -> torch.device:
        if self._device is None:
            self._device = default_device()
        return self._device

    def _context(self) -> FedAvgContext:
        assert self.__native_layout is not None
        key = (self.device, self.__native_layout, self.split_policy)
        if self.__ctx is None or self.__ctx_key != key:
            if self.__ctx is not None:
                self.__ctx.close()
            self.__ctx = FedAvgContext(self.__native_layout, self.device, split_policy=self.split_policy)
            self.__ctx_key = key
        return self.__ctx

    def _set_layout(self, parameter: ModelParameter) -> None:
        self.__layout = ModelLayout.from_parameters(parameter)
        self.__native_layout, self.__keep = split_empty(self.__layout)

    # ---- per arrival (fed_avg_algorithm.py:20-41) --------------------------------------
    def process_worker_data(
        self,
        worker_id: int,
        worker_data: Message | None,
    ) -> bool:
        res = super().process_worker_data(worker_id=worker_id, worker_data=worker_data)
        if not res:
            return False
        worker_data = self._all_worker_data.get(worker_id, None)
        if worker_data is None:
            return True
        # messages are recognised by their dataclass fields, not by class identity: the
        # reference's own server passes simulation_lib.message objects (message.py)
        if is_delta_message(worker_data) and not (self.accumulate and self._delta_fusable(worker_data)):
            # a delta the fold cannot take (consistency-check fields, or the ratio path keeps
            # whole updates): restore it on the host exactly as the reference server does
            # (aggregation_server.py:123-125) and keep the full update in its place
            assert self._old_parameter is not None, "a delta update needs the cached global model"
            worker_data = worker_data.restore(self._old_parameter)
            self._all_worker_data[worker_id] = worker_data
        if is_delta_message(worker_data):
            # restore() fused into the fold: x = old + delta in the kernel (message.py:40-61)
            assert self._old_parameter is not None
            assert len(worker_data.delta_parameter) == len(self._old_parameter)
            if self.__layout is None:
                self._set_layout(self._old_parameter)
            self.__row = {}
            for name, delta in worker_data.delta_parameter.items():
                weight = self._get_weight(worker_data=worker_data, name=name, parameter=delta)
                self.__row[name] = (delta, weight)
            worker_data.delta_parameter = {}
            self._stage_client(delta=True)
            return True
        if not is_parameter_message(worker_data):
            return True
        self.__row = {}
        for name, parameter in worker_data.parameter.items():
            self._accumulate_parameter(worker_data=worker_data, name=name, parameter=parameter)
        if self.accumulate:
            self._stage_client()
        return True

    # The server hands DeltaParameterMessages straight to this algorithm (with the cached global
    # model set through set_old_parameter) instead of restoring them on the host first.
    accepts_delta_messages = True

    def _delta_fusable(self, msg: DeltaParameterMessage) -> bool:
        # the consistency-check fields of restore() (message.py:42-59) need the host path
        return self._old_parameter is not None and msg.old_parameter is None and msg.new_parameter is None

    def set_old_parameter(self, old_parameter: ModelParameter) -> None:
        if old_parameter is not self._old_parameter:
            self.__base = None
        super().set_old_parameter(old_parameter)

    def _delta_base(self) -> OutputTable:
        """The cached global model as fp64 device tensors in native-layout order."""
        if self.__base is None:
            assert self._old_parameter is not None and self.__native_layout is not None and self.__layout is not None
            names = [self.__layout.names[i] for i in self.__keep]
            tensors = [self._old_parameter[n].to(device=self.device, dtype=torch.float64).contiguous().view(-1)
                       for n in names]
            self.__base = OutputTable(tensors, self.__native_layout, self.device, torch.float64)
        return self.__base

    def _accumulate_parameter(
        self,
        worker_data: ParameterMessage,
        name: str,
        parameter: torch.Tensor,
    ) -> None:
        """Stage (tensor, weight) for the next GPU wave; releases the payload like :64."""
        if not self.accumulate:
            return
        weight = self._get_weight(worker_data=worker_data, name=name, parameter=parameter)
        # host tensors are packed and DMA'd per client in _stage_client (ingest.HostIngest)
        self.__row[name] = (parameter, weight)
        # release to reduce memory pressure (fed_avg_algorithm.py:63-64)
        worker_data.parameter = {}

    def _get_weight(self, worker_data: ParameterMessage, name: str, parameter: Any) -> Any:
        return worker_data.aggregation_weight

    def _apply_total_weight(self, name: str, parameter: torch.Tensor, total_weight: Any) -> torch.Tensor:
        return parameter / total_weight

    def _stage_client(self, delta: bool = False) -> None:
        row = self.__row
        self.__row = {}
        if not row:
            return
        if self.__layout is None:
            self._set_layout({k: v[0] for k, v in row.items()})
        assert self.__layout is not None
        unknown = [k for k in row if k not in self.__layout.names]
        if unknown:
            raise NotImplementedError(
                f"tensors {unknown} were not in the first client's update; complete() the "
                "message against the global model first (aggregation_server.py:126-128)"
            )
        if self.__native_layout is None:
            self.__has_data = True
            return
        tensors: list[torch.Tensor | None] = []
        weights: list[float] = []
        for i in self.__keep:
            name = self.__layout.names[i]
            if name in row:
                t, w = row[name]
                if tuple(t.shape) != self.__layout.shapes[i]:
                    raise ValueError(f"shape of {name} changed: {tuple(t.shape)} vs {self.__layout.shapes[i]}")
                assert w is not None, "aggregation_weight is None"
                tensors.append(t)
                weights.append(float(w))
            else:
                tensors.append(None)
                weights.append(0.0)
        present = [t for t in tensors if t is not None]
        codecs = {t.codec for t in present if isinstance(t, QuantizedTensor)}
        if codecs and len(codecs) == 1 and all(isinstance(t, QuantizedTensor) for t in present):
            # quantised update: the records are the kernel operands (dequantised in the fold)
            dt = codecs.pop()
            tensors = self._records_to_device(tensors)
        else:
            if codecs:  # mixed with dense tensors (e.g. complete()-d keys): dequantise here
                tensors = [dequantize_tensor(t) if isinstance(t, QuantizedTensor) else t for t in tensors]
            tensors = self._to_device_row(tensors)
            present = [t for t in tensors if t is not None]
            if present:
                unified, dt = unify_dtype(present)
                it = iter(unified)
                tensors = [next(it) if t is not None else None for t in tensors]
            else:
                dt = self.__table_dtype or torch.float32
        if self.__table is not None and (self.__table_dtype != dt or self.__table_delta != delta):
            self._flush()
        if self.__table is None:
            self.__table = ClientTable(len(self.__keep))
            self.__table_dtype = dt
            self.__table_delta = delta
        self.__table.add_client(tensors, weights)
        self.__has_data = True
        if self.__table.num_clients >= self.wave_size:
            self._flush()

    def _to_device_row(self, tensors: list[torch.Tensor | None]) -> list[torch.Tensor | None]:
        """One client's tensors in HBM. Host tensors of one kernel dtype go through the pinned
        ingest (one packed DMA per client); anything else moves tensor by tensor."""
        host = [t for t in tensors if t is not None and t.device.type == "cpu"]
        if not host:
            return [None if t is None else to_device_operand(t, self.device) for t in tensors]
        dtypes = {t.dtype for t in host}
        if len(dtypes) == 1 and next(iter(dtypes)) in (torch.float32, torch.float16, torch.bfloat16, torch.float64):
            if self.__ingest is None:
                self.__ingest = HostIngest(self.device)
            assert self.__native_layout is not None
            moved = self.__ingest.to_device(
                self.__native_layout, [t if t is not None and t.device.type == "cpu" else None for t in tensors],
                next(iter(dtypes)),
            )
            return [
                None if t is None else (m if m is not None else to_device_operand(t, self.device))
                for t, m in zip(tensors, moved)
            ]
        return [None if t is None else to_device_operand(t, self.device) for t in tensors]

    # Quantised updates (StochasticQuantServerEndpoint, quantized_endpoint.py:69-77,102-111) are
    # handed over as QSGD records; the kernel dequantises them inside the fold.
    accepts_quantized_messages = True

    def _records_to_device(self, tensors: list) -> list[torch.Tensor | None]:
        """One client's QSGD records in HBM: host records go through the pinned ingest (one
        packed DMA per client), device records are used where they are."""
        host = [q for q in tensors if q is not None and q.device.type == "cpu"]
        moved: list[torch.Tensor | None] = [None] * len(tensors)
        if host:
            if self.__ingest is None:
                self.__ingest = HostIngest(self.device)
            numels = tuple(q.numel if q is not None else 1 for q in tensors)
            rl = self.__record_layouts.get(numels)
            if rl is None:
                rl = self.__record_layouts[numels] = record_layout(list(numels))
            staged = self.__ingest.to_device(
                rl,
                [q.record if q is not None and q.device.type == "cpu" else None for q in tensors],
                torch.uint8,
            )
            moved = list(staged)
        out: list[torch.Tensor | None] = []
        for q, m in zip(tensors, moved):
            if q is None:
                out.append(None)
            elif m is not None:
                out.append(m)
            else:
                out.append(q.record if q.device == self.device else q.record.to(self.device))
        return out

    def _flush(self) -> None:
        """Fold the staged wave into the device accumulator (one kernel launch)."""
        if self.__table is None or self.__table.num_clients == 0:
            return
        ctx = self._context()
        table, dt = self.__table, self.__table_dtype
        assert dt is not None
        self.__table, self.__table_dtype = None, None
        if self.__table_delta:
            ctx.accumulate_delta(table, dt, self._delta_base())
        else:
            ctx.accumulate(table, dt)

    # ---- end of round (fed_avg_algorithm.py:76-113) ------------------------------------
    def _aggregate_parameter(self, chosen_worker_ids: set[int] | None = None) -> ModelParameter:
        self.__result_flat = None
        if not self.accumulate:
            worker_data: MutableMapping[int, Message] = self._all_worker_data
            if chosen_worker_ids is not None:
                worker_data = {k: worker_data[k] for k in chosen_worker_ids}
            return AggregationAlgorithm.weighted_avg(
                worker_data, AggregationAlgorithm.get_ratios(worker_data), device=self.device
            )
        assert self.__has_data
        assert chosen_worker_ids is None
        layout = self.__layout
        assert layout is not None
        result: ModelParameter = {}
        if self.__native_layout is not None:
            result.update(self._finish_native())
        for i, name in enumerate(layout.names):
            if i not in self.__keep:
                result[name] = torch.empty(layout.shapes[i], dtype=self.result_dtype, device=self.device)
        self.__has_data = False
        out = {name: result[name] for name in layout.names}
        if self.result_device is not None:
            out = self._move_result(out)
        return out

    def _move_result(self, out: ModelParameter) -> ModelParameter:
        """Results to ``result_device``: the native part lives in one flat device buffer, so a
        host destination takes ONE device-to-host copy of it (not one per tensor)."""
        assert self.result_device is not None
        flat = self.__result_flat
        if self.result_device.type != "cpu" or flat is None:
            return {k: v.to(self.result_device) for k, v in out.items()}
        # through torch's caching pinned-host allocator: a DMA at full PCIe rate instead of a
        # pageable copy (the pinned block is reused once the previous round's result is freed)
        host = torch.empty(flat.shape, dtype=flat.dtype, pin_memory=True)
        host.copy_(flat)
        moved: ModelParameter = {}
        for name, v in out.items():
            if v.numel() and v.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr():
                off = v.storage_offset() - flat.storage_offset()
                moved[name] = host[off : off + v.numel()].view(v.shape)
            else:
                moved[name] = v.to(self.result_device)
        return moved

    def _finish_native(self) -> ModelParameter:
        ctx = self._context()
        native = self.__native_layout
        layout = self.__layout
        assert native is not None and layout is not None
        table, dt = self.__table, self.__table_dtype
        self.__table, self.__table_dtype = None, None
        pending = [(table, dt)] if table is not None and dt is not None else []
        custom_divide = type(self)._apply_total_weight is not FedAVGAlgorithm._apply_total_weight
        out_dtype = torch.float64 if custom_divide else self.result_dtype
        flat = torch.empty(native.padded_offsets(8 if out_dtype == torch.float64 else 4)[1],
                           dtype=out_dtype, device=self.device)
        self.__result_flat = None if custom_divide else flat
        offs, _ = native.padded_offsets(flat.element_size())
        outs = [flat[o : o + n] for o, n in zip(offs, native.numels)]
        delta = self.__table_delta and table is not None
        try:
            if not custom_divide:
                if delta:
                    ctx.aggregate_delta(table, dt, self._delta_base(), outs, out_dtype)
                else:
                    ctx.aggregate(table, dt or torch.float32, outs, out_dtype)
                ctx.raise_on_nan(pending)
            else:
                # a subclass divides: finalize with a unit divisor (exact), then call its hook
                if table is not None and dt is not None:
                    if delta:
                        ctx.accumulate_delta(table, dt, self._delta_base())
                    else:
                        ctx.accumulate(table, dt)
                totals = ctx.total_weights()
                ctx.set_accumulated([1.0] * native.num_segments)
                ctx.finalize_range(outs, torch.float64)
                ctx.raise_on_nan(pending)
        except NaNAggregationError:
            ctx.reset()
            raise
        result: ModelParameter = {}
        for j, i in enumerate(self.__keep):
            name = layout.names[i]
            value = outs[j].view(layout.shapes[i])
            if custom_divide:
                value = self._apply_total_weight(name=name, parameter=value, total_weight=totals[j])
                assert not value.isnan().any().cpu()
                value = value.to(self.result_dtype)
            result[name] = value
        ctx.reset()
        return result

    def aggregate_worker_data(self) -> ParameterMessage:
        parameter = self._aggregate_parameter()
        other_data: dict[str, Any] = {}
        if self.aggregate_loss:
            other_data |= self.__aggregate_loss(self._all_worker_data)
        other_data |= self.__check_and_reduce_other_data(self._all_worker_data)
        first = next(iter(self._all_worker_data.values()))
        # the caller's own ParameterMessage class: the reference server matches the result
        # with `case ParameterMessageBase()` (aggregation_server.py:87) and caches it (:148-167)
        return wire_class(first, "ParameterMessage")(
            parameter=parameter,
            end_training=first.end_training,
            in_round=first.in_round,
            other_data=other_data,
        )

    def clear_worker_data(self) -> None:
        super().clear_worker_data()
        self.__table, self.__table_dtype = None, None
        self.__row = {}
        self.__has_data = False
        if self.__ctx is not None:
            self.__ctx.reset()

    def exit(self) -> None:
        if self.__ctx is not None:
            self.__ctx.close()
            self.__ctx = None

    @classmethod
    def __aggregate_loss(cls, all_worker_data: MutableMapping[int, Message]) -> dict[str, Any]:
        """Ratio-weighted training/validation loss (fed_avg_algorithm.py:115-134)."""
        assert all_worker_data
        first = next(iter(all_worker_data.values()))
        loss_types = [t for t in ("training_loss", "validation_loss") if t in first.other_data]
        ratios = AggregationAlgorithm.get_ratios(all_worker_data)
        loss_dict = {
            t: AggregationAlgorithm.weighted_avg_for_scalar(all_worker_data, ratios, scalar_key=t)
            for t in loss_types
        }
        assert loss_dict
        for msg in all_worker_data.values():
            for t in ("training_loss", "validation_loss"):
                msg.other_data.pop(t, None)
        return loss_dict

    @classmethod
    def __check_and_reduce_other_data(cls, all_worker_data: MutableMapping[int, Message]) -> dict[str, Any]:
        """Every client must agree on every other_data key (fed_avg_algorithm.py:136-149)."""
        merged: dict[str, Any] = {}
        for msg in all_worker_data.values():
            for k, v in msg.other_data.items():
                if k in merged and v != merged[k]:
                    raise RuntimeError(f"different values on key {k}")
                merged.setdefault(k, v)
        return merged
