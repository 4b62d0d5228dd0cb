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

The hooks keep the reference's full semantics (golden cases in tests/golden, generated from the
reference's own code):
  * ``_get_weight`` may return a number, a 0-dim tensor — whose total then accumulates in the
    tensor's dtype through the reference's ``total += weight`` (:59-62, reproduced on the host
    with the very same objects) — or a tensor of the parameter's shape (per-element weights:
    ``fedavg_accumulate_elementwise`` keeps a per-element total on the GPU);
  * ``_apply_total_weight`` overridden by a subclass receives the fp64 weighted sum and the
    same total object the reference would pass;
  * a tensor name that first appears in a later client grows the layout (:55-62), keeping the
    accumulated state; output keys come in first-seen order.

Differences a caller can observe, all documented in DESIGN.md:
  * the NaN assertion on an arriving update (:35) fires at the wave flush / aggregate unless
    ``eager_nan_check`` (or ``FEDAVG_EAGER_NAN=1``) scans every arrival on the GPU first;
  * ``aggregate_worker_data`` returns float64 tensors on the GPU (``result_device`` moves
    them, e.g. to ``"cpu"`` as the reference's server does on caching).
"""

from __future__ import annotations

from collections.abc import MutableMapping, Sequence
from typing import Any

import numpy as np
import torch

from .. import _native, _staging
from .._staging import NativeClientTable, TableTail
from ..fedavg import ClientTable, FedAvgContext, ModelLayout, NaNAggregationError, OutputTable
from ..ingest import HostIngest
from ..multi_device import MultiDeviceContext
from ..message import (
    KIND_DELTA,
    KIND_PARAMETER,
    DeltaParameterMessage,
    Message,
    ModelParameter,
    ParameterMessage,
    message_kind,
    wire_class,
)
from ..quantized import QuantizedTensor, dequantize_tensor, record_layout
from .dynamic_wave import DynamicWave, PluginSettings
from .aggregation_algorithm import (
    AggregationAlgorithm,
    default_device,
    split_empty,
    to_device_operand,
    unify_dtype,
)


_KERNEL_DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.float64)
_STAGING_DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.float64)  # staging_ext.cpp codes
_STAGING_CODES = {dt: code for code, dt in enumerate(_STAGING_DTYPES)}
# what a device entry of the multi-device mode keeps for itself (the rest of the round's state —
# layout, per-name totals, flags — is one for the whole round)
_LANE_ATTRS = ("_device", "_FedAVGAlgorithm__table", "_FedAVGAlgorithm__table_dtype",
               "_FedAVGAlgorithm__table_delta", "_FedAVGAlgorithm__ingest", "_FedAVGAlgorithm__fast",
               "_FedAVGAlgorithm__base", "_FedAVGAlgorithm__wave_event")


def _is_elementwise(weight: Any, parameter: Any) -> bool:
    """A _get_weight value that is a tensor of the parameter's shape (not a scalar)."""
    if type(weight) in (int, float):  # the default hook's dataset-size weight: the common case
        return False
    if isinstance(weight, torch.Tensor) and weight.numel() != 1:
        if isinstance(parameter, torch.Tensor) and tuple(weight.shape) == tuple(parameter.shape):
            return True
        raise NotImplementedError(
            f"a _get_weight tensor of shape {tuple(weight.shape)} for a parameter of shape "
            f"{tuple(getattr(parameter, 'shape', ()))}: scalars and per-element weights are supported"
        )
    if isinstance(weight, np.ndarray) and weight.size != 1:
        raise NotImplementedError("per-element weights must be torch tensors")
    return False


def _total_is_fp32(weight: Any) -> bool:
    """The reference's `total = weight; total += ...` keeps the first weight's dtype."""
    dt = getattr(weight, "dtype", None)
    if dt in (torch.float32, np.float32):
        return True
    if dt in (torch.float16, torch.bfloat16, np.float16):
        raise NotImplementedError("fp16 / bf16 weight tensors are not supported (fp32 / fp64 / numbers are)")
    return False


class FedAVGAlgorithm(AggregationAlgorithm):
    """The reference's ``FedAVGAlgorithm`` (fed_avg_algorithm.py:12-149) folding on MI355X.

    One device (``device``, the default): every result is bit-identical to the reference's single
    arrival-order fp64 chain. ``devices=[...]`` (one server process, several GPUs): arrivals are
    dealt to the entries in turn and each entry's chain is summed in entry order, so a result
    depends on the entry count and on which client lands on which entry, and matches the
    reference's single chain to fp64 reassociation only — |Δ| ≤ 1e-12 · Σ|w x| / |W| per element,
    ≤ 1 ulp after an fp32 cast (tests/test_multi_tolerance.py, tests/test_gpu_multi_device.py);
    ``bit_exact_with_reference`` says which of the two a given object gives.
    """

    def __init__(
        self,
        device: torch.device | str | None = None,
        wave_size: int | None = None,
        result_dtype: torch.dtype = torch.float64,
        result_device: torch.device | str | None = None,
        split_policy: int = 1,
        eager_nan_check: bool | None = None,
        devices: Sequence[int | str | torch.device] | None = None,
        exchange: str = "peer",
        wave_min: int | None = None,
        dynamic_wave: bool | None = None,
        settings: PluginSettings | None = None,
    ) -> None:
        super().__init__()
        self.accumulate: bool = True
        self.aggregate_loss: bool = False
        self._device = torch.device(device) if device is not None else None
        # the tuning knobs: one settings object (PluginSettings.from_env() unless given), single
        # fields overridden by the keyword arguments
        self.settings = (settings or PluginSettings.from_env()).with_overrides(
            wave_size=wave_size or None, wave_min=wave_min, eager_nan_check=eager_nan_check, dynamic_wave=dynamic_wave)
        # 64: with an update staged in ~2.6 us, folding half a 64-client round early no longer
        # pays for the extra wave's fp64 accumulator round trip and launch ramp (0.756 vs 0.789 ms
        # per device-resident 64 x ResNet-18 round; 32 was faster while
        # staging took ~4 us per update)
        self.wave_size = self.settings.wave_size
        # early waves: a wave of at least ``wave_min`` staged clients is also folded when the next
        # update arrives while the GPU has finished every wave so far (0 = only full waves), so the
        # fold starts after the first few arrivals instead of after ``wave_size`` of them
        self.wave_min = self.settings.wave_min
        self.__wave_event: torch.cuda.Event | None = None  # recorded after each flushed wave
        # The round's first wave as a dynamic wave (algorithm/dynamic_wave.py): launched at the
        # round's first staged update, handed the staged rows while it folds the ones it has, closed
        # by the wave's flush or by aggregate_worker_data (which then divides in the same kernel) —
        # the GPU works through the arrival phase instead of after it. Any update it cannot take (an
        # absent tensor, per-tensor weights, unaligned tensors) closes it early: it keeps the rows it
        # folded and the ordinary waves fold the rest, with the same bits.
        self.__dyn = DynamicWave(self.settings.dynamic)
        self.__round_updates = 0
        self.result_dtype = result_dtype
        self.result_device = torch.device(result_device) if result_device is not None else None
        self.split_policy = split_policy
        # the reference asserts each arriving tensor is NaN-free (fed_avg_algorithm.py:34-35);
        # by default the fused flags report it at the wave flush, eagerly on request
        self.eager_nan_check = self.settings.eager_nan_check
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
        # (key, flat, output table, views) of the last round's result buffer (_result_buffer)
        self.__result_pool: tuple | None = None
        self.__record_layouts: dict[tuple, ModelLayout] = {}
        # fed_avg_algorithm.py:59-62, kept with the hook's own objects (scalar weights)
        self.__host_totals: dict[str, Any] = {}
        # while every staged update of the round carried every name of the layout, all per-name
        # totals are one value: kept once (``__uniform_total`` after ``__uniform_count`` updates)
        # and written into __host_totals only when an update needs per-name bookkeeping
        self.__uniform_total: Any = None
        self.__uniform_count = 0
        self.__round_fresh = True  # no update of this round seen yet
        # per-element weights: decided by the round's first update
        self.__ew: bool | None = None
        # no per-tensor hook overridden: a scalar-weighted arrival is staged in one pass
        # (process_worker_data), with the default hooks' exact effect
        self.__result_geo: dict = {}
        self.__fast: tuple | None = None  # _fast_maps(): (layout, name -> native segment, shapes, device)
        cls = type(self)
        self.__default_hooks = all(getattr(cls, h) is getattr(FedAVGAlgorithm, h)
                                   for h in ("_accumulate_parameter", "_get_weight", "_note_total"))
        self.__tot_fp32: dict[str, bool] = {}
        self.__ew_totals: torch.Tensor | None = None
        # Multi-device mode (one server process, several MI355X; include/fedavg_hip.h fedavg_multi_*):
        # arrivals are dealt to the device entries in turn (an update already resident on a GPU goes
        # to an entry of that GPU), each entry folds its shard in waves like the single-device path,
        # and aggregate_worker_data sums the G partials in entry order on the GPUs (``exchange``:
        # "peer" stores over xGMI, or "reduce": RCCL) and divides into the first entry's device.
        self.__multi_devices: list[torch.device] | None = None
        self.__multi: MultiDeviceContext | None = None
        self.__lanes: list[dict[str, Any]] = []
        self.__lane = 0
        self.__arrivals = 0
        self.exchange = exchange
        self.bit_exact_with_reference = True
        if devices is not None:
            devs = [torch.device("cuda", d) if isinstance(d, int) else torch.device(d) for d in devices]
            if not devs or any(d.type != "cuda" for d in devs):
                raise ValueError("devices: a non-empty list of GPU devices")
            if device is not None and torch.device(device) != devs[0]:
                raise ValueError("device must be the first entry of devices (the result's device)")
            self._device = devs[0]
            self.__multi_devices = devs
            # entry-ordered sums of per-entry chains: the reference's result to fp64 reassociation
            self.bit_exact_with_reference = len(devs) == 1
            self.__lanes = [{a: getattr(self, a) for a in _LANE_ATTRS} for _ in devs]
            for lane, d in zip(self.__lanes, devs):
                lane["_device"] = d

    # ---- setup -------------------------------------------------------------------------
    @property
    def dynamic_wave(self) -> bool:
        return self.__dyn.settings.enabled

    @dynamic_wave.setter
    def dynamic_wave(self, on: bool) -> None:
        self.settings = self.settings.with_overrides(dynamic_wave=bool(on))
        self.__dyn.settings = self.settings.dynamic

    @property
    def dyn_stats(self) -> dict[str, int]:
        """Dynamic waves opened, rows they folded, waves that wrote the round's result, continued
        launches after a wave ended itself, opens the library refused (DynamicWave.stats)."""
        return self.__dyn.stats

    @property
    def device(self) -> torch.device:
        if self._device is None:
            self._device = default_device()
        return self._device

    @property
    def devices(self) -> list[torch.device]:
        """The device entries (multi-device mode), or the one device."""
        return list(self.__multi_devices) if self.__multi_devices is not None else [self.device]

    def _select_lane(self, g: int) -> None:
        """Make device entry g's wave, ingest and device the current ones (multi-device mode)."""
        if g == self.__lane:
            return
        cur = self.__lanes[self.__lane]
        for a in _LANE_ATTRS:
            cur[a] = getattr(self, a)
        for a, v in self.__lanes[g].items():
            setattr(self, a, v)
        self.__lane = g

    def _lane_for(self, worker_data: Any) -> int:
        """The entry of an arrival: an update resident on a GPU goes to the entries of that GPU in
        turn, any other update to all entries in turn; a round of per-element weights stays on the
        first entry (its per-element totals are one arrival-order chain)."""
        devs = self.__multi_devices
        assert devs is not None
        i = self.__arrivals
        self.__arrivals += 1
        if self.__ew:
            return 0
        payload = getattr(worker_data, "parameter", None) or getattr(worker_data, "delta_parameter", None)
        first = next(iter(payload.values()), None) if isinstance(payload, dict) else None
        if isinstance(first, torch.Tensor) and first.is_cuda:
            on = [g for g, d in enumerate(devs) if d.index == first.get_device()]
            if on:
                return on[i % len(on)]
        return i % len(devs)

    def _multi(self) -> MultiDeviceContext:
        assert self.__native_layout is not None and self.__multi_devices is not None
        m = self.__multi
        if m is None or m.layout != self.__native_layout:
            if m is not None:
                m.close()
            m = self.__multi = MultiDeviceContext(self.__native_layout, self.__multi_devices)
            if self.split_policy != 1:
                for c in m.contexts:
                    _native.check(c._lib.fedavg_set_split_policy(c._h, self.split_policy))
            self.__ew_totals = None
        return m

    def _context(self) -> FedAvgContext:
        assert self.__native_layout is not None
        if self.__multi_devices is not None:
            return self._multi().contexts[self.__lane]
        key = (self.device, self.__native_layout, self.split_policy)
        if self.__ctx is None or self.__ctx_key != key:
            if self.__ctx is not None:
                self.__ctx.close()
            self.__ctx = FedAvgContext(self.__native_layout, self.device, split_policy=self.split_policy)
            self.__ctx_key = key
            self.__ew_totals = None
        return self.__ctx

    def _set_layout(self, parameter: ModelParameter) -> None:
        self.__layout = ModelLayout.from_parameters(parameter)
        self.__native_layout, self.__keep = split_empty(self.__layout)

    def _grow_layout(self, unknown: list[str], row: dict[str, tuple[Any, Any]]) -> None:
        """Names first seen in a later client (fed_avg_algorithm.py:55-62): append them to the
        layout, moving what is accumulated so far into a context of the grown layout."""
        if self.__multi_devices is not None:
            self._grow_layout_multi(unknown, row)
            return
        self._flush()
        old_layout, old_native, old_ctx = self.__layout, self.__native_layout, self.__ctx
        assert old_layout is not None
        # what the old context holds, read before it is replaced
        old_state = None
        if old_ctx is not None and old_native is not None:
            old_state = ([old_ctx.segment_offset(j) for j in range(old_native.num_segments)],
                         old_ctx.total_weights(), old_ctx.accumulator, self.__ew_totals)
        self.__layout = ModelLayout(names=old_layout.names + tuple(unknown),
                                    shapes=old_layout.shapes + tuple(tuple(row[k][0].shape) for k in unknown))
        self.__native_layout, self.__keep = split_empty(self.__layout)
        self.__base = None
        if old_state is None or self.__native_layout is None:
            return
        old_offs, old_totals, old_acc, old_ew = old_state
        new_ctx = self._context()  # closes the old context
        index = {n: i for i, n in enumerate(self.__native_layout.names)}
        totals = [0.0] * self.__native_layout.num_segments
        valid = [0] * self.__native_layout.num_segments
        for j, (name, n) in enumerate(zip(old_native.names, old_native.numels)):
            k = index[name]
            src, dst = old_offs[j], new_ctx.segment_offset(k)
            new_ctx.accumulator[dst : dst + n].copy_(old_acc[src : src + n])
            if old_ew is not None:
                self._ew_totals_buffer()[dst : dst + n].copy_(old_ew[src : src + n])
            totals[k], valid[k] = old_totals[j], 1
        new_ctx.set_segment_state(totals, valid)

    def _grow_layout_multi(self, unknown: list[str], row: dict[str, tuple[Any, Any]]) -> None:
        """_grow_layout for every device entry: each entry's folded segments move into the grown
        layout's context of the same entry."""
        here = self.__lane
        for g in range(len(self.__lanes)):
            self._select_lane(g)
            self._flush()
        self._select_lane(here)
        old_layout, old_native, old_multi = self.__layout, self.__native_layout, self.__multi
        assert old_layout is not None
        old_state = None
        if old_multi is not None and old_native is not None and old_multi.layout == old_native:
            # what each entry's context holds, read before the object is replaced
            old_state = [([c.segment_offset(j) for j in range(old_native.num_segments)], *c.segment_state(),
                          c.accumulator) for c in old_multi.contexts]
        self.__layout = ModelLayout(names=old_layout.names + tuple(unknown),
                                    shapes=old_layout.shapes + tuple(tuple(row[k][0].shape) for k in unknown))
        self.__native_layout, self.__keep = split_empty(self.__layout)
        for lane in self.__lanes:
            lane["_FedAVGAlgorithm__base"] = None
        self.__base = None
        if old_state is None or self.__native_layout is None:
            return
        new_multi = self._multi()  # closes the old object (its accumulators stay alive here)
        index = {n: i for i, n in enumerate(self.__native_layout.names)}
        for g, (old_offs, old_totals, old_valid, old_acc) in enumerate(old_state):
            new_ctx = new_multi.contexts[g]
            totals = [0.0] * self.__native_layout.num_segments
            valid = [0] * self.__native_layout.num_segments
            for j, (name, n) in enumerate(zip(old_native.names, old_native.numels)):
                k = index[name]
                if not old_valid[j]:
                    continue  # this entry never folded the segment
                src, dst = old_offs[j], new_ctx.segment_offset(k)
                new_ctx.accumulator[dst : dst + n].copy_(old_acc[src : src + n])
                totals[k], valid[k] = old_totals[j], 1
            new_ctx.set_segment_state(totals, valid)

    # ---- per arrival (fed_avg_algorithm.py:20-41) --------------------------------------
    def process_worker_data(
        self,
        worker_id: int,
        worker_data: Message | None,
    ) -> bool:
        self.__round_updates += 1
        if self.__round_updates == 1 and self._device_update(worker_data):
            self.__dyn.preopen(self._context, self._dyn_eligible(), self.__table is not None, self.wave_size)
        if worker_data is not None and self._arrive_quick(worker_id, worker_data):
            return True
        res = super().process_worker_data(worker_id, worker_data)
        if not res:
            return False
        worker_data = self._all_worker_data.get(worker_id, None)
        if worker_data is None:
            return True
        if self.__multi_devices is not None and self.accumulate:
            self._select_lane(self._lane_for(worker_data))
        # messages are recognised by their dataclass fields, not by class identity: the
        # reference's own server passes simulation_lib.message objects (message.py)
        kind = message_kind(worker_data)
        if kind == KIND_DELTA and not (self.accumulate and self._delta_fusable(worker_data) and not self.__ew):
            worker_data = self._restore_on_host(worker_id, worker_data)
            kind = message_kind(worker_data)
        if kind == KIND_DELTA:
            # restore() fused into the fold: x = old + delta in the kernel (message.py:40-61)
            assert self._old_parameter is not None
            assert len(worker_data.delta_parameter) == len(self._old_parameter)
            if self.__layout is None:
                self._set_layout(self._old_parameter)
            # a delta stages against the current layout: a later full update of this round must
            # not replace it (its names are matched by name, new ones grow the layout)
            self.__round_fresh = False
            w = worker_data.aggregation_weight
            if self.__default_hooks and isinstance(w, (int, float)) and \
                    self._stage_natively(worker_data.delta_parameter, w, delta=True):
                worker_data.delta_parameter = {}
                return True
            row = {}
            for name, delta in worker_data.delta_parameter.items():
                row[name] = (delta, self._get_weight(worker_data=worker_data, name=name, parameter=delta))
            if any(_is_elementwise(w, t) for t, w in row.values()):
                # per-element weights take the dense elementwise fold: restore first
                worker_data = self._restore_on_host(worker_id, worker_data)
                kind = message_kind(worker_data)
            else:
                self._materialize_totals()
                for name, (delta, weight) in row.items():
                    self._note_total(name, weight, delta)
                self.__row = row
                worker_data.delta_parameter = {}
                self._stage_client(delta=True, worker_id=worker_id)
                return True
        if kind != KIND_PARAMETER:
            return True
        if self.__round_fresh and self.accumulate and not self.__has_data:
            # the reference's per-name dicts start empty every round (:55-62): the round's first
            # update sets the names and their order (a layout equal to the last round's keeps its
            # context); later names grow it (_grow_layout). Only while nothing is staged: staged
            # rows and folded waves are laid out in the current layout.
            self.__round_fresh = False
            params = worker_data.parameter
            if isinstance(params, dict) and params and (self.__layout is None or tuple(params) != self.__layout.names):
                self._set_layout(params)
        w = worker_data.aggregation_weight
        if self.accumulate and self.__default_hooks and isinstance(w, (int, float)):
            # the default _accumulate_parameter / _get_weight / _note_total for every tensor of
            # the update (fed_avg_algorithm.py:43-69: the message's weight, the per-name total
            # += w in arrival order, the payload released), without a hook call per tensor
            params = worker_data.parameter
            if self._stage_natively(params, w):
                worker_data.parameter = {}
                return True
            self._materialize_totals()
            totals = self.__host_totals
            for name in params:
                if name in totals:
                    totals[name] += w
                else:
                    totals[name] = w
            self.__row = {name: (t, w) for name, t in params.items()}
            worker_data.parameter = {}
            self._stage_client(worker_id=worker_id)
            return True
        self.__row = {}
        self._materialize_totals()
        for name, parameter in worker_data.parameter.items():
            self._accumulate_parameter(worker_data=worker_data, name=name, parameter=parameter)
        if self.accumulate:
            self._stage_client(worker_id=worker_id)
        return True

    def _arrive_quick(self, worker_id: int, worker_data: Any) -> bool:
        """The common arrival in one short pass: a full ParameterMessage with a number weight,
        after the round's first arrival, into the wave's native table while it has room. The same
        state changes as the general flow below (the message recorded (aggregation_algorithm.py:
        93-102), its update appended to the wave (``Rows.append``), the totals += w (:59-62), the
        payload released (:64)); False with nothing changed for anything else."""
        table = self.__table
        if (type(table) is not NativeClientTable or self.__round_fresh or self.__ew is not False or self.__table_delta
                or self.__multi_devices is not None or not self.accumulate or not self.__default_hooks
                or message_kind(worker_data) != KIND_PARAMETER):
            return False
        w = worker_data.aggregation_weight
        params = worker_data.parameter
        fast = self.__fast
        if (type(w) not in (int, float) or type(params) is not dict or fast is None
                or fast[0] is not self.__layout or self._wave_due(table.num_clients)):
            return False
        want = _STAGING_CODES.get(self.__table_dtype, -3)
        if want == -3:
            return False
        rc = table.rows.append(params, fast[1], fast[2], w, want)
        if rc < 0:
            return False  # nothing changed: the general flow decides
        if rc & 16 and not self.__host_totals:
            self.__uniform_total = w if self.__uniform_count == 0 else self.__uniform_total + w
            self.__uniform_count += 1
        else:
            self._materialize_totals()
            totals = self.__host_totals
            for name in params:
                if name in totals:
                    totals[name] += w
                else:
                    totals[name] = w
        self._all_worker_data[worker_id] = worker_data
        self.__has_data = True
        worker_data.parameter = {}
        self._dyn_arrival()
        return True

    def _stage_natively(self, params: Any, w: Any, delta: bool = False) -> bool:
        """The default hooks' per-tensor walk of an update in one native call
        (csrc/staging_ext.cpp). A device-resident update is checked (known name, contiguous, on
        the device, one kernel dtype, the layout's shape) and written straight into the wave's
        native client table (``Rows.append``); the per-name totals `+= w` (:59-62) take one
        addition while every update of the round carries every name. A contiguous host update of
        one dtype is checked, its totals updated, and it is packed and moved by the pinned ingest
        from its pointers. ``delta``: the tensors are a DeltaParameterMessage's deltas, folded with
        restore() fused (x = old + delta). False (nothing changed) when the extension is absent or
        the update needs the general path."""
        if self.__ew or not isinstance(params, dict):
            return False
        fast = self.__fast
        if fast is None or fast[0] is not self.__layout:
            fast = self.__fast = self._fast_maps()
            if fast is None:
                return False
        _, index, shapes, dev_idx = fast
        if self.__table is not None and self._wave_due(self.__table.num_clients):
            self._flush()  # a full wave is folded when the next update arrives (see _stage_client)
        table = self.__table
        fresh = table is None
        want = -1
        if not fresh:
            want = _STAGING_CODES.get(self.__table_dtype, -3) if type(table) is NativeClientTable else -3
            if want == -3 or self.__table_delta != delta:
                want = -3  # the wave so far is not a native table of this kind: general path below
        if want != -3:
            if fresh:
                table = NativeClientTable(len(self.__keep), dev_idx)
            rc = table.rows.append(params, index, shapes, w, want)
            if rc <= -2:  # a valid update of another dtype: the wave so far is folded first
                self._flush()
                table, fresh = NativeClientTable(len(self.__keep), dev_idx), True
                rc = table.rows.append(params, index, shapes, w, -1)
            if rc >= 0:
                if rc & 16 and not self.__host_totals:
                    # a complete update while every total is still the same value
                    self.__uniform_total = w if self.__uniform_count == 0 else self.__uniform_total + w
                    self.__uniform_count += 1
                else:
                    self._materialize_totals()
                    totals = self.__host_totals
                    for name in params:
                        if name in totals:
                            totals[name] += w
                        else:
                            totals[name] = w
                if fresh:
                    self.__table = table
                    self.__table_dtype = _STAGING_DTYPES[rc & 15]
                    self.__table_delta = delta
                self.__ew = False
                self.__has_data = True
                self._dyn_arrival(next(iter(params.values()), None))
                return True
        first = next(iter(params.values()), None)
        host = isinstance(first, torch.Tensor) and first.device.type == "cpu"
        if not host and want != -3:
            return False  # a device update the native check refused: the general path
        self._materialize_totals()
        res = _staging.module().stage_resident(params, index, shapes, -1 if host else dev_idx,
                                               self.__host_totals, w)
        if res is None:
            return False
        ptrs, nums, weights, code, keep = res
        self.__ew = False
        dt = _STAGING_DTYPES[code]
        if host:
            # host update: one packed DMA per client through the pinned ingest (ingest.py), the
            # row's device pointers computed from the bucket's segment offsets
            if self.__ingest is None:
                self.__ingest = HostIngest(self.device)
            bucket, ptrs = self.__ingest.to_device_pointers(self.__native_layout, ptrs, nums, dt)
            keep = [bucket]
        if self.__table is not None and (self.__table_dtype != dt or self.__table_delta != delta):
            self._flush()
        if self.__table is None:
            self.__table = self._new_table(dev_idx)
            self.__table_dtype = dt
            self.__table_delta = delta
        self.__table.add_resident_client(ptrs, weights, nums, dt.itemsize, dev_idx, keep)
        self.__has_data = True
        if host:
            # host rows: the round is PCIe-bound (the fold hides behind the DMAs), so no wave holds
            # the GPU for it — nor, pre-opened, for the next round
            self.__dyn.not_this_round()
        elif type(self.__table) is NativeClientTable:
            self._dyn_arrival(keep[0] if keep else None)
        else:
            self.__dyn.not_this_round()
        return True

    def _fast_maps(self) -> tuple | None:
        """(layout, name -> native segment, native shapes, device index) of the native staging,
        or None where it does not apply (no extension, no GPU device, eager NaN scans, nothing
        native in the layout)."""
        if (_staging.module() is None or self.__native_layout is None or self.__layout is None
                or self.eager_nan_check):
            return None
        dev = self.device
        if dev.type != "cuda":
            return None
        dev_idx = dev.index if dev.index is not None else torch.cuda.current_device()
        index = {n: -1 for n in self.__layout.names}
        for j, i in enumerate(self.__keep):
            index[self.__layout.names[i]] = j
        shapes = [tuple(self.__layout.shapes[i]) for i in self.__keep]
        return (self.__layout, index, shapes, dev_idx)

    def _materialize_totals(self) -> None:
        """Write the running total of the complete updates into every name's total (what the
        reference's dict holds at this point: each name saw exactly those updates, in order)."""
        if self.__uniform_count:
            assert self.__layout is not None and not self.__host_totals
            total = self.__uniform_total
            self.__host_totals = {name: total for name in self.__layout.names}
            self.__uniform_total, self.__uniform_count = None, 0

    def _new_table(self, dev_idx: int) -> ClientTable | NativeClientTable:
        """The wave's client table: native rows when the staging extension is built (scalar
        weights), else the Python table; per-element weights always take the Python table."""
        if not self.__ew and _staging.module() is not None and self.device.type == "cuda":
            return NativeClientTable(len(self.__keep), dev_idx)
        return ClientTable(len(self.__keep))

    def _restore_on_host(self, worker_id: int, worker_data: Any) -> Any:
        """A delta the fold cannot take (consistency-check fields, the ratio path, per-element
        weights): restore it with its own restore() exactly as the reference server does
        (aggregation_server.py:123-125) and keep the full update in its place."""
        assert self._old_parameter is not None, "a delta update needs the cached global model"
        restored = worker_data.restore(self._old_parameter)
        self._all_worker_data[worker_id] = restored
        return restored

    # The server hands DeltaParameterMessages straight to this algorithm (with the cached global
    # model set through set_old_parameter) instead of restoring them on the host first.
    accepts_delta_messages = True

    def _delta_fusable(self, msg: DeltaParameterMessage) -> bool:
        # the consistency-check fields of restore() (message.py:42-59) need the host path
        return self._old_parameter is not None and msg.old_parameter is None and msg.new_parameter is None

    def set_old_parameter(self, old_parameter: ModelParameter) -> None:
        if old_parameter is not self._old_parameter:
            self.__base = None
            for lane in self.__lanes:
                lane["_FedAVGAlgorithm__base"] = None
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
        self._note_total(name, weight, parameter)
        # host tensors are packed and DMA'd per client in _stage_client (ingest.HostIngest)
        self.__row[name] = (parameter, weight)
        # release to reduce memory pressure (fed_avg_algorithm.py:63-64)
        worker_data.parameter = {}

    def _note_total(self, name: str, weight: Any, parameter: Any) -> None:
        """fed_avg_algorithm.py:59-62 with the hook's own objects (a 0-dim tensor total stays a
        tensor of its dtype, updated in place). Per-element totals live on the GPU instead."""
        if _is_elementwise(weight, parameter):
            return
        if name not in self.__host_totals:
            self.__host_totals[name] = weight
        else:
            self.__host_totals[name] += weight

    def _get_weight(self, worker_data: ParameterMessage, name: str, parameter: Any) -> Any:
        return worker_data.aggregation_weight

    def _apply_total_weight(self, name: str, parameter: torch.Tensor, total_weight: Any) -> torch.Tensor:
        return parameter / total_weight

    def _stage_client(self, delta: bool = False, worker_id: int | None = None) -> None:
        row = self.__row
        self.__row = {}
        if not row:
            return
        if self.__layout is None:
            self._set_layout({k: v[0] for k, v in row.items()})
        assert self.__layout is not None
        known = set(self.__layout.names)
        unknown = [k for k in row if k not in known]
        if unknown:
            if delta:
                raise NotImplementedError(f"delta tensors {unknown} are not in the cached global model")
            self._grow_layout(unknown, row)
        if self.__native_layout is None:
            self.__has_data = True
            return
        ew_here = any(_is_elementwise(w, t) for t, w in row.values())
        if self.__ew is None:
            self.__ew = ew_here
        elif ew_here and not self.__ew:
            raise NotImplementedError(
                "per-element weights must be returned from the round's first update on "
                "(the reference's scalar total cannot be added in place into a tensor, fed_avg_algorithm.py:62)"
            )
        tensors: list[torch.Tensor | None] = []
        weights: list[float] = []
        weight_tensors: list[torch.Tensor | None] = []
        names, shapes, ew = self.__layout.names, self.__layout.shapes, self.__ew
        dev = self.device
        dev_idx = dev.index if dev.index is not None else (torch.cuda.current_device() if dev.type == "cuda" else -1)
        # the common arrival — dense tensors of one kernel dtype, contiguous, already on this
        # device — is recognised in this one pass and staged without the general path's passes
        in_place, dtypes = True, set()
        # the client-table row of the common arrival, built in the same pass (pointers, sizes)
        ptrs: list[int] = []
        nums: list[int] = []
        keep: list[torch.Tensor] = []
        numels = self.__layout.numels
        for i in self.__keep:
            name = names[i]
            if name in row:
                t, w = row[name]
                if t.shape != shapes[i]:  # torch.Size / tuple compare as tuples
                    raise ValueError(f"shape of {name} changed: {tuple(t.shape)} vs {shapes[i]}")
                assert w is not None, "aggregation_weight is None"
                tensors.append(t)
                if in_place:
                    if isinstance(t, torch.Tensor) and t.get_device() == dev_idx and t.is_contiguous():
                        dtypes.add(t.dtype)
                        ptrs.append(t.data_ptr())
                        nums.append(numels[i])
                        keep.append(t)
                    else:
                        in_place = False
                if ew:
                    self.__tot_fp32.setdefault(name, _total_is_fp32(w))
                    if _is_elementwise(w, t):
                        wt = w.detach().to(device=dev).contiguous()
                        if wt.dtype not in (torch.float32, torch.float64):
                            wt = wt.to(torch.float64)
                        weight_tensors.append(wt)
                        weights.append(0.0)
                        continue
                weight_tensors.append(None)
                weights.append(float(w))
            else:
                tensors.append(None)
                weights.append(0.0)
                weight_tensors.append(None)
                ptrs.append(0)
                nums.append(-1)
        resident = False
        q_row: tuple | None = None  # (device pointers, record bytes, keep) of packed host records
        if in_place and len(dtypes) == 1 and next(iter(dtypes)) in _KERNEL_DTYPES:
            dt = next(iter(dtypes))
            resident = True
        elif in_place and not dtypes:
            dt = self.__table_dtype or torch.float32
        else:
            present = [t for t in tensors if t is not None]
            codecs = {t.codec for t in present if isinstance(t, QuantizedTensor)}
            if codecs and len(codecs) == 1 and all(isinstance(t, QuantizedTensor) for t in present) and not ew:
                # quantised update: the records are the kernel operands (dequantised in the fold)
                dt = codecs.pop()
                recs = [None if t is None else t.record for t in tensors]
                if self.settings.qsgd_host_pointers and not self.eager_nan_check and \
                        all(r is None or (r.device.type == "cpu" and r.is_contiguous()) for r in recs):
                    # host records: packed from their pointers, one DMA, row pointers from the
                    # bucket offsets (no per-record views, no second per-record pass)
                    q_row = self._host_records_to_device(tensors, recs)
                else:
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
        if self.eager_nan_check:
            self._scan_arrival(tensors, dt, worker_id, delta)
        # A full wave is folded when the next update arrives, not when it fills: the round's last
        # wave then always reaches aggregate_worker_data unfolded and is folded and divided in one
        # launch (fedavg_aggregate) instead of an accumulate launch plus a finalize pass.
        if self.__table is not None and (self.__table_dtype != dt or self.__table_delta != delta
                                         or self._wave_due(self.__table.num_clients)):
            self._flush()
        if self.__table is None:
            self.__table = self._new_table(dev_idx)
            self.__table_dtype = dt
            self.__table_delta = delta
        if resident and not self.__ew:
            self.__table.add_resident_client(ptrs, weights, nums, dt.itemsize, dev_idx, keep)
        elif q_row is not None:
            self.__table.add_resident_client(q_row[0], weights, q_row[1], 1, dev_idx, q_row[2])
        else:
            self.__table.add_client(tensors, weights, weight_tensors if self.__ew else None)
        self.__has_data = True
        if resident and type(self.__table) is NativeClientTable:
            self._dyn_arrival(keep[0] if keep else None)
        else:
            self.__dyn.not_this_round()  # host / converted rows, quantised records, per-element weights

    def _scan_arrival(self, tensors: list, dt: Any, worker_id: int | None, delta: bool) -> None:
        """fed_avg_algorithm.py:34-35 at the arrival: one GPU scan of the staged update."""
        if delta:
            return  # the delta fold restores first; its NaN surfaces at the flush (:93)
        t1 = ClientTable(len(tensors))
        t1.add_client(tensors, [1.0] * len(tensors))
        if self._context().find_nan_clients(t1, dt):
            raise NaNAggregationError("input", f"NaN in the update of worker {worker_id} (fed_avg_algorithm.py:35)",
                                      [worker_id] if worker_id is not None else [])

    def _to_device_row(self, tensors: list[torch.Tensor | None]) -> list[torch.Tensor | None]:
        """One client's tensors in HBM. Host tensors of one kernel dtype go through the pinned
        ingest (one packed DMA per client); anything else moves tensor by tensor."""
        host = [t for t in tensors if t is not None and not t.is_cuda]
        if not host:
            dev = self.device
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
            # device tensors already in place (the common case) are used as they are
            return [t if t is None or (t.get_device() == idx and t.is_contiguous()) else to_device_operand(t, dev)
                    for t in tensors]
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

    # Quantised updates (StochasticQuantServerEndpoint / NNADQServerEndpoint, quantized_endpoint.py:
    # 69-77,102-142) are handed over as QSGD / NNADQ records; the kernel dequantises them inside
    # the fold.
    accepts_quantized_messages = True

    def _host_records_to_device(self, tensors: list, recs: list) -> tuple[list[int], list[int], list]:
        """One client's host QSGD records through the pinned ingest by pointer (HostIngest
        .to_device_pointers): (device pointers, record bytes (-1 absent), [bucket])."""
        if self.__ingest is None:
            self.__ingest = HostIngest(self.device)
        numels = tuple(1 if q is None else q.numel for q in tensors)
        codec = next(q.codec for q in tensors if q is not None)
        rl = self.__record_layouts.get((numels, codec))
        if rl is None:
            rl = self.__record_layouts[(numels, codec)] = record_layout(list(numels), codec)
        nums = [-1 if r is None else r.numel() for r in recs]
        bucket, dptrs = self.__ingest.to_device_pointers(rl, [0 if r is None else r.data_ptr() for r in recs],
                                                         nums, torch.uint8)
        return dptrs, nums, [bucket]

    def _records_to_device(self, tensors: list) -> list[torch.Tensor | None]:
        """One client's QSGD records in HBM: host records go through the pinned ingest (one
        packed DMA per client), device records are used where they are."""
        host = [q for q in tensors if q is not None and q.device.type == "cpu"]
        moved: list[torch.Tensor | None] = [None] * len(tensors)
        if host:
            if self.__ingest is None:
                self.__ingest = HostIngest(self.device)
            numels = tuple(q.numel if q is not None else 1 for q in tensors)
            codec = host[0].codec
            rl = self.__record_layouts.get((numels, codec))
            if rl is None:
                rl = self.__record_layouts[(numels, codec)] = record_layout(list(numels), codec)
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

    def _ew_totals_buffer(self) -> torch.Tensor:
        """Per-element totals (fp64, accumulator coordinates) of the elementwise fold."""
        ctx = self._context()
        if self.__ew_totals is None or self.__ew_totals.numel() != ctx.acc_numel:
            self.__ew_totals = torch.zeros(ctx.acc_numel, dtype=torch.float64, device=self.device)
        return self.__ew_totals

    def _tot_fp32_flags(self) -> list[bool]:
        assert self.__native_layout is not None
        return [self.__tot_fp32.get(n, False) for n in self.__native_layout.names]

    def _wave_due(self, staged: int) -> bool:
        """Fold the staged wave before the arriving update joins it: it is full, or it holds at
        least ``wave_min`` clients and the GPU has finished every wave flushed so far."""
        if staged >= self.wave_size:
            return True
        if not self.wave_min or staged < self.wave_min:
            return False
        ev = self.__wave_event
        return ev is None or ev.query()

    # ---- the dynamic wave (algorithm/dynamic_wave.py) -----------------------------------
    def _dyn_eligible(self) -> bool:
        """The round may fold through a dynamic wave (one device, the default hooks, no early
        waves or eager scans, scalar weights, full updates)."""
        return (self.dynamic_wave and self.device.type == "cuda" and self.__multi_devices is None and self.accumulate
                and self.__default_hooks and not self.wave_min and not self.eager_nan_check
                and self.__ew is not True and not self.__table_delta and self.__native_layout is not None)

    def _dyn_arrival(self, probe: Any = None) -> None:
        """A device-resident row joined the table (``probe``: one of its tensors, checked at the
        round's first row only)."""
        dyn = self.__dyn
        if dyn.table is not None:
            dyn.more(self.__table)  # the common arrival: at most one publication
        elif not dyn.decided:
            dyn.arrival(self.__table, self._context,
                        self._dyn_eligible() and self.__ew is False and not self._shared_device(probe),
                        self.__table_dtype, self.wave_size)

    @staticmethod
    def _device_update(worker_data: Any) -> bool:
        """The update's first tensor is already on a GPU (a round that may take a wave: host
        updates never do, so no wave is opened ahead of them)."""
        payload = getattr(worker_data, "parameter", None)
        if not isinstance(payload, dict) or not payload:
            return False
        first = next(iter(payload.values()))
        return isinstance(first, torch.Tensor) and first.is_cuda

    @staticmethod
    def _shared_device(t: Any) -> bool:
        """The row's memory came from another process (CUDA IPC from a worker — which then holds a
        context on this GPU and computes there — or external memory): the wave stays off for the
        round, since its workgroups hold the register file while they wait for rows."""
        ext = _staging.module()
        return isinstance(t, torch.Tensor) and ext is not None and bool(ext.foreign(t))

    def _flush(self) -> None:
        """Fold the staged wave into the device accumulator (one kernel launch)."""
        self.__dyn.unpre()
        if self.__table is None or self.__table.num_clients == 0:
            return
        ctx = self._context()
        table, dt = self.__table, self.__table_dtype
        assert dt is not None
        self.__table, self.__table_dtype = None, None
        self.__dyn.flush(table)  # a full dynamic wave: its rows stay in the accumulator
        table = self.__dyn.rest(table)
        if table is None:
            return
        if self.__ew:
            ctx.accumulate_elementwise(table, dt, self._ew_totals_buffer(), self._tot_fp32_flags())
        elif self.__table_delta:
            ctx.accumulate_delta(table, dt, self._delta_base())
        else:
            ctx.accumulate(table, dt)
        if self.wave_min:
            if self.__wave_event is None:
                self.__wave_event = torch.cuda.Event()
            self.__wave_event.record(torch.cuda.current_stream(self.device))

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
        try:
            if self.__native_layout is not None:
                result.update(self._finish_native())
        finally:
            self._reset_round()
        if len(self.__keep) == layout.num_segments:
            out = result  # no zero-element tensors: the native segments are the layout, in order
        else:
            kept = set(self.__keep)
            for i, name in enumerate(layout.names):
                if i not in kept:
                    result[name] = torch.empty(layout.shapes[i], dtype=self.result_dtype, device=self.device)
            out = {name: result[name] for name in layout.names}
        if self.result_device is not None:
            out = self._move_result(out)
        return out

    def _reset_round(self) -> None:
        self.__dyn.end_round(self.__round_updates)  # an abandoned round's wave ends with its rows
        self.__round_updates = 0
        self.__arrivals = 0
        self.__has_data = False
        self.__host_totals = {}
        self.__uniform_total, self.__uniform_count = None, 0
        self.__round_fresh = True
        self.__ew = None
        self.__tot_fp32 = {}

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
        self.__dyn.unpre()
        if self.__dyn.table is not None and self.__dyn.table is self.__table:
            self.__dyn.publish()  # the last rows to the wave first: it folds them while the result is prepared
        if self.__multi_devices is not None:
            if not self.__ew:
                return self._finish_multi()
            self._select_lane(0)  # a round of per-element weights lives on the first entry
        ctx = self._context()
        native = self.__native_layout
        layout = self.__layout
        assert native is not None and layout is not None
        table, dt = self.__table, self.__table_dtype
        self.__table, self.__table_dtype = None, None
        pending = [(table, dt)] if table is not None and dt is not None else []
        custom_divide = type(self)._apply_total_weight is not FedAVGAlgorithm._apply_total_weight
        # a 0-dim tensor (or other non-number) total: divide by the host total the reference has
        # (the one running total of complete updates is always a number)
        host_divide = False
        if not self.__ew and not (self.__uniform_count and not self.__host_totals):
            self._materialize_totals()
            host_divide = any(not isinstance(self.__host_totals.get(layout.names[i], 0), (int, float))
                              for i in self.__keep)
        out_dtype = torch.float64 if custom_divide else self.result_dtype
        offs, total, shapes = self._result_geometry(out_dtype)
        flat, outs, views = self._result_buffer(out_dtype, reuse=not custom_divide)
        self.__result_flat = None if custom_divide else flat
        delta = self.__table_delta and table is not None
        # the dynamic wave wrote the result (else its rows are in the accumulator: the rest below)
        done = self.__dyn.finish(table, None if (self.__ew or custom_divide or host_divide or delta) else outs,
                                 out_dtype, torch.cuda.current_stream(self.device)) if table is not None else False
        if not done and table is not None:
            table = self.__dyn.rest(table)
        try:
            if done:
                pass
            elif self.__ew:
                if table is not None and dt is not None:
                    ctx.accumulate_elementwise(table, dt, self._ew_totals_buffer(), self._tot_fp32_flags())
                if not custom_divide:
                    ctx.finalize_elementwise(self._ew_totals_buffer(), outs, out_dtype)
                else:
                    ctx.set_accumulated([1.0] * native.num_segments)
                    ctx.finalize_range(outs, torch.float64)
            elif not custom_divide and not host_divide:
                if delta:
                    ctx.aggregate_delta(table, dt, self._delta_base(), outs, out_dtype)
                else:
                    ctx.aggregate(table, dt or torch.float32, outs, out_dtype)
            else:
                # fold the last wave, then divide by the host totals (exact float values of the
                # reference's total objects) or by 1 for a subclass hook (exact: x / 1.0 == x)
                if table is not None and dt is not None:
                    if delta:
                        ctx.accumulate_delta(table, dt, self._delta_base())
                    else:
                        ctx.accumulate(table, dt)
                if custom_divide:
                    ctx.set_accumulated([1.0] * native.num_segments)
                    ctx.finalize_range(outs, torch.float64)
                else:
                    ctx.set_accumulated([float(self.__host_totals[layout.names[i]]) for i in self.__keep])
                    ctx.finalize_range(outs, out_dtype)
            result: ModelParameter = {}
            if not custom_divide:
                # the segments as shaped views of the flat result (one native call when the staging
                # extension is built), made while the kernel runs — or the reused buffer's own
                if views is None:
                    views = self._result_views(flat, outs, out_dtype)
                for j, i in enumerate(self.__keep):
                    result[layout.names[i]] = views[j]
            ctx.raise_on_nan(pending)  # the round ends on the host: :93 / :97 asserted
        except NaNAggregationError:
            ctx.reset()
            raise
        if not custom_divide:
            ctx.reset()
            return result
        # a subclass's _apply_total_weight runs where the reference runs it — on host fp64
        # tensors (torch's GPU division by a scalar multiplies by its reciprocal, which does not
        # round like the reference's CPU division); one D2H copy of the weighted sums
        host = torch.empty(flat.shape, dtype=flat.dtype, pin_memory=True)
        host.copy_(flat)
        self._materialize_totals()
        for j, i in enumerate(self.__keep):
            name = layout.names[i]
            total = self._total_for(name, j)
            if isinstance(total, torch.Tensor):
                total = total.cpu()
            value = host[offs[j] : offs[j] + native.numels[j]].view(layout.shapes[i])
            value = self._apply_total_weight(name=name, parameter=value, total_weight=total)
            assert not value.isnan().any()  # fed_avg_algorithm.py:97
            result[name] = value.to(device=self.device, dtype=self.result_dtype)
        ctx.reset()
        return result

    def _finish_multi(self) -> ModelParameter:
        """The end of a multi-device round: every entry folds its last wave into its accumulator
        (its shard's arrival-order partial), then the partials are summed in entry order on the
        GPUs and divided by the round's arrival-order totals into the first entry's device
        (``MultiDeviceContext.combine``), with the reference's NaN assertions."""
        native, layout = self.__native_layout, self.__layout
        assert native is not None and layout is not None
        pending: list[list[tuple[ClientTable, Any]]] = []
        for g in range(len(self.__lanes)):
            self._select_lane(g)
            table, dt = self.__table, self.__table_dtype
            pending.append([(table, dt)] if table is not None and dt is not None else [])
            self._flush()
        self._select_lane(0)
        m = self._multi()
        custom_divide = type(self)._apply_total_weight is not FedAVGAlgorithm._apply_total_weight
        if custom_divide:
            totals = [1.0] * native.num_segments  # x / 1.0 == x: the hook divides on the host
        elif self.__uniform_count and not self.__host_totals:
            totals = [float(self.__uniform_total)] * native.num_segments
        else:
            self._materialize_totals()
            totals = [float(self.__host_totals[layout.names[i]]) for i in self.__keep]
        out_dtype = torch.float64 if custom_divide else self.result_dtype
        offs, total, shapes = self._result_geometry(out_dtype)
        flat, outs, views = self._result_buffer(out_dtype, reuse=not custom_divide)
        self.__result_flat = None if custom_divide else flat
        try:
            m.combine(totals, outs, out_dtype, root=0, exchange=self.exchange)
        except Exception:
            m.reset()
            raise
        m.raise_on_nan(pending)  # the round ends on the host: :35 / :93 / :97 asserted
        result: ModelParameter = {}
        if not custom_divide:
            if views is None:
                views = self._result_views(flat, outs, out_dtype)
            for j, i in enumerate(self.__keep):
                result[layout.names[i]] = views[j]
            return result
        host = torch.empty(flat.shape, dtype=flat.dtype, pin_memory=True)
        host.copy_(flat)
        self._materialize_totals()
        for j, i in enumerate(self.__keep):
            name = layout.names[i]
            tot = self._total_for(name, j)
            if isinstance(tot, torch.Tensor):
                tot = tot.cpu()
            value = host[offs[j] : offs[j] + native.numels[j]].view(layout.shapes[i])
            value = self._apply_total_weight(name=name, parameter=value, total_weight=tot)
            assert not value.isnan().any()  # fed_avg_algorithm.py:97
            result[name] = value.to(device=self.device, dtype=self.result_dtype)
        return result

    def _result_geometry(self, out_dtype: torch.dtype) -> tuple[list[int], int, list[tuple[int, ...]]]:
        """(element offsets, flat size, shapes) of the native segments in a flat result buffer of
        ``out_dtype`` — cached per layout, reused every round."""
        native = self.__native_layout
        assert native is not None and self.__layout is not None
        key = (native, out_dtype)
        geo = self.__result_geo.get(key)
        if geo is None:
            offs, total = native.padded_offsets(torch.empty((), dtype=out_dtype).element_size())
            geo = (list(offs), int(total), [tuple(self.__layout.shapes[i]) for i in self.__keep])
            self.__result_geo = {key: geo}
        return geo

    def _result_buffer(self, out_dtype: torch.dtype, reuse: bool = True) -> tuple[torch.Tensor, OutputTable, list | None]:
        """(flat result buffer, its OutputTable, its segment views or None) for this round. The
        reference hands out fresh tensors every round; a buffer of an earlier round is written
        again only when nothing outside this object can still see it — no result tensor, view of
        one or storage handle kept by the caller, no in-place change to the views
        (``unobserved``, csrc/staging_ext.cpp) — so no caller can tell the difference. Otherwise
        (or with ``reuse`` False) a fresh buffer; its views are made by ``_result_views``."""
        native = self.__native_layout
        assert native is not None
        offs, total, shapes = self._result_geometry(out_dtype)
        pool, ext = self.__result_pool, _staging.module()
        if reuse and pool is not None and ext is not None and pool[0] == (native, out_dtype, self.device):
            _, flat, outs, views = pool
            if ext.unobserved(flat, views, offs, shapes):
                return flat, outs, views
        self.__result_pool = None  # the old buffer stays with whoever still holds its results
        flat = torch.empty(total, dtype=out_dtype, device=self.device)
        return flat, OutputTable.from_flat(flat, offs, native), None

    def _result_views(self, flat: torch.Tensor, outs: OutputTable, out_dtype: torch.dtype) -> list[torch.Tensor]:
        """The segments of a fresh result buffer as shaped views (one native call when the staging
        extension is built); the buffer joins the pool for a later round."""
        native = self.__native_layout
        assert native is not None
        offs, _, shapes = self._result_geometry(out_dtype)
        ext = _staging.module()
        if ext is None:
            return [flat[o : o + n].view(sh) for o, n, sh in zip(offs, native.numels, shapes)]
        views = ext.views(flat, offs, shapes)
        self.__result_pool = ((native, out_dtype, self.device), flat, outs, views)
        return views

    def _total_for(self, name: str, seg: int) -> Any:
        """The total object the reference hands _apply_total_weight (fed_avg_algorithm.py:95)."""
        if not self.__ew:
            return self.__host_totals[name]
        ctx = self._context()
        native = self.__native_layout
        assert native is not None
        o = ctx.segment_offset(seg)
        tot = self._ew_totals_buffer()[o : o + native.numels[seg]].view(native.shapes[seg])
        return tot.to(torch.float32) if self.__tot_fp32.get(name) else tot.clone()

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
        for g in range(len(self.__lanes)):
            self._select_lane(g)
            self.__table, self.__table_dtype = None, None
        if self.__lanes:
            self._select_lane(0)
        self.__table, self.__table_dtype = None, None
        self.__row = {}
        self._reset_round()
        if self.__ctx is not None:
            self.__ctx.reset()
        if self.__multi is not None:
            self.__multi.reset()

    def exit(self) -> None:
        self.__result_pool = None
        if self.__ctx is not None:
            self.__ctx.close()
            self.__ctx = None
        if self.__multi is not None:
            self.__multi.close()
            self.__multi = None

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
