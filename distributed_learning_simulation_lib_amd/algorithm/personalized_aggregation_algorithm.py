"""PersonalizedFedAVG on MI355X: every receiver's FedAvg and the centralized average in one launch.

Same plugin surface as the reference's ``PersonalizedFedAVGAlgorithm``
(``simulation_lib/algorithm/personalized_aggregation_algorithm.py:9-57``):
``set_worker_weights`` (:15-21), ``process_worker_data`` (:23-43), ``aggregate_worker_data``
(:45-57) returning a ``MultipleWorkerMessage`` whose ``worker_data`` holds one
``ParameterMessage`` per receiver (in ``worker_weights`` key order) and whose
``other_data["centralized_parameter"]`` is the equal-weight average of them.

The reference deep-copies every arriving update into M-1 per-receiver ``FedAVGAlgorithm``s
and reduces each on the CPU (M² fp64 passes over the model). Here an arrival is staged once
in HBM and, at the end of the round, one HIP launch folds all N arrivals into all M receivers
(arrival-order fp64 chains, bit-identical to the reference) and the centralized average
(``personalized_kernels.hip``). Observable differences (as for ``FedAVGAlgorithm``): the NaN
assertions fire at ``aggregate_worker_data``, results are float64 tensors on the GPU (or on
``result_device``), and a tensor name absent from the first arrival raises
``NotImplementedError``.
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch

from .. import _native, _staging
from ..fedavg import ModelLayout, NaNAggregationError
from ..ingest import HostIngest
from ..message import Message, ModelParameter, MultipleWorkerMessage, ParameterMessage, is_parameter_message, wire_class
from ..personalized import FlatOutputs, PersonalizedContext
from .aggregation_algorithm import (
    AggregationAlgorithm,
    context_for,
    default_device,
    split_empty,
    to_device_operand,
    unify_dtype,
)


_STAGING_DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.float64)  # staging_ext.cpp codes


class PersonalizedFedAVGAlgorithm(AggregationAlgorithm):
    def __init__(
        self,
        device: torch.device | str | None = None,
        result_dtype: torch.dtype = torch.float64,
        result_device: torch.device | str | None = None,
    ) -> None:
        super().__init__()
        self._worker_weights: dict[int, dict[int, float]] = {}
        self._device = torch.device(device) if device is not None else None
        self.result_dtype = result_dtype
        self.result_device = torch.device(result_device) if result_device is not None else None
        self.__arrivals: list[tuple[int, ParameterMessage, list[torch.Tensor | None]]] = []
        self.__layout: ModelLayout | None = None
        self.__ctx: PersonalizedContext | None = None
        self.__ingest: HostIngest | None = None
        self.__stage_maps: tuple | None = None  # (layout, name -> position, shapes) for staging_ext
        # dtype codes of this round's natively staged arrivals (None once one took the general path)
        self.__native_codes: set[int] | None = set()
        self.__ptr_rows: list[bytes] = []  # the natively staged arrivals' device addresses
        # ((receivers, arrival ids), [M][N] weights, copies of the receivers' weight dicts)
        self.__weights_memo: tuple | None = None
        self.__geometry: tuple | None = None  # (native layout, offsets, flat size, shapes)
        # (key, [(buffer, views)] per receiver, (buffer, views) centralized) of the last round's
        # result buffers, written again only while nobody outside can see them (_result_rows)
        self.__result_pool: tuple | None = None

    @property
    def device(self) -> torch.device:
        if self._device is None:
            self._device = default_device()
        return self._device

    # :15-21
    def set_worker_weights(self, worker_weights: dict[int, dict[int, float]]) -> None:
        assert not self._worker_weights
        self._worker_weights = worker_weights

    # :23-43 — the update is staged once in HBM instead of deep-copied per receiver
    def process_worker_data(self, worker_id: int, worker_data: Message | None) -> bool:
        assert self._worker_weights
        if worker_data is None:
            return True  # every receiver records a skipped worker (aggregation_algorithm.py:98-100)
        if not any(j != worker_id for j in self._worker_weights):
            return True  # nobody else receives it: the reference never touches it
        assert is_parameter_message(worker_data)
        if self.__layout is None:
            self.__layout = ModelLayout.from_parameters(worker_data.parameter)
        staged = self._resident_row(worker_data.parameter)
        if staged is not None:
            row_native, code, ptr_row = staged
            self.__arrivals.append((worker_id, worker_data, row_native))
            if self.__native_codes is not None:
                self.__native_codes.add(code)
                self.__ptr_rows.append(ptr_row)
            return True
        self.__native_codes = None
        unknown = [k for k in worker_data.parameter if k not in self.__layout.names]
        if unknown:
            raise NotImplementedError(
                f"tensors {unknown} were not in the first update; complete() the message against the "
                "global model first (aggregation_server.py:126-128)"
            )
        row: list[torch.Tensor | None] = []
        for name, shape in zip(self.__layout.names, self.__layout.shapes):
            t = worker_data.parameter.get(name)
            if t is not None and tuple(t.shape) != shape:
                raise ValueError(f"shape of {name} changed: {tuple(t.shape)} vs {shape}")
            row.append(t)
        self.__arrivals.append((worker_id, worker_data, self._to_device_row(row)))
        return True

    def _resident_row(self, params: Any) -> tuple[list[torch.Tensor | None], int, bytes] | None:
        """An update already in HBM (contiguous, one kernel dtype, the layout's names and shapes)
        in layout order with its dtype code and device addresses, checked in one native call
        (csrc/staging_ext.cpp); None: the general path below (which also raises the errors)."""
        ext = _staging.module()
        dev = self.device
        if ext is None or dev.type != "cuda" or not isinstance(params, dict):
            return None
        layout = self.__layout
        assert layout is not None
        if self.__stage_maps is None or self.__stage_maps[0] is not layout:
            self.__stage_maps = (layout, {n: i for i, n in enumerate(layout.names)},
                                 [tuple(sh) for sh in layout.shapes])
        _, index, shapes = self.__stage_maps
        res = ext.resident_row(params, index, shapes,
                               dev.index if dev.index is not None else torch.cuda.current_device())
        return None if res is None else (res[0], res[1], res[2])

    def _to_device_row(self, row: list[torch.Tensor | None]) -> list[torch.Tensor | None]:
        assert self.__layout is not None
        host = [t for t in row if t is not None and t.device.type == "cpu"]
        dtypes = {t.dtype for t in host}
        if host and len(host) == sum(t is not None for t in row) and len(dtypes) == 1 and \
                next(iter(dtypes)) in (torch.float32, torch.float16, torch.bfloat16, torch.float64):
            # one packed DMA per client through pinned memory (ingest.py)
            if self.__ingest is None:
                self.__ingest = HostIngest(self.device)
            return self.__ingest.to_device(self.__layout, row, next(iter(dtypes)))
        return [None if t is None else to_device_operand(t, self.device) for t in row]

    # :45-57
    def aggregate_worker_data(self) -> MultipleWorkerMessage:
        receivers = list(self._worker_weights)
        folded = {j: [n for n, (wid, _, _) in enumerate(self.__arrivals) if wid != j] for j in receivers}
        for j in receivers:
            # a receiver that heard from nobody: FedAVGAlgorithm._aggregate_parameter's
            # `assert self.__parameter` (fed_avg_algorithm.py:88)
            assert folded[j], f"receiver {j} received no update"
        layout = self.__layout
        assert layout is not None
        msgs_of: dict[int, list[Message]] = {}

        def receivers_messages() -> None:
            # the receiver's FedAVGAlgorithm keeps _all_worker_data[worker_id] = update: a worker
            # that reported twice keeps its first position and its last message (built while the
            # kernel runs)
            for j in receivers:
                by_id: dict[int, Message] = {}
                for n in folded[j]:
                    by_id[self.__arrivals[n][0]] = self.__arrivals[n][1]
                msgs_of[j] = list(by_id.values())

        parameters, central = self._reduce(receivers, under_kernel=receivers_messages)
        if not msgs_of:
            receivers_messages()
        # answer in the caller's wire classes (the reference server matches
        # `case MultipleWorkerMessage()`, aggregation_server.py:84-86)
        like = self.__arrivals[0][1] if self.__arrivals else None
        param_cls = wire_class(like, "ParameterMessage")
        results: dict[int, ParameterMessage] = {}
        # no arrival carries other_data: every receiver's merge is an empty dict (:136-149)
        no_other = all(not getattr(m, "other_data", None) for _, m, _ in self.__arrivals)
        for j in receivers:
            msgs = msgs_of[j]
            results[j] = param_cls(
                parameter=parameters[j],
                end_training=msgs[0].end_training,
                in_round=msgs[0].in_round,
                other_data={} if no_other else self._check_and_reduce_other_data(msgs),
            )
        return wire_class(like, "MultipleWorkerMessage")(worker_data=results,
                                                         other_data={"centralized_parameter": central})

    def _reduce(self, receivers: list[int], under_kernel: Any = None) -> tuple[dict[int, ModelParameter], ModelParameter]:
        layout = self.__layout
        assert layout is not None
        native, keep = split_empty(layout)
        M = len(receivers)
        out: dict[int, ModelParameter] = {j: {} for j in receivers}
        central: ModelParameter = {}
        whole = native is not None and len(keep) == layout.num_segments
        if native is not None:
            codes = self.__native_codes
            client_ptrs = None
            if whole and codes is not None and len(codes) == 1:
                # every arrival staged natively in one kernel dtype, no empty tensors: the rows are
                # already the kernel's operands, checked and addressed at arrival
                rows = [row for _, _, row in self.__arrivals]
                dt = _STAGING_DTYPES[next(iter(codes))]
                client_ptrs = b"".join(self.__ptr_rows)
            else:
                rows = [[row[i] for i in keep] for _, _, row in self.__arrivals]
                present = [t for r in rows for t in r if t is not None]
                unified, dt = unify_dtype(present)
                it = iter(unified)
                rows = [[None if t is None else next(it) for t in r] for r in rows]
            ids = [wid for wid, _, _ in self.__arrivals]
            weights = self._weights(receivers, ids)
            if self.__ctx is None or self.__ctx.layout != native or self.__ctx.device != self.device:
                if self.__ctx is not None:
                    self.__ctx.close()
                self.__ctx = PersonalizedContext(native, self.device)
            res_dtype = self.result_dtype if self.result_dtype in (torch.float32, torch.float64) else torch.float64
            offs, padded, shapes = self._geometry(native)
            rows_out, cent_out = self._result_rows(native, M, res_dtype, offs, padded, shapes)
            try:
                self.__ctx.aggregate(rows, dt, ids, weights, receivers,
                                     FlatOutputs([b for b, _ in rows_out], offs), res_dtype,
                                     FlatOutputs([cent_out[0]], offs), torch.float64, client_ptrs)
            except _native.NativeError as e:
                if e.status == _native.ERR_STATE:
                    # every update a receiver folds lacks some tensor: the reference would leave
                    # the key out of that receiver's model; complete() the messages instead
                    raise NotImplementedError(str(e)) from e
                raise
            # the M x T result tensors, made while the kernel runs (one native call per receiver
            # when the staging extension is built), or the reused buffers' own
            outs = [v if v is not None else self._views(b, offs, shapes, native) for b, v in rows_out]
            couts = cent_out[1] if cent_out[1] is not None else self._views(cent_out[0], offs, shapes, native)
            self.__result_pool = ((native, res_dtype, self.device), list(zip([b for b, _ in rows_out], outs)),
                                  (cent_out[0], couts))
            kept_names = [layout.names[i] for i in keep]
            for r, j in enumerate(receivers):
                out[j].update(zip(kept_names, outs[r]))
            central.update(zip(kept_names, couts))
            if under_kernel is not None:
                under_kernel()  # the caller's host work that needs no result values
            flags = self.__ctx.check()
            if flags:
                self._raise_nan(flags, rows, dt, native, outs, receivers)
        if whole:
            ordered, central_ordered = out, central  # already every name, in layout order
        else:
            for i, name in enumerate(layout.names):
                if i not in keep:
                    for j in receivers:
                        out[j][name] = torch.empty(layout.shapes[i], dtype=self.result_dtype, device=self.device)
                    central[name] = torch.empty(layout.shapes[i], dtype=torch.float64, device=self.device)
            ordered = {j: {n: out[j][n] for n in layout.names} for j in receivers}
            central_ordered = {n: central[n] for n in layout.names}
        if self.result_device is not None:
            ordered = {j: {k: v.to(self.result_device) for k, v in p.items()} for j, p in ordered.items()}
            central_ordered = {k: v.to(self.result_device) for k, v in central_ordered.items()}
        return ordered, central_ordered

    def _geometry(self, native: ModelLayout) -> tuple[list[int], int, list[tuple[int, ...]]]:
        """(element offsets, flat size, shapes) of a result buffer, one set of objects per layout
        (the staging extension parses a shapes list once per list object)."""
        memo = self.__geometry
        if memo is None or memo[0] is not native:
            offs, padded = native.padded_offsets(8)
            memo = self.__geometry = (native, list(offs), int(padded), [tuple(sh) for sh in native.shapes])
        return memo[1], memo[2], memo[3]

    def _weights(self, receivers: list[int], ids: list[int]) -> np.ndarray:
        """weights[r][n] = worker_weights[receiver r].get(arrival n's worker, 0) (:36). The
        reference reads the caller's dicts live on every arrival, so the matrix of the last
        (receivers, arrival order) is reused only while every receiver's dict still equals the copy
        taken with it (one C-level dict comparison per receiver): a caller that changes a weight in
        place between rounds gets it, as in the reference."""
        key = (tuple(receivers), tuple(ids))
        memo = self.__weights_memo
        if (memo is not None and memo[0] == key
                and all(self._worker_weights[j] == snap for j, snap in zip(receivers, memo[2]))):
            return memo[1]
        weights = np.zeros((len(receivers), len(ids)), dtype=np.float64)
        for r, j in enumerate(receivers):
            wj = self._worker_weights[j]
            for n, wid in enumerate(ids):
                weights[r, n] = float(wj.get(wid, 0))
        self.__weights_memo = (key, weights, [dict(self._worker_weights[j]) for j in receivers])
        return weights

    @staticmethod
    def _views(buf: torch.Tensor, offs, shapes, native: ModelLayout) -> list[torch.Tensor]:
        ext = _staging.module()
        if ext is not None:
            return ext.views(buf, offs, shapes)
        return [buf[o : o + n].view(sh) for o, n, sh in zip(offs, native.numels, shapes)]

    def _result_rows(self, native: ModelLayout, M: int, res_dtype: torch.dtype, offs, padded: int, shapes):
        """(buffer, views or None) per receiver and for the centralized model. A buffer of the
        last round is written again only when nothing outside this object can see it (``unobserved``,
        csrc/staging_ext.cpp: its views referenced by the pool alone, nothing else on its storage,
        geometry untouched) — the caller cannot tell it from a fresh one; otherwise a new buffer."""
        ext = _staging.module()
        pool, self.__result_pool = self.__result_pool, None
        old_rows: list = []
        old_cent = None
        if pool is not None and ext is not None and pool[0] == (native, res_dtype, self.device):
            old_rows, old_cent = pool[1], pool[2]
        rows = []
        for r in range(M):
            if r < len(old_rows) and ext.unobserved(old_rows[r][0], old_rows[r][1], offs, shapes):
                rows.append(old_rows[r])
            else:
                rows.append((torch.empty(padded, dtype=res_dtype, device=self.device), None))
        if old_cent is not None and ext.unobserved(old_cent[0], old_cent[1], offs, shapes):
            cent = old_cent
        else:
            cent = (torch.empty(padded, dtype=torch.float64, device=self.device), None)
        return rows, cent

    def _raise_nan(self, flags: int, rows, dt, native: ModelLayout, outs, receivers) -> None:
        """Map the fused flags onto the reference's assertions (error path only)."""
        if flags & (_native.FLAG_ACC_NAN | _native.FLAG_RESULT_NAN):
            if flags & _native.FLAG_ACC_NAN:
                from ..fedavg import ClientTable

                table = ClientTable(native.num_segments)
                for r in rows:
                    table.add_client(r, [1.0] * native.num_segments)
                bad = context_for(native, self.device).find_nan_clients(table, dt)
                if bad:
                    ids = [self.__arrivals[n][0] for n in bad]
                    raise NaNAggregationError("input", f"NaN in the update(s) of worker(s) {ids} "
                                                       "(fed_avg_algorithm.py:35)", bad)
                raise NaNAggregationError("accumulator", "NaN in a receiver's weighted sum, e.g. inf * 0 or "
                                                         "inf - inf (fed_avg_algorithm.py:93)")
            raise NaNAggregationError("result", "NaN in a receiver's average, e.g. 0 / 0 "
                                                "(fed_avg_algorithm.py:97)")
        raise NaNAggregationError("result", "NaN in the centralized average (aggregation_algorithm.py:73)")

    @staticmethod
    def _check_and_reduce_other_data(msgs: list[Message]) -> dict[str, Any]:
        """fed_avg_algorithm.py:136-149, over the updates one receiver folded."""
        merged: dict[str, Any] = {}
        for msg in msgs:
            for k, v in msg.other_data.items():
                if k in merged and v != merged[k]:
                    raise RuntimeError(f"different values on key {k}")
                merged.setdefault(k, v)
        return merged

    def clear_worker_data(self) -> None:
        super().clear_worker_data()
        self.__arrivals = []
        self.__native_codes = set()
        self.__ptr_rows = []

    def exit(self) -> None:
        self.__result_pool = None
        if self.__ctx is not None:
            self.__ctx.close()
            self.__ctx = None
