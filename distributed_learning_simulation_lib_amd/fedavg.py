"""Host-side handle on the HIP FedAvg library: model layouts, client tables, error mapping.

A ``ModelLayout`` is the ordered list of named tensors of a model — the keys of
``ParameterMessage.parameter`` (reference ``simulation_lib/message.py:24-31``). A
``FedAvgContext`` owns one native context (``include/fedavg_hip.h``) for one layout on one
device: the fp64 accumulator the streaming path folds clients into
(``fed_avg_algorithm.py:43-64``), the per-segment total weights, and the fused
finalize/NaN checks (``fed_avg_algorithm.py:76-99``).

Every method launches asynchronously on the current torch stream of the context's device
(``torch.cuda.current_stream``); PyTorch is only the allocator and stream provider here. The
arithmetic runs in the HIP kernels of ``csrc/fedavg_kernels.hip``; there is no CPU path.
"""

from __future__ import annotations

import ctypes
import weakref
from collections.abc import Mapping, Sequence
from dataclasses import dataclass
from functools import cached_property
from typing import Any

import numpy as np
import torch

from . import _native

DTYPE_CODES: dict[torch.dtype, int] = {
    torch.float32: _native.F32,
    torch.float16: _native.F16,
    torch.bfloat16: _native.BF16,
    torch.float64: _native.F64,
}
OUT_CODES: dict[torch.dtype, int] = {torch.float32: _native.F32, torch.float64: _native.F64}

_PTR = ctypes.POINTER(ctypes.c_void_p)
_DBL = ctypes.POINTER(ctypes.c_double)


class NaNAggregationError(AssertionError):
    """Raised where the reference's NaN assertions fire (fed_avg_algorithm.py:35,93,97).

    Subclasses ``AssertionError`` so callers that expect the reference's ``assert`` keep
    working. ``stage`` is ``"input"`` (:35), ``"accumulator"`` (:93) or ``"result"`` (:97).
    """

    def __init__(self, stage: str, message: str, bad_clients: Sequence[int] = ()) -> None:
        super().__init__(message)
        self.stage = stage
        self.bad_clients = list(bad_clients)


@dataclass(frozen=True)
class ModelLayout:
    """Names, shapes and element counts of a model's tensors, in dict order."""

    names: tuple[str, ...]
    shapes: tuple[tuple[int, ...], ...]

    @classmethod
    def from_parameters(cls, parameter: Mapping[str, torch.Tensor]) -> ModelLayout:
        return cls(
            names=tuple(parameter.keys()),
            shapes=tuple(tuple(t.shape) for t in parameter.values()),
        )

    @classmethod
    def flat(cls, numel: int, name: str = "bucket") -> ModelLayout:
        return cls(names=(name,), shapes=((int(numel),),))

    @cached_property
    def numels(self) -> list[int]:
        # cached: the staging path asks for it per client (np.prod per tensor is ~2 us)
        return [int(np.prod(s, dtype=np.int64)) for s in self.shapes]

    @property
    def num_segments(self) -> int:
        return len(self.names)

    @property
    def total_numel(self) -> int:
        return sum(self.numels)

    def padded_offsets(self, elem_bytes: int) -> tuple[list[int], int]:
        """Element offsets of each tensor in a flat buffer whose segments start 16-B aligned."""
        cache = self.__dict__.setdefault("_padded_cache", {})
        if elem_bytes not in cache:
            cache[elem_bytes] = self._padded_offsets(elem_bytes)
        offs, total = cache[elem_bytes]
        return list(offs), total

    def _padded_offsets(self, elem_bytes: int) -> tuple[list[int], int]:
        align = max(1, 16 // elem_bytes)
        offs, pos = [], 0
        for n in self.numels:
            offs.append(pos)
            pos += (n + align - 1) // align * align
        return offs, pos


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_EMPTY_ARRAYS = (np.zeros(1, np.uint64), np.zeros(1, np.float64))  # module-lifetime storage
_EMPTY_TABLE = (_EMPTY_ARRAYS[0].ctypes.data, _EMPTY_ARRAYS[1].ctypes.data)


def _table_args(table: ClientTable) -> tuple[Any, Any]:
    """The client table's pointer and weight arrays as C-ABI arguments: the staging extension's
    raw addresses when the table has them, else ctypes pointers that keep its numpy arrays alive
    for the call."""
    addresses = getattr(table, "addresses", None)
    if addresses is not None:
        return addresses()
    p, w = table.arrays()
    return p.ctypes.data_as(_PTR), w.ctypes.data_as(_DBL)


def _stream_handle(device: torch.device) -> ctypes.c_void_p:
    """torch's current stream on ``device`` (the raw handle without building a Stream object:
    this runs on every launch)."""
    if _raw_stream is not None and device.index is not None:
        return ctypes.c_void_p(_raw_stream(device.index))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def dtype_code(dtype) -> int:
    """C-ABI input format of a torch dtype, or of a quantised record format
    (``quantized.QSGD_F32`` / ``QSGD_F64`` / ``NNADQ_F32`` / ``NNADQ_F64``, which carry their
    own code)."""
    if not isinstance(dtype, torch.dtype):
        code = getattr(dtype, "code", None)
        if code in _native.RECORD_CODES:
            return int(code)
        raise TypeError(f"no HIP FedAvg kernel for input format {dtype}")
    try:
        return DTYPE_CODES[dtype]
    except KeyError:
        raise TypeError(f"no HIP FedAvg kernel for input dtype {dtype}") from None


def out_code(dtype: torch.dtype) -> int:
    try:
        return OUT_CODES[dtype]
    except KeyError:
        raise TypeError(f"aggregated output dtype must be float32 or float64, not {dtype}") from None


class ClientTable:
    """Row-major [num_clients][num_segments] device pointers + fp64 weights for one call.

    ``None`` entries are absent tensors (skipped, never counted in the segment's total
    weight). The tensors are kept alive by the table until the caller drops it.
    """

    def __init__(self, num_segments: int) -> None:
        self.num_segments = num_segments
        self._ptrs: list[int] = []
        self._weights: list[float] = []
        self._keep: list[torch.Tensor] = []
        # per entry: element count, element size, device (-1 = host) — checked against the
        # layout and input format before any launch (an undersized operand would be read out
        # of bounds by the kernel); -1 / 0 / -2 for absent entries
        self._numel: list[int] = []
        self._esize: list[int] = []
        self._dev: list[int] = []
        self._validated: set = set()
        self.num_clients = 0
        self._arrays: tuple[np.ndarray, np.ndarray] | None = None
        # per-element weights (fedavg_accumulate_elementwise): pointer + dtype code per entry
        self._wptrs: list[int] = []
        self._wdts: list[int] = []

    def add_client(self, tensors: Sequence[torch.Tensor | None], weights: Sequence[float],
                   weight_tensors: Sequence[torch.Tensor | None] | None = None) -> None:
        """One client row. ``weight_tensors`` (optional): per-element weight tensors (fp32 / fp64,
        the segment's size) where a _get_weight override returned one; None = the scalar."""
        T = self.num_segments
        if len(tensors) != T or len(weights) != T:
            raise ValueError("client row does not match the layout")
        if weight_tensors is not None and len(weight_tensors) != T:
            raise ValueError("weight row does not match the layout")
        # the row is built in locals and committed at the end: a rejected row leaves the table as
        # it was (this runs once per client on the plugin path, so it is kept lean)
        ptrs, ws, numel, esize, dev, keep = [], [], [], [], [], []
        for t, w in zip(tensors, weights):
            if t is None:
                ptrs.append(0)
                ws.append(0.0)
                numel.append(-1)
                esize.append(0)
                dev.append(-2)
            else:
                if not t.is_contiguous():
                    raise ValueError("client tensors must be contiguous (the kernel reads them as flat buffers)")
                ptrs.append(t.data_ptr())
                ws.append(float(w))
                numel.append(t.numel())
                esize.append(t.element_size())
                dev.append(t.get_device())  # -1 for host tensors
                keep.append(t)
        wptrs, wdts = [0] * T, [_native.F64] * T
        if weight_tensors is not None:
            for i, (t, wt) in enumerate(zip(tensors, weight_tensors)):
                if t is None or wt is None:
                    continue
                if wt.dtype not in (torch.float32, torch.float64) or not wt.is_contiguous() \
                        or wt.numel() != t.numel() or wt.device != t.device:
                    raise ValueError("per-element weights: contiguous fp32 / fp64 of the tensor's size and device")
                wptrs[i] = wt.data_ptr()
                wdts[i] = _native.F32 if wt.dtype == torch.float32 else _native.F64
                keep.append(wt)
        self._ptrs += ptrs
        self._weights += ws
        self._numel += numel
        self._esize += esize
        self._dev += dev
        self._wptrs += wptrs
        self._wdts += wdts
        self._keep += keep
        self._validated.clear()
        self.num_clients += 1
        self._arrays = None

    def add_resident_client(self, ptrs: list[int], weights: list[float], numels: list[int], esize: int,
                            device_index: int, keep: list[torch.Tensor]) -> None:
        """One client row whose present tensors the caller has already checked: contiguous, on
        ``device_index``, ``esize``-byte elements, ``numels[seg]`` elements each (``ptrs[seg]``
        == 0 and ``numels[seg]`` == -1 for an absent tensor). The plugin's staging pass proves
        all of that while it recognises the common arrival, so the row is committed without
        touching the tensors again; ``validate`` still checks the recorded sizes before a launch."""
        T = self.num_segments
        if len(ptrs) != T or len(weights) != T or len(numels) != T:
            raise ValueError("client row does not match the layout")
        self._ptrs += ptrs
        self._weights += weights
        self._numel += numels
        self._esize += [esize if n >= 0 else 0 for n in numels]
        self._dev += [device_index if n >= 0 else -2 for n in numels]
        self._wptrs += [0] * T
        self._wdts += [_native.F64] * T
        self._keep += keep
        self._validated.clear()
        self.num_clients += 1
        self._arrays = None

    def elementwise_arrays(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Weight pointers and dtype codes, [num_clients][num_segments] (0 = scalar weight)."""
        return (np.asarray(self._wptrs or [0], dtype=np.uint64), np.asarray(self._wdts or [0], dtype=np.int32),
                np.asarray(self._weights or [0.0], dtype=np.float64))

    def validate(self, numels: Sequence[int], esize: int, device_index: int, key) -> None:
        """Every present entry holds exactly ``numels[seg]`` elements of ``esize`` bytes on the
        device (checked once per table and ``key``). Raises ValueError naming the first bad one."""
        if key in self._validated or self.num_clients == 0:
            return
        T = self.num_segments
        have = np.asarray(self._numel, dtype=np.int64).reshape(self.num_clients, T)
        es = np.asarray(self._esize, dtype=np.int64).reshape(self.num_clients, T)
        dev = np.asarray(self._dev, dtype=np.int64).reshape(self.num_clients, T)
        want = np.broadcast_to(np.asarray(numels, dtype=np.int64), have.shape)
        present = have >= 0
        bad = present & ((have != want) | (es != esize) | (dev != device_index))
        if bad.any():
            k, t = (int(x) for x in np.argwhere(bad)[0])
            raise ValueError(
                f"client {k}, tensor {t}: {have[k, t]} elements of {es[k, t]} bytes on device {dev[k, t]}; "
                f"the layout and input format need {want[k, t]} of {esize} bytes on device {device_index}")
        self._validated.add(key)

    def arrays(self) -> tuple[np.ndarray, np.ndarray]:
        """The C-ABI arrays (built once per table and cached: a table can be reduced many times)."""
        if self._arrays is None:
            ptrs = np.asarray(self._ptrs, dtype=np.uint64) if self._ptrs else np.zeros(1, np.uint64)
            ws = np.asarray(self._weights, dtype=np.float64) if self._weights else np.zeros(1, np.float64)
            self._arrays = (ptrs, ws)
        return self._arrays

    def rows(self) -> list[list[int]]:
        T = self.num_segments
        return [self._ptrs[k * T : (k + 1) * T] for k in range(self.num_clients)]


class OutputTable:
    """Validated per-segment output tensors of one dtype (built once, reusable across calls)."""

    def __init__(self, outs: Sequence[torch.Tensor], layout: ModelLayout, device: torch.device,
                 dtype: torch.dtype) -> None:
        if len(outs) != layout.num_segments:
            raise ValueError("one output tensor per segment is required")
        for o, n in zip(outs, layout.numels):
            if o.dtype != dtype or o.device != device or o.numel() != n or not o.is_contiguous():
                raise ValueError("output tensors must be contiguous, on the context device, of the layout size")
        self.tensors = list(outs)
        self.dtype = dtype
        self.layout = layout
        self.device = device
        self.c_array = (ctypes.c_void_p * len(outs))(*[o.data_ptr() for o in outs])

    @classmethod
    def from_flat(cls, flat: torch.Tensor, offsets: Sequence[int], layout: ModelLayout) -> OutputTable:
        """Segments of one flat contiguous buffer at element ``offsets`` (no tensor per segment:
        the pointer array is computed from the buffer's address)."""
        if flat.dim() != 1 or not flat.is_contiguous() or len(offsets) != layout.num_segments:
            raise ValueError("a flat contiguous buffer and one offset per segment are required")
        offs = np.asarray(offsets, dtype=np.int64)
        if layout.num_segments and (offs.min() < 0 or int((offs + np.asarray(layout.numels)).max()) > flat.numel()):
            raise ValueError("segment outside the flat output buffer")
        self = cls.__new__(cls)
        self.tensors = [flat]
        self.dtype = flat.dtype
        self.layout = layout
        self.device = flat.device
        ptrs = np.uint64(flat.data_ptr()) + offs.astype(np.uint64) * np.uint64(flat.element_size())
        self.c_array = (ctypes.c_void_p * layout.num_segments).from_buffer_copy(ptrs.tobytes())
        return self


class FedAvgContext:
    """One native FedAvg context: layout + device + fp64 accumulator."""

    def __init__(
        self,
        layout: ModelLayout,
        device: torch.device | str | int | None = None,
        split_policy: int | None = None,
        lib: ctypes.CDLL | None = None,
    ) -> None:
        self._lib = lib if lib is not None else _native.load()
        self._plans: weakref.WeakSet[AggregatePlan] = weakref.WeakSet()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("the FedAvg HIP path runs on a GPU device")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.layout = layout
        if layout.num_segments == 0 or min(layout.numels) <= 0:
            raise ValueError("a native layout needs at least one tensor and no empty tensors")
        numels = (ctypes.c_int64 * layout.num_segments)(*layout.numels)
        # the accumulator is a torch tensor so collectives (RCCL) can run on it
        acc_numel = self._padded_acc_numel(layout, self._lib)
        self.accumulator = torch.zeros(acc_numel, dtype=torch.float64, device=device)
        handle = ctypes.c_void_p()
        _native.check(
            self._lib.fedavg_ctx_create(
                ctypes.byref(handle),
                device.index,
                numels,
                layout.num_segments,
                ctypes.c_void_p(self.accumulator.data_ptr()),
            )
        )
        self._h = handle
        assert self._lib.fedavg_acc_numel(self._h) == acc_numel
        if split_policy is not None:
            _native.check(self._lib.fedavg_set_split_policy(self._h, split_policy))

    @classmethod
    def borrowed(cls, lib: ctypes.CDLL, handle: int, layout: ModelLayout, device: torch.device,
                 accumulator: torch.Tensor) -> FedAvgContext:
        """A view of a native context owned by another object (a device entry of
        ``multi_device.MultiDeviceContext``): same methods, but ``close`` leaves it alone."""
        self = cls.__new__(cls)
        self._lib = lib
        self._plans = weakref.WeakSet()
        self.device = device
        self.layout = layout
        self.accumulator = accumulator
        self._h = ctypes.c_void_p(handle)
        self._borrowed = True
        return self

    @staticmethod
    def _padded_acc_numel(layout: ModelLayout, lib: ctypes.CDLL) -> int:
        """Accumulator elements: every segment starts at a multiple of FEDAVG_ACC_ALIGN (32)."""
        numels = (ctypes.c_int64 * layout.num_segments)(*layout.numels)
        n = int(lib.fedavg_layout_acc_numel(numels, layout.num_segments))
        if n < 0:
            raise ValueError("bad layout")
        return n

    @property
    def acc_numel(self) -> int:
        return self.accumulator.numel()

    # -- lifecycle -------------------------------------------------------------------
    def close(self) -> None:
        for plan in list(getattr(self, "_plans", ())):
            plan.close()  # before the native context goes: a plan reads it
        if getattr(self, "_borrowed", False):
            self._h = ctypes.c_void_p()  # the owner destroys it
            return
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.fedavg_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self) -> None:  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    # -- helpers ---------------------------------------------------------------------
    @property
    def stream(self) -> ctypes.c_void_p:
        return _stream_handle(self.device)

    def segment_offset(self, seg: int) -> int:
        return int(self._lib.fedavg_segment_offset(self._h, seg))

    @property
    def num_tiles(self) -> int:
        return int(self._lib.fedavg_num_tiles(self._h))

    def tile_range(self, tile_begin: int, tile_end: int) -> tuple[int, int]:
        b, e = ctypes.c_int64(), ctypes.c_int64()
        _native.check(self._lib.fedavg_tile_range(self._h, tile_begin, tile_end, ctypes.byref(b), ctypes.byref(e)))
        return b.value, e.value

    def total_weights(self) -> list[float]:
        out = (ctypes.c_double * self.layout.num_segments)()
        _native.check(self._lib.fedavg_total_weights(self._h, out))
        return list(out)

    def _out_table(self, outs: Sequence[torch.Tensor] | OutputTable, out_dtype: torch.dtype) -> ctypes.Array:
        if isinstance(outs, OutputTable):
            if outs.dtype != out_dtype or outs.layout != self.layout or outs.device != self.device:
                raise ValueError("output table was built for another dtype, layout or device")
            return outs.c_array
        return OutputTable(outs, self.layout, self.device, out_dtype).c_array

    def _check_table(self, table: ClientTable, in_dtype: torch.dtype) -> None:
        if table.num_segments != self.layout.num_segments:
            raise ValueError("client table does not match the layout")
        code = dtype_code(in_dtype)
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        if code in _native.RECORD_CODES:
            # one uint8 record per tensor (include/fedavg_hip.h record layouts)
            nbytes = (self._lib.fedavg_qsgd_record_bytes if code in (_native.QSGD_F32, _native.QSGD_F64)
                      else self._lib.fedavg_nnadq_record_bytes)
            need = [int(nbytes(n)) for n in self.layout.numels]
            table.validate(need, 1, dev, ("record", tuple(need), dev))
        else:
            # the key is built once per (dtype, device): this runs per wave launch
            keys = self.__dict__.setdefault("_dense_keys", {})
            key = keys.get((in_dtype, dev))
            if key is None:
                key = keys[(in_dtype, dev)] = (in_dtype, tuple(self.layout.numels), dev)
            table.validate(self.layout.numels, in_dtype.itemsize, dev, key)

    # -- hot path --------------------------------------------------------------------
    def accumulate(self, table: ClientTable, in_dtype: torch.dtype) -> None:
        """Fold a wave of clients into the accumulator (fed_avg_algorithm.py:43-64)."""
        self._check_table(table, in_dtype)
        if table.num_clients == 0:
            return
        p, w = _table_args(table)
        _native.check(
            self._lib.fedavg_accumulate(self._h, p, dtype_code(in_dtype), w, table.num_clients, self.stream)
        )

    def aggregate(
        self,
        table: ClientTable | None,
        in_dtype: torch.dtype,
        outs: Sequence[torch.Tensor] | OutputTable,
        out_dtype: torch.dtype,
    ) -> None:
        """Fold the last wave (optional) then out = acc / total_weight (fed_avg_algorithm.py:76-99)."""
        n = 0 if table is None else table.num_clients
        if table is not None:
            self._check_table(table, in_dtype)
            p, w = _table_args(table)
        else:
            p, w = _EMPTY_TABLE
        ot = self._out_table(outs, out_dtype)
        _native.check(
            self._lib.fedavg_aggregate(
                self._h, p, dtype_code(in_dtype) if n else _native.F32, w, n, ot, out_code(out_dtype), self.stream,
            )
        )

    def _base_table(self, base: Sequence[torch.Tensor] | OutputTable) -> ctypes.Array:
        return self._out_table(base, torch.float64)

    def accumulate_delta(self, table: ClientTable, in_dtype: torch.dtype,
                         base: Sequence[torch.Tensor] | OutputTable) -> None:
        """Fold a wave of DELTA clients: x = base + delta (fp64), message.py:40-61 fused."""
        self._check_table(table, in_dtype)
        if table.num_clients == 0:
            return
        p, w = table.arrays()
        bt = self._base_table(base)
        _native.check(
            self._lib.fedavg_accumulate_delta(
                self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype), w.ctypes.data_as(_DBL),
                table.num_clients, bt, self.stream,
            )
        )

    def aggregate_delta(self, table: ClientTable, in_dtype: torch.dtype,
                        base: Sequence[torch.Tensor] | OutputTable,
                        outs: Sequence[torch.Tensor] | OutputTable, out_dtype: torch.dtype) -> None:
        """Last wave of delta clients + divide (fedavg_aggregate with the restore fused)."""
        self._check_table(table, in_dtype)
        p, w = table.arrays()
        bt = self._base_table(base)
        ot = self._out_table(outs, out_dtype)
        _native.check(
            self._lib.fedavg_aggregate_delta(
                self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype), w.ctypes.data_as(_DBL),
                table.num_clients, bt, ot, out_code(out_dtype), self.stream,
            )
        )

    def weighted_avg(
        self, table: ClientTable, in_dtype: torch.dtype, outs: Sequence[torch.Tensor], out_dtype: torch.dtype
    ) -> None:
        """out = sum_k ratio_k * x_k in fp64, table weights are the ratios (aggregation_algorithm.py:51-76)."""
        self._check_table(table, in_dtype)
        p, w = table.arrays()
        ot = self._out_table(outs, out_dtype)
        _native.check(
            self._lib.fedavg_weighted_avg(
                self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype), w.ctypes.data_as(_DBL),
                table.num_clients, ot, out_code(out_dtype), self.stream,
            )
        )

    def partial(
        self,
        table: ClientTable | None,
        in_dtype: torch.dtype,
        zero_init: bool = True,
        tile_begin: int = 0,
        tile_end: int = -1,
    ) -> None:
        """acc[tiles] = (0 | acc) + sum_k w_k x_k (the shard step of the multi-GPU path)."""
        n = 0 if table is None else table.num_clients
        if table is not None:
            self._check_table(table, in_dtype)
            p, w = table.arrays()
        else:
            p, w = np.zeros(1, np.uint64), np.zeros(1, np.float64)
        _native.check(
            self._lib.fedavg_partial(
                self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype) if n else _native.F32,
                w.ctypes.data_as(_DBL), n, 1 if zero_init else 0, tile_begin, tile_end, self.stream,
            )
        )

    def segment_state(self) -> tuple[list[float], list[int]]:
        """(per-segment total weight, 1 = the accumulator holds folded data) — what
        ``set_segment_state`` sets."""
        tw = (ctypes.c_double * self.layout.num_segments)()
        vv = (ctypes.c_int32 * self.layout.num_segments)()
        _native.check(self._lib.fedavg_segment_state(self._h, tw, vv))
        return list(tw), list(vv)

    def set_segment_state(self, total_weights: Sequence[float], valid: Sequence[int]) -> None:
        """Per-segment accumulated state (a layout grown mid-round keeps its folded segments)."""
        tw = (ctypes.c_double * self.layout.num_segments)(*[float(x) for x in total_weights])
        vv = (ctypes.c_int32 * self.layout.num_segments)(*[1 if v else 0 for v in valid])
        _native.check(self._lib.fedavg_set_segment_state(self._h, tw, vv))

    def accumulate_elementwise(self, table: ClientTable, in_dtype: torch.dtype, totals: torch.Tensor,
                               total_fp32: Sequence[bool]) -> None:
        """Fold a wave with per-element weights (fed_avg_algorithm.py:51-62 with a tensor-valued
        _get_weight): acc += x * w and totals += w elementwise; ``totals`` is an fp64 buffer in
        accumulator coordinates, rounded to fp32 per segment where ``total_fp32``."""
        self._check_table(table, in_dtype)
        if table.num_clients == 0:
            return
        if totals.dtype != torch.float64 or totals.numel() < self.acc_numel or totals.device != self.device:
            raise ValueError("totals: an fp64 buffer of the accumulator's size on the context device")
        p, _ = table.arrays()
        wp, wd, ws = table.elementwise_arrays()
        flags = (ctypes.c_int32 * self.layout.num_segments)(*[1 if f else 0 for f in total_fp32])
        _native.check(self._lib.fedavg_accumulate_elementwise(
            self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype), wp.ctypes.data_as(_PTR),
            wd.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ws.ctypes.data_as(_DBL), flags, table.num_clients,
            ctypes.c_void_p(totals.data_ptr()), self.stream))

    def finalize_elementwise(self, totals: torch.Tensor, outs: Sequence[torch.Tensor] | OutputTable,
                             out_dtype: torch.dtype) -> None:
        """out = acc / totals elementwise (fed_avg_algorithm.py:94-97); resets the state."""
        ot = self._out_table(outs, out_dtype)
        _native.check(self._lib.fedavg_finalize_elementwise(self._h, ctypes.c_void_p(totals.data_ptr()), ot,
                                                            out_code(out_dtype), self.stream))

    def set_accumulated(self, total_weights: Sequence[float]) -> None:
        tw = (ctypes.c_double * self.layout.num_segments)(*[float(x) for x in total_weights])
        _native.check(self._lib.fedavg_set_accumulated(self._h, tw))

    def finalize_range(
        self, outs: Sequence[torch.Tensor], out_dtype: torch.dtype, tile_begin: int = 0, tile_end: int = -1
    ) -> None:
        ot = self._out_table(outs, out_dtype)
        _native.check(
            self._lib.fedavg_finalize_range(self._h, ot, out_code(out_dtype), tile_begin, tile_end, self.stream)
        )

    def plan(
        self, table: ClientTable, in_dtype: torch.dtype, outs: Sequence[torch.Tensor] | OutputTable,
        out_dtype: torch.dtype,
    ) -> AggregatePlan:
        """Prepare ``aggregate(table, in_dtype, outs, out_dtype)`` once; ``plan.run()`` repeats it
        with no host staging (the table's tensors and the outputs must stay alive)."""
        self._check_table(table, in_dtype)
        p, w = table.arrays()
        ot = self._out_table(outs, out_dtype)
        h = ctypes.c_void_p()
        _native.check(
            self._lib.fedavg_plan_create(
                self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype), w.ctypes.data_as(_DBL),
                table.num_clients, ot, out_code(out_dtype), ctypes.byref(h),
            )
        )
        return AggregatePlan(self, h, keep=(table, outs))

    def plan_partial(self, table: ClientTable | None, in_dtype: torch.dtype, zero_init: bool = True) -> AggregatePlan:
        """Prepared shard partial; ``plan.run_range(tb, te)`` == ``partial(table, ..., tb, te)``."""
        n = 0 if table is None else table.num_clients
        if table is not None:
            self._check_table(table, in_dtype)
            p, w = table.arrays()
        else:
            p, w = np.zeros(1, np.uint64), np.zeros(1, np.float64)
        h = ctypes.c_void_p()
        _native.check(
            self._lib.fedavg_plan_create_partial(
                self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype) if n else _native.F32,
                w.ctypes.data_as(_DBL), n, 1 if zero_init else 0, ctypes.byref(h),
            )
        )
        return AggregatePlan(self, h, keep=(table,))

    def plan_finalize(self, total_weights: Sequence[float], outs: Sequence[torch.Tensor] | OutputTable,
                      out_dtype: torch.dtype) -> AggregatePlan:
        """Prepared finalize with baked totals; ``plan.run_range(tb, te)`` == ``finalize_range``."""
        ot = self._out_table(outs, out_dtype)
        tw = (ctypes.c_double * self.layout.num_segments)(*[float(x) for x in total_weights])
        h = ctypes.c_void_p()
        _native.check(self._lib.fedavg_plan_create_finalize(self._h, tw, ot, out_code(out_dtype), ctypes.byref(h)))
        return AggregatePlan(self, h, keep=(outs,))

    def set_fused_fold(self, enable: bool) -> None:
        """Allow the one-instruction fold when every product is provably exact (default on)."""
        _native.check(self._lib.fedavg_set_fused_fold(self._h, 1 if enable else 0))

    def reset(self) -> None:
        _native.check(self._lib.fedavg_reset(self._h, self.stream))

    # -- dynamic waves (fedavg_dyn_*: the round's first wave folded while clients arrive) -
    def dyn_open(self, in_dtype: torch.dtype, max_clients: int) -> None:
        _native.check(self._lib.fedavg_dyn_open(self._h, dtype_code(in_dtype), int(max_clients), self.stream))

    def dyn_publish(self, table: ClientTable) -> int:
        """Hand the table's unpublished rows to the open wave; the rows published now (0 while
        the current stream still has unfinished work). NativeError for a row the wave cannot take
        (its ``published``: the rows before it, published)."""
        p, w = _table_args(table)
        n = ctypes.c_int32()
        st = self._lib.fedavg_dyn_publish(self._h, p, w, table.num_clients, self.stream, ctypes.byref(n))
        if st != _native.OK:  # the rows before the one it cannot take were published: e.published
            err = _native.NativeError(st, _native.last_error())
            err.published = int(n.value)
            raise err
        return int(n.value)

    def dyn_close(self, outs: Sequence[torch.Tensor] | OutputTable | None = None,
                  out_dtype: torch.dtype = torch.float64, join: bool = True) -> tuple[int, bool]:
        """(rows folded, finalized): with ``outs`` the wave divides into them (finalized), else —
        or when it ended itself — it leaves rows [0, folded) in the accumulator. ``join=False``:
        a finalized wave's outputs are complete after the next ``flags`` / ``raise_on_nan``."""
        ot = self._out_table(outs, out_dtype) if outs is not None else None
        folded, fin = ctypes.c_int32(), ctypes.c_int32()
        _native.check(self._lib.fedavg_dyn_close(self._h, ot, out_code(out_dtype), 1 if join else 0, self.stream,
                                                 ctypes.byref(folded), ctypes.byref(fin)))
        return int(folded.value), bool(fin.value)

    def dyn_prof_collect(self) -> tuple[float, int]:
        """(ms, waves): the closed dynamic waves' body launches, enqueue to end, while profiling."""
        ms, n = ctypes.c_double(), ctypes.c_int32()
        _native.check(self._lib.fedavg_dyn_prof_collect(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def dyn_state(self) -> tuple[bool, int]:
        a, p = ctypes.c_int32(), ctypes.c_int32()
        _native.check(self._lib.fedavg_dyn_state(self._h, ctypes.byref(a), ctypes.byref(p)))
        return bool(a.value), int(p.value)

    def dyn_configure(self, idle_us: int = 0, life_us: int = 0) -> None:
        """The wave's idle limit / lifetime (µs) for the following launches (0: unchanged)."""
        _native.check(self._lib.fedavg_dyn_configure(self._h, int(idle_us), int(life_us)))

    def dyn_timing(self) -> dict[str, float]:
        """fedavg_dyn_timing of the last completed wave (µs, GPU clock; -1 where not recorded)."""
        v = (ctypes.c_double * 3)()
        _native.check(self._lib.fedavg_dyn_timing(self._h, v, 3))
        return dict(zip(("rows_to_end_us", "close_to_end_us", "rows_to_close_us"), (float(x) for x in v)))

    def dyn_info(self) -> dict[str, int]:
        """fedavg_dyn_info: the open wave's state and this context's continued waves / launches."""
        v = (ctypes.c_int32 * 5)()
        _native.check(self._lib.fedavg_dyn_info(self._h, v, 5))
        return dict(zip(("active", "published", "base", "reopens", "launches"), (int(x) for x in v)))

    # -- fault reporting ---------------------------------------------------------------
    def flags(self) -> int:
        """Synchronise the stream and return the latched NaN flag bits."""
        f = ctypes.c_uint32()
        st = self._lib.fedavg_check(self._h, self.stream, ctypes.byref(f))
        if st not in (_native.OK, _native.ERR_NAN_ACCUM, _native.ERR_NAN_RESULT):
            _native.check(st)
        return int(f.value)

    def find_nan_clients(self, table: ClientTable, in_dtype: torch.dtype) -> list[int]:
        p, _ = table.arrays()
        out = (ctypes.c_int32 * table.num_clients)()
        _native.check(
            self._lib.fedavg_find_nan_clients(
                self._h, p.ctypes.data_as(_PTR), dtype_code(in_dtype), table.num_clients, out, self.stream
            )
        )
        return [i for i in range(table.num_clients) if out[i]]

    def raise_on_nan(self, tables: Sequence[tuple[ClientTable, torch.dtype]] = ()) -> None:
        """Map the latched flags onto the reference's assertions.

        Input NaN (fed_avg_algorithm.py:35) and an accumulator NaN (:93) both leave the fp64
        accumulator NaN; the client tables still held by the caller are scanned to tell them
        apart and name the offending clients.
        """
        f = self.flags()
        if f == 0:
            return
        # the flag is sticky until reset: clear it so the context stays usable
        self.reset()
        if f & _native.FLAG_ACC_NAN:
            for table, dt in tables:
                bad = self.find_nan_clients(table, dt)
                if bad:
                    raise NaNAggregationError("input", f"NaN in client update(s) at table rows {bad}", bad)
            raise NaNAggregationError("accumulator", "NaN in the weighted sum (e.g. inf - inf)")
        raise NaNAggregationError("result", "NaN after dividing by the total weight (e.g. 0 / 0)")

    # -- measurement -------------------------------------------------------------------
    def prof_enable(self, on: bool = True) -> None:
        _native.check(self._lib.fedavg_prof_enable(self._h, 1 if on else 0))

    def prof_collect(self) -> tuple[float, int]:
        ms, n = ctypes.c_double(), ctypes.c_int32()
        _native.check(self._lib.fedavg_prof_collect(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


class AggregatePlan:
    """A prepared fused aggregation (``fedavg_plan_*``)."""

    def __init__(self, ctx: FedAvgContext, handle: ctypes.c_void_p, keep: tuple) -> None:
        self.ctx = ctx
        self._h = handle
        self._keep = keep
        ctx._plans.add(self)  # closed with the context (a native plan points at its context)

    def run(self) -> None:
        _native.check(self.ctx._lib.fedavg_plan_run(self._h, self.ctx.stream))

    def run_range(self, tile_begin: int, tile_end: int) -> None:
        _native.check(self.ctx._lib.fedavg_plan_run_range(self._h, tile_begin, tile_end, self.ctx.stream))

    # -- scatter exchange pieces (finalize plans; sharded.py) ---------------------------
    @property
    def out_dtype(self) -> torch.dtype:
        code = int(self.ctx._lib.fedavg_plan_out_dtype(self._h))
        return {_native.F32: torch.float32, _native.F64: torch.float64}[code]

    def finalize_window(self, src: torch.Tensor, lo: int, hi: int, res: torch.Tensor) -> None:
        """res[p] = src[p - lo] / W[seg(p)] over accumulator positions [lo, hi) (padding skipped);
        ``res`` is in accumulator coordinates, of the plan's out dtype."""
        if src.dtype != torch.float64 or src.numel() < hi - lo or res.dtype != self.out_dtype \
                or res.numel() < self.ctx.acc_numel or not (src.is_contiguous() and res.is_contiguous()):
            raise ValueError("window buffers do not match the plan")
        _native.check(self.ctx._lib.fedavg_plan_finalize_window(
            self._h, ctypes.c_void_p(src.data_ptr()), lo, hi, ctypes.c_void_p(res.data_ptr()), self.ctx.stream))

    def copy_out(self, res: torch.Tensor) -> None:
        """The plan's outputs <- res (accumulator coordinates)."""
        if res.dtype != self.out_dtype or res.numel() < self.ctx.acc_numel or not res.is_contiguous():
            raise ValueError("result buffer does not match the plan")
        _native.check(self.ctx._lib.fedavg_plan_copy_out(self._h, ctypes.c_void_p(res.data_ptr()), self.ctx.stream))

    def close(self) -> None:
        if self._h is not None and self._h.value:
            self.ctx._lib.fedavg_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self) -> None:  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def bw_probe(src: torch.Tensor, dst: torch.Tensor, mode: int) -> None:
    """HBM ceiling probe: mode 0 copies src->dst (16-B lanes), mode 1 only reads src."""
    lib = _native.load()
    nbytes = src.numel() * src.element_size()
    _native.check(
        lib.fedavg_bw_probe(
            ctypes.c_void_p(src.data_ptr()), nbytes, ctypes.c_void_p(dst.data_ptr()), mode,
            _stream_handle(src.device),
        )
    )
