"""Host-side handle on the PersonalizedFedAVG kernel (``fedavg_pers_*`` of include/fedavg_hip.h).

One ``PersonalizedContext`` per (layout, device). ``aggregate`` launches the whole round of
the reference's ``PersonalizedFedAVGAlgorithm`` (personalized_aggregation_algorithm.py:23-57)
— M per-receiver FedAvgs over N arrivals plus the centralized average — asynchronously on the
current torch stream; ``check`` drains the stream and reports the fused NaN assertions.
The arithmetic runs in ``csrc/personalized_kernels.hip``; there is no CPU path.
"""

from __future__ import annotations

import ctypes
from collections.abc import Sequence
from dataclasses import dataclass

import numpy as np
import torch

from . import _native, _staging
from .fedavg import ModelLayout, dtype_code, out_code

_PTR = ctypes.POINTER(ctypes.c_void_p)
# dtype codes of csrc/staging_ext.cpp (the kernel input / output dtypes)
_STAGING_CODES = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float64: 3}
_DBL = ctypes.POINTER(ctypes.c_double)
_I64 = ctypes.POINTER(ctypes.c_int64)


@dataclass(frozen=True)
class FlatOutputs:
    """Output rows as flat contiguous buffers, one per receiver (or one for the centralized
    model): segment t of row r starts at element ``offsets[t]`` of ``buffers[r]``. The table takes
    the pointers from the buffers' addresses — no tensor per segment is needed before the
    launch, so the per-segment result views can be made while the kernel runs."""

    buffers: Sequence[torch.Tensor]
    offsets: Sequence[int]


@dataclass(frozen=True)
class PersonalizedTables:
    """Validated device pointers of one round's clients and outputs (C-ABI arrays)."""

    num_clients: int
    num_receivers: int
    in_dtype: torch.dtype
    out_dtype: torch.dtype
    central_dtype: torch.dtype
    ptrs: np.ndarray
    optrs: np.ndarray
    cptrs: np.ndarray | None
    keep: tuple


class PersonalizedContext:
    def __init__(self, layout: ModelLayout, device: torch.device | str | int | None = None) -> None:
        self._lib = _native.load()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("the personalized HIP path runs on a GPU device")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if layout.num_segments == 0 or min(layout.numels) <= 0:
            raise ValueError("a native layout needs at least one tensor and no empty tensors")
        self.device = device
        self.layout = layout
        numels = (ctypes.c_int64 * layout.num_segments)(*layout.numels)
        handle = ctypes.c_void_p()
        _native.check(self._lib.fedavg_pers_create(ctypes.byref(handle), device.index, numels, layout.num_segments))
        self._h = handle
        self._keep: tuple = ()

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.fedavg_pers_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self) -> None:  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> ctypes.c_void_p:
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def set_fused_fold(self, enable: bool) -> None:
        _native.check(self._lib.fedavg_pers_set_fused_fold(self._h, 1 if enable else 0))

    def tables(
        self,
        clients: Sequence[Sequence[torch.Tensor | None]],
        in_dtype: torch.dtype,
        outs: Sequence[Sequence[torch.Tensor]] | FlatOutputs,
        out_dtype: torch.dtype,
        central: Sequence[torch.Tensor] | FlatOutputs | None = None,
        central_dtype: torch.dtype = torch.float64,
        client_ptrs: bytes | None = None,
    ) -> PersonalizedTables:
        """Validate the tensors of a round once (persistent client / output slots reuse it).
        ``client_ptrs``: the rows' device addresses ([N][T] uint64) when the caller already checked
        every client tensor against the layout and ``in_dtype`` (the staging extension's
        ``resident_row``); the rows are then only kept alive, not walked again."""
        T = self.layout.num_segments
        numels = self.layout.numels
        keep: list = []
        if client_ptrs is not None:
            ptrs = np.frombuffer(client_ptrs, dtype=np.uint64)
            if ptrs.size != len(clients) * T:
                raise ValueError("client pointer rows do not match the clients and the layout")
            keep.append(clients)
            clients_to_walk: Sequence = ()
        else:
            ptrs = np.zeros(len(clients) * T, dtype=np.uint64)
            clients_to_walk = clients
        # the checks + pointer pass of a row in one native call (csrc/staging_ext.cpp) when built;
        # a row it refuses goes through the loop below, which names the offending tensor
        ext = _staging.module() if self.device.type == "cuda" else None
        dev_idx = -1
        if ext is not None:
            dev_idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        in_code, out_code_, c_code = (_STAGING_CODES.get(in_dtype, -9), _STAGING_CODES.get(out_dtype, -9),
                                      _STAGING_CODES.get(central_dtype, -9))
        for k, row in enumerate(clients_to_walk):
            if len(row) != T:
                raise ValueError("client row does not match the layout")
            got = ext.row_pointers(list(row), numels, dev_idx, in_code) if ext is not None else None
            if got is not None:
                ptrs[k * T : (k + 1) * T] = got
                keep.append(row)
                continue
            for t, x in enumerate(row):
                if x is None:
                    continue
                if x.device != self.device or x.dtype != in_dtype or x.numel() != numels[t] or not x.is_contiguous():
                    raise ValueError("client tensors must be contiguous, on the device, of the input dtype and size")
                ptrs[k * T + t] = x.data_ptr()
                keep.append(x)
        n_recv = len(outs.buffers) if isinstance(outs, FlatOutputs) else len(outs)
        if isinstance(outs, FlatOutputs):
            optrs = self._flat_pointers(outs, out_dtype)
            keep.append(outs)
            outs = ()
        else:
            optrs = np.zeros(len(outs) * T, dtype=np.uint64)
        for j, row in enumerate(outs):
            got = ext.row_pointers(list(row), numels, dev_idx, out_code_) if ext is not None and len(row) == T else None
            if got is not None:
                optrs[j * T : (j + 1) * T] = got
                keep.append(row)
                continue
            for t, o in enumerate(row):
                if o.device != self.device or o.dtype != out_dtype or o.numel() != numels[t] or not o.is_contiguous():
                    raise ValueError("output tensors must be contiguous, on the device, of the output dtype and size")
                optrs[j * T + t] = o.data_ptr()
                keep.append(o)
        cptrs = None
        if isinstance(central, FlatOutputs):
            if len(central.buffers) != 1:
                raise ValueError("the centralized model is one flat buffer")
            cptrs = self._flat_pointers(central, central_dtype)
            keep.append(central)
            central = None
        elif central is not None:
            cptrs = np.zeros(T, dtype=np.uint64)
            got = ext.row_pointers(list(central), numels, dev_idx, c_code) if ext is not None and len(central) == T \
                else None
            for t, o in enumerate(central if got is None else ()):
                if o.device != self.device or o.dtype != central_dtype or o.numel() != numels[t] or not o.is_contiguous():
                    raise ValueError("centralized outputs must be contiguous, on the device, of the dtype and size")
                cptrs[t] = o.data_ptr()
                keep.append(o)
            if got is not None:
                cptrs[:] = got
                keep.append(central)
        return PersonalizedTables(len(clients), n_recv, in_dtype, out_dtype, central_dtype, ptrs, optrs, cptrs,
                                  tuple(keep))

    def _flat_pointers(self, flat: FlatOutputs, dtype: torch.dtype) -> np.ndarray:
        """[rows][T] segment pointers of flat output buffers (each checked: contiguous, 1-D, on the
        device, of ``dtype``, holding every segment)."""
        T = self.layout.num_segments
        offs = np.asarray(flat.offsets, dtype=np.int64)
        if offs.shape != (T,) or (T and offs.min() < 0):
            raise ValueError("one non-negative element offset per segment is required")
        need = int((offs + np.asarray(self.layout.numels, dtype=np.int64)).max()) if T else 0
        bases = []
        for b in flat.buffers:
            if (b.device != self.device or b.dtype != dtype or b.dim() != 1 or not b.is_contiguous()
                    or b.numel() < need):
                raise ValueError("flat outputs must be contiguous 1-D buffers on the device, of the output "
                                 "dtype, holding every segment")
            bases.append(b.data_ptr())
        esize = torch.empty((), dtype=dtype).element_size()
        return (np.asarray(bases, dtype=np.uint64)[:, None]
                + (offs.astype(np.uint64) * np.uint64(esize))[None, :]).reshape(-1)

    def aggregate(
        self,
        clients: Sequence[Sequence[torch.Tensor | None]] | PersonalizedTables,
        in_dtype: torch.dtype,
        client_ids: Sequence[int],
        weights: np.ndarray,
        receiver_ids: Sequence[int],
        outs: Sequence[Sequence[torch.Tensor]] | FlatOutputs | None = None,
        out_dtype: torch.dtype = torch.float64,
        central: Sequence[torch.Tensor] | FlatOutputs | None = None,
        central_dtype: torch.dtype = torch.float64,
        client_ptrs: bytes | None = None,
    ) -> None:
        """clients[N][T] (None = tensor not sent) or prepared tables, weights[M][N] float64
        (``client_ptrs``: see ``tables``)."""
        tab = clients if isinstance(clients, PersonalizedTables) else \
            self.tables(clients, in_dtype, outs or (), out_dtype, central, central_dtype, client_ptrs)
        N, M = tab.num_clients, len(receiver_ids)
        w = np.ascontiguousarray(weights, dtype=np.float64)
        if w.shape != (M, N) or len(client_ids) != N or tab.num_receivers != M:
            raise ValueError("clients, weights, ids and outputs disagree on N / M")
        cid = np.asarray(client_ids, dtype=np.int64)
        rid = np.asarray(receiver_ids, dtype=np.int64)
        self._keep = (tab, cid, rid, w)
        _native.check(
            self._lib.fedavg_pers_aggregate(
                self._h, tab.ptrs.ctypes.data_as(_PTR), dtype_code(tab.in_dtype), N, cid.ctypes.data_as(_I64),
                w.ctypes.data_as(_DBL), rid.ctypes.data_as(_I64), M, tab.optrs.ctypes.data_as(_PTR),
                out_code(tab.out_dtype), None if tab.cptrs is None else tab.cptrs.ctypes.data_as(_PTR),
                out_code(tab.central_dtype), self.stream,
            )
        )

    def check(self) -> int:
        """Drain the stream; returns the NaN flag bits (FLAG_ACC_NAN / RESULT / CENTRAL) and clears them."""
        flags = ctypes.c_uint32()
        self._lib.fedavg_pers_check(self._h, self.stream, ctypes.byref(flags))
        return int(flags.value)

    def prof_enable(self, on: bool = True) -> None:
        _native.check(self._lib.fedavg_pers_prof_enable(self._h, 1 if on else 0))

    def prof_collect(self) -> tuple[float, int]:
        ms, n = ctypes.c_double(), ctypes.c_int32()
        _native.check(self._lib.fedavg_pers_prof_collect(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


def fp64_probe(device: torch.device, waves: int = 256 * 4 * 8, iters: int = 4096) -> float:
    """Measured fp64 VALU ceiling (TFLOP/s) of independent v_fma_f64 chains."""
    lib = _native.load()
    out = ctypes.c_double()
    with torch.cuda.device(device):
        _native.check(lib.fedavg_fp64_probe(waves, iters, ctypes.byref(out),
                                            ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)))
    return out.value
