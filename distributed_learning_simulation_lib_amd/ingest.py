"""Host-to-HBM ingest of client updates that arrive in host memory.

The reference server receives every update as CPU tensors unpickled from a pipe
(aggregation_server.py:129, aggregation_worker.py:152). Moving such a pageable tensor with
``t.to(device)`` goes through the runtime's own bounce buffers at ~19 GB/s
(``scripts/ingest_probe.py``). Here each client's tensors are packed into a pinned staging
bucket (a ring of two) by ONE native call (``fedavg_host_pack``: a pool of host threads copies
equal byte ranges across the tensors), then one asynchronous DMA moves the bucket into a
device bucket on the compute stream — the host packs client k+1 while the DMA of client k
runs.

The device bucket uses 16-byte aligned segment offsets, so the fold kernel takes its
vector path. Ordering: the DMA and the fold kernel are on the same stream; a pinned bucket
is reused only after the DMA that read it has completed (event wait on the host).
"""

from __future__ import annotations

import ctypes
from collections.abc import Sequence

import torch

from . import _native
from .fedavg import ModelLayout


class HostIngest:
    def __init__(self, device: torch.device, ring: int = 2) -> None:
        self.device = device
        self.ring = ring
        self._pinned: dict[tuple[torch.dtype, int], list[torch.Tensor]] = {}
        self._events: dict[tuple[torch.dtype, int], list[torch.cuda.Event | None]] = {}
        self._next: dict[tuple[torch.dtype, int], int] = {}
        self.bytes_moved = 0
        self._lib = _native.load()

    def _slot(self, dtype: torch.dtype, numel: int) -> tuple[torch.Tensor, int, tuple[torch.dtype, int]]:
        key = (dtype, numel)
        if key not in self._pinned:
            self._pinned[key] = [torch.empty(numel, dtype=dtype).pin_memory() for _ in range(self.ring)]
            self._events[key] = [None] * self.ring
            self._next[key] = 0
        i = self._next[key]
        self._next[key] = (i + 1) % self.ring
        ev = self._events[key][i]
        if ev is not None:
            ev.synchronize()  # the DMA that last read this pinned bucket has finished
        return self._pinned[key][i], i, key

    def to_device(
        self, layout: ModelLayout, tensors: Sequence[torch.Tensor | None], dtype: torch.dtype
    ) -> list[torch.Tensor | None]:
        """Device copies of one client's tensors (``None`` stays ``None``), in layout order."""
        elem = torch.empty((), dtype=dtype).element_size()
        offs, padded = layout.padded_offsets(elem)
        host, i, key = self._slot(dtype, padded)
        # one native call packs every tensor (host_pack.cpp, a pool of host threads)
        srcs = [None if t is None else (t if t.is_contiguous() else t.contiguous()) for t in tensors]
        n = len(srcs)
        ptrs = (ctypes.c_void_p * n)(*[0 if t is None else t.data_ptr() for t in srcs])
        nbytes = (ctypes.c_int64 * n)(*[0 if t is None else t.numel() * elem for t in srcs])
        doff = (ctypes.c_int64 * n)(*[o * elem for o in offs])
        _native.check(self._lib.fedavg_host_pack(ctypes.c_void_p(host.data_ptr()), ptrs, nbytes, doff, n))
        stream = torch.cuda.current_stream(self.device)
        bucket = torch.empty(padded, dtype=dtype, device=self.device)
        bucket.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        self._events[key][i] = ev
        self.bytes_moved += padded * elem
        return [None if t is None else bucket[o : o + n] for t, o, n in zip(tensors, offs, layout.numels)]

    def to_device_pointers(
        self, layout: ModelLayout, ptrs: Sequence[int], numels: Sequence[int], dtype: torch.dtype
    ) -> tuple[torch.Tensor, list[int]]:
        """The same transfer for a row the caller has already checked (contiguous host tensors of
        ``dtype``: their data pointers, ``numels`` = -1 where absent, layout order). Returns the
        device bucket (keep it alive with the row) and the device pointer of each segment
        (0 where absent) — no per-tensor views are made."""
        elem = dtype.itemsize
        offs, padded = layout.padded_offsets(elem)
        host, i, key = self._slot(dtype, padded)
        n = len(ptrs)
        _native.check(self._lib.fedavg_host_pack(
            ctypes.c_void_p(host.data_ptr()), (ctypes.c_void_p * n)(*ptrs),
            (ctypes.c_int64 * n)(*[m * elem if m > 0 else 0 for m in numels]),
            (ctypes.c_int64 * n)(*[o * elem for o in offs]), n))
        stream = torch.cuda.current_stream(self.device)
        bucket = torch.empty(padded, dtype=dtype, device=self.device)
        bucket.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        self._events[key][i] = ev
        self.bytes_moved += padded * elem
        base = bucket.data_ptr()
        return bucket, [base + o * elem if m >= 0 else 0 for o, m in zip(offs, numels)]
