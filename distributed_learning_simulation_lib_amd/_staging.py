"""Loader of the host-side staging extension (``csrc/staging_ext.cpp``, built in-tree by
``build.build_staging``). Loaded from its file without any build step at run time; ``None`` when
it is absent, and the plugin then stages updates in Python (same results, more host time)."""

from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import warnings
from types import ModuleType

import torch  # noqa: F401  (the extension links against torch's libraries)

from .build import STAGING_NAME, STAGING_PATH

_module: ModuleType | None = None
_tried = False


def module() -> ModuleType | None:
    global _module, _tried
    if not _tried:
        _tried = True
        if STAGING_PATH.exists() and os.environ.get("FEDAVG_PY_STAGING") != "1":
            try:
                loader = importlib.machinery.ExtensionFileLoader(STAGING_NAME, str(STAGING_PATH))
                spec = importlib.util.spec_from_file_location(STAGING_NAME, str(STAGING_PATH), loader=loader)
                assert spec is not None
                mod = importlib.util.module_from_spec(spec)
                loader.exec_module(mod)
                _module = mod
            except (ImportError, OSError) as e:  # e.g. built against another torch: stage in Python
                warnings.warn(f"staging extension {STAGING_PATH} not loadable ({e}); staging in Python",
                              RuntimeWarning, stacklevel=2)
    return _module


class NativeClientTable:
    """The ``fedavg.ClientTable`` protocol over the extension's native ``Rows`` (one wave's
    [num_clients][num_segments] pointers / weights / element counts, kept in C++ and appended to
    by one call per update: ``rows.append``, staging_ext.cpp). Scalar weights only: per-element
    weights use ``ClientTable``. The cached arrays and validations are keyed by the row count, so
    appends straight to ``rows`` need no bookkeeping here."""

    def __init__(self, num_segments: int, device_index: int) -> None:
        mod = module()
        if mod is None:
            raise RuntimeError("the staging extension is not built")
        self.rows = mod.Rows(num_segments, device_index)
        self.num_segments = num_segments
        self.device_index = device_index
        self._validated: set = set()
        self._arrays = None

    @property
    def num_clients(self) -> int:
        return self.rows.num_clients

    def add_resident_client(self, ptrs, weights, numels, esize, device_index, keep) -> None:
        if device_index != self.device_index:
            raise ValueError(f"a row on device {device_index} for a table of device {self.device_index}")
        self.rows.append_row(list(ptrs), [float(w) for w in weights], list(numels), esize, list(keep))

    def add_client(self, tensors, weights, weight_tensors=None) -> None:
        if weight_tensors is not None and any(w is not None for w in weight_tensors):
            raise ValueError("per-element weights need fedavg.ClientTable")
        if len(tensors) != self.num_segments or len(weights) != self.num_segments:
            raise ValueError("client row does not match the layout")
        ptrs, nums, ws, keep, esize = [], [], [], [], 0
        for t, w in zip(tensors, weights):
            if t is None:
                ptrs.append(0)
                nums.append(-1)
                ws.append(0.0)
                continue
            if not t.is_contiguous():
                raise ValueError("client tensors must be contiguous (the kernel reads them as flat buffers)")
            if t.get_device() != self.device_index:
                raise ValueError(f"a tensor on device {t.get_device()} for a table of device {self.device_index}")
            if esize and t.element_size() != esize:
                raise ValueError("one element size per client row")
            esize = t.element_size()
            ptrs.append(t.data_ptr())
            nums.append(t.numel())
            ws.append(float(w))
            keep.append(t)
        self.add_resident_client(ptrs, ws, nums, esize or (self.rows.esize or 4), self.device_index, keep)

    def validate(self, numels, esize: int, device_index: int, key) -> None:
        n = self.num_clients
        if (key, n) in self._validated or n == 0:
            return
        msg = self.rows.validate([int(x) for x in numels], int(esize), int(device_index))
        if msg:
            raise ValueError(msg)
        self._validated.add((key, n))

    def arrays(self):
        import numpy as np

        n = self.num_clients
        if self._arrays is None or self._arrays[0] != n:
            if n == 0:
                arrs = (np.zeros(1, np.uint64), np.zeros(1, np.float64))
            else:
                arrs = (np.frombuffer(self.rows.ptr_bytes(), dtype=np.uint64),
                        np.frombuffer(self.rows.weight_bytes(), dtype=np.float64))
            self._arrays = (n, arrs)
        return self._arrays[1]

    def addresses(self) -> tuple[int, int]:
        """Host addresses of the pointer / weight arrays (valid until the next append)."""
        return self.rows.ptr_addr(), self.rows.weight_addr()

    def elementwise_arrays(self):
        raise NotImplementedError("per-element weights need fedavg.ClientTable")


class TableTail:
    """Rows [offset, n) of a NativeClientTable (the ClientTable protocol): what the ordinary
    waves still fold after a dynamic wave folded rows [0, offset) (fedavg_dyn_close)."""

    def __init__(self, table: NativeClientTable, offset: int) -> None:
        self.table = table
        self.offset = int(offset)
        self.num_segments = table.num_segments
        self.device_index = table.device_index

    @property
    def num_clients(self) -> int:
        return self.table.num_clients - self.offset

    def validate(self, numels, esize: int, device_index: int, key) -> None:
        self.table.validate(numels, esize, device_index, key)

    def arrays(self):
        p, w = self.table.arrays()
        o = self.offset * self.num_segments
        return p[o:], w[o:]

    def addresses(self) -> tuple[int, int]:
        p, w = self.table.addresses()
        o = self.offset * self.num_segments * 8
        return p + o, w + o

    def elementwise_arrays(self):
        raise NotImplementedError("per-element weights need fedavg.ClientTable")
