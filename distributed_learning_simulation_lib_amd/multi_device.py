"""One server process, several MI355X: the single-process multi-device mode of the FedAvg reduce.

The reference aggregates in ONE server process: ``Server.start`` polls the workers
(``simulation_lib/server/server.py:122-152``) and ``AggregationServer._process_worker_data``
hands every update to the algorithm (``simulation_lib/server/aggregation_server.py:111-145``).
``MultiDeviceContext`` lets that process spread the client sum of ``fed_avg_algorithm.py:43-64``
over a device list (``include/fedavg_hip.h`` ``fedavg_multi_*``, ``csrc/multi_device.cpp``):

  * one ``FedAvgContext`` per device entry (``contexts[g]``): the shard's arrival-order fold, with
    every single-device call (waves, deltas, quantised records, plans);
  * ``round``: one round of device-resident clients from per-device partial plans — chunked, with
    the peer-window exchange (each device stores its fp64 partial of window j straight into device
    j's receive slot over xGMI; device j sums the G partials in device order and divides into the
    root's outputs) or an in-process RCCL reduce;
  * ``combine``: the streaming form — every context's accumulator already holds its shard's
    partial (``FedAVGAlgorithm(devices=[...])`` folds its waves per device), one exchange.

Parity: each device's fold is the reference's chain over its clients; ``peer`` sums the partials
in device order, so a result equals the host composition S_0 + S_1 + ... + S_{G-1} divided by the
arrival-order total weight bit for bit (and the reference's single chain to fp64 rounding).
Entries may repeat a device (``devices=[0, 0, 0, 0]``): the tests run the whole exchange on one GPU.
"""

from __future__ import annotations

import ctypes
from collections.abc import Sequence

import torch

from . import _native
from .fedavg import AggregatePlan, ClientTable, FedAvgContext, ModelLayout, NaNAggregationError, OutputTable, out_code

EXCHANGES = {"peer": _native.EXCHANGE_PEER, "reduce": _native.EXCHANGE_REDUCE}


def _as_device(d: int | str | torch.device) -> torch.device:
    dev = torch.device("cuda", d) if isinstance(d, int) else torch.device(d)
    if dev.type != "cuda":
        raise ValueError(f"the multi-device FedAvg path runs on GPU devices, not {dev}")
    return torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())


def exchange_code(exchange: str) -> int:
    try:
        return EXCHANGES[exchange]
    except KeyError:
        raise ValueError(f"exchange must be one of {sorted(EXCHANGES)}, not {exchange!r}") from None


def window_bounds(tb: int, te: int, world: int) -> list[tuple[int, int]]:
    """The G windows of chunk [tb, te): entry j owns tiles [tb + span*j//G, tb + span*(j+1)//G)
    (multi_device.cpp's split)."""
    span = te - tb
    return [(tb + span * j // world, tb + span * (j + 1) // world) for j in range(world)]


class MultiDeviceContext:
    """``fedavg_multi``: the per-device contexts of one layout and the exchange between them."""

    def __init__(self, layout: ModelLayout, devices: Sequence[int | str | torch.device],
                 lib: ctypes.CDLL | None = None) -> None:
        self._lib = lib if lib is not None else _native.load()
        self.devices = [_as_device(d) for d in devices]
        if not 1 <= len(self.devices) <= _native.MULTI_MAX_DEVICES:
            raise ValueError(f"1 to {_native.MULTI_MAX_DEVICES} device entries")
        if layout.num_segments == 0 or min(layout.numels) <= 0:
            raise ValueError("a native layout needs at least one tensor and no empty tensors")
        self.layout = layout
        G = len(self.devices)
        acc_numel = FedAvgContext._padded_acc_numel(layout, self._lib)
        # caller-owned accumulators (torch tensors): views, collectives and layout migrations use them
        self._accs = [torch.zeros(acc_numel, dtype=torch.float64, device=d) for d in self.devices]
        devs = (ctypes.c_int32 * G)(*[d.index for d in self.devices])
        numels = (ctypes.c_int64 * layout.num_segments)(*layout.numels)
        accs = (ctypes.c_void_p * G)(*[a.data_ptr() for a in self._accs])
        h = ctypes.c_void_p()
        _native.check(self._lib.fedavg_multi_create(ctypes.byref(h), devs, G, numels, layout.num_segments, accs))
        self._h = h
        self.contexts = [
            FedAvgContext.borrowed(self._lib, self._lib.fedavg_multi_context(h, g), layout, self.devices[g], self._accs[g])
            for g in range(G)
        ]

    @property
    def world(self) -> int:
        return len(self.devices)

    @property
    def peer_access(self) -> bool:
        return bool(self._lib.fedavg_multi_peer_access(self._h))

    @property
    def num_tiles(self) -> int:
        return self.contexts[0].num_tiles

    def _streams(self) -> ctypes.Array:
        """The current torch stream of every entry (the order the caller's work runs in)."""
        return (ctypes.c_void_p * self.world)(*[torch.cuda.current_stream(d).cuda_stream for d in self.devices])

    def _outs(self, outs: Sequence[torch.Tensor] | OutputTable, out_dtype: torch.dtype, root: int) -> ctypes.Array:
        if isinstance(outs, OutputTable):
            if outs.dtype != out_dtype or outs.layout != self.layout or outs.device != self.devices[root]:
                raise ValueError("output table was built for another dtype, layout or device")
            return outs.c_array
        return OutputTable(outs, self.layout, self.devices[root], out_dtype).c_array

    def plan_partials(self, tables: Sequence[ClientTable | None], in_dtype: torch.dtype) -> list[AggregatePlan | None]:
        """One zero-initialised partial plan per entry (None where the entry holds no client)."""
        if len(tables) != self.world:
            raise ValueError("one client table (or None) per device entry")
        return [None if t is None or t.num_clients == 0 else self.contexts[g].plan_partial(t, in_dtype, zero_init=True)
                for g, t in enumerate(tables)]

    def round(self, partials: Sequence[AggregatePlan | None], total_weights: Sequence[float],
              outs: Sequence[torch.Tensor] | OutputTable, out_dtype: torch.dtype, root: int = 0,
              edges: Sequence[int] | None = None, exchange: str = "peer") -> None:
        """One round of device-resident clients (``fedavg_multi_round``), asynchronous on the
        entries' current streams; ``check`` / ``raise_on_nan`` read the NaN flags."""
        if len(partials) != self.world:
            raise ValueError("one partial plan (or None) per device entry")
        for g, p in enumerate(partials):
            if p is not None and p.ctx is not self.contexts[g]:
                raise ValueError(f"partial plan {g} was not made on entry {g}'s context")
        plans = (ctypes.c_void_p * self.world)(*[None if p is None else p._h.value for p in partials])
        tw = (ctypes.c_double * self.layout.num_segments)(*[float(w) for w in total_weights])
        e = list(edges) if edges is not None else [0, self.num_tiles]
        ea = (ctypes.c_int32 * len(e))(*e)
        _native.check(self._lib.fedavg_multi_round(self._h, plans, tw, self._outs(outs, out_dtype, root),
                                                   out_code(out_dtype), root, ea, len(e), exchange_code(exchange),
                                                   self._streams()))

    def combine(self, total_weights: Sequence[float], outs: Sequence[torch.Tensor] | OutputTable,
                out_dtype: torch.dtype, root: int = 0, exchange: str = "peer") -> None:
        """Sum the contexts' accumulators (each a shard's partial) in device order, divide by
        ``total_weights`` into the root's outputs; resets every context's accumulated state."""
        tw = (ctypes.c_double * self.layout.num_segments)(*[float(w) for w in total_weights])
        _native.check(self._lib.fedavg_multi_combine(self._h, tw, self._outs(outs, out_dtype, root), out_code(out_dtype),
                                                     root, exchange_code(exchange), self._streams()))

    def flags(self, round_only: bool = False) -> int:
        """Synchronise every stream of the object (``round_only``: wait for the end of the last
        round / combine alone, ``fedavg_multi_round_check``); the OR of every entry's NaN flag bits."""
        f = ctypes.c_uint32()
        fn = self._lib.fedavg_multi_round_check if round_only else self._lib.fedavg_multi_check
        st = fn(self._h, ctypes.byref(f))
        if st not in (_native.OK, _native.ERR_NAN_ACCUM, _native.ERR_NAN_RESULT):
            _native.check(st)
        return int(f.value)

    def reset(self) -> None:
        _native.check(self._lib.fedavg_multi_reset(self._h))

    def prof_enable(self, on: bool = True) -> None:
        """Time every following round with events on entry 0's stream (fedavg_multi_prof_enable)."""
        _native.check(self._lib.fedavg_multi_prof_enable(self._h, 1 if on else 0))

    def prof_collect(self) -> tuple[float, float, int]:
        """(fold ms, tail ms, rounds) summed over the rounds timed since the last collect: entry 0's
        round start -> its last chunk fold, and that fold -> the round's end behind every exchange."""
        fold, tail, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
        _native.check(self._lib.fedavg_multi_prof_collect(self._h, ctypes.byref(fold), ctypes.byref(tail),
                                                          ctypes.byref(n)))
        return float(fold.value), float(tail.value), int(n.value)

    def raise_on_nan(self, pending: Sequence[Sequence[tuple[ClientTable, torch.dtype]]] = (),
                     round_only: bool = False) -> None:
        """The reference's assertions (fed_avg_algorithm.py:35,93,97) for the whole round: an input
        NaN in a table the caller still holds (``pending[g]``: entry g's tables) names its clients
        (:35); otherwise a NaN sum (e.g. inf - inf across shards) is :93, a NaN quotient :97.
        ``round_only``: the per-round form — wait for the last round's end event only."""
        f = self.flags(round_only)
        if f == 0:
            return
        self.reset()
        if f & _native.FLAG_ACC_NAN:
            for g, tables in enumerate(pending):
                for table, dt in tables:
                    bad = self.contexts[g].find_nan_clients(table, dt)
                    if bad:
                        raise NaNAggregationError("input", f"NaN in client update(s) at table rows {bad} of device "
                                                  f"entry {g}", bad)
            raise NaNAggregationError("accumulator", "NaN in the weighted sum (e.g. inf - inf)")
        raise NaNAggregationError("result", "NaN after dividing by the total weight (e.g. 0 / 0)")

    def close(self) -> None:
        for c in getattr(self, "contexts", []):
            c.close()
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.fedavg_multi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self) -> None:  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

