"""Clients sharded across the GPUs of a node, one RCCL reduce of the fp64 partials.

The reference has no collectives: every client update goes to the one server process
(SURVEY.md §5). When N × model bytes outgrows one GPU (BASELINE.json configs 3 and 5), the
clients are partitioned over the ranks (one process per GPU, ``torch.distributed`` with the
``nccl`` backend = RCCL over xGMI):

    rank r:  S_r = sum_{k in shard r} w_k x_k           (fp64, HIP partial kernel)
    root:    S   = sum_r S_r                            (RCCL reduce, chunked)
    root:    out = S / W                                (HIP finalize kernel, per chunk)

The partial is produced and reduced in chunks of tiles: the kernel for chunk c+1 runs on
the compute stream while RCCL reduces chunk c on its own stream; the root finalizes every
tile in one launch once the last reduce has landed. This is the only exchange step of the
path.

Numerics: each rank accumulates its clients in arrival order exactly like the single-GPU
kernel; the cross-rank sum reorders fp64 additions, so results match the reference to fp64
rounding (|Δ| ≤ 1e-12 relative; after an fp32 cast, identical in practice) instead of
bit-for-bit. Total weights: integer weights sum exactly; float weights to fp64 rounding.

``LocalReducer`` is the per-rank compute interface; ``HipLocalReducer`` is the product
implementation. Tests on CPU (gloo) plug a plain torch reducer in its place to cover the
chunking / collective / finalize logic without a GPU.
"""

from __future__ import annotations

import ctypes
from collections.abc import Sequence
from typing import Protocol

import torch
import torch.distributed as dist

from . import _native
from .fedavg import ClientTable, FedAvgContext, OutputTable


class LocalReducer(Protocol):
    accumulator: torch.Tensor

    @property
    def num_tiles(self) -> int: ...

    def tile_range(self, tile_begin: int, tile_end: int) -> tuple[int, int]: ...

    def partial(self, tile_begin: int, tile_end: int) -> None: ...

    def set_accumulated(self, total_weights: Sequence[float]) -> None: ...

    def finalize_range(self, tile_begin: int, tile_end: int) -> None: ...

    def fused(self) -> None: ...

    def prefold(self) -> None: ...


class HipLocalReducer:
    """The shard's clients, reduced by the HIP kernels of one FedAvgContext.

    ``prior_waves`` are client tables folded into the accumulator before the chunked last
    wave (streaming waves: BASELINE config 5 folds 1024 clients in waves).
    """

    def __init__(
        self,
        ctx: FedAvgContext,
        table: ClientTable | None,
        in_dtype: torch.dtype,
        outs: Sequence[torch.Tensor] | OutputTable | None,
        out_dtype: torch.dtype,
        prior_waves: Sequence[ClientTable] = (),
        use_plan: bool = True,
    ) -> None:
        self.ctx = ctx
        self.use_plan = use_plan
        self._plan = None
        self.table = table
        self.in_dtype = in_dtype
        self.outs = outs
        self.out_dtype = out_dtype
        self.prior_waves = list(prior_waves)
        self.accumulator = ctx.accumulator
        self._partial_plan = None
        self._finalize_plan = None
        self._finalize_totals: list[float] | None = None

    @property
    def num_tiles(self) -> int:
        return self.ctx.num_tiles

    def tile_range(self, tile_begin: int, tile_end: int) -> tuple[int, int]:
        return self.ctx.tile_range(tile_begin, tile_end)

    def prefold(self) -> None:
        """Fold the prior waves (if any) into the accumulator, in order."""
        self.ctx.reset()
        for t in self.prior_waves:
            self.ctx.accumulate(t, self.in_dtype)

    def partial(self, tile_begin: int, tile_end: int) -> None:
        # prepared once: each chunk is a bare launch (the host must stay ahead of 8 chunk
        # kernels of ~65 us each, or the GPU idles between them)
        if self.use_plan:
            if self._partial_plan is None:
                self._partial_plan = self.ctx.plan_partial(self.table, self.in_dtype, zero_init=not self.prior_waves)
            self._partial_plan.run_range(tile_begin, tile_end)
        else:
            self.ctx.partial(self.table, self.in_dtype, zero_init=not self.prior_waves,
                             tile_begin=tile_begin, tile_end=tile_end)

    def set_accumulated(self, total_weights: Sequence[float]) -> None:
        totals = [float(w) for w in total_weights]
        if self.use_plan:
            if self._finalize_plan is None or self._finalize_totals != totals:
                assert self.outs is not None
                self._finalize_plan = self.ctx.plan_finalize(totals, self.outs, self.out_dtype)
                self._finalize_totals = totals
        else:
            self.ctx.set_accumulated(totals)

    def finalize_range(self, tile_begin: int, tile_end: int) -> None:
        assert self.outs is not None
        if self.use_plan:
            assert self._finalize_plan is not None
            self._finalize_plan.run_range(tile_begin, tile_end)
        else:
            self.ctx.finalize_range(self.outs, self.out_dtype, tile_begin, tile_end)

    def native_round(self, comm: RcclComm, total_weights: Sequence[float], chunks: int, root: int) -> None:
        """One round through the library's own RCCL pipeline (``fedavg_sharded_round``): the
        chunk launches, the reduces and the finalize are enqueued by one native call."""
        assert self.use_plan and self.table is not None
        if self._partial_plan is None:
            self._partial_plan = self.ctx.plan_partial(self.table, self.in_dtype, zero_init=not self.prior_waves)
        fin = None
        if comm.rank == root:
            self.set_accumulated(total_weights)
            fin = self._finalize_plan._h
        _native.check(self.ctx._lib.fedavg_sharded_round(comm.handle, self.ctx._h, self._partial_plan._h, fin,
                                                         chunks, root, self.ctx.stream))

    def fused(self) -> None:
        """Single-rank shortcut: fold + divide in the last wave's launch, no extra fp64 pass."""
        assert self.outs is not None
        if self.use_plan and not self.prior_waves and self.table is not None:
            # persistent client slots: the table is staged once, each round is one launch
            if self._plan is None:
                self._plan = self.ctx.plan(self.table, self.in_dtype, self.outs, self.out_dtype)
            self._plan.run()
            return
        self.prefold()
        self.ctx.aggregate(self.table, self.in_dtype, self.outs, self.out_dtype)


class RcclComm:
    """The library's own RCCL communicator (``fedavg_comm_*``), one per process / GPU.

    Rank 0 of ``group`` makes the RCCL unique id; it is shipped to the other ranks over the
    existing process group (any backend), then every rank joins (collective). The library binds
    the process's RCCL (torch's) at run time; see ``sharded_comm.cpp``.
    """

    def __init__(self, device: torch.device, group: dist.ProcessGroup | None = None) -> None:
        self._lib = _native.load()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        uid = torch.zeros(_native.COMM_ID_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            _native.check(self._lib.fedavg_comm_unique_id(ctypes.c_void_p(uid.data_ptr())))
        on_device = dist.get_backend(group) == "nccl"
        t = uid.to(device) if on_device else uid
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(t, src=src, group=group)
        uid = t.cpu() if on_device else t
        h = ctypes.c_void_p()
        _native.check(self._lib.fedavg_comm_create(ctypes.byref(h), ctypes.c_void_p(uid.data_ptr()), self.world,
                                                   self.rank, device.index or 0))
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None) is not None and self.handle.value:
            self._lib.fedavg_comm_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self) -> None:  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def chunk_bounds(num_tiles: int, chunks: int) -> list[tuple[int, int]]:
    chunks = max(1, min(chunks, num_tiles))
    edges = [round(i * num_tiles / chunks) for i in range(chunks + 1)]
    return [(edges[i], edges[i + 1]) for i in range(chunks) if edges[i + 1] > edges[i]]


def sharded_reduce(
    reducer: LocalReducer,
    local_total_weights: Sequence[float],
    chunks: int = 4,
    root: int = 0,
    group: dist.ProcessGroup | None = None,
    global_total_weights: Sequence[float] | None = None,
    force_collective: bool = False,
    comm: RcclComm | None = None,
) -> list[float]:
    """One FedAvg reduce over every rank's shard; the result lands in the root's outputs.

    ``local_total_weights`` are this rank's per-segment sums of client weights. When the
    caller already knows the global totals (the dispatcher that assigned clients to ranks
    knows every client's weight) it passes ``global_total_weights`` and no collective is
    spent on them; otherwise they are all-reduced first. Returns the global totals. On a
    one-rank world the fused single-launch kernel is used (no fp64 round trip) unless
    ``force_collective`` (tests / measurement of the sharded path on one GPU). With ``comm``
    (the library's own RCCL communicator) a HIP reducer runs the whole round in one native call
    (``fedavg_sharded_round``); otherwise the chunks' reduces go through ``torch.distributed``.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1 and not (force_collective and dist.is_initialized()):
        reducer.fused()
        return list(local_total_weights)
    rank = dist.get_rank(group)
    if global_total_weights is None:
        totals = torch.tensor([float(w) for w in local_total_weights], dtype=torch.float64,
                              device=reducer.accumulator.device)
        dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)
        global_total_weights = totals.tolist()
    global_totals = [float(w) for w in global_total_weights]
    reducer.prefold()
    if comm is not None and hasattr(reducer, "native_round"):
        reducer.native_round(comm, global_totals, chunks, root)
        return global_totals
    bounds = chunk_bounds(reducer.num_tiles, chunks)
    acc = reducer.accumulator
    # Each chunk's reduce is issued right after its partial kernel, from the compute stream:
    # the process group's RCCL stream waits only for that chunk's kernel (an event on the
    # compute stream) and reduces chunk c while the kernel for chunk c+1 runs. No intermediate
    # "comm" stream: HIP maps streams onto a few hardware queues in order, and a wait parked
    # in a queue shared with the compute stream would hold every reduce behind the last
    # partial (kernel traces: scripts/gpu_sharded_trace.sh).
    works = []
    for tb, te in bounds:
        reducer.partial(tb, te)
        a, b = reducer.tile_range(tb, te)
        works.append(dist.reduce(acc[a:b], dst=root, op=dist.ReduceOp.SUM, group=group, async_op=True))
    # The collectives of one process group run on one RCCL stream and complete in issue
    # order, so on the GPU one wait (the last reduce) covers every chunk: one cross-stream
    # dependency instead of one per chunk. Host backends (gloo) wait for each work.
    for w in (works[-1:] if acc.is_cuda else works):
        w.wait()
    if rank == root:
        reducer.set_accumulated(global_totals)
        reducer.finalize_range(0, reducer.num_tiles)  # one launch over every tile
    return global_totals
