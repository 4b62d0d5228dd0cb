"""Client updates sharded by element range across the GPUs of a node (the
alternative to sharding by client).

Rank r owns the flat element range [lo_r, hi_r) of the model — its tensors in dict order,
concatenated — and folds that range over *every* client in arrival order. Each element therefore
goes through the reference's single chain (fed_avg_algorithm.py:43-64, then the division at
:76-99) on exactly one GPU: the result is bit-identical to the one-GPU kernel and to the
reference at any world size, with no cross-rank fp64 sum. The exchange is a gather of the
finished result, in the output dtype, to the root — (G-1)/G of the fp32 model into the root
instead of the fp64 partial of the client-sharded round — plus one flag word for the NaN
assertions (:35, :93, :97), which every rank raises together.

It fits when updates arrive in host memory (the bytes of range r of each client cross rank r's own
PCIe link, so ingest scales with the GPUs) or are produced distributed. BASELINE config 3 itself
shards whole clients (``sharded.py``); ``bench.py --shard elements`` runs this form on the same
256 × ResNet-18 job.
"""

from __future__ import annotations

import bisect
from collections.abc import Sequence
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .fedavg import ClientTable, FedAvgContext, ModelLayout, NaNAggregationError, OutputTable
from . import _native
from .sharded import union_flags

RANGE_ALIGN = 4096  # range boundaries fall on multiples of this many elements (16-B aligned views)
_FLAG_LOCAL_ERROR = 0x100  # a rank's fold raised (e.g. nothing to aggregate): every rank raises


def element_ranges(total: int, world: int, align: int = RANGE_ALIGN) -> list[tuple[int, int]]:
    """[lo, hi) per rank: contiguous, covering [0, total), boundaries at multiples of ``align``,
    as even as that allows (a rank may get an empty range when total < world * align)."""
    if world < 1 or total < 0 or align < 1:
        raise ValueError("bad world / total / align")
    units = -(-total // align)
    per, extra = divmod(units, world)
    out, u = [], 0
    for r in range(world):
        n = per + (1 if r < extra else 0)
        lo, hi = min(u * align, total), min((u + n) * align, total)
        out.append((lo, hi))
        u += n
    return out


def layout_ranges(layout: ModelLayout, world: int, align: int = RANGE_ALIGN) -> list[tuple[int, int]]:
    """[lo, hi) per rank over the flat layout, cut only where a piece starts on a multiple of
    ``align`` elements *of its own segment* (or at a segment start), so every rank's views keep
    the tensors' 16-B alignment (the kernel's vector path), as close to equal as those cuts allow."""
    if world < 1 or align < 1:
        raise ValueError("bad world / align")
    cuts, off = [], 0
    for n in layout.numels:
        cuts.extend(range(off, off + n, align))
        off += n
    total = off
    cuts.append(total)
    bounds = [0]
    for r in range(1, world):
        target = round(r * total / world)
        i = bisect.bisect_left(cuts, target)
        cand = [c for c in (cuts[i - 1] if i > 0 else None, cuts[i] if i < len(cuts) else None) if c is not None]
        best = min(cand, key=lambda c: (abs(c - target), c))
        bounds.append(max(best, bounds[-1]))
    bounds.append(total)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


@dataclass(frozen=True)
class RangePiece:
    """Elements [lo, hi) of segment ``seg`` (segment-local indices)."""

    seg: int
    lo: int
    hi: int


def range_pieces(layout: ModelLayout, lo: int, hi: int) -> list[RangePiece]:
    """The segments' parts that fall in the flat range [lo, hi), in layout order."""
    out, off = [], 0
    for s, n in enumerate(layout.numels):
        a, b = max(lo, off), min(hi, off + n)
        if b > a:
            out.append(RangePiece(s, a - off, b - off))
        off += n
    return out


class RangeShard:
    """This rank's element range: its pieces, their sub-layout and a FedAvgContext over it."""

    def __init__(self, layout: ModelLayout, world: int, rank: int, device: torch.device | None,
                 align: int = RANGE_ALIGN) -> None:
        self.layout = layout
        self.world, self.rank = world, rank
        self.ranges = layout_ranges(layout, world, align)
        self.lo, self.hi = self.ranges[rank]
        self.pieces = range_pieces(layout, self.lo, self.hi)
        self.sub_layout = ModelLayout(
            names=tuple(f"{layout.names[p.seg]}[{p.lo}:{p.hi}]" for p in self.pieces),
            shapes=tuple((p.hi - p.lo,) for p in self.pieces),
        ) if self.pieces else None
        self.device = device
        self.ctx = FedAvgContext(self.sub_layout, device) if (self.pieces and device is not None) else None
        self._outs: dict[torch.dtype, tuple[torch.Tensor, OutputTable]] = {}

    def views(self, tensors: Sequence[torch.Tensor | None]) -> list[torch.Tensor | None]:
        """One client's tensors (the full layout, contiguous) -> this rank's pieces (views)."""
        out = []
        for p in self.pieces:
            t = tensors[p.seg]
            out.append(None if t is None else t.reshape(-1)[p.lo:p.hi])
        return out

    def local_output(self, out_dtype: torch.dtype) -> tuple[torch.Tensor, OutputTable | None]:
        """The rank's result, contiguous (hi - lo elements), and its per-piece output table."""
        if out_dtype not in self._outs:
            flat = torch.empty(self.hi - self.lo, dtype=out_dtype, device=self.device)
            table = None
            if self.pieces and self.ctx is not None:
                offs, pos = [], 0
                for p in self.pieces:
                    offs.append(pos)
                    pos += p.hi - p.lo
                table = OutputTable([flat[o : o + p.hi - p.lo] for o, p in zip(offs, self.pieces)],
                                    self.sub_layout, self.device, out_dtype)
            self._outs[out_dtype] = (flat, table)
        return self._outs[out_dtype]

    def fold(self, table: ClientTable | None, in_dtype: torch.dtype, out_dtype: torch.dtype) -> torch.Tensor:
        """Fold + divide this rank's range (one fused launch); returns the local result. A rank
        with elements but no clients raises, as the reference does with nothing accumulated."""
        flat, outs = self.local_output(out_dtype)
        if self.ctx is not None:
            if table is None or table.num_clients == 0:
                raise RuntimeError("nothing to aggregate in this rank's range (fed_avg_algorithm.py:88)")
            self.ctx.aggregate(table, in_dtype, outs, out_dtype)
        return flat

    def flags(self) -> int:
        return self.ctx.flags() if self.ctx is not None else 0

    def raise_local(self, tables: Sequence[tuple[ClientTable, torch.dtype]]) -> None:
        if self.ctx is not None:
            self.ctx.raise_on_nan(tables)


def range_sharded_reduce(
    shard: RangeShard,
    table: ClientTable | None,
    in_dtype: torch.dtype,
    out: torch.Tensor | None,
    out_dtype: torch.dtype = torch.float32,
    root: int = 0,
    group: dist.ProcessGroup | None = None,
) -> None:
    """One FedAvg round over element ranges; the root's ``out`` (flat, layout.total_numel
    elements of ``out_dtype``, tensors concatenated in layout order) receives the model.

    ``table`` holds this rank's views of every client (``shard.views``) with the segment weights.
    Collective over ``group`` (``root`` is a group rank). The NaN assertions
    (fed_avg_algorithm.py:35,93,97) fire on every rank together: the flags are combined first, so
    no rank is left waiting in the gather.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world != shard.world:
        raise ValueError(f"the shard was cut for {shard.world} ranks, the group has {world}")
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    # a rank whose fold fails — or a root without a usable output — still joins the flag
    # reduction below, so no rank waits forever in a collective the failing rank never reaches
    error: Exception | None = None
    try:
        if rank == root and (out is None or out.numel() != shard.layout.total_numel or out.dtype != out_dtype
                             or not out.is_contiguous()):
            raise ValueError("the root needs a contiguous flat output of the layout's size and dtype")
        local = shard.fold(table, in_dtype, out_dtype)
        flags = shard.flags()
    except (RuntimeError, ValueError) as e:
        error, local, flags = e, torch.empty(0, dtype=out_dtype, device=shard.device), _FLAG_LOCAL_ERROR
    if world > 1:
        global_flags = union_flags(flags, group, shard.device)
    else:
        global_flags = flags
    if global_flags & _FLAG_LOCAL_ERROR:
        if error is not None:
            raise error
        raise RuntimeError("another rank's fold of its element range failed")
    if global_flags:
        if flags:
            shard.raise_local([(table, in_dtype)] if table is not None else [])
        if global_flags & _native.FLAG_ACC_NAN:
            raise NaNAggregationError("accumulator", "NaN in another rank's element range (input or weighted sum)")
        raise NaNAggregationError("result", "NaN after dividing by the total weight in another rank's range")
    if world == 1:
        out.copy_(local)
        return
    root_global = dist.get_global_rank(group, root) if group is not None else root
    width = max(hi - lo for lo, hi in shard.ranges)
    host = dist.get_backend(group) == "gloo" and local.is_cuda
    send = torch.zeros(width, dtype=out_dtype, device="cpu" if host else local.device)
    send[: local.numel()].copy_(local)
    recv = [torch.empty_like(send) for _ in range(world)] if rank == root else None
    dist.gather(send, recv, dst=root_global, group=group)
    if rank == root:
        for (lo, hi), part in zip(shard.ranges, recv):
            if hi > lo:
                out[lo:hi].copy_(part[: hi - lo])


def segment_views(out: torch.Tensor, layout: ModelLayout) -> dict[str, torch.Tensor]:
    """The flat result as the layout's named tensors (views)."""
    res, off = {}, 0
    for name, shape, n in zip(layout.names, layout.shapes, layout.numels):
        res[name] = out[off : off + n].view(shape)
        off += n
    return res
