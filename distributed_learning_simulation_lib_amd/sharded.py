"""Clients sharded across the GPUs of a node, one RCCL reduce of the fp64 partials.

The reference has no collectives: every client update goes to the one server process
(SURVEY.md §5). When N × model bytes outgrows one GPU (BASELINE.json configs 3 and 5), the
clients are partitioned over the ranks (one process per GPU, ``torch.distributed`` with the
``nccl`` backend = RCCL over xGMI):

    rank r:  S_r = sum_{k in shard r} w_k x_k           (fp64, HIP partial kernel)
    root:    S   = sum_r S_r                            (RCCL reduce, chunked)
    root:    out = S / W                                (HIP finalize kernel, per chunk)

The partial is produced and exchanged in chunks of tiles: the kernel for chunk c+1 runs on
the compute stream while RCCL exchanges chunk c on its own stream. Two exchanges (DESIGN.md §5
cost table), both the one exchange step of the path:

  * ``reduce``:  ncclReduce of each chunk to the root; the root finalizes every tile at the end.
  * ``scatter``: ncclReduceScatter of each chunk (rank r owns the sums of the chunk's r-th
    window), every rank divides its own window, ncclGather brings the windows (output dtype)
    to the root, which copies them into its outputs. Root ingress (G-1)/G x (fp64 partial +
    result) instead of the whole fp64 partial; all ranks do equal exchange work.

``exchange="auto"`` picks scatter at 2 ranks and reduce above (the cost model of DESIGN.md §5);
``tune_exchange`` instead times every (exchange, chunks) candidate on the live job and returns
the fastest, the same answer on every rank.
A process group on the ``gloo`` backend with GPU accumulators stages each chunk through host
memory (tests and hosts without RCCL); ``nccl`` (= RCCL) works on HBM directly.

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
import time
from collections.abc import Sequence
from typing import Protocol

import torch
import torch.distributed as dist

from . import _native
from .fedavg import ClientTable, FedAvgContext, NaNAggregationError, OutputTable


EXCHANGES = ("auto", "reduce", "scatter")
# chunk shapes: equal ranges; the last chunk half the others (a short exchange tail when the
# exchange keeps up with the fold); the first chunk half the others (the exchange starts sooner
# when it does not); the last chunk a quarter of the others (a shorter tail still, for links
# fast enough to keep up with three full chunks)
CHUNK_SHAPES = ("even", "taper", "ramp", "tail")


FLAG_BITS = 16  # NaN flag words are bit sets: FLAG_ACC_NAN / RESULT / CENTRAL, local-error bits above


def union_flags(flags: int, group: dist.ProcessGroup | None = None, device: torch.device | str | None = None) -> int:
    """Bitwise OR of every rank's flag word (collective over ``group``).

    The backends reduce with SUM / MAX / MIN only, so each bit travels as its own int32 and the
    bits are MAX-reduced: every rank gets the union, e.g. FLAG_ACC_NAN from one rank and
    FLAG_RESULT_NAN from another give both, and every rank raises the same (first) assertion."""
    if not 0 <= flags < (1 << FLAG_BITS):
        raise ValueError(f"flag word {flags:#x} outside {FLAG_BITS} bits")
    on_host = device is None or dist.get_backend(group) == "gloo" or torch.device(device).type != "cuda"
    bits = torch.tensor([(flags >> b) & 1 for b in range(FLAG_BITS)], dtype=torch.int32,
                        device="cpu" if on_host else device)
    dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=group)
    return sum(1 << b for b, v in enumerate(bits.tolist()) if v)


def raise_for_flags(flags: int, where: str) -> None:
    """The reference's assertion for a flag word that another rank raised (fed_avg_algorithm.py:93 / :97)."""
    if flags & _native.FLAG_ACC_NAN:
        raise NaNAggregationError("accumulator", f"NaN in the weighted sum ({where}: an input or inf - inf)")
    if flags:
        raise NaNAggregationError("result", f"NaN after dividing by the total weight ({where})")


def resolve_exchange(exchange: str, world: int) -> str:
    if exchange not in EXCHANGES:
        raise ValueError(f"exchange must be one of {EXCHANGES}, not {exchange!r}")
    if exchange == "auto":
        return "scatter" if world == 2 else "reduce"
    return exchange


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

    # scatter exchange: window finalize into a result buffer in accumulator coordinates, then
    # the root's copy into its outputs
    def result_buffer(self) -> torch.Tensor: ...

    def finalize_window(self, src: torch.Tensor, lo: int, hi: int, res: torch.Tensor) -> None: ...

    def copy_out(self, res: torch.Tensor) -> None: ...

    def nan_flags(self) -> int: ...

    def raise_on_nan(self) -> None: ...


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
        self._res: torch.Tensor | None = None

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
            self._plan_finalize(totals)
        else:
            self.ctx.set_accumulated(totals)

    def _plan_finalize(self, totals: list[float]) -> None:
        if self._finalize_plan is None or self._finalize_totals != totals:
            if self.outs is None:
                # a non-root rank of the scatter exchange finalizes windows only: its plan needs
                # outputs of the layout, which it never copies into
                offs, total = self.ctx.layout.padded_offsets(torch.empty((), dtype=self.out_dtype).element_size())
                flat = torch.empty(total, dtype=self.out_dtype, device=self.ctx.device)
                self.outs = OutputTable([flat[o : o + m] for o, m in zip(offs, self.ctx.layout.numels)],
                                        self.ctx.layout, self.ctx.device, self.out_dtype)
            self._finalize_plan = self.ctx.plan_finalize(totals, self.outs, self.out_dtype)
            self._finalize_totals = totals

    def finalize_range(self, tile_begin: int, tile_end: int) -> None:
        assert self.outs is not None
        if self.use_plan:
            assert self._finalize_plan is not None
            self._finalize_plan.run_range(tile_begin, tile_end)
        else:
            self.ctx.finalize_range(self.outs, self.out_dtype, tile_begin, tile_end)

    def native_round(self, comm: RcclComm, total_weights: Sequence[float], chunks: int, root: int,
                     exchange: str = "reduce", shape: str = "even") -> None:
        """One round through the library's own RCCL pipeline (``fedavg_sharded_round`` /
        ``_scatter``, or ``fedavg_sharded_round_edges`` for an uneven chunk ``shape``): the chunk
        launches, the exchange and the finalize are enqueued by one native call."""
        assert self.use_plan and self.table is not None
        if self._partial_plan is None:
            self._partial_plan = self.ctx.plan_partial(self.table, self.in_dtype, zero_init=not self.prior_waves)
        lib = self.ctx._lib
        fin = None
        if exchange == "scatter":
            self._plan_finalize([float(w) for w in total_weights])
            fin = self._finalize_plan._h
        elif comm.rank == root:
            self.set_accumulated(total_weights)
            fin = self._finalize_plan._h
        if shape != "even":
            edges = chunk_edges(self.num_tiles, chunks, shape)
            arr = (ctypes.c_int32 * len(edges))(*edges)
            ex = _native.EXCHANGE_SCATTER if exchange == "scatter" else _native.EXCHANGE_REDUCE
            _native.check(lib.fedavg_sharded_round_edges(comm.handle, self.ctx._h, self._partial_plan._h, fin, arr,
                                                         len(edges), ex, root, self.ctx.stream))
        elif exchange == "scatter":
            _native.check(lib.fedavg_sharded_round_scatter(comm.handle, self.ctx._h, self._partial_plan._h, fin,
                                                           chunks, root, self.ctx.stream))
        else:
            _native.check(lib.fedavg_sharded_round(comm.handle, self.ctx._h, self._partial_plan._h, fin,
                                                   chunks, root, self.ctx.stream))

    # -- scatter exchange pieces (host-driven path) -----------------------------------------
    def result_buffer(self) -> torch.Tensor:
        if self._res is None or self._res.dtype != self.out_dtype:
            self._res = torch.empty(self.ctx.acc_numel, dtype=self.out_dtype, device=self.ctx.device)
        return self._res

    def finalize_window(self, src: torch.Tensor, lo: int, hi: int, res: torch.Tensor) -> None:
        assert self._finalize_plan is not None, "set_accumulated first"
        self._finalize_plan.finalize_window(src, lo, hi, res)

    def copy_out(self, res: torch.Tensor) -> None:
        assert self._finalize_plan is not None, "set_accumulated first"
        self._finalize_plan.copy_out(res)

    def nan_flags(self) -> int:
        """This rank's latched NaN flag bits (drains the stream; does not clear them)."""
        return self.ctx.flags()

    def raise_on_nan(self) -> None:
        """The reference's NaN assertions (fed_avg_algorithm.py:35,93,97) on this rank's flags."""
        self.ctx.raise_on_nan([(t, self.in_dtype) for t in [*self.prior_waves, self.table] if t is not None])

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


def chunk_edges(num_tiles: int, chunks: int, shape: str = "even") -> list[int]:
    """Tile edges 0 = e[0] < ... < e[-1] = num_tiles of ``chunks`` ranges of the given shape."""
    if shape not in CHUNK_SHAPES:
        raise ValueError(f"shape must be one of {CHUNK_SHAPES}, not {shape!r}")
    chunks = max(1, min(chunks, num_tiles))
    if shape == "even" or chunks == 1:
        weights = [1.0] * chunks
    elif shape == "tail":
        weights = [4.0] * chunks
        weights[-1] = 1.0
    else:
        weights = [2.0] * chunks
        weights[-1 if shape == "taper" else 0] = 1.0
    total, acc, edges = sum(weights), 0.0, [0]
    for w in weights:
        acc += w
        e = round(acc / total * num_tiles)
        if e > edges[-1]:
            edges.append(e)
    edges[-1] = num_tiles
    return edges


def chunk_bounds(num_tiles: int, chunks: int, shape: str = "even") -> list[tuple[int, int]]:
    edges = chunk_edges(num_tiles, chunks, shape)
    return [(edges[i], edges[i + 1]) for i in range(len(edges) - 1)]


class ExchangeModel:
    """Per-round cost model of the client-sharded reduce: G ranks, each folding
    its shard into an fp64 partial in tile chunks, the exchange of chunk c on the comm stream
    behind the fold of chunk c, the root's division of every chunk but the last overlapped with
    the last exchange (``fedavg_sharded_round``), the last chunk's exchange and division exposed.

    The rates: ``fold_rate`` and ``hbm_rate`` are measured on one MI355X (the partial kernel's
    6.45 TB/s over a 256 x ResNet-18 shard, profiles/r02_sharded_and_anchor.jsonl; the finalize is
    an HBM stream at the same rate); ``link_rate`` is the quoted xGMI rate per link and direction
    (7 links per GPU, one per peer) and ``link_eff`` the share of it RCCL is assumed to reach —
    neither is measurable on the one-GPU boxes this build is tested on, so the tuner
    (``tune_exchange``) has the last word on a node. ``underfill_ms``: a chunk of fewer than
    ``full_chunk_tiles`` 4096-element tiles leaves CUs idle at its end (measured: 8 chunks of
    357 tiles +0.07 ms per one-rank round against 2-4 chunks)."""

    def __init__(self, fold_rate: float = 6.45e12, hbm_rate: float = 6.5e12, link_rate: float = 153e9,
                 link_eff: float = 0.75, full_chunk_tiles: int = 512, underfill_ms: float = 0.009,
                 sync_ms: float = 0.008) -> None:
        self.fold_rate, self.hbm_rate = fold_rate, hbm_rate
        self.link_rate, self.link_eff = link_rate, link_eff
        self.full_chunk_tiles, self.underfill_ms = full_chunk_tiles, underfill_ms
        # the peer exchange's cross-device hand-off after the last chunk (event marker, a peer's wait,
        # the combine launch): assumed, not measurable on one GPU
        self.sync_ms = sync_ms

    def one_gpu_ms(self, numel: int, n_clients: int, in_bytes: int, out_bytes: int) -> float:
        """The fused single-launch round on one GPU (the strong-scaling anchor)."""
        return (n_clients * numel * in_bytes + numel * out_bytes) / self.fold_rate * 1e3

    def round_ms(self, world: int, numel: int, n_clients: int, in_bytes: int, out_bytes: int,
                 edges: Sequence[int], exchange: str, root_clients: int | None = None) -> dict[str, float]:
        """Predicted terms of one round. Every rank's HBM carries its fold (its clients + the fp64
        partial write) and its share of the exchange (RCCL reads the partial and writes the
        received sums: ~2 x the chunk per rank); the root's also the division. The exchange of
        chunk c starts once every rank has folded chunk c and the previous exchange is done; it
        is link-bound. ``root_clients``: the root's shard (default: an even split), the others
        share the rest — a smaller root shard leaves HBM time for the root's division."""
        G = world
        n_root = -(-n_clients // G) if root_clients is None else root_clients
        n_peer = -(-(n_clients - n_root) // (G - 1)) if G > 1 else 0
        link = self.link_rate * self.link_eff
        rate = self.fold_rate / 1e3  # bytes per ms
        part_b, res_b = numel * 8, numel * out_bytes
        total_tiles = edges[-1]
        fracs = [(b - a) / total_tiles for a, b in zip(edges, edges[1:])]
        under = [self.underfill_ms if b - a < self.full_chunk_tiles else 0.0 for a, b in zip(edges, edges[1:])]
        if exchange == "peer":
            return self._peer_round_ms(G, numel, n_clients, in_bytes, out_bytes, fracs, under, n_root, n_peer)
        root_t = peer_t = x_end = 0.0
        xs, x_ends = [], []
        for c, f in enumerate(fracs):
            # the exchange of the previous chunk shares HBM with this chunk's fold on every rank
            xh = 2 * fracs[c - 1] * part_b if c else 0.0
            root_t += (f * (n_root * numel * in_bytes + part_b) + xh) / rate + under[c]
            peer_t += (f * (n_peer * numel * in_bytes + part_b) + xh) / rate + under[c]
            ready = max(root_t, peer_t if G > 1 else 0.0)
            if exchange == "reduce":
                x = f * part_b / ((G - 1) * link) * 1e3  # the root takes the partial over G - 1 links
            else:  # reduce-scatter out of / into every rank over G - 1 links, then the result gather
                x = (f * part_b / G + f * res_b / G) / link * 1e3 + f * (part_b + res_b) / G / rate
            x_end = max(x_end, ready) + x
            xs.append(x)
            x_ends.append(x_end)
        last = fracs[-1]
        if exchange == "reduce":
            # the root divides the head chunks once they are reduced, during the last exchange
            head_div = (1 - last) * (part_b + res_b) / rate if len(fracs) > 1 else 0.0
            head_end = max(root_t, x_ends[-2]) + head_div if len(fracs) > 1 else 0.0
            last_div = last * (part_b + res_b) / rate
            step = max(x_end, head_end) + last_div
        else:
            last_div = 2 * res_b / rate  # the root's copy-out of the gathered result
            step = x_end + last_div
        fold = max(root_t, peer_t if G > 1 else 0.0)
        t1 = self.one_gpu_ms(numel, n_clients, in_bytes, out_bytes)
        return {"fold_ms": round(fold, 4), "exposed_exchange_and_finalize_ms": round(step - fold, 4),
                "last_chunk_exchange_ms": round(xs[-1], 4), "last_finalize_ms": round(last_div, 4),
                "root_clients": n_root, "peer_clients": n_peer,
                "step_ms": round(step, 4), "one_gpu_ms": round(t1, 4), "speedup": round(t1 / step, 3)}

    def _peer_round_ms(self, G: int, numel: int, n_clients: int, in_bytes: int, out_bytes: int, fracs: list[float],
                       under: list[float], n_root: int, n_peer: int) -> dict[str, float]:
        """The single-process peer-window exchange (multi_device.cpp). Per chunk every
        device folds its clients over the other windows, each tile's fp64 partial stored straight into
        the window owner's receive slot (a peer store: S/G per peer link per round, the receiver's HBM
        takes it), and then folds its own window with the G - 1 received partials of it added in entry
        order in the same kernel, dividing and storing 1/G of the result into the root. A device's HBM
        per chunk: its clients, the (G-1)/G of the chunk's partial arriving from peers, the own-window
        kernel's read of those same bytes, and on the root every result window; the other windows'
        fold cannot end before its peer stores have drained over the links. The last chunk's own-window
        kernel (it waits for every peer's stores) and the result's trip to the root are the tail, plus
        a cross-device hand-off."""
        link = self.link_rate * self.link_eff
        rate = self.fold_rate / 1e3
        part_b, res_b = numel * 8, numel * out_bytes
        share = (G - 1) / G  # the partial bytes of a chunk a device receives (and its own window re-reads)

        def own_window(f: float, n: int, root: bool) -> float:
            """Bytes of one device's own-window kernel for a chunk of fraction f."""
            return f / G * n * numel * in_bytes + share * f * part_b + (f * res_b if root else f * res_b / G)

        root_t = peer_t = 0.0
        for c, f in enumerate(fracs):
            last = c == len(fracs) - 1
            drain = f * part_b / G / link * 1e3 if G > 1 else 0.0  # one window per peer link
            others_root = (1 - 1 / G) * f * n_root * numel * in_bytes + share * f * part_b
            others_peer = (1 - 1 / G) * f * n_peer * numel * in_bytes + share * f * part_b
            own_root = 0.0 if last else own_window(f, n_root, True)
            own_peer = 0.0 if last else own_window(f, n_peer, False)
            root_t += max((others_root + own_root) / rate, drain) + under[c]
            peer_t += max((others_peer + own_peer) / rate, drain) + under[c]
        last = fracs[-1]
        own_last = max(own_window(last, n_root, True), own_window(last, n_peer, False) if G > 1 else 0.0) / rate
        result_link = last * res_b / G / link * 1e3 if G > 1 else 0.0
        fold = max(root_t, peer_t if G > 1 else 0.0)
        tail = own_last + result_link + (self.sync_ms if G > 1 else 0.0)
        step = fold + tail
        t1 = self.one_gpu_ms(numel, n_clients, in_bytes, out_bytes)
        return {"fold_ms": round(fold, 4), "exposed_exchange_and_finalize_ms": round(tail, 4),
                "last_chunk_exchange_ms": round(result_link, 4), "last_finalize_ms": round(own_last, 4),
                "root_clients": n_root, "peer_clients": n_peer,
                "step_ms": round(step, 4), "one_gpu_ms": round(t1, 4), "speedup": round(t1 / step, 3)}

    def best(self, world: int, numel: int, n_clients: int, in_bytes: int, out_bytes: int, num_tiles: int,
             candidates: Sequence[tuple[str, int, str]] | None = None,
             balance_root: bool = True) -> tuple[tuple[str, int, str], dict]:
        """The candidate (exchange, chunks, shape) — and, with ``balance_root``, the root's shard
        (an even split or up to 8 clients fewer) — with the smallest predicted step."""
        cands = list(candidates) if candidates is not None else exchange_candidates()
        even = -(-n_clients // world)
        roots = range(max(1, even - 8), even + 1) if balance_root and world > 1 else [even]
        best = None
        for i, (ex, ch, sh) in enumerate(cands):
            edges = chunk_edges(num_tiles, ch, sh)
            for nr in roots:
                r = self.round_ms(world, numel, n_clients, in_bytes, out_bytes, edges, ex, nr)
                key = (r["step_ms"], -nr, i)
                if best is None or key < best[0]:
                    best = (key, cands[i], r)
        assert best is not None
        return best[1], best[2]


def sharded_reduce(
    reducer: LocalReducer,
    local_total_weights: Sequence[float],
    chunks: int = 4,
    root: int = 0,
    group: dist.ProcessGroup | None = None,
    global_total_weights: Sequence[float] | None = None,
    force_collective: bool = False,
    comm: RcclComm | None = None,
    exchange: str = "auto",
    check_nan: bool = True,
    shape: str = "even",
) -> list[float]:
    """One FedAvg reduce over every rank's shard; the result lands in the root's outputs.

    ``local_total_weights`` are this rank's per-segment sums of client weights. When the
    caller already knows the global totals (the dispatcher that assigned clients to ranks
    knows every client's weight) it passes ``global_total_weights`` and no collective is
    spent on them; otherwise they are all-reduced first. Returns the global totals. On a
    one-rank world the fused single-launch kernel is used (no fp64 round trip) unless
    ``force_collective`` (tests / measurement of the sharded path on one GPU). With ``comm``
    (the library's own RCCL communicator) a HIP reducer runs the whole round in one native call
    (``fedavg_sharded_round[_scatter]``); otherwise the exchange goes through
    ``torch.distributed``. ``shape`` is the chunk shape (``CHUNK_SHAPES``). ``root`` is a rank of
    ``group``. With ``check_nan`` every rank raises the reference's NaN assertions
    (fed_avg_algorithm.py:35,93,97) before returning when any rank's flags are set (one small
    all-reduce of the flag bits; the root raises the precise stage). Without it the caller reads
    the flags itself (``reducer.raise_on_nan`` / ``nan_flags``) and owns the agreement.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1 and not (force_collective and dist.is_initialized()):
        reducer.fused()
        if check_nan:
            reducer.raise_on_nan()
        return list(local_total_weights)
    rank = dist.get_rank(group)
    # torch.distributed addresses the root by its global rank (RcclComm takes the group rank)
    root_global = dist.get_global_rank(group, root) if group is not None else root
    acc = reducer.accumulator
    host_staged = acc.is_cuda and dist.get_backend(group) == "gloo"  # gloo reduces host memory
    if global_total_weights is None:
        totals = torch.tensor([float(w) for w in local_total_weights], dtype=torch.float64,
                              device="cpu" if host_staged or not acc.is_cuda else acc.device)
        dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)
        global_total_weights = totals.tolist()
    global_totals = [float(w) for w in global_total_weights]
    mode = resolve_exchange(exchange, world)
    reducer.prefold()
    if comm is not None and hasattr(reducer, "native_round"):
        reducer.native_round(comm, global_totals, chunks, root, exchange=mode, shape=shape)
    else:
        bounds = chunk_bounds(reducer.num_tiles, chunks, shape)
        if mode == "scatter":
            _scatter_exchange(reducer, global_totals, bounds, world, rank, root, root_global, group, host_staged)
        else:
            _reduce_exchange(reducer, global_totals, bounds, rank, root, root_global, group, host_staged)
    if check_nan:
        # every rank raises together: the flag words (the root's finalize; under the scatter
        # exchange each rank's window finalize too) are OR-ed across ranks before anyone raises,
        # so no rank returns normally and then waits in the next round's collectives
        dev = acc.device if acc.is_cuda and not host_staged else None
        local = reducer.nan_flags()
        flags = union_flags(local, group, dev)
        if flags:
            if rank == root or local:
                # the reference's stage from this rank's own flags: a rank whose shard holds the
                # NaN input scans its own tables and names its clients (:35); the root names the
                # stage of its finalize (:93 / :97)
                reducer.raise_on_nan()
            raise_for_flags(flags, f"reported by the sharded round on rank {rank}")
    return global_totals


def exchange_candidates(chunks: int | None = None, shapes: Sequence[str] = CHUNK_SHAPES,
                        exchanges: Sequence[str] = ("reduce", "scatter")) -> list[tuple[str, int, str]]:
    """(exchange, chunks, shape) triples ``tune_exchange`` tries: both exchanges at 2 / 4 / 6 / 8
    chunks (or the given count only), every chunk shape (one shape when there is one chunk).
    ``exchanges=("peer", "reduce")``: the single-process multi-device round's candidates."""
    out = []
    for ex in exchanges:
        for c in ((chunks,) if chunks else (2, 4, 6, 8)):
            for sh in (shapes if c > 1 else ("even",)):
                out.append((ex, c, sh))
    return out


def tune_exchange(
    reducer: LocalReducer,
    local_total_weights: Sequence[float],
    candidates: Sequence[tuple[str, int, str]] | None = None,
    rounds: int = 3,
    root: int = 0,
    group: dist.ProcessGroup | None = None,
    global_total_weights: Sequence[float] | None = None,
    comm: RcclComm | None = None,
    force_collective: bool = False,
    check_nan: bool = True,
    budget_s: float | None = None,
) -> tuple[tuple[str, int, str], dict[tuple[str, int, str], float]]:
    """Pick the exchange, chunk count and chunk shape by timing the job itself.

    The cost model of DESIGN.md §5 rests on a link rate no single-GPU box can measure, so the
    multi-GPU round can instead be tuned on the node it runs on: each candidate runs one
    untimed round (plans and scratch), then ``rounds`` rounds between a barrier and a device
    sync; the time of a candidate is the max over ranks (one all-reduce), so every rank ranks
    the candidates identically and returns the same choice. Each round ends as a server's does,
    with the root reading the NaN flags (``check_nan``): without that host sync, back-to-back
    rounds overlap one round's exchange with the next round's fold, a pipelining no
    round-by-round server gets, and the candidates would be ranked on it. Ties go to the earlier candidate.
    ``budget_s``: once this many seconds of tuning have passed (the max over ranks, taken with each
    candidate's time, so every rank stops after the same candidate) the rest are not timed.
    Returns ``((exchange, chunks, shape), {candidate: ms per round})`` — the candidates timed.
    Collective: every rank of ``group`` calls it with the same candidates.
    """
    cands = list(candidates) if candidates is not None else exchange_candidates()
    if not cands:
        raise ValueError("no candidates to tune")
    for ex, ch, sh in cands:
        resolve_exchange(ex, 2)
        if ch < 1:
            raise ValueError(f"chunks must be >= 1, not {ch}")
        if sh not in CHUNK_SHAPES:
            raise ValueError(f"shape must be one of {CHUNK_SHAPES}, not {sh!r}")
    acc = reducer.accumulator
    on_host = not acc.is_cuda or dist.get_backend(group) == "gloo"

    def settle() -> None:
        if acc.is_cuda:
            torch.cuda.synchronize(acc.device)

    times: dict[tuple[str, int, str], float] = {}
    t_start = time.perf_counter()
    for ex, ch, sh in cands:
        kw = dict(chunks=ch, root=root, group=group, global_total_weights=global_total_weights,
                  force_collective=force_collective, comm=comm, exchange=ex, check_nan=check_nan, shape=sh)
        sharded_reduce(reducer, local_total_weights, **kw)
        settle()
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(max(1, rounds)):
            sharded_reduce(reducer, local_total_weights, **kw)
        settle()
        now = time.perf_counter()
        el = torch.tensor([now - t0, now - t_start], dtype=torch.float64, device="cpu" if on_host else acc.device)
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=group)
        times[(ex, ch, sh)] = float(el[0].item()) / max(1, rounds) * 1e3
        if budget_s is not None and float(el[1].item()) > budget_s:
            break
    timed = [i for i in range(len(cands)) if cands[i] in times]
    best = min(timed, key=lambda i: (times[cands[i]], i))
    return cands[best], times


def _reduce_exchange(reducer: LocalReducer, global_totals: list[float], bounds: list[tuple[int, int]], rank: int,
                     root: int, root_global: int, group: dist.ProcessGroup | None, host_staged: bool) -> None:
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
        if host_staged:
            h = acc[a:b].cpu()
            dist.reduce(h, dst=root_global, op=dist.ReduceOp.SUM, group=group)
            if rank == root:
                acc[a:b].copy_(h)
        else:
            works.append(dist.reduce(acc[a:b], dst=root_global, op=dist.ReduceOp.SUM, group=group, async_op=True))
    # The collectives of one process group run on one RCCL stream and complete in issue
    # order, so on the GPU one wait (the last reduce) covers every chunk: one cross-stream
    # dependency instead of one per chunk. Host backends (gloo) wait for each work.
    if rank == root:
        reducer.set_accumulated(global_totals)
    if acc.is_cuda and len(works) >= 2 and rank == root:
        # the chunks already reduced are divided while the last one is still being reduced
        # (fedavg_sharded_round does the same): only the last chunk's division
        # follows the last collective
        works[-2].wait()
        reducer.finalize_range(0, bounds[-1][0])
        works[-1].wait()
        reducer.finalize_range(bounds[-1][0], reducer.num_tiles)
        return
    for w in (works[-1:] if acc.is_cuda else works):
        w.wait()
    if rank == root:
        reducer.finalize_range(0, reducer.num_tiles)  # one launch over every tile


def scatter_windows(a: int, b: int, world: int) -> tuple[int, int]:
    """Chunk [a, b) of the accumulator -> (L, R): rank r owns [a + r*L, a + (r+1)*L), the
    R-element tail [a + world*L, b) is reduced to the root (R = 0 whenever world divides 32)."""
    return divmod(b - a, world)


def _scatter_exchange(reducer: LocalReducer, global_totals: list[float], bounds: list[tuple[int, int]], world: int,
                      rank: int, root: int, root_global: int, group: dist.ProcessGroup | None,
                      host_staged: bool) -> None:
    """Host-driven form of fedavg_sharded_round_scatter (same windows, same arithmetic)."""
    acc = reducer.accumulator
    reducer.set_accumulated(global_totals)  # every rank divides its own windows
    res = reducer.result_buffer()
    for tb, te in bounds:
        reducer.partial(tb, te)
        a, b = reducer.tile_range(tb, te)
        L, R = scatter_windows(a, b, world)
        lo = a + rank * L
        if L > 0:
            src = acc[a : a + world * L]
            if host_staged:
                mine = torch.empty(L, dtype=torch.float64)
                dist.reduce_scatter_tensor(mine, src.cpu(), op=dist.ReduceOp.SUM, group=group)
                mine = mine.to(acc.device)
            else:
                mine = torch.empty(L, dtype=torch.float64, device=acc.device)
                dist.reduce_scatter_tensor(mine, src, op=dist.ReduceOp.SUM, group=group)
            reducer.finalize_window(mine, lo, lo + L, res)
        if R > 0:
            tail = acc[a + world * L : b]
            h = tail.cpu() if host_staged else tail
            dist.reduce(h, dst=root_global, op=dist.ReduceOp.SUM, group=group)
            if rank == root:
                reducer.finalize_window(h.to(acc.device) if host_staged else tail, a + world * L, b, res)
        if L > 0:
            send = res[lo : lo + L]
            if host_staged:
                recv = [torch.empty(L, dtype=res.dtype) for _ in range(world)] if rank == root else None
                dist.gather(send.cpu(), recv, dst=root_global, group=group)
                if rank == root:
                    for i, t in enumerate(recv):
                        if i != root:
                            res[a + i * L : a + (i + 1) * L].copy_(t)
            else:
                recv = [res[a + i * L : a + (i + 1) * L] for i in range(world)] if rank == root else None
                dist.gather(send, recv, dst=root_global, group=group)
    if rank == root:
        reducer.copy_out(res)
