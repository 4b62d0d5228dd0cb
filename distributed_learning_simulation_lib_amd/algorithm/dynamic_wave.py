"""The plugin's settings and the controller of its dynamic wave.

``PluginSettings`` is the one place the plugin's tuning knobs are read from the environment
(``PluginSettings.from_env``); ``FedAVGAlgorithm(settings=...)`` takes an explicit object instead,
and its keyword arguments override single fields.

``DynamicWave`` drives the round's dynamic wave (include/fedavg_hip.h ``fedavg_dyn_*``) for one
``FedAVGAlgorithm``: the reference folds every update as it arrives
(``simulation_lib/algorithm/fed_avg_algorithm.py:20-64``) while its server hands them over from its
poll loop (``simulation_lib/server/server.py:133-146``, via ``aggregation_server.py:111-145``). Here
the first wave of the round is launched at the round's first staged update with an open client
count; the staged rows are handed to it every ``batch`` arrivals while it folds the ones it has,
and the close — the wave's flush or ``aggregate_worker_data`` — either divides in the same kernel
(the round's result) or leaves the rows it folded in the fp64 accumulator for the ordinary waves.
A wave that ends itself after ``idle_us`` without a row is continued by the library at the next
publication (a fresh launch that starts from the accumulator), so each burst of arrivals is
folded while it arrives. Per element the fold is the reference's arrival-order chain in every
case: the results are bit-identical to the one-launch kernel's.
"""

from __future__ import annotations

import os
from collections.abc import Callable, Mapping
from dataclasses import dataclass, field, replace
from typing import Any

import torch

from .. import _native
from .._staging import NativeClientTable, TableTail

DYN_DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.float64)  # dyn_wave_kernel inputs


@dataclass(frozen=True)
class DynamicWaveSettings:
    """The dynamic wave's knobs (environment names in brackets, read by ``PluginSettings.from_env``).

    * ``enabled`` (``FEDAVG_DYN``, default on): use the wave at all. While open, its workgroups hold
      the register file of every CU they occupy (they spin on the row count), so a GPU shared with
      training kernels that must never wait should turn it off.
    * ``batch`` (``FEDAVG_DYN_BATCH``, 2): staged rows handed over per publication (the first at once).
    * ``min_rows`` (``FEDAVG_DYN_MIN_ROWS``, 4): a round after one of fewer updates skips the wave.
    * ``idle_us`` (``FEDAVG_DYN_IDLE_US``, 200): the wave ends itself after this long without a row,
      freeing the GPU between bursts; the next publication continues it from the accumulator.
    * ``life_us`` (``FEDAVG_DYN_LIFE_US``, 2 s): the longest one launch spins; likewise continued.
    """

    enabled: bool = True
    batch: int = 2
    min_rows: int = 4
    idle_us: int = 200
    life_us: int = 2_000_000

    def __post_init__(self) -> None:
        if self.batch < 1 or self.min_rows < 0 or self.idle_us < 1 or self.life_us < 1:
            raise ValueError(f"invalid dynamic-wave settings: {self}")


@dataclass(frozen=True)
class PluginSettings:
    """``FedAVGAlgorithm``'s tuning knobs.

    * ``wave_size`` (``FEDAVG_WAVE_SIZE``, 64): clients per launch; the last wave of a round is folded
      and divided in one launch.
    * ``wave_min`` (``FEDAVG_WAVE_MIN``, 0): early waves — a staged wave of at least this many clients
      is also folded when the GPU has finished every wave so far (0 = full waves only).
    * ``eager_nan_check`` (``FEDAVG_EAGER_NAN=1``): scan every arrival for NaN on the GPU and raise on
      that arrival (fed_avg_algorithm.py:34-35) instead of at the flush.
    * ``qsgd_host_pointers`` (``FEDAVG_QSGD_HOST_PTRS``, on): host QSGD records packed by pointer.
    * ``dynamic``: ``DynamicWaveSettings``.
    """

    wave_size: int = 64
    wave_min: int = 0
    eager_nan_check: bool = False
    qsgd_host_pointers: bool = True
    dynamic: DynamicWaveSettings = field(default_factory=DynamicWaveSettings)

    def __post_init__(self) -> None:
        if self.wave_size < 1 or self.wave_min < 0:
            raise ValueError(f"invalid plugin settings: {self}")

    @classmethod
    def from_env(cls, environ: Mapping[str, str] | None = None) -> PluginSettings:
        env = os.environ if environ is None else environ
        d = DynamicWaveSettings()
        dyn = DynamicWaveSettings(
            enabled=env.get("FEDAVG_DYN", "1") != "0",
            batch=max(1, int(env.get("FEDAVG_DYN_BATCH", d.batch))),
            min_rows=int(env.get("FEDAVG_DYN_MIN_ROWS", d.min_rows)),
            idle_us=int(env.get("FEDAVG_DYN_IDLE_US", d.idle_us)),
            life_us=int(env.get("FEDAVG_DYN_LIFE_US", d.life_us)),
        )
        return cls(
            wave_size=int(env.get("FEDAVG_WAVE_SIZE", cls.wave_size)),
            wave_min=int(env.get("FEDAVG_WAVE_MIN", cls.wave_min)),
            eager_nan_check=env.get("FEDAVG_EAGER_NAN") == "1",
            qsgd_host_pointers=env.get("FEDAVG_QSGD_HOST_PTRS", "1") != "0",
            dynamic=dyn,
        )

    def with_overrides(self, **kw: Any) -> PluginSettings:
        """A copy with the fields given (None values ignored; ``dynamic_wave`` sets dynamic.enabled)."""
        kw = {k: v for k, v in kw.items() if v is not None}
        dyn = kw.pop("dynamic_wave", None)
        out = replace(self, **kw)
        if dyn is not None:
            out = replace(out, dynamic=replace(out.dynamic, enabled=bool(dyn)))
        return out


class DynamicWave:
    """The round's dynamic wave of one algorithm object (one device context at a time).

    ``stats``: waves opened (``waves``), rows they folded (``rows``), waves that wrote the round's
    result themselves (``finalized``), continued launches after a wave ended itself (``reopens``),
    and opens the library refused (``open_failures``, with ``last_error``) — a refused open is
    never silent: the round then folds in ordinary waves, with the same bits.
    """

    def __init__(self, settings: DynamicWaveSettings) -> None:
        self.settings = settings
        self.table: Any = None        # the table the open wave reads
        self.published = 0            # its rows published so far
        self.closed: Any = None       # (table, rows folded) of the round's closed wave
        self.decided = False          # the round's first wave has been decided
        self.prev_arrivals: int | None = None  # the previous round's process_worker_data calls
        # the input dtype of the last round's wave: the next round opens its wave with it before its
        # first update is staged (bound to that update's row, or closed empty if it differs)
        self.last_dtype: Any = None
        self.pre_dtype: Any = None    # the dtype of a wave opened before its first row
        self.pre_ctx: Any = None      # ... and the context it was opened on
        self._ctx: Any = None         # the context of the open wave
        self._reopens0 = 0            # the library's continued-wave count at the open
        self._configured: Any = None  # the context idle_us / life_us were handed to
        self.last_error: str | None = None
        self.stats = {"waves": 0, "rows": 0, "finalized": 0, "reopens": 0, "open_failures": 0}

    # -- opening ------------------------------------------------------------------------
    def _round_allowed(self) -> bool:
        # rounds after one of fewer updates than min_rows skip the wave: its open / close cost more
        # than the arrivals it hides
        return self.prev_arrivals is None or self.prev_arrivals >= self.settings.min_rows

    def _open(self, ctx: Any, dtype: torch.dtype, wave_size: int) -> bool:
        if self._configured is not ctx:
            ctx.dyn_configure(self.settings.idle_us, self.settings.life_us)
            self._configured = ctx
        try:
            ctx.dyn_open(dtype, wave_size)
        except _native.NativeError as e:  # e.g. the accumulator already holds data
            self.stats["open_failures"] += 1
            self.last_error = str(e)
            return False
        self._reopens0 = ctx.dyn_info()["reopens"]
        return True

    def preopen(self, ctx_fn: Callable[[], Any], eligible: bool, staged: bool, wave_size: int) -> None:
        """The round's first update is arriving: open the wave with the last round's input dtype
        now, so the launch overlaps this update's staging (its row binds it in ``arrival``)."""
        if not (self.settings.enabled and eligible and not staged and self.last_dtype is not None
                and not self.decided and self.table is None and self._round_allowed()):
            return
        ctx = ctx_fn()
        if self._open(ctx, self.last_dtype, wave_size):
            self.pre_dtype, self.pre_ctx = self.last_dtype, ctx

    def unpre(self) -> None:
        """Close a wave opened before its first row that no row will bind (it folded nothing)."""
        if self.pre_dtype is not None:
            ctx, self.pre_dtype, self.pre_ctx = self.pre_ctx, None, None
            try:
                ctx.dyn_close(None)
            except _native.NativeError:
                pass  # its context was replaced (a grown layout): closing it ended the wave

    def not_this_round(self) -> None:
        """The round's first row cannot use the wave: no wave this round, none pre-opened next."""
        if not self.decided and self.table is None:
            self.decided = True
            self.unpre()
            self.last_dtype = None

    def arrival(self, table: Any, ctx_fn: Callable[[], Any], eligible: bool, dtype: Any, wave_size: int) -> None:
        """The round's first row joined a table: open the round's wave for it (when the round
        qualifies) and hand it the row; later rows go through ``more``."""
        if self.table is not None:
            self.more(table)
            return
        if self.decided:
            return
        self.decided = True
        if not (self.settings.enabled and eligible and type(table) is NativeClientTable
                and table.num_clients == 1 and dtype in DYN_DTYPES and self._round_allowed()):
            self.unpre()
            self.last_dtype = None
            return
        ctx = ctx_fn()
        if self.pre_dtype is not None and (self.pre_dtype != dtype or self.pre_ctx is not ctx):
            self.unpre()  # opened for another dtype or context: reopen for this one
        if self.pre_dtype is None and not self._open(ctx, dtype, wave_size):
            return  # the ordinary waves fold the round
        self.pre_dtype = self.pre_ctx = None
        self.last_dtype = dtype
        self.table, self.published, self.closed, self._ctx = table, 0, None, ctx
        self.stats["waves"] += 1
        self.publish()  # the first row at once: the wave starts folding

    def more(self, table: Any) -> None:
        """A later row joined the wave's table: the staged rows to the wave every ``batch`` rows."""
        if self.table is table and (table.num_clients - self.published >= self.settings.batch or self.published == 0):
            self.publish()

    # -- handing over and closing -------------------------------------------------------------
    def publish(self) -> None:
        """Every staged row of the wave's table to the wave (none while the current stream has
        unfinished work); a row it cannot take closes it with the rows it has."""
        try:
            self.published += self._ctx.dyn_publish(self.table)
        except _native.NativeError as e:
            self.published += getattr(e, "published", 0)
            self.close(None)

    def close(self, outs: Any, out_dtype: torch.dtype = torch.float64, join: bool = True) -> bool:
        """Close the open wave: into ``outs`` (True: the round's result is written) or into the
        accumulator (the rows it folded; ``rest`` gives the ordinary calls the rest)."""
        table, ctx = self.table, self._ctx
        self.table = None
        try:
            folded, finalized = ctx.dyn_close(outs, out_dtype, join)
        finally:
            self.stats["reopens"] += ctx.dyn_info()["reopens"] - self._reopens0
        self.closed = (table, folded)
        self.stats["rows"] += folded
        self.stats["finalized"] += int(finalized)
        return finalized

    def rest(self, table: Any) -> Any:
        """The part of ``table`` the ordinary calls fold: all of it, its rows after those a closed
        wave folded (``TableTail``), or None when the wave folded every row."""
        closed = self.closed
        if closed is None or closed[0] is not table or not closed[1]:
            return table
        self.closed = None
        return TableTail(table, closed[1]) if closed[1] < table.num_clients else None

    def flush(self, table: Any) -> None:
        """The wave's table is flushed as a full wave: its rows stay in the accumulator."""
        if self.table is table:
            self.publish()
            if self.table is table:
                self.close(None)

    def finish(self, table: Any, outs: Any, out_dtype: torch.dtype, stream: torch.cuda.Stream) -> bool:
        """The round's end for the wave holding ``table`` (its last wave): every row published,
        then closed into ``outs`` (None: into the accumulator). True when the wave wrote the result;
        the caller then checks the round (its flags wait for the wave)."""
        if table is None or self.table is not table:
            return False
        if self.published < table.num_clients:
            # the last arrivals' copies / conversions were still running at the last publication:
            # wait for them, as the one-launch path would, so the wave can take every row
            stream.synchronize()
            self.publish()  # (a row it cannot take closes the wave here: the rest is the caller's)
        if self.table is table and self.published < table.num_clients:
            self.close(None)  # rows left unpublished: the wave keeps its rows
        if self.table is table:
            # join=False: the caller's NaN check waits for the wave before anything reads the outputs
            return self.close(outs, out_dtype, join=False)
        return False

    def end_round(self, round_updates: int) -> None:
        """The round is over (aggregated or dropped): an abandoned wave ends with its rows."""
        try:
            self.unpre()
        except _native.NativeError:
            self.pre_dtype = None
        if self.table is not None:
            try:
                self.close(None)
            except _native.NativeError:
                pass
        self.closed, self.decided = None, False
        if round_updates:
            self.prev_arrivals = round_updates
