"""DynamicWave (algorithm/dynamic_wave.py): the round's wave bookkeeping against a recording fake
context (CPU). The kernels themselves are covered by tests/test_gpu_dynamic_wave.py."""

from __future__ import annotations

import pytest
import torch

from distributed_learning_simulation_lib_amd import _native
from distributed_learning_simulation_lib_amd._staging import TableTail
from distributed_learning_simulation_lib_amd.algorithm import dynamic_wave as dw
from distributed_learning_simulation_lib_amd.algorithm.dynamic_wave import DynamicWave, DynamicWaveSettings


class FakeTable:
    def __init__(self, n: int = 0) -> None:
        self.num_clients = n
        self.num_segments = 1
        self.device_index = 0


class FakeStream:
    def synchronize(self) -> None:
        pass


class FakeCtx:
    """Records the fedavg_dyn_* calls; a publish takes every row, a close folds what was published."""

    def __init__(self, refuse_open: bool = False, bad_row: int | None = None, ended_at: int | None = None) -> None:
        self.calls: list = []
        self.refuse_open = refuse_open
        self.bad_row = bad_row
        self.published = 0
        self.reopens = 0
        self.ended_at = ended_at  # the wave ends itself after this many rows (a continued wave follows)

    def dyn_configure(self, idle_us: int, life_us: int) -> None:
        self.calls.append(("configure", idle_us, life_us))

    def dyn_open(self, dtype, max_clients) -> None:
        if self.refuse_open:
            raise _native.NativeError(_native.ERR_STATE, "the accumulator already holds data")
        self.calls.append(("open", dtype, max_clients))
        self.published = 0

    def dyn_publish(self, table) -> int:
        k = table.num_clients
        if self.bad_row is not None and k > self.bad_row >= self.published:
            n = self.bad_row - self.published
            self.published = self.bad_row
            e = _native.NativeError(_native.ERR_INVALID, "a row the wave cannot take")
            e.published = n
            raise e
        if self.ended_at is not None and self.published >= self.ended_at and k > self.published:
            self.reopens += 1
            self.ended_at = None
        n = k - self.published
        self.published = k
        self.calls.append(("publish", n))
        return n

    def dyn_close(self, outs, out_dtype=torch.float64, join=True):
        fin = outs is not None
        self.calls.append(("close", fin))
        return self.published, fin

    def dyn_info(self) -> dict:
        return {"reopens": self.reopens}


@pytest.fixture(autouse=True)
def _fake_tables(monkeypatch):
    # the controller takes native client tables only: the fake stands in for one here
    monkeypatch.setattr(dw, "NativeClientTable", FakeTable)


def _kinds(ctx):
    return [c[0] for c in ctx.calls]


def test_first_row_opens_then_every_batch_publishes():
    ctx = FakeCtx()
    w = DynamicWave(DynamicWaveSettings(batch=2))
    t = FakeTable(1)
    w.arrival(t, lambda: ctx, True, torch.float32, 64)
    assert _kinds(ctx) == ["configure", "open", "publish"] and w.table is t
    for n in range(2, 6):
        t.num_clients = n
        w.more(t)
    assert [c for c in ctx.calls if c[0] == "publish"] == [("publish", 1), ("publish", 2), ("publish", 2)]
    t.num_clients = 6
    assert w.finish(t, ["out"], torch.float64, FakeStream()) is True  # the last row, then the final close
    assert ctx.calls[-1] == ("close", True) and w.stats["rows"] == 6 and w.stats["finalized"] == 1


def test_ineligible_first_row_means_no_wave_and_no_preopen_next_round():
    ctx = FakeCtx()
    w = DynamicWave(DynamicWaveSettings())
    w.last_dtype = torch.float32
    w.arrival(FakeTable(1), lambda: ctx, False, torch.float32, 64)
    assert ctx.calls == [] and w.decided and w.last_dtype is None
    w.end_round(8)
    w.preopen(lambda: ctx, True, False, 64)  # nothing to pre-open with
    assert ctx.calls == []


def test_not_this_round_closes_a_preopened_wave():
    ctx = FakeCtx()
    w = DynamicWave(DynamicWaveSettings())
    w.last_dtype = torch.float16
    w.preopen(lambda: ctx, True, False, 64)
    assert _kinds(ctx) == ["configure", "open"] and w.pre_dtype == torch.float16
    w.not_this_round()  # e.g. the round's first update arrived in host memory
    assert ctx.calls[-1] == ("close", False) and w.pre_dtype is None and w.last_dtype is None and w.decided


def test_refused_open_is_counted_not_silent():
    ctx = FakeCtx(refuse_open=True)
    w = DynamicWave(DynamicWaveSettings())
    w.arrival(FakeTable(1), lambda: ctx, True, torch.float32, 64)
    assert w.table is None and w.stats["open_failures"] == 1 and "accumulator" in w.last_error
    assert w.stats["waves"] == 0


def test_row_it_cannot_take_closes_with_the_rows_before():
    ctx = FakeCtx(bad_row=3)
    w = DynamicWave(DynamicWaveSettings(batch=1))
    t = FakeTable(1)
    w.arrival(t, lambda: ctx, True, torch.float32, 64)
    for n in range(2, 6):
        t.num_clients = n
        w.more(t)
    assert w.table is None and w.closed == (t, 3)
    rest = w.rest(t)
    assert isinstance(rest, TableTail) and rest.offset == 3


def test_small_previous_round_skips_the_wave():
    ctx = FakeCtx()
    w = DynamicWave(DynamicWaveSettings(min_rows=16))
    w.end_round(8)
    w.arrival(FakeTable(1), lambda: ctx, True, torch.float32, 64)
    assert ctx.calls == [] and w.table is None


def test_continued_waves_are_counted():
    ctx = FakeCtx(ended_at=2)
    w = DynamicWave(DynamicWaveSettings(batch=1))
    t = FakeTable(1)
    w.arrival(t, lambda: ctx, True, torch.float32, 64)
    for n in range(2, 5):
        t.num_clients = n
        w.more(t)
    w.finish(t, ["out"], torch.float64, FakeStream())
    assert w.stats["reopens"] == 1 and w.stats["finalized"] == 1


def test_abandoned_round_closes_its_wave():
    ctx = FakeCtx()
    w = DynamicWave(DynamicWaveSettings())
    w.arrival(FakeTable(1), lambda: ctx, True, torch.float32, 64)
    w.end_round(1)
    assert ctx.calls[-1] == ("close", False) and w.table is None and not w.decided and w.prev_arrivals == 1


def test_dtypes_the_kernel_takes():
    assert dw.DYN_DTYPES == (torch.float32, torch.float16, torch.bfloat16, torch.float64)
