"""Host logic of the staging extension (csrc/staging_ext.cpp) on CPU tensors: what it refuses
(everything that is not resident on the GPU goes back to the Python staging unchanged), the
views it makes, and that a refusal leaves the per-name totals untouched."""

from __future__ import annotations

import pytest
import torch

from distributed_learning_simulation_lib_amd import _staging

ext = _staging.module()
pytestmark = pytest.mark.skipif(ext is None, reason="staging extension not built")


def test_host_tensors_are_refused_and_totals_untouched():
    params = {"a": torch.ones(3), "b": torch.ones(2, 2)}
    totals = {"a": 5.0}
    res = ext.stage_resident(params, {"a": 0, "b": 1}, [(3,), (2, 2)], 0, totals, 2.0)
    assert res is None
    assert totals == {"a": 5.0}
    assert ext.resident_row(params, {"a": 0, "b": 1}, [(3,), (2, 2)], 0) is None
    assert ext.row_pointers([torch.ones(3), None], [3, 4], 0, 0) is None


def test_unknown_names_and_non_tensors_are_refused():
    assert ext.stage_resident({"z": torch.ones(1)}, {"a": 0}, [(1,)], 0, {}, 1.0) is None
    assert ext.stage_resident({"a": [1.0]}, {"a": 0}, [(1,)], 0, {}, 1.0) is None
    assert ext.stage_resident({"a": torch.ones(1)}, {"a": 0}, [(1,)], 0, {}, object()) is None


def test_views_of_a_flat_buffer():
    flat = torch.arange(40, dtype=torch.float64)
    vs = ext.views(flat, [0, 8, 24, 39], [(2, 4), (4, 4), (), (1,)])
    assert [tuple(v.shape) for v in vs] == [(2, 4), (4, 4), (), (1,)]
    assert torch.equal(vs[0], flat[:8].view(2, 4))
    assert torch.equal(vs[1], flat[8:24].view(4, 4))
    assert float(vs[2]) == 24.0 and float(vs[3][0]) == 39.0
    assert all(v.is_contiguous() for v in vs)
    vs[1][0, 0] = -1.0  # views, not copies
    assert flat[8] == -1.0
    with pytest.raises(IndexError):
        ext.views(flat, [38], [(4,)])  # outside the buffer


def test_native_rows_refuse_host_updates_unchanged():
    rows = ext.Rows(2, 0)
    params = {"a": torch.ones(3), "b": torch.ones(2, 2)}
    assert rows.append(params, {"a": 0, "b": 1}, [(3,), (2, 2)], 2.0, -1) == -1
    assert rows.append({"z": torch.ones(1)}, {"a": 0, "b": 1}, [(3,), (2, 2)], 2.0, -1) == -1
    assert rows.append(params, {"a": 0, "b": 1}, [(3,), (2, 2)], object(), -1) == -1
    assert rows.num_clients == 0 and rows.ptr_bytes() == b""


def test_native_rows_general_appends_and_validation():
    import numpy as np

    t = _staging.NativeClientTable(3, 0)
    t.add_resident_client([16, 0, 48], [2.0, 0.0, 2.0], [5, -1, 7], 4, 0, [])
    t.add_resident_client([64, 80, 96], [3, 3, 3], [5, 6, 7], 4, 0, [])
    assert t.num_clients == 2
    p, w = t.arrays()
    assert p.tolist() == [16, 0, 48, 64, 80, 96] and w.tolist() == [2.0, 0.0, 2.0, 3.0, 3.0, 3.0]
    assert np.frombuffer(t.rows.numel_bytes(), dtype=np.int64).tolist() == [5, -1, 7, 5, 6, 7]
    t.validate([5, 6, 7], 4, 0, "k")  # absent entries are skipped
    with pytest.raises(ValueError, match="client 0, tensor 2: 7 elements; the layout needs 8"):
        t.validate([5, 6, 8], 4, 0, "k2")
    with pytest.raises(ValueError, match="input format needs 2 bytes"):
        t.validate([5, 6, 7], 2, 0, "k3")
    with pytest.raises(ValueError, match="device"):
        t.add_resident_client([1, 2, 3], [1, 1, 1], [5, 6, 7], 4, 1, [])
    with pytest.raises(ValueError):
        t.add_resident_client([1, 2], [1, 1], [5, 6], 4, 0, [])  # not a full row
    with pytest.raises(ValueError):
        t.add_resident_client([1, 2, 3], [1, 1, 1], [5, 6, 7], 8, 0, [])  # another element size
    assert t.num_clients == 2


def test_shape_checks_follow_the_shapes_list_passed():
    """The layout's shapes are parsed once per list object (csrc/staging_ext.cpp ShapeCache):
    alternating lists, a same-numel reshape and a malformed list are each judged on the list
    actually passed."""
    s1, s2 = [(2, 3), (4,)], [(3, 2), (4,)]
    idx = {"a": 0, "b": 1}
    good = {"a": torch.ones(2, 3), "b": torch.ones(4)}
    flipped = {"a": torch.ones(3, 2), "b": torch.ones(4)}
    for _ in range(2):
        assert ext.stage_resident(good, idx, s1, -1, {}, 1.0) is not None
        assert ext.stage_resident(flipped, idx, s1, -1, {}, 1.0) is None  # same numel, other shape
        assert ext.stage_resident(flipped, idx, s2, -1, {}, 1.0) is not None
        assert ext.stage_resident(good, idx, s2, -1, {}, 1.0) is None
        assert ext.stage_resident({"a": torch.ones(6)}, idx, s1, -1, {}, 1.0) is None  # other rank
    assert ext.stage_resident(good, idx, [(2, 3), [4]], -1, {}, 1.0) is None  # not a tuple
    assert ext.stage_resident(good, idx, [(2, 3), ("4",)], -1, {}, 1.0) is None  # not an int
    assert ext.stage_resident(good, idx, s1, -1, {}, 1.0) is not None


def test_result_buffer_is_reused_only_when_nobody_can_see_it():
    """``unobserved`` (FedAVGAlgorithm._result_buffer): a result buffer of an earlier round is
    written again only when its views are referenced by the pool list alone, untouched."""
    flat = torch.zeros(40, dtype=torch.float64)
    offs, shapes = [0, 8, 24], [(2, 4), (4, 4), (3,)]
    views = ext.views(flat, offs, shapes)
    assert ext.unobserved(flat, views, offs, shapes)
    kept = views[1]  # a result the caller kept
    assert not ext.unobserved(flat, views, offs, shapes)
    del kept
    assert ext.unobserved(flat, views, offs, shapes)
    row = views[0][0]  # a view of a result
    assert not ext.unobserved(flat, views, offs, shapes)
    del row
    alias = flat.view(4, 10)  # another tensor on the buffer
    assert not ext.unobserved(flat, views, offs, shapes)
    del alias
    assert ext.unobserved(flat, views, offs, shapes)
    assert not ext.unobserved(flat, views, [0, 8, 25], shapes)  # not where the views are
    assert not ext.unobserved(flat, views, offs, [(2, 4), (4, 4), (1, 3)])
    views[2].foo = 1  # a Python attribute on a result
    assert not ext.unobserved(flat, views, offs, shapes)
    for make in (lambda v: v.unsqueeze_(0), lambda v: v.requires_grad_()):
        views = ext.views(flat, offs, shapes)
        assert ext.unobserved(flat, views, offs, shapes)
        make(views[0])  # an in-place change of a result's metadata
        assert not ext.unobserved(flat, views, offs, shapes)
    # a storage handle (torch may keep its Python object for the storage's lifetime: the buffer
    # is then never reused, which only costs a fresh allocation per round)
    flat = torch.zeros(40, dtype=torch.float64)
    views = ext.views(flat, offs, shapes)
    st = views[2].untyped_storage()
    assert not ext.unobserved(flat, views, offs, shapes)


def test_a_buffer_shared_with_another_process_is_never_reused():
    """torch.multiprocessing sharing leaves the reference counts as they were but moves the buffer
    (host: into shared memory; CUDA: behind the IPC limbo's deleter): ``unobserved`` also requires
    the allocator's own deleter, so such a buffer is never written again."""
    from multiprocessing.reduction import ForkingPickler

    import torch.multiprocessing as _torch_mp  # noqa: F401  (registers the tensor reducers)

    flat = torch.zeros(40, dtype=torch.float64)
    offs, shapes = [0, 8, 24], [(2, 4), (4, 4), (3,)]
    views = ext.views(flat, offs, shapes)
    assert ext.unobserved(flat, views, offs, shapes)
    payload = ForkingPickler.dumps(views[1])  # what a Queue / Pipe put of the result does
    import gc

    gc.collect()
    assert not ext.unobserved(flat, views, offs, shapes)
    del payload


def test_table_arguments_reach_a_c_abi_pointer_parameter():
    """fedavg._table_args: the native table's raw addresses and a ClientTable's numpy arrays both
    pass through a c_void_p parameter (the hot entry points' client table arguments) with the
    table's contents behind them."""
    import ctypes

    import numpy as np

    from distributed_learning_simulation_lib_amd.fedavg import _EMPTY_TABLE, ClientTable, _table_args

    memcpy = ctypes.CDLL(None).memcpy
    memcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    native = _staging.NativeClientTable(3, 0)
    native.add_resident_client([16, 0, 48], [2.0, 0.0, 2.5], [5, -1, 7], 4, 0, [])
    general = ClientTable(2)
    general.add_client([torch.ones(3), None], [1.5, 0.0])
    for table, n in ((native, 3), (general, 2)):
        want_p, want_w = table.arrays()
        p, w = _table_args(table)
        got_p, got_w = np.zeros(n, np.uint64), np.zeros(n, np.float64)
        memcpy(got_p.ctypes.data, p, 8 * n)
        memcpy(got_w.ctypes.data, w, 8 * n)
        assert got_p.tolist() == want_p.tolist() and got_w.tolist() == want_w.tolist()
    one = np.ones(1, np.float64)
    memcpy(one.ctypes.data, _EMPTY_TABLE[1], 8)
    assert one[0] == 0.0
