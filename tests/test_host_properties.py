"""CPU property tests (hypothesis) of host-side pieces: the native host packer, layouts. No GPU
and no compute kernels: runs in the CPU suite."""

from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from distributed_learning_simulation_lib_amd import ParameterMessage, _native
from distributed_learning_simulation_lib_amd.build import build
from distributed_learning_simulation_lib_amd.fedavg import ModelLayout


@pytest.fixture(scope="module")
def lib():
    build()
    return _native.load()


@settings(max_examples=40, deadline=None)
@given(sizes=st.lists(st.integers(0, 300_000), min_size=1, max_size=12),
       elem=st.sampled_from([2, 4, 8]), absent=st.lists(st.booleans(), min_size=12, max_size=12))
def test_host_pack_places_every_tensor_at_its_aligned_offset(lib, sizes, elem, absent):
    """fedavg_host_pack == per-tensor copies into ModelLayout.padded_offsets (byte-exact)."""
    dtype = {2: np.uint16, 4: np.uint32, 8: np.uint64}[elem]
    rng = np.random.default_rng(len(sizes) * 7 + elem)
    srcs = [None if (absent[i] or n == 0) else rng.integers(0, 2**15, size=n).astype(dtype) for i, n in enumerate(sizes)]
    layout = ModelLayout(names=tuple(f"t{i}" for i in range(len(sizes))), shapes=tuple((n,) for n in sizes))
    offs, padded = layout.padded_offsets(elem)
    dst = np.full(padded + 1, 0xAB, dtype=dtype)
    ptrs = (ctypes.c_void_p * len(srcs))(*[0 if s is None else s.ctypes.data for s in srcs])
    nbytes = (ctypes.c_int64 * len(srcs))(*[0 if s is None else s.size * elem for s in srcs])
    doff = (ctypes.c_int64 * len(srcs))(*[o * elem for o in offs])
    assert lib.fedavg_host_pack(ctypes.c_void_p(dst.ctypes.data), ptrs, nbytes, doff, len(srcs)) == 0
    want = np.full(padded + 1, 0xAB, dtype=dtype)
    for s, o in zip(srcs, offs):
        if s is not None:
            want[o : o + s.size] = s
    assert np.array_equal(dst, want)


def test_host_pack_rejects_bad_arguments(lib):
    assert lib.fedavg_host_pack(None, None, None, None, 3) == _native.ERR_INVALID
    assert lib.fedavg_host_pack_threads() >= 1


@settings(max_examples=40, deadline=None)
@given(shapes=st.lists(st.lists(st.integers(0, 9), min_size=0, max_size=3), min_size=1, max_size=8),
       elem=st.sampled_from([2, 4, 8]))
def test_padded_offsets_are_aligned_and_disjoint(shapes, elem):
    lay = ModelLayout(names=tuple(f"p{i}" for i in range(len(shapes))), shapes=tuple(tuple(s) for s in shapes))
    offs, total = lay.padded_offsets(elem)
    ends = [o + n for o, n in zip(offs, lay.numels)]
    assert all(o * elem % 16 == 0 for o in offs)
    assert all(e <= o2 for e, o2 in zip(ends, offs[1:])) and (not ends or ends[-1] <= total)
