"""The native multi-rank round (``fedavg_sharded_round`` / ``fedavg_sharded_round_scatter`` at
world 2, 3 and 4) on the one GPU of a test box: ``tests/native/threaded_ranks.cpp`` runs every
rank as a thread of one process, and ``FEDAVG_RCCL_LIB`` points the library's run-time RCCL
binding at ``tests/native/fake_rccl.cpp`` (real RCCL refuses two ranks on one GPU). Covers what a
one-rank RCCL world cannot: chunk windows split over G ranks, the scatter tail (G = 3), the gather
placement, roots 0 and G - 1, fp32 / fp64 outputs, two rounds on the same plans, a NaN in another
rank's shard — bit-for-bit against the host composition. The send / recv gather
fallback runs with the stand-in built without ``ncclGather``."""

from __future__ import annotations

import ctypes
import os
import subprocess

import pytest

from distributed_learning_simulation_lib_amd.build import FAKE_RCCL, LIB_DIR

# the RCCL entry points sharded_comm.cpp binds by name (ncclGather optional)
BOUND = ["ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclReduce", "ncclReduceScatter",
         "ncclGroupStart", "ncclGroupEnd", "ncclSend", "ncclRecv", "ncclGetErrorString"]


@pytest.mark.parametrize("lib", sorted(FAKE_RCCL))
def test_fake_rccl_exports_what_the_library_binds(lib):
    so = LIB_DIR / lib
    assert so.exists(), "test libraries not built: run __graft_entry__.build()"
    h = ctypes.CDLL(str(so))
    for name in BOUND:
        assert hasattr(h, name), name
    assert hasattr(h, "ncclGather") == ("nogather" not in lib)


@pytest.mark.gpu
@pytest.mark.parametrize("lib", sorted(FAKE_RCCL))
def test_native_round_with_threaded_ranks(lib):
    exe = LIB_DIR / "threaded_ranks"
    assert exe.exists(), "test programs not built: run __graft_entry__.build()"
    env = dict(os.environ, FEDAVG_RCCL_LIB=str(LIB_DIR / lib))
    proc = subprocess.run([str(exe)], capture_output=True, text=True, timeout=150, env=env)
    assert proc.returncode == 0, proc.stdout + proc.stderr
    for g in (2, 3, 4):
        assert f"G={g} root=0: 40 root rounds checked" in proc.stdout, proc.stdout
        assert f"G={g} root={g - 1}: 40 root rounds checked" in proc.stdout, proc.stdout
    assert proc.stdout.count("sweep G=") == 6, proc.stdout  # the randomised layouts
    assert proc.stdout.strip().endswith("PASS")
