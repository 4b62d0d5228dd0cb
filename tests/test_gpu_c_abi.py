"""The drop-in boundary used without Python: examples/c_abi_round.cpp drives a streamed round and
a sharded round (one-rank RCCL world, ``fedavg_comm_*`` + ``fedavg_sharded_round``) through
include/fedavg_hip.h alone and checks both bit-for-bit against a host fp64 fold in arrival order.
Built by ``build()`` next to the library; run here as a child process."""

from __future__ import annotations

import subprocess

import pytest

from distributed_learning_simulation_lib_amd.build import LIB_DIR

pytestmark = pytest.mark.gpu


def test_c_abi_round_binary():
    exe = LIB_DIR / "c_abi_round"
    assert exe.exists(), "examples not built: run __graft_entry__.build()"
    proc = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert "streamed round: bit-identical" in proc.stdout
    assert "sharded round 2: bit-identical" in proc.stdout
    assert proc.stdout.strip().endswith("PASS")
