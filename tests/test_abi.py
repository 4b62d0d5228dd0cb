"""The C ABI surface: header <-> binding <-> exported symbols (CPU only, no compute calls)."""

import re

import pytest
import subprocess
from pathlib import Path

from distributed_learning_simulation_lib_amd import _native
from distributed_learning_simulation_lib_amd.build import LIB_PATH, build

HEADER = Path(__file__).resolve().parent.parent / "include" / "fedavg_hip.h"


def header_functions() -> set[str]:
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(fedavg_[a-z0-9_]+)\s*\(", text))


def test_binding_covers_header_exactly():
    assert header_functions() == set(_native.SIGNATURES)


def test_library_builds_loads_and_exports_every_symbol():
    build()  # no-op when up to date; hipcc cross-compiles gfx950 without a GPU
    assert LIB_PATH.exists()
    lib = _native.load()
    assert lib.fedavg_abi_version() == _native.ABI_VERSION
    nm = subprocess.run(["nm", "-D", "--defined-only", str(LIB_PATH)], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (fedavg_[a-z0-9_]+)\b", nm.stdout))
    assert header_functions() <= exported


def test_gfx950_code_object_present():
    # the offload bundle embedded in .hip_fatbin names its target
    assert b"amdgcn-amd-amdhsa--gfx950" in LIB_PATH.read_bytes()


def test_null_context_is_rejected_without_a_gpu():
    lib = _native.load()
    assert lib.fedavg_reset(None, None) == _native.ERR_INVALID
    assert "null context" in _native.last_error()


def test_product_build_is_not_an_ablation_build():
    lib = _native.load()
    assert lib.fedavg_build_flags() == 0


def test_layout_acc_numel_aligns_segments():
    import ctypes

    lib = _native.load()
    numels = [1, 31, 32, 33, 4097]
    arr = (ctypes.c_int64 * len(numels))(*numels)
    want = sum((n + _native.ACC_ALIGN - 1) // _native.ACC_ALIGN * _native.ACC_ALIGN for n in numels)
    assert lib.fedavg_layout_acc_numel(arr, len(numels)) == want
    assert lib.fedavg_layout_acc_numel(arr, 0) == -1


def test_kernel_constants_are_readable_without_a_gpu():
    """fedavg_kernel_constant: the geometry the GPU property tests place their sizes around."""
    from distributed_learning_simulation_lib_amd._native import NativeError, kernel_constant

    assert kernel_constant("tile") == 4096 and kernel_constant("tile_wide") in (0, 4096, 8192)
    for d in ("f32", "f16", "bf16", "f64"):
        ae, lanes = kernel_constant(f"ae_{d}"), kernel_constant(f"lanes_{d}")
        assert ae > 0 and lanes % 64 == 0 and kernel_constant(f"group_{d}") >= 2
        assert kernel_constant(f"ae4096_{d}") * kernel_constant(f"lanes4096_{d}") == 4096
        assert kernel_constant(f"pipe_{d}") >= 0
    assert kernel_constant("pers_group") % kernel_constant("pers_jb") == 0
    assert kernel_constant("qsgd_tile") == kernel_constant("qsgd_ae") * 256
    for bad in ("nope", "ae_f8", "pers_nope", ""):
        with pytest.raises(NativeError):
            kernel_constant(bad)
