"""ctypes binding of the C ABI in ``include/fedavg_hip.h``.

There is no CPU fallback: if the in-tree HIP library is missing or fails to load, every
entry point raises. The symbols bound here are exactly the ones the header declares
(``tests/test_abi.py`` checks that list against the header text).
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int32, c_int64, c_uint32, c_void_p
from typing import Any

from .build import LIB_PATH

# enum fedavg_dtype
F32, F16, BF16, F64 = 0, 1, 2, 3
QSGD_F32, QSGD_F64 = 4, 5  # quantised records (quantized.py)
NNADQ_F32, NNADQ_F64 = 6, 7
RECORD_CODES = (QSGD_F32, QSGD_F64, NNADQ_F32, NNADQ_F64)
# enum fedavg_status
OK = 0
ERR_NAN_INPUT = 1
ERR_NAN_ACCUM = 2
ERR_NAN_RESULT = 3
ERR_INVALID = 4
ERR_HIP = 5
ERR_STATE = 6
ERR_RCCL = 7
COMM_ID_BYTES = 128
EXCHANGE_REDUCE, EXCHANGE_SCATTER = 0, 1  # FEDAVG_EXCHANGE_* (fedavg_sharded_round_edges)
EXCHANGE_PEER = 2  # fedavg_multi_round / _combine: peer-window stores, no collective library
MULTI_MAX_DEVICES = 16
FLAG_ACC_NAN = 0x1
FLAG_RESULT_NAN = 0x2
FLAG_CENTRAL_NAN = 0x4
ABI_VERSION = 1
ACC_ALIGN = 32  # FEDAVG_ACC_ALIGN: accumulator segments start at multiples of 32 elements
BUILD_ABLATE_EPILOGUE = 0x1
BUILD_ABLATE_QSGD = 0x2

_PP = POINTER(c_void_p)
_PD = POINTER(c_double)

# name -> (restype, argtypes); the full exported surface of the library
SIGNATURES: dict[str, tuple[Any, list[Any]]] = {
    "fedavg_abi_version": (c_int32, []),
    "fedavg_build_flags": (c_int32, []),
    "fedavg_kernel_constant": (c_int32, [ctypes.c_char_p, POINTER(c_int64)]),
    "fedavg_layout_acc_numel": (c_int64, [POINTER(c_int64), c_int32]),
    "fedavg_last_error": (ctypes.c_char_p, []),
    "fedavg_qsgd_record_bytes": (c_int64, [c_int64]),
    "fedavg_qsgd_sign_offset": (c_int64, [c_int64]),
    "fedavg_nnadq_record_bytes": (c_int64, [c_int64]),
    "fedavg_ctx_create": (
        c_int32,
        [POINTER(c_void_p), c_int32, POINTER(c_int64), c_int32, c_void_p],
    ),
    "fedavg_ctx_destroy": (c_int32, [c_void_p]),
    "fedavg_acc_numel": (c_int64, [c_void_p]),
    "fedavg_segment_offset": (c_int64, [c_void_p, c_int32]),
    "fedavg_accumulator": (c_void_p, [c_void_p]),
    "fedavg_set_split_policy": (c_int32, [c_void_p, c_int32]),
    "fedavg_set_fused_fold": (c_int32, [c_void_p, c_int32]),
    "fedavg_reset": (c_int32, [c_void_p, c_void_p]),
    "fedavg_total_weights": (c_int32, [c_void_p, _PD]),
    # the client table arguments are c_void_p: numpy / ctypes pointers or the staging extension's
    # raw addresses (no conversion objects per launch)
    "fedavg_accumulate": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_void_p]),
    "fedavg_aggregate": (
        c_int32,
        [c_void_p, c_void_p, c_int32, c_void_p, c_int32, _PP, c_int32, c_void_p],
    ),
    "fedavg_accumulate_delta": (c_int32, [c_void_p, _PP, c_int32, _PD, c_int32, _PP, c_void_p]),
    "fedavg_aggregate_delta": (
        c_int32,
        [c_void_p, _PP, c_int32, _PD, c_int32, _PP, _PP, c_int32, c_void_p],
    ),
    "fedavg_weighted_avg": (
        c_int32,
        [c_void_p, _PP, c_int32, _PD, c_int32, _PP, c_int32, c_void_p],
    ),
    "fedavg_partial": (
        c_int32,
        [c_void_p, _PP, c_int32, _PD, c_int32, c_int32, c_int32, c_int32, c_void_p],
    ),
    "fedavg_num_tiles": (c_int32, [c_void_p]),
    "fedavg_tile_range": (
        c_int32,
        [c_void_p, c_int32, c_int32, POINTER(c_int64), POINTER(c_int64)],
    ),
    "fedavg_set_accumulated": (c_int32, [c_void_p, _PD]),
    "fedavg_finalize_range": (
        c_int32,
        [c_void_p, _PP, c_int32, c_int32, c_int32, c_void_p],
    ),
    "fedavg_plan_create": (
        c_int32,
        [c_void_p, _PP, c_int32, _PD, c_int32, _PP, c_int32, POINTER(c_void_p)],
    ),
    "fedavg_plan_run": (c_int32, [c_void_p, c_void_p]),
    "fedavg_plan_create_partial": (
        c_int32,
        [c_void_p, _PP, c_int32, _PD, c_int32, c_int32, POINTER(c_void_p)],
    ),
    "fedavg_plan_create_finalize": (c_int32, [c_void_p, _PD, _PP, c_int32, POINTER(c_void_p)]),
    "fedavg_plan_run_range": (c_int32, [c_void_p, c_int32, c_int32, c_void_p]),
    "fedavg_plan_destroy": (c_int32, [c_void_p]),
    "fedavg_set_segment_state": (c_int32, [c_void_p, _PD, POINTER(c_int32)]),
    "fedavg_segment_state": (c_int32, [c_void_p, _PD, POINTER(c_int32)]),
    "fedavg_accumulate_elementwise": (
        c_int32, [c_void_p, _PP, c_int32, _PP, POINTER(c_int32), _PD, POINTER(c_int32), c_int32, c_void_p, c_void_p]),
    "fedavg_finalize_elementwise": (c_int32, [c_void_p, c_void_p, _PP, c_int32, c_void_p]),
    "fedavg_plan_finalize_window": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "fedavg_plan_copy_out": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "fedavg_plan_out_dtype": (c_int32, [c_void_p]),
    "fedavg_check": (c_int32, [c_void_p, c_void_p, POINTER(c_uint32)]),
    "fedavg_find_nan_clients": (
        c_int32,
        [c_void_p, _PP, c_int32, c_int32, POINTER(c_int32), c_void_p],
    ),
    "fedavg_prof_enable": (c_int32, [c_void_p, c_int32]),
    "fedavg_prof_collect": (c_int32, [c_void_p, _PD, POINTER(c_int32)]),
    "fedavg_bw_probe": (c_int32, [c_void_p, c_int64, c_void_p, c_int32, c_void_p]),
    # PersonalizedFedAVG (personalized_kernels.hip)
    "fedavg_pers_create": (c_int32, [POINTER(c_void_p), c_int32, POINTER(c_int64), c_int32]),
    "fedavg_pers_destroy": (c_int32, [c_void_p]),
    "fedavg_pers_set_fused_fold": (c_int32, [c_void_p, c_int32]),
    "fedavg_pers_aggregate": (
        c_int32,
        [c_void_p, _PP, c_int32, c_int32, POINTER(c_int64), _PD, POINTER(c_int64), c_int32, _PP, c_int32,
         _PP, c_int32, c_void_p],
    ),
    "fedavg_pers_check": (c_int32, [c_void_p, c_void_p, POINTER(c_uint32)]),
    "fedavg_pers_prof_enable": (c_int32, [c_void_p, c_int32]),
    "fedavg_pers_prof_collect": (c_int32, [c_void_p, _PD, POINTER(c_int32)]),
    "fedavg_fp64_probe": (c_int32, [c_int64, c_int32, _PD, c_void_p]),
    # host ingest (host_pack.cpp)
    "fedavg_host_pack": (c_int32, [c_void_p, _PP, POINTER(c_int64), POINTER(c_int64), c_int32]),
    "fedavg_host_pack_threads": (c_int32, []),
    "fedavg_comm_unique_id": (c_int32, [c_void_p]),
    "fedavg_comm_create": (c_int32, [_PP, c_void_p, c_int32, c_int32, c_int32]),
    "fedavg_comm_destroy": (c_int32, [c_void_p]),
    "fedavg_sharded_round": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "fedavg_sharded_round_scatter": (
        c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "fedavg_sharded_round_edges": (
        c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, POINTER(c_int32), c_int32, c_int32, c_int32, c_void_p]),
    # dynamic waves (dyn_wave_kernel)
    "fedavg_dyn_open": (c_int32, [c_void_p, c_int32, c_int32, c_void_p]),
    "fedavg_dyn_publish": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, POINTER(c_int32)]),
    "fedavg_dyn_close": (c_int32, [c_void_p, _PP, c_int32, c_int32, c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    "fedavg_dyn_state": (c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    "fedavg_dyn_info": (c_int32, [c_void_p, POINTER(c_int32), c_int32]),
    "fedavg_dyn_configure": (c_int32, [c_void_p, c_int64, c_int64]),
    "fedavg_dyn_timing": (c_int32, [c_void_p, POINTER(c_double), c_int32]),
    "fedavg_dyn_prof_collect": (c_int32, [c_void_p, POINTER(c_double), POINTER(c_int32)]),
    # single-process multi-device mode (multi_device.cpp)
    "fedavg_multi_create": (c_int32, [POINTER(c_void_p), POINTER(c_int32), c_int32, POINTER(c_int64), c_int32, _PP]),
    "fedavg_multi_destroy": (c_int32, [c_void_p]),
    "fedavg_multi_num_devices": (c_int32, [c_void_p]),
    "fedavg_multi_device": (c_int32, [c_void_p, c_int32]),
    "fedavg_multi_context": (c_void_p, [c_void_p, c_int32]),
    "fedavg_multi_stream": (c_void_p, [c_void_p, c_int32]),
    "fedavg_multi_peer_access": (c_int32, [c_void_p]),
    "fedavg_multi_round": (
        c_int32, [c_void_p, _PP, _PD, _PP, c_int32, c_int32, POINTER(c_int32), c_int32, c_int32, _PP]),
    "fedavg_multi_combine": (c_int32, [c_void_p, _PD, _PP, c_int32, c_int32, c_int32, _PP]),
    "fedavg_multi_check": (c_int32, [c_void_p, POINTER(c_uint32)]),
    "fedavg_multi_round_check": (c_int32, [c_void_p, POINTER(c_uint32)]),
    "fedavg_multi_reset": (c_int32, [c_void_p]),
    "fedavg_multi_prof_enable": (c_int32, [c_void_p, c_int32]),
    "fedavg_multi_prof_collect": (c_int32, [c_void_p, POINTER(c_double), POINTER(c_double), POINTER(c_int32)]),
}

_lib: ctypes.CDLL | None = None


class NativeError(RuntimeError):
    """A non-NaN failure reported by the HIP library."""

    def __init__(self, status: int, message: str) -> None:
        super().__init__(f"fedavg_hip status {status}: {message}")
        self.status = status


def load(path: str | None = None, allow_ablated: bool = False) -> ctypes.CDLL:
    """Load the in-tree HIP library (raises if it is absent — there is no fallback).

    A timing-only ablation build (``fedavg_build_flags() != 0``: results wrong by design) is
    refused unless ``allow_ablated`` or ``FEDAVG_ALLOW_ABLATED=1`` (the A/B scripts)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # FEDAVG_HIP_LIB: load a tuning build instead of the in-tree library (scripts/ A/B runs)
    lib_path = path or os.environ.get("FEDAVG_HIP_LIB") or str(LIB_PATH)
    try:
        lib = ctypes.CDLL(lib_path)
    except OSError as e:
        raise ImportError(
            f"MI355X FedAvg library not loadable at {lib_path}: {e}. "
            "Build it with `python -c 'import __graft_entry__ as g; g.build()'`."
        ) from e
    tuning_build = lib_path != str(LIB_PATH)
    for name, (restype, argtypes) in SIGNATURES.items():
        if tuning_build and not hasattr(lib, name):
            continue  # a tuning build from older sources: A/B runs use the timed entry points only
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    if lib.fedavg_abi_version() != ABI_VERSION:
        raise ImportError("fedavg_hip ABI version mismatch")
    flags = lib.fedavg_build_flags()
    if flags and not (allow_ablated or os.environ.get("FEDAVG_ALLOW_ABLATED") == "1"):
        raise ImportError(
            f"{lib_path} is a timing-only ablation build (fedavg_build_flags = {flags:#x}: "
            "its results are wrong by design); set FEDAVG_ALLOW_ABLATED=1 to load it for A/B timing"
        )
    if path is None:
        _lib = lib
    return lib


def kernel_constant(name: str) -> int:
    """A compile-time constant of the kernels' geometry (``fedavg_kernel_constant``)."""
    v = c_int64()
    check(load().fedavg_kernel_constant(name.encode(), ctypes.byref(v)))
    return int(v.value)


def last_error() -> str:
    msg = load().fedavg_last_error()
    return msg.decode() if msg else ""


def check(status: int) -> None:
    if status != OK:
        raise NativeError(status, last_error())
