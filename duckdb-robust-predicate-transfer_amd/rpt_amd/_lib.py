"""ctypes binding of librpt_gpu.so (the C-ABI declared in include/rpt_gpu.h).

The library is built in-tree (``make -C duckdb-robust-predicate-transfer_amd``) and loaded from
``duckdb-robust-predicate-transfer_amd/build/librpt_gpu.so``. There is no fallback: if the library
is missing, every call raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "build", "librpt_gpu.so")

RPT_OK = 0
RPT_ERR_INVALID_ARGUMENT = 1
RPT_ERR_HIP = 2
RPT_ERR_OUT_OF_MEMORY = 3
RPT_ERR_WORKSPACE = 4
RPT_ERR_SHAPE_MISMATCH = 5
RPT_ERR_COLLECTIVE = 6
RPT_ERR_COMM_ABORTED = 7

RPT_PROBE_AUTO = 0
RPT_PROBE_GATHER = 1
RPT_PROBE_LDS = 2
RPT_PROBE_PARTITIONED = 3
RPT_PROBE_BUCKETED = 4

RPT_INSERT_AUTO = 0
RPT_INSERT_ATOMIC = 1
RPT_INSERT_PARTITIONED = 2
RPT_INSERT_BUCKETED = 3

RPT_KEY_I64 = 0
RPT_KEY_I32 = 1
RPT_KEY_HASH = 2


class RptError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"rpt status {status}: {message}")
        self.status = status


class KeyColumn(ctypes.Structure):
    """rpt_key_column (include/rpt_gpu.h)."""

    _fields_ = [
        ("key_type", c_int32),
        ("keys", c_void_p),
        ("key_sel", c_void_p),
        ("validity", c_void_p),
    ]


class BfInfo(ctypes.Structure):
    """rpt_bf_info (include/rpt_gpu.h)."""

    _fields_ = [
        ("device", c_int32),
        ("log_num_blocks", c_int32),
        ("num_blocks", c_uint64),
        ("sized_for_rows", c_uint64),
        ("has_data", c_int32),
        ("finalized", c_int32),
        ("words", c_void_p),
    ]


class KernelStat(ctypes.Structure):
    """rpt_kernel_stat (include/rpt_gpu.h)."""

    _fields_ = [("name", ctypes.c_char * 48), ("launches", c_uint64), ("total_ms", ctypes.c_double)]


# name -> (restype, argtypes); every symbol include/rpt_gpu.h and include/rpt_gpu_synth.h declare.
SIGNATURES = {
    "rpt_abi_version": (c_int, []),
    "rpt_status_string": (c_char_p, [c_int]),
    "rpt_last_error": (c_char_p, []),
    "rpt_bf_log_num_blocks_for_rows": (c_int, [c_uint64]),
    "rpt_bf_needs_resize": (c_int, [c_uint64, c_uint64]),
    "rpt_bf_needs_resize_alloc": (c_int, [c_void_p, c_uint64]),
    "rpt_probe_workspace_bytes": (c_size_t, [c_uint64, c_int]),
    "rpt_bf_set_probe_strategy": (c_int, [c_void_p, c_int]),
    "rpt_probe_strategy_supported": (c_int, [c_int, c_int]),
    "rpt_bf_probe_strategy": (c_int, [c_void_p]),
    "rpt_bf_probe_strategy_for": (c_int, [c_void_p, c_uint64]),
    "rpt_bf_probe_is_fused": (c_int, [c_void_p, c_uint64]),
    "rpt_bf_insert_strategy_for": (c_int, [c_void_p, c_uint64]),
    "rpt_bf_probe_workspace_bytes": (c_size_t, [c_void_p, c_uint64]),
    "rpt_bf_create": (c_int, [c_int, c_uint64, POINTER(c_void_p)]),
    "rpt_bf_create_log_blocks": (c_int, [c_int, c_int, POINTER(c_void_p)]),
    "rpt_bf_destroy": (c_int, [c_void_p]),
    "rpt_bf_get_info": (c_int, [c_void_p, POINTER(BfInfo)]),
    "rpt_bf_reinitialize": (c_int, [c_void_p, c_uint64]),
    "rpt_bf_set_finalized": (c_int, [c_void_p, c_int]),
    "rpt_bf_clear": (c_int, [c_void_p, c_void_p]),
    "rpt_bf_settle": (c_int, [c_void_p, c_void_p]),
    "rpt_bf_insert": (c_int, [c_void_p, POINTER(KeyColumn), c_uint64, c_void_p]),
    "rpt_insert_workspace_bytes": (c_size_t, [c_uint64, c_int]),
    "rpt_bf_insert_workspace_bytes": (c_size_t, [c_void_p, c_uint64]),
    "rpt_bf_insert_ws": (c_int, [c_void_p, POINTER(KeyColumn), c_uint64, c_void_p, c_size_t, c_void_p]),
    "rpt_bf_set_insert_strategy": (c_int, [c_void_p, c_int]),
    "rpt_bf_get_minmax": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int), c_void_p]),
    "rpt_bf_set_minmax": (c_int, [c_void_p, c_int64, c_int64, c_int, c_void_p]),
    "rpt_bf_probe": (
        c_int,
        [c_void_p, POINTER(KeyColumn), c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "rpt_bf_probe_chain": (
        c_int, [c_void_p, POINTER(KeyColumn), ctypes.c_uint32, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]
    ),
    "rpt_bf_probe_phase1": (
        c_int, [c_void_p, POINTER(KeyColumn), c_void_p, c_uint64, c_void_p, c_size_t, c_void_p]
    ),
    "rpt_bf_probe_phase2": (
        c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    ),
    "rpt_bf_find_bits": (c_int, [c_void_p, POINTER(KeyColumn), c_uint64, c_void_p, c_void_p]),
    "rpt_hash_keys": (c_int, [POINTER(KeyColumn), c_uint64, c_void_p, c_void_p]),
    "rpt_hash_combine": (c_int, [POINTER(KeyColumn), c_uint64, c_void_p, c_void_p]),
    "rpt_keys_widen": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    "rpt_bf_probe_bits": (c_int, [c_void_p, POINTER(KeyColumn), c_void_p, c_uint64, c_void_p, c_void_p, c_size_t, c_void_p]),
    "rpt_bf_merge_or": (c_int, [c_void_p, c_void_p, c_void_p]),
    "rpt_bf_allreduce_or": (c_int, [c_void_p, c_void_p, c_void_p]),
    "rpt_bf_allreduce_or_ws": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "rpt_allreduce_workspace_bytes": (c_size_t, [c_int, c_int]),
    "rpt_collective_set_timeout_ms": (c_int, [c_uint64]),
    "rpt_collective_timeout_ms": (c_uint64, []),
    "rpt_collective_set_abort_on_error": (c_int, [c_int]),
    "rpt_collective_abort_on_error": (c_int, []),
    "rpt_rccl_available": (c_int, [c_int]),
    "rpt_rccl_get_unique_id": (c_int, [c_void_p]),
    "rpt_rccl_comm_init_rank": (c_int, [c_int, c_int, c_void_p, c_int, POINTER(c_void_p)]),
    "rpt_rccl_comm_init_rank_nonblocking": (c_int, [c_int, c_int, c_void_p, c_int, POINTER(c_void_p)]),
    "rpt_rccl_comm_destroy": (c_int, [c_void_p]),
    "rpt_words_or": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_words_or_slices": (c_int, [c_void_p, c_void_p, c_uint32, c_uint64, c_void_p]),
    "rpt_bf_count_bits": (c_int, [c_void_p, POINTER(c_uint64)]),
    "rpt_bf_is_same_as": (c_int, [c_void_p, c_void_p, POINTER(c_int), POINTER(c_uint64)]),
    "rpt_bf_fold": (c_int, [c_void_p, POINTER(c_int)]),
    "rpt_bf_export_words": (c_int, [c_void_p, c_void_p, c_uint64]),
    "rpt_bf_import_words": (c_int, [c_void_p, c_void_p, c_uint64]),
    "rpt_bf_copy_words_to": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_bf_copy_words_from": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_bf_set_has_data": (c_int, [c_void_p, c_int]),
    "rpt_profiling_enable": (c_int, [c_int]),
    "rpt_profiling_reset": (c_int, []),
    "rpt_profiling_read": (c_int, [POINTER(KernelStat), c_int]),
    "rpt_synth_build_keys": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p]),
    "rpt_synth_probe_keys": (c_int, [c_void_p, c_uint64, c_uint32, c_uint64, c_uint64, c_void_p]),
    "rpt_stream_sink_words": (c_uint64, [c_int]),
    "rpt_stream_read": (c_int, [c_void_p, c_uint64, c_void_p, c_void_p]),
    "rpt_stream_copy": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
}

_lib = None


def _bind(p: str) -> ctypes.CDLL:
    if not os.path.exists(p):
        raise RptError(-1, f"librpt_gpu.so not found at {p}; build it with `make -C {PKG_DIR}`")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and return librpt_gpu.so. Raises if it is missing: there is no CPU fallback."""
    global _lib
    if _lib is None:
        _lib = _bind(path or os.environ.get("RPT_GPU_LIB", LIB_PATH))
    return _lib


def load_variant(path: str) -> ctypes.CDLL:
    """Bind another build of the same C-ABI (the test build tests/loopback/build/librpt_gpu_testing.so)
    beside the product library; handles from one build must not be passed to the other."""
    return _bind(path)


def check(status: int, lib=None) -> None:
    """Raise RptError for a non-OK status with the message of `lib` (the library that returned it; default the
    product library)."""
    if status != RPT_OK:
        lib = lib if lib is not None else load()
        raise RptError(status, lib.rpt_last_error().decode(errors="replace"))


def kernel_times() -> dict:
    """{kernel name: (launches, total_ms)} recorded since the last reset (see rpt_profiling_*)."""
    lib = load()
    n = lib.rpt_profiling_read(None, 0)
    if n < 0:
        check(-n)
    arr = (KernelStat * max(n, 1))()
    n = lib.rpt_profiling_read(arr, n)
    return {arr[i].name.decode(): (arr[i].launches, arr[i].total_ms) for i in range(n)}


def profiling(enable: bool) -> None:
    check(load().rpt_profiling_enable(int(enable)))


def profiling_reset() -> None:
    check(load().rpt_profiling_reset())
