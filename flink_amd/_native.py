"""ctypes binding of ``include/gwo.h`` (libgwo.so, built in-tree for gfx950).

The product path has exactly one implementation: the HIP kernels behind this library.  If the
library is missing or cannot be loaded, importing this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# GWO_LIB_PATH selects an alternative build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("GWO_LIB_PATH") or os.path.join(_HERE, "libgwo.so")

GWO_ABI_VERSION = 4
GWO_MAX_AGGS = 4

# gwo_status
GWO_OK = 0
STATUS_NAMES = {
    0: "GWO_OK", 1: "GWO_ERR_INVALID_ARGUMENT", 2: "GWO_ERR_NO_TIMESTAMP", 3: "GWO_ERR_KEY_GROUP",
    4: "GWO_ERR_OUT_OF_MEMORY", 5: "GWO_ERR_HIP", 6: "GWO_ERR_UNSUPPORTED", 7: "GWO_ERR_MERGE_LATE",
    8: "GWO_ERR_COMM", 9: "GWO_ERR_STATE", 10: "GWO_ERR_CAPACITY",
}
globals().update({name: code for code, name in STATUS_NAMES.items()})
ASSIGNER_TUMBLING, ASSIGNER_SLIDING, ASSIGNER_SESSION = 0, 1, 2
AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG = 0, 1, 2, 3, 4
DTYPE_INT64, DTYPE_FLOAT64 = 0, 1
KEY_LONG, KEY_INT, KEY_STRING = 0, 1, 2
STATE_AUTO, STATE_TABLE, STATE_LOG = 0, 1, 2
KERNEL_SCAN, KERNEL_INSERT, KERNEL_FIRE, KERNEL_PARTITION, KERNEL_EXCHANGE, KERNEL_SLIDE, KERNEL_SESSION = range(7)
COMM_ID_BYTES = 128


class GwoConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("assigner", C.c_int32),
        ("size", C.c_int64), ("slide", C.c_int64), ("offset", C.c_int64), ("gap", C.c_int64),
        ("allowed_lateness", C.c_int64),
        ("num_aggs", C.c_int32), ("aggs", C.c_int32 * GWO_MAX_AGGS),
        ("value_dtype", C.c_int32), ("key_kind", C.c_int32), ("max_parallelism", C.c_int32),
        ("key_group_start", C.c_int32), ("key_group_end", C.c_int32), ("device", C.c_int32),
        ("side_output", C.c_int32), ("state_layout", C.c_int32), ("expected_keys", C.c_int64),
        ("stream", C.c_void_p),
    ]


class GwoOut(C.Structure):
    _fields_ = [("key", C.c_void_p), ("start", C.c_void_p), ("end", C.c_void_p),
                ("result", C.c_void_p * GWO_MAX_AGGS)]


class GwoSideOut(C.Structure):
    _fields_ = [("key", C.c_void_p), ("ts", C.c_void_p), ("value", C.c_void_p)]


class GwoStateRows(C.Structure):
    _fields_ = [("key", C.c_void_p), ("window_start", C.c_void_p), ("window_end", C.c_void_p), ("words", C.c_void_p),
                ("key_group", C.c_void_p), ("timer", C.c_void_p)]


class GwoCommWaits(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("routed_batches", "count_waits", "wm_waits", "flow_count_waits",
                                         "flow_wm_waits", "count_wait_ns", "wm_wait_ns", "flow_wait_ns")]


class GwoHeapStateIds(C.Structure):
    _fields_ = [("window_contents", C.c_int16), ("merging_window_set", C.c_int16), ("event_timers", C.c_int16),
                ("processing_timers", C.c_int16)]


class GwoGenSpec(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64), ("first_index", C.c_int64), ("total_records", C.c_int64),
        ("num_keys", C.c_int64), ("span_ms", C.c_int64), ("disorder_ms", C.c_int64), ("t0", C.c_int64),
        ("value_range", C.c_int64), ("value_dtype", C.c_int32), ("key_mode", C.c_int32),
    ]


# (name, restype, argtypes) -- every symbol include/gwo.h declares
_P = C.c_void_p
_I64P = C.POINTER(C.c_int64)
SIGNATURES = [
    ("gwo_config_init", None, [C.POINTER(GwoConfig)]),
    ("gwo_create", C.c_int, [C.POINTER(GwoConfig), C.POINTER(_P)]),
    ("gwo_destroy", C.c_int, [_P]),
    ("gwo_submit", C.c_int, [_P, _P, _P, _P, C.c_int64]),
    ("gwo_wait_stream", C.c_int, [_P, _P]),
    ("gwo_host_register", C.c_int, [_P, C.c_int64]),
    ("gwo_host_unregister", C.c_int, [_P]),
    ("gwo_submit_utf16", C.c_int, [_P, _P, _P, _P, _P, C.c_int64]),
    ("gwo_intern_utf16", C.c_int, [_P, _P, _P, C.c_int64, _P]),
    ("gwo_key_strings", C.c_int, [_P, _P, C.c_int64, _P, _P, C.c_int64, _I64P]),
    ("gwo_advance_watermark", C.c_int, [_P, C.c_int64]),
    ("gwo_end_input", C.c_int, [_P]),
    ("gwo_output_count", C.c_int, [_P, _I64P]),
    ("gwo_rows_emitted", C.c_int, [_P, _I64P]),
    ("gwo_drain", C.c_int, [_P, C.POINTER(GwoOut), C.c_int64, _I64P]),
    ("gwo_output_view", C.c_int, [_P, C.POINTER(GwoOut), _I64P]),
    ("gwo_discard_output", C.c_int, [_P]),
    ("gwo_result_dtype", C.c_int, [_P, C.c_int32, C.POINTER(C.c_int32)]),
    ("gwo_late_dropped", C.c_int, [_P, _I64P]),
    ("gwo_side_output_count", C.c_int, [_P, _I64P]),
    ("gwo_drain_side_output", C.c_int, [_P, C.POINTER(GwoSideOut), C.c_int64, _I64P]),
    ("gwo_current_watermark", C.c_int, [_P, _I64P]),
    ("gwo_get_config", C.c_int, [_P, C.POINTER(GwoConfig)]),
    ("gwo_state_size", C.c_int, [_P, _I64P]),
    ("gwo_snapshot_rows", C.c_int, [_P, _I64P, C.POINTER(C.c_int32)]),
    ("gwo_snapshot", C.c_int, [_P, C.POINTER(GwoStateRows), C.c_int64, _I64P, _I64P]),
    ("gwo_restore", C.c_int, [_P, C.POINTER(GwoStateRows), C.c_int32, C.c_int64, C.c_int64]),
    ("gwo_export_heap_state", C.c_int, [_P, C.POINTER(GwoHeapStateIds), _P, C.c_int64, _I64P, _P, _I64P]),
    ("gwo_import_heap_state", C.c_int, [_P, C.POINTER(GwoHeapStateIds), _P, C.c_int64, C.c_int64]),
    ("gwo_export_heap_state_begin", C.c_int, [_P, C.POINTER(GwoHeapStateIds), _I64P, _I64P, _I64P]),
    ("gwo_export_heap_state_read", C.c_int, [_P, C.c_int64, _P, C.c_int64]),
    ("gwo_export_heap_state_end", C.c_int, [_P]),
    ("gwo_sync", C.c_int, [_P]),
    ("gwo_wait_fires", C.c_int, [_P]),
    ("gwo_get_stream", C.c_int, [_P, C.POINTER(_P)]),
    ("gwo_last_error", C.c_char_p, [_P]),
    ("gwo_status_string", C.c_char_p, [C.c_int]),
    ("gwo_set_profiling", C.c_int, [_P, C.c_int32]),
    ("gwo_set_profiling_mask", C.c_int, [_P, C.c_uint32]),
    ("gwo_set_pipelined_submit", C.c_int, [_P, C.c_int32]),
    ("gwo_kernel_stats", C.c_int, [_P, C.c_int32, _I64P, C.POINTER(C.c_double), _I64P]),
    ("gwo_reset_stats", C.c_int, [_P]),
    ("gwo_assign_key_groups", C.c_int, [_P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _P, _P, C.c_int32]),
    ("gwo_assign_key_groups_utf16", C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P, C.c_int32]),
    ("gwo_window_starts", C.c_int, [_P, C.c_int64, C.c_int64, C.c_int64, _P, C.c_int32]),
    ("gwo_comm_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("gwo_comm_init", C.c_int, [_P, C.POINTER(C.c_uint8), C.c_int32, C.c_int32]),
    ("gwo_comm_set_async_watermark", C.c_int, [_P, C.c_int32]),
    ("gwo_comm_stats", C.c_int, [_P, _I64P, _I64P, _I64P]),
    ("gwo_comm_wait_stats", C.c_int, [_P, _P]),
    ("gwo_partition_by_operator", C.c_int, [_P, _P, _P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _P, C.c_int64,
                                            _P, C.c_int32]),
    ("gwo_generate", C.c_int, [C.POINTER(GwoGenSpec), C.c_int64, _P, _P, _P, _P, C.c_int32]),
]


class NativeLibraryMissing(RuntimeError):
    pass


def _share_hip_runtime_with_torch():
    """PyTorch-ROCm wheels bundle their own libamdhip64/libhsa-runtime64 (same SONAMEs as
    /opt/rocm's).  Two HSA runtimes in one process break GPU discovery for whichever loads second,
    so when torch is importable it is loaded first and libgwo.so binds to the runtime it brought."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load(path: str = LIB_PATH):
    _share_hip_runtime_with_torch()
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} is missing: build it with `make` (or __graft_entry__.build()). "
            "flink_amd has no CPU fallback.")
    lib = C.CDLL(path)
    for name, res, args in SIGNATURES:
        if os.environ.get("GWO_LIB_PATH") and not hasattr(lib, name):
            continue   # an older build under A/B comparison: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


class GwoError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status
        self.status_name = STATUS_NAMES.get(status, str(status))


def check(status: int, handle=None, what: str = ""):
    if status != GWO_OK:
        msg = ""
        if handle is not None:
            raw = lib().gwo_last_error(handle)
            msg = raw.decode() if raw else ""
        raise GwoError(status, f"{what}: {msg}" if what else msg)
