"""ctypes driver of oracle/window_oracle.c (the C restatement used as bench.py's cpu_baseline and
for large parity runs) -- TEST INFRASTRUCTURE ONLY."""
import ctypes as C
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libwindow_oracle.so")
_lib = None


def available() -> bool:
    return os.path.exists(LIB)


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(LIB)
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def run_tumbling(keys, ts, vals, batches, size, offset=0, lateness=0, threads=1, max_par=128, rows=True):
    """Returns (rows[n,7] = key, start, end, sum, min, max, count | None, checksum, late)."""
    k = np.ascontiguousarray(keys, np.int64)
    t = np.ascontiguousarray(ts, np.int64)
    v = None if vals is None else np.ascontiguousarray(vals, np.int64)
    be = np.array([b[0] for b in batches], np.int64)
    bw = np.array([b[1] for b in batches], np.int64)
    f = lib().wo_tumbling
    f.restype = C.c_int64
    cs = C.c_uint64()
    late = C.c_int64()
    args = lambda out: (_p(k), _p(t), _p(v), C.c_int64(len(k)), _p(be), _p(bw), C.c_int(len(be)), C.c_int64(size),
                        C.c_int64(offset), C.c_int64(lateness), C.c_int(threads), C.c_int32(max_par), out,
                        C.byref(cs), C.byref(late))
    if not rows:
        f(*args(None))
        return None, cs.value, late.value
    g = lib().wo_tumbling_rows
    g.restype = C.c_int64
    buf = C.c_void_p()
    n = g(_p(k), _p(t), _p(v), C.c_int64(len(k)), _p(be), _p(bw), C.c_int(len(be)), C.c_int64(size),
          C.c_int64(offset), C.c_int64(lateness), C.c_int(threads), C.c_int32(max_par), C.byref(buf),
          C.byref(cs), C.byref(late))
    out = np.empty((n, 7), np.int64)
    if n:
        C.memmove(out.ctypes.data, buf, n * 7 * 8)
    lib().wo_free(buf)
    return out, cs.value, late.value


def time_tumbling(keys, ts, vals, batches, size, threads):
    t0 = time.perf_counter()
    run_tumbling(keys, ts, vals, batches, size, threads=threads, rows=False)
    return time.perf_counter() - t0


def row_checksum(rows) -> int:
    """The C twin's order-independent output checksum (window_oracle.c emit()): the wrapping sum over
    rows of an FNV-1a-style hash of the row's 7 words (key, start, end, sum, min, max, count)."""
    r = np.ascontiguousarray(rows, np.int64).view(np.uint64)
    h = np.full(r.shape[0], 1469598103934665603, np.uint64)
    with np.errstate(over="ignore"):
        for c in range(r.shape[1]):
            h = (h ^ r[:, c]) * np.uint64(1099511628211)
        return int(h.sum(dtype=np.uint64))
