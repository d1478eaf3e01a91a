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


AGG_CODES = {"count": 0, "sum": 1, "min": 2, "max": 3, "avg": 4}


def _run_sw(fn, head, keys, ts, vals, batches, aggs, lateness, threads, max_par, keep_steps):
    k = np.ascontiguousarray(keys, np.int64)
    t = np.ascontiguousarray(ts, np.int64)
    v = None if vals is None else np.ascontiguousarray(vals, np.int64)
    be = np.array([b[0] for b in batches], np.int64)
    bw = np.array([b[1] for b in batches], np.int64)
    nb = len(be)
    ag = np.array([AGG_CODES[a] if isinstance(a, str) else a for a in aggs], np.int32)
    keep = None
    if keep_steps is not None:
        keep = np.zeros(nb + 1, np.uint8)
        keep[list(keep_steps)] = 1
    step_rows = np.zeros(nb + 1, np.int64)
    step_cs = np.zeros(nb + 1, np.uint64)
    buf = C.c_void_p()
    nrows = C.c_int64()
    late = C.c_int64()
    fn.restype = C.c_int
    st = fn(_p(k), _p(t), _p(v), C.c_int64(len(k)), _p(be), _p(bw), C.c_int(nb), *head, C.c_int64(lateness),
            _p(ag), C.c_int(len(ag)), C.c_int(threads), C.c_int32(max_par), _p(keep), _p(step_rows), _p(step_cs),
            C.byref(buf) if keep is not None else None, C.byref(nrows), C.byref(late))
    rows = None
    if keep is not None:
        w = 4 + len(ag)
        rows = np.empty((nrows.value, w), np.int64)
        if nrows.value:
            C.memmove(rows.ctypes.data, buf, nrows.value * w * 8)
        lib().wo_free(buf)
    if st != 0:
        raise RuntimeError("GWO_ERR_MERGE_LATE" if st == 7 else f"window oracle error {st}")
    return rows, step_rows, step_cs, late.value


def run_sliding(keys, ts, vals, batches, size, slide, offset=0, lateness=0, aggs=("avg",), threads=1, max_par=128,
                keep_steps=None):
    """C restatement of WindowOperator over SlidingEventTimeWindows (window_oracle_sw.c).  Returns (rows | None,
    step_rows[nb+1], step_checksum[nb+1] (uint64), late).  rows (kept steps only): key, start, end, result...,
    step -- AVG results as float64 bits."""
    return _run_sw(lib().wo_sliding, (C.c_int64(size), C.c_int64(slide), C.c_int64(offset)), keys, ts, vals, batches,
                   aggs, lateness, threads, max_par, keep_steps)


def run_sessions(keys, ts, vals, batches, gap, lateness=0, aggs=("sum",), threads=1, max_par=128, keep_steps=None):
    """C restatement of WindowOperator over EventTimeSessionWindows + MergingWindowSet (window_oracle_sw.c); same
    returns as run_sliding.  A merge into a late window raises RuntimeError('GWO_ERR_MERGE_LATE')."""
    return _run_sw(lib().wo_sessions, (C.c_int64(gap),), keys, ts, vals, batches, aggs, lateness, threads, max_par,
                   keep_steps)


def rows_checksum(cols) -> int:
    """The checksum window_oracle_sw.c keeps per step: wrapping sum over rows of an FNV-1a hash of the row's words
    (key, start, end, results as int64 bit patterns)."""
    r = [np.ascontiguousarray(c).view(np.uint64) for c in cols]
    if not len(r[0]):
        return 0
    h = np.full(len(r[0]), 1469598103934665603, np.uint64)
    with np.errstate(over="ignore"):
        for c in r:
            h = (h ^ c) * np.uint64(1099511628211)
        return int(h.sum(dtype=np.uint64))
