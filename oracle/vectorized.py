"""Vectorised (numpy) restatement of WindowOperator for tumbling/sliding windows with
allowedLateness = 0 -- TEST INFRASTRUCTURE ONLY.

For lateness 0 the reference's per-record loop (SJ/runtime/operators/windowing/WindowOperator.java:
386-427) reduces to set algebra:
  * a record is added to window W iff W.maxTimestamp() > wm, the watermark in effect when the record
    arrives (isWindowLate, :578-580; cleanupTime == maxTs for lateness 0, :639-646);
  * it counts in numLateRecordsDropped iff it reaches no window and ts <= wm (isElementLate, :588-591);
  * W fires exactly once, with every record it accepted, when a watermark >= W.maxTimestamp()
    arrives (EventTimeTrigger.java:37-52), and is cleared at the same timer.
So the output is a group-by over accepted (key, window) pairs of windows whose maxTimestamp is <= the
final watermark.  tests/test_oracle.py pins this restatement against the record-at-a-time oracle
(oracle/flink_oracle.py) on randomized streams.
"""
from __future__ import annotations

import numpy as np

LONG_MIN = -(1 << 63)
AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG = 0, 1, 2, 3, 4


def java_window_start(ts, offset, size):
    """TimeWindow.getWindowStartWithOffset with Java's truncating '%' (np.fmod on integers)."""
    with np.errstate(over="ignore"):
        return ts - np.fmod(ts - offset + size, size)


def wm_per_record(n, batches):
    """batches: [(end_index, watermark)], records [prev_end, end) see the previous watermark."""
    wm = np.full(n, LONG_MIN, dtype=np.int64)
    prev_end, prev_wm = 0, LONG_MIN
    for end, w in batches:
        wm[prev_end:end] = prev_wm
        prev_end, prev_wm = end, w
    wm[prev_end:] = prev_wm
    return wm, prev_wm


def _order_key(x):
    bits = x.view(np.int64).copy()
    nan = np.isnan(x)
    bits[nan] = 0x7FF8000000000000
    neg = bits < 0
    bits[neg] ^= 0x7FFFFFFFFFFFFFFF
    return bits


def _from_order_key(k):
    b = k.copy()
    neg = b < 0
    b[neg] ^= 0x7FFFFFFFFFFFFFFF
    return b.view(np.float64)


def group_aggregate(keys, starts, vals, kinds, value_is_f64):
    """Group rows by (key, start); returns sorted unique (key, start) and one result array per agg."""
    if len(keys) == 0:
        return np.empty(0, np.int64), np.empty(0, np.int64), [np.empty(0) for _ in kinds]
    order = np.lexsort((keys, starts))
    k, s = keys[order], starts[order]
    v = vals[order] if vals is not None else None
    brk = np.ones(len(k), dtype=bool)
    brk[1:] = (k[1:] != k[:-1]) | (s[1:] != s[:-1])
    idx = np.flatnonzero(brk)
    counts = np.diff(np.append(idx, len(k)))
    res = []
    with np.errstate(over="ignore"):
        for kind in kinds:
            if kind == AGG_COUNT:
                res.append(counts.astype(np.int64))
            elif kind == AGG_SUM:
                res.append(np.add.reduceat(v, idx))
            elif kind in (AGG_MIN, AGG_MAX):
                f = np.minimum if kind == AGG_MIN else np.maximum
                if value_is_f64:
                    res.append(_from_order_key(f.reduceat(_order_key(v), idx)))
                else:
                    res.append(f.reduceat(v, idx))
            elif kind == AGG_AVG:
                sm = np.add.reduceat(v, idx)
                res.append(sm.astype(np.float64) / counts.astype(np.float64))
            else:
                raise ValueError(kind)
    return k[idx], s[idx], res


def tumbling_lateness0(keys, ts, vals, batches, size, offset, kinds, value_is_f64=False):
    """Returns ((key, start, end, results...) arrays, late_count)."""
    n = len(keys)
    wm, final_wm = wm_per_record(n, batches)
    off = int(np.fmod(offset, size))
    start = java_window_start(ts, off, size)
    with np.errstate(over="ignore"):
        max_ts = start + size - 1
    accepted = max_ts > wm
    late = int(np.count_nonzero(~accepted & (ts <= wm)))
    fired = accepted & (max_ts <= final_wm)
    k, s, res = group_aggregate(keys[fired], start[fired], vals[fired] if vals is not None else None, kinds,
                                value_is_f64)
    return (k, s, s + size, res), late


def sliding_lateness0(keys, ts, vals, batches, size, slide, offset, kinds, value_is_f64=False):
    n = len(keys)
    wm, final_wm = wm_per_record(n, batches)
    last = java_window_start(ts, offset, slide)
    nwin = -(-size // slide) + 1
    ks, ss, vs = [], [], []
    any_acc = np.zeros(n, dtype=bool)
    for j in range(nwin):
        st = last - j * slide
        inw = st > ts - size
        acc = inw & (st + size - 1 > wm)
        any_acc |= acc
        fired = acc & (st + size - 1 <= final_wm)
        ks.append(keys[fired])
        ss.append(st[fired])
        if vals is not None:
            vs.append(vals[fired])
    late = int(np.count_nonzero(~any_acc & (ts <= wm)))
    k = np.concatenate(ks)
    s = np.concatenate(ss)
    v = np.concatenate(vs) if vals is not None else None
    k, s, res = group_aggregate(k, s, v, kinds, value_is_f64)
    return (k, s, s + size, res), late


def key_groups(keys, max_parallelism, parallelism=1):
    """numpy restatement of ``KeyGroupRangeAssignment.assignToKeyGroup`` for Long keys
    (``Long.hashCode`` -> ``MathUtils.murmurHash`` -> ``% maxParallelism``,
    RT/state/KeyGroupRangeAssignment.java:60-73, CO/util/MathUtils.java:134-198) and
    ``computeOperatorIndexForKeyGroup`` (:118-119).  Returns (key_group, operator_index)."""
    k = np.asarray(keys, dtype=np.int64).view(np.uint64)
    h = ((k ^ (k >> np.uint64(32))) & np.uint64(0xFFFFFFFF)).astype(np.uint32)

    def rotl(x, r):
        return (x << np.uint32(r)) | (x >> np.uint32(32 - r))

    with np.errstate(over="ignore"):
        c = h * np.uint32(0xCC9E2D51)
        c = rotl(c, 15)
        c = c * np.uint32(0x1B873593)
        c = rotl(c, 13)
        c = c * np.uint32(5) + np.uint32(0xE6546B64)
        c = c ^ np.uint32(4)
        c ^= c >> np.uint32(16)
        c = c * np.uint32(0x85EBCA6B)
        c ^= c >> np.uint32(13)
        c = c * np.uint32(0xC2B2AE35)
        c ^= c >> np.uint32(16)
    s = c.view(np.int32).astype(np.int64)
    s = np.where(s >= 0, s, np.where(s == -(1 << 31), 0, -s))
    kg = s % max_parallelism
    return kg, kg * parallelism // max_parallelism
