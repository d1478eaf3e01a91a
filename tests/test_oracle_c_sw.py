"""CPU: pin the C restatement of WindowOperator for SLIDING and SESSION windows (oracle/window_oracle_sw.c, the
checker of the full-size C3 and C5 GPU parity tests) against the record-at-a-time Python oracle
(oracle/flink_oracle.py, pinned by the reference's golden vectors in test_oracle.py).

Compared per watermark step: the rows a step emits (the batch's per-element re-fires and the timers its
watermark fires), their per-step checksum, and numLateRecordsDropped -- random streams with lateness 0 and > 0,
several thread counts and maxParallelism 128 / 32768, negative timestamps and offsets, sessions with heavy
disorder (merges, bridging records, late drops, re-fires)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import cbaseline
from oracle import flink_oracle as O
from oracle import gen as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LONG_MAX = (1 << 63) - 1


@pytest.fixture(scope="module", autouse=True)
def c_oracle():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    assert cbaseline.available()


def _agg(names):
    m = {"sum": O.SumLongAgg, "count": O.CountAgg, "min": O.MinAgg, "max": O.MaxAgg, "avg": O.AvgAgg}
    return O.MultiAgg([m[n]() for n in names])


def _loop(assigner, names, lateness, keys, ts, vals, batches):
    """Loop oracle; rows tagged with the batch whose records or watermark emitted them."""
    op = O.WindowOperatorOracle(assigner, _agg(names), lateness)
    prev, rows = 0, []
    for b, (end, wm) in enumerate(batches):
        for i in range(prev, end):
            op.process_element(int(keys[i]), int(ts[i]), int(vals[i]))
        op.process_watermark(wm)
        prev = end
        rows += [(r.key, r.start, r.end, *_bits(r.result), b) for r in op.output]
        op.output.clear()
    return sorted(rows), op.num_late_records_dropped


def _bits(res):
    return tuple(int(np.float64(x).view(np.int64)) if isinstance(x, float) else int(x) for x in res)


def _stream(seed, n, nkeys, span, disorder, every, lag, neg=False):
    rng = np.random.default_rng(seed)
    keys = rng.integers(-nkeys, nkeys, n).astype(np.int64)
    ts = (np.sort(rng.integers(0, span, n)) + rng.integers(0, disorder, n)).astype(np.int64)
    if neg:
        ts -= span // 2
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    return keys, ts, vals, G.punctuated_watermarks(ts, every, lag) + [(n, LONG_MAX)]


def _check(kind, params, names, lateness, keys, ts, vals, batches, threads, maxp):
    if kind == "sliding":
        size, slide, off = params
        assigner = O.SlidingEventTimeWindows(size, slide, off)
        rows, srows, scs, late = cbaseline.run_sliding(keys, ts, vals, batches, size, slide, off, lateness, names,
                                                       threads, maxp, keep_steps=range(len(batches) + 1))
    else:
        assigner = O.EventTimeSessionWindows(params)
        rows, srows, scs, late = cbaseline.run_sessions(keys, ts, vals, batches, params, lateness, names, threads,
                                                        maxp, keep_steps=range(len(batches) + 1))
    want, want_late = _loop(assigner, names, lateness, keys, ts, vals, batches)
    got = sorted(map(tuple, rows.tolist()))
    assert got == want
    assert late == want_late
    # per-step counts and checksums agree with the kept rows
    for b in range(len(batches) + 1):
        sel = rows[rows[:, -1] == b]
        assert srows[b] == len(sel)
        assert int(scs[b]) == cbaseline.rows_checksum([sel[:, c] for c in range(sel.shape[1] - 1)])
    return want


@pytest.mark.parametrize("lateness", [0, 700, 2500])
@pytest.mark.parametrize("threads,maxp", [(1, 128), (4, 32768)])
@pytest.mark.parametrize("params", [(3000, 1000, 0), (4000, 1500, 300), (2000, 2000, 0)])
def test_sliding_c_twin_matches_loop_oracle(lateness, threads, maxp, params):
    keys, ts, vals, batches = _stream(lateness + threads + params[1], 3000, 40, 20000, 2500, 97, 300)
    want = _check("sliding", params, ["sum", "count", "min", "max"], lateness, keys, ts, vals, batches, threads, maxp)
    assert len(want) > 500


@pytest.mark.parametrize("lateness", [0, 1500])
def test_sliding_c_twin_avg_negative_time_and_offset(lateness):
    keys, ts, vals, batches = _stream(31 + lateness, 3000, 30, 30000, 3000, 113, 500, neg=True)
    _check("sliding", (5000, 1000, -300), ["avg"], lateness, keys, ts, vals, batches, 3, 128)


@pytest.mark.parametrize("lateness", [0, 900, 5000])
@pytest.mark.parametrize("threads,maxp", [(1, 128), (5, 32768)])
def test_sessions_c_twin_matches_loop_oracle(lateness, threads, maxp):
    keys, ts, vals, batches = _stream(lateness + threads, 4000, 50, 200_000, 6000, 131, 800)
    want = _check("sessions", 2000, ["sum", "count", "max"], lateness, keys, ts, vals, batches, threads, maxp)
    assert len(want) > 500


def test_sessions_c_twin_generated_c5_shape():
    """The C5 generator's shape (bursty sessions, 0.5 % of events delayed beyond the lag) at a small size."""
    k, t, v, _ = G.session_stream(300, 20_000, late_fraction=0.005, seed=3, late_extra=30_000)
    b = G.punctuated_watermarks(t, 200, 5_000) + [(len(k), LONG_MAX)]
    _check("sessions", 30_000, ["sum", "count", "min", "max"], 0, k, t, v, b, 4, 128)


def test_sessions_c_twin_late_window_retired_and_merge_refire():
    """A late record's own session window is retired and the record counted (WindowOperator.java:358-362,420-426);
    a record merging into a fired-but-kept session re-fires the merged window (EventTimeTrigger.onElement).  (The
    late-merge UnsupportedOperationException of :318-323 cannot arise from a stream: every in-flight member's
    cleanup time exceeds the watermark, and the merge result ends no earlier.)"""
    keys = np.array([1, 1, 1], np.int64)
    vals = np.array([1, 2, 3], np.int64)
    # [0, 1000) and [5000, 6000), lateness 500, watermark 6000: the first is fired and cleaned, the second fired and
    # kept until 6499; a record at 2000 makes [2000, 3000), already late: retired, the record dropped
    rows, _, _, late = cbaseline.run_sessions(keys, np.array([0, 5000, 2000]), vals, [(2, 6000), (3, LONG_MAX)], 1000,
                                              500, ["sum"], 1, 128, keep_steps=[0, 1, 2])
    assert late == 1 and sorted(r[:4] for r in rows.tolist()) == [[1, 0, 1000, 1], [1, 5000, 6000, 2]]
    # a record at 4500 merges into [5000, 6000): [4500, 6000) is re-fired on the element with the merged sum
    rows, _, _, late = cbaseline.run_sessions(keys, np.array([0, 5000, 4500]), vals, [(2, 6000), (3, LONG_MAX)], 1000,
                                              500, ["sum"], 1, 128, keep_steps=[0, 1, 2])
    assert late == 0 and [1, 4500, 6000, 5, 1] in rows.tolist()
