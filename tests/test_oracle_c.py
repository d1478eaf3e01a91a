"""CPU: pin the C restatement of WindowOperator (oracle/window_oracle.c, driven by oracle/cbaseline.py)
against the record-at-a-time Python oracle (oracle/flink_oracle.py, itself pinned by the reference's
golden vectors in test_oracle.py).  The C twin is what the full-scale GPU parity test
(tests/test_gpu_fullscale.py) and bench.py's cpu_baseline run, so it must agree row for row --
including per-element re-fires with allowedLateness > 0 (EventTimeTrigger.java:37-45,
WindowOperator.java:393-406), numLateRecordsDropped (:420-426) and the key-group sharding of its
threads (KeyGroupRangeAssignment.java:60-73,118-119) at maxParallelism 128 and 32768."""
import os
import subprocess

import numpy as np
import pytest

from oracle import cbaseline
from oracle import flink_oracle as O
from oracle import gen as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def c_oracle():
    if not cbaseline.available():
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    assert cbaseline.available()


def _stream(seed, n, nkeys, span, disorder, every, lag, extreme=False):
    rng = np.random.default_rng(seed)
    keys = rng.integers(-nkeys, nkeys, n).astype(np.int64)
    if extreme:   # Long.MIN/MAX keys and values: wrap-around sums, sign of Long.hashCode
        keys[::97] = np.iinfo(np.int64).min
        keys[5::89] = np.iinfo(np.int64).max
    ts = np.sort(rng.integers(0, span, n)) + rng.integers(0, disorder, n)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    if extreme:
        vals[::53] = np.iinfo(np.int64).max
        vals[7::61] = np.iinfo(np.int64).min
    batches = G.punctuated_watermarks(ts, every, lag)
    return keys, ts.astype(np.int64), vals, batches


def _loop_rows(keys, ts, vals, batches, size, offset, lateness):
    op = O.WindowOperatorOracle(O.TumblingEventTimeWindows(size, offset),
                                O.MultiAgg([O.SumLongAgg(), O.MinAgg(), O.MaxAgg(), O.CountAgg()]), lateness)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(keys[i]), int(ts[i]), int(vals[i]))
        op.process_watermark(wm)
        prev = end
    rows = sorted((r.key, r.start, r.end, *r.result) for r in op.output)
    return rows, op.num_late_records_dropped


def _c_rows(keys, ts, vals, batches, size, offset, lateness, threads, maxp):
    rows, cs, late = cbaseline.run_tumbling(keys, ts, vals, batches, size, offset=offset, lateness=lateness,
                                            threads=threads, max_par=maxp)
    return sorted(map(tuple, rows.tolist())), cs, late


@pytest.mark.parametrize("lateness", [0, 400, 2500])
@pytest.mark.parametrize("threads,maxp", [(1, 128), (3, 128), (4, 32768), (8, 32768)])
def test_c_twin_matches_loop_oracle(lateness, threads, maxp):
    keys, ts, vals, batches = _stream(lateness * 7 + threads, 5000, 60, 24000, 1800, 113, 300)
    want, want_late = _loop_rows(keys, ts, vals, batches, 1000, 100, lateness)
    got, _, late = _c_rows(keys, ts, vals, batches, 1000, 100, lateness, threads, maxp)
    assert got == want
    assert late == want_late


@pytest.mark.parametrize("lateness", [0, 3000])
def test_c_twin_extremes_and_negative_offset(lateness):
    keys, ts, vals, batches = _stream(11 + lateness, 4000, 30, 30000, 4000, 71, 1000, extreme=True)
    ts = ts - 15000   # negative timestamps: Java '%' path of getWindowStartWithOffset
    batches = [(e, w - 15000) for e, w in batches]
    want, want_late = _loop_rows(keys, ts, vals, batches, 3000, -700, lateness)
    got, _, late = _c_rows(keys, ts, vals, batches, 3000, -700, lateness, 4, 32768)
    assert got == want
    assert late == want_late


def test_c_twin_checksum_is_order_independent_and_thread_invariant():
    keys, ts, vals, batches = _stream(5, 20000, 500, 60000, 2000, 500, 500)
    base = None
    for threads, maxp in [(1, 128), (2, 128), (16, 32768), (7, 32768)]:
        rows, cs, late = cbaseline.run_tumbling(keys, ts, vals, batches, 5000, threads=threads, max_par=maxp)
        assert cbaseline.row_checksum(rows) == cs
        cur = (len(rows), cs, late)
        assert base is None or cur == base
        base = cur


def test_c_twin_final_watermark_fires_everything():
    # a stream ended with processWatermark(Long.MAX_VALUE) (StreamSource.java:122) fires every window
    keys, ts, vals, batches = _stream(9, 3000, 40, 20000, 500, 300, 600)
    batches = batches + [(len(keys), np.iinfo(np.int64).max)]
    want, _ = _loop_rows(keys, ts, vals, batches, 2000, 0, 0)
    got, _, _ = _c_rows(keys, ts, vals, batches, 2000, 0, 0, 4, 32768)
    assert got == want
    assert sum(r[6] for r in got) == len(keys)   # no record lost: every record is in exactly one row
