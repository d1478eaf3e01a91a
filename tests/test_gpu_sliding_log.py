"""GPU parity of the sliding-window log layout: panes logged by K1 + pass 2, the running
total of the last fired window partitioned like the pane logs and advanced by one window step per window
(gwo_slog.hip) -- against the oracle's SlidingEventTimeWindows (SlidingEventTimeWindows.java:68-82,
WindowOperator.java:294-473).  Integer aggregates and the int64 accumulators of AverageAggregate: bit-exact
(the double average is computed from identical (sum, count) words, so it is bit-exact too)."""
import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G
from oracle import vectorized as V

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    return flink_amd


def _stream(n, nkeys, every, lag, disorder, seed, span=60_000):
    spec = G.GenSpec(seed=seed, total_records=n, num_keys=nkeys, span_ms=span, disorder_ms=disorder,
                     value_range=1000)
    k, t, v = G.generate(spec, n)
    return k, t, v, G.punctuated_watermarks(t, every, lag)


def _run(op, k, t, v, batches, start=0, end_input=True):
    prev = start
    for end, wm in batches:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        prev = end
    if end_input:
        op.end_input()
    return prev


def _want(k, s, e, res):
    return sorted(zip(k.tolist(), s.tolist(), e.tolist(), *[x.tolist() for x in res]))


def _got(op):
    return sorted((a, s, e, *(r if isinstance(r, tuple) else (r,))) for a, s, e, r in op.output)


def _final(b):
    return b + [(b[-1][0], LONG_MAX)]


@pytest.mark.parametrize("size,slide,offset", [(60_000, 1_000, 0), (3_000, 1_000, 0), (6_000, 2_000, -1_000),
                                               (5_000, 5_000, 0), (3_000, 1_000, 500)])
def test_sliding_log_avg_bit_exact(F, size, slide, offset):
    k, t, v, b = _stream(150_000, 20_000, 5_000, 500, 900, 5)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(size, slide, offset), F.AverageAggregate(),
                             state_layout="log")
    _run(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), size, slide, offset, [4])
    got = _got(op)
    assert len(got) == len(wk)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


@pytest.mark.parametrize("layout", ["log", "table"])
def test_sliding_log_late_records_late_pass(F, layout):
    """lag 0 with 4.5 s of disorder: many records arrive after the window ending at their pane fired but
    while later windows holding the pane are open (the late pass), many others after every window of
    their pane fired (dropped and counted)."""
    k, t, v, b = _stream(100_000, 3_000, 2_000, 0, 4_500, 9)
    agg = F.MultiAggregate(F.SumAggregate(), F.CountAggregate())
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(4_000, 1_000), agg, state_layout=layout)
    _run(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 4_000, 1_000, 0, [1, 0])
    assert _got(op) == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late > 0
    op.close()


def test_sliding_log_side_output(F):
    k, t, v, b = _stream(60_000, 2_000, 1_500, 0, 4_000, 19)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3_000, 1_000), F.CountAggregate(), state_layout="log",
                             side_output_late_data=True)
    _run(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 3_000, 1_000, 0, [0])
    assert _got(op) == _want(wk, ws, we, res)
    assert len(op.side_output) == late > 0
    assert op.num_late_records_dropped == 0   # side output instead of the counter (WindowOperator.java:420-426)
    op.close()


def test_sliding_log_gap_rebuilds_running_total(F):
    """A hole of many windows in event time: the running total empties, the window steps skip to the next
    pane holding records and rebuild from its window's panes."""
    k1, t1, v1, _ = _stream(20_000, 500, 2_000, 1_000, 1_000, 21)
    k = np.concatenate([k1, k1])
    t = np.concatenate([t1, t1 + 10_000_000])
    v = np.concatenate([v1, v1])
    b = G.punctuated_watermarks(t, 2_000, 1_000)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3_000, 1_000), F.SumAggregate(), state_layout="log")
    _run(op, k, t, v, b)
    (wk, ws, we, res), _ = V.sliding_lateness0(k, t, v, _final(b), 3_000, 1_000, 0, [1])
    assert _got(op) == _want(wk, ws, we, res)
    op.close()


def test_sliding_log_partition_growth_and_lds_rounds(F):
    """No key-count hint: the running total starts at 256 partitions, so 600K keys overflow the LDS table
    (range rounds) until the partitions split (each split doubles them; older panes are read at their own
    coarser partitioning)."""
    k, t, v, b = _stream(1_200_000, 600_000, 100_000, 1_000, 1_000, 23, span=20_000)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(8_000, 1_000), F.AverageAggregate(), state_layout="log")
    _run(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 8_000, 1_000, 0, [4])
    got = _got(op)
    assert len(got) == len(wk) > 1_000_000
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


def test_sliding_log_extreme_keys_and_min_key(F):
    """Long.MIN_VALUE (the LDS table's free marker: held in the side slot) and the int64 extremes."""
    rng = np.random.default_rng(4)
    n = 40_000
    k = rng.choice(np.array([-(1 << 63), (1 << 63) - 1, 0, -1, 1, 12345], dtype=np.int64), n)
    t = np.sort(rng.integers(0, 30_000, n)).astype(np.int64)
    v = rng.integers(-1 << 40, 1 << 40, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 1_000, 200)
    agg = F.MultiAggregate(F.SumAggregate(), F.AverageAggregate())
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(5_000, 1_000), agg, state_layout="log")
    _run(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 5_000, 1_000, 0, [1, 4])
    assert _got(op) == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


@pytest.mark.parametrize("restore_layout", ["log", "table"])
def test_sliding_log_checkpoint_continues_exactly(F, restore_layout):
    """Checkpoint rows are (key, pane, raw words) as the table layout writes them, so a checkpoint of either
    layout restores into the other; the running total is rebuilt from the restored panes."""
    k, t, v, b = _stream(80_000, 5_000, 2_000, 300, 700, 31)
    want, late = None, None
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 6_000, 2_000, 0, [4, 0])
    want = _want(wk, ws, we, res)
    agg = F.MultiAggregate(F.AverageAggregate(), F.CountAggregate())
    mk = lambda layout: F.GpuWindowOperator(F.SlidingEventTimeWindows.of(6_000, 2_000), agg, state_layout=layout)
    for cut in (len(b) // 3, len(b) // 2 + 1):
        a = mk("log")
        prev = _run(a, k, t, v, b[:cut], end_input=False)
        snap = a.snapshot_state()
        rows, late_a = list(a.output), a.num_late_records_dropped
        a.close()
        c = mk(restore_layout)
        c.restore_state(snap)
        _run(c, k, t, v, b[cut:], start=prev)
        assert sorted((x, s, e, *r) for x, s, e, r in rows + list(c.output)) == want
        assert late_a + c.num_late_records_dropped == late
        c.close()
    # and a table-layout checkpoint restored into the log layout
    a = mk("table")
    prev = _run(a, k, t, v, b[:len(b) // 2], end_input=False)
    snap = a.snapshot_state()
    rows = list(a.output)
    a.close()
    c = mk("log")
    c.restore_state(snap)
    _run(c, k, t, v, b[len(b) // 2:], start=prev)
    assert sorted((x, s, e, *r) for x, s, e, r in rows + list(c.output)) == want
    c.close()


def test_sliding_log_matches_loop_oracle_reference_stream(F, golden):
    """The reference's sliding 3 s / 1 s stream (WindowOperatorTest.java:111-184) on the log layout."""
    s = next(x for x in golden["operator_streams"] if x["name"] == "sliding_3s_1s")
    a = s["assigner"]
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(a["size"], a["slide"], a["offset"]), F.SumAggregate(),
                             allowed_lateness=s["lateness"], state_layout="log")
    for ev in s["events"]:
        if ev[0] == "e":
            op.process_element(ev[1], ev[2], ev[3])
        else:
            op.process_watermark(ev[1])
    op.end_input()
    got = sorted(op.output)
    if "expected" in s:
        assert got == sorted(map(tuple, s["expected"]))
    else:
        assert sorted((r[0], r[1], r[3]) for r in got) == sorted(map(tuple, s["expected_key_start_sum"]))
    op.close()


def test_sliding_log_rejected_configurations(F):
    from flink_amd import _native as N
    for kw in [dict(aggregate=F.MinAggregate()),                                   # not invertible
               dict(aggregate=F.SumAggregate(), allowed_lateness=1_000),           # re-fires need the table path
               dict(aggregate=F.AverageAggregate("float64")),                      # float sums are not a group
               dict(aggregate=F.SumAggregate(), size=5_000, slide=2_000)]:         # slide does not divide size
        size, slide = kw.pop("size", 3_000), kw.pop("slide", 1_000)
        with pytest.raises(N.GwoError) as ei:
            F.GpuWindowOperator(F.SlidingEventTimeWindows.of(size, slide), kw.pop("aggregate"), state_layout="log",
                                **kw)
        assert ei.value.status_name == "GWO_ERR_UNSUPPORTED"


def test_sliding_log_sharded_union(F):
    """Four handles, each owning a quarter of the key groups (maxParallelism 128), as four subtasks of one
    job: the union of their rows is the single-operator oracle's."""
    k, t, v, b = _stream(120_000, 30_000, 6_000, 500, 800, 41)
    par = 4
    kg, owner = F.assign_key_groups(k, 128, par)
    rows = []
    for i in range(par):
        lo, hi = (i * 128 + par - 1) // par, ((i + 1) * 128 - 1) // par
        m = owner == i
        ki, ti, vi = k[m], t[m], v[m]
        idx = np.flatnonzero(m)
        bi = [(int(np.searchsorted(idx, e)), wm) for e, wm in b]
        op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(10_000, 1_000), F.SumAggregate(), state_layout="log",
                                 key_group_range=(lo, hi))
        _run(op, ki, ti, vi, bi)
        rows += list(op.output)
        op.close()
    (wk, ws, we, res), _ = V.sliding_lateness0(k, t, v, _final(b), 10_000, 1_000, 0, [1])
    assert sorted(rows) == _want(wk, ws, we, res)


def test_sliding_log_many_small_batches_and_restore_rebuild(F):
    """Batches of 150 records: ~20 segments per pane, so a window step (entering + leaving pane) and the rebuild
    after a restore (every pane of a 20-pane window) take more segments than one launch holds -- chunked steps,
    entering segments first, rows from the last chunk only."""
    k, t, v, _ = _stream(60_000, 2_000, 150, 300, 300, 51, span=20_000)
    b = G.punctuated_watermarks(t, 150, 300)
    agg = F.MultiAggregate(F.SumAggregate(), F.CountAggregate())
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 20_000, 1_000, 0, [1, 0])
    want = _want(wk, ws, we, res)
    mk = lambda: F.GpuWindowOperator(F.SlidingEventTimeWindows.of(20_000, 1_000), agg, state_layout="log")
    op = mk()
    _run(op, k, t, v, b)
    assert _got(op) == want and op.num_late_records_dropped == late
    op.close()
    cut = len(b) // 2
    a = mk()
    prev = _run(a, k, t, v, b[:cut], end_input=False)
    snap = a.snapshot_state()
    rows, late_a = list(a.output), a.num_late_records_dropped
    a.close()
    c = mk()
    c.restore_state(snap)
    _run(c, k, t, v, b[cut:], start=prev)
    assert sorted((x, s, e, *r) for x, s, e, r in rows + list(c.output)) == want
    assert late_a + c.num_late_records_dropped == late
    c.close()


def test_sliding_log_hot_key_pass2_overflow_redo(F):
    """One key holds half of every batch: its partition outgrows pass 2's speculative capacity, so the window step
    queued behind that pass 2 (fire_slog no longer waits for it) reads an incomplete segment -- its rows are
    rewound, the split redone exactly and the step run again.  Same rows as the oracle."""
    k, t, v, b = _stream(400_000, 100_000, 20_000, 500, 900, 41, span=20_000)
    k = k.copy()
    k[::2] = 77   # the hot key
    # a large key-count hint: pass 2 splits every coarse bucket into many partitions (a partition's capacity is a
    # share of its bucket, which the hot key's records exceed)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3_000, 1_000),
                             F.MultiAggregate(F.SumAggregate(), F.CountAggregate()), state_layout="log",
                             expected_keys=4_000_000)
    _run(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 3_000, 1_000, 0, [1, 0])
    assert _got(op) == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()
