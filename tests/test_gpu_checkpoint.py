"""GPU checkpoint / restore of the keyed window state (gwo.h gwo_snapshot / gwo_restore) for every assigner and
state layout, checked against the oracle:

* the reference's own snapshot points (WindowOperatorTest.java:150-160, 266-276, 396-404, 543-551: snapshot,
  close, initializeState into a fresh operator, continue) replayed on the golden streams;
* continue-after-restore on random streams for the log layout (the C4 default), sessions and tumbling tables;
* rescaling by key-group range (HeapRestoreOperation reads only the subtask's key groups), including subtasks
  checkpointed at different watermarks;
* the checkpoint format: rows grouped by key group with KeyGroupRangeAssignment's key groups, the fire-timer
  flag per row, and validation that leaves a handle untouched.
Integer aggregates: bit-exact.
"""
import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G

pytestmark = pytest.mark.gpu

LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    return flink_amd


def _assigner(F, a):
    if a["kind"] == "tumbling":
        return F.TumblingEventTimeWindows.of(a["size"], a["offset"])
    if a["kind"] == "sliding":
        return F.SlidingEventTimeWindows.of(a["size"], a["slide"], a["offset"])
    return F.EventTimeSessionWindows.withGap(a["gap"])


def _feed(op, events):
    for ev in events:
        if ev[0] == "e":
            op.process_element(ev[1], ev[2], ev[3])
        else:
            op.process_watermark(ev[1])


@pytest.mark.parametrize("name,layout", [("tumbling_3s", "table"), ("tumbling_3s", "log"), ("sliding_3s_1s", "auto"),
                                         ("session_list_3s", "auto"), ("session_reduce_3s", "auto")])
def test_reference_snapshot_points(F, golden, name, layout):
    """WindowOperatorTest snapshots mid-stream, closes the operator and continues in a restored one; the
    combined output is the test's expected output."""
    s = next(x for x in golden["operator_streams"] if x["name"] == name)
    cut = s["snapshot_after"] + 1
    mk = lambda: F.GpuWindowOperator(_assigner(F, s["assigner"]), F.SumAggregate(), allowed_lateness=s["lateness"],
                                     side_output_late_data=s["side_output"], state_layout=layout)
    a = mk()
    _feed(a, s["events"][:cut])
    snap = a.snapshot_state()
    before = list(a.output)
    a.close()
    b = mk()
    b.restore_state(snap)
    _feed(b, s["events"][cut:])
    b.end_input()
    got = sorted(before + list(b.output))
    if "expected" in s:
        assert got == sorted(map(tuple, s["expected"]))
    else:
        assert sorted((r[0], r[1], r[3]) for r in got) == sorted(map(tuple, s["expected_key_start_sum"]))
    b.close()


def _oracle_rows(assigner, agg, k, t, v, batches, lateness=0):
    op = O.WindowOperatorOracle(assigner, agg, lateness)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(k[i]), int(t[i]), int(v[i]))
        op.process_watermark(wm)
        prev = end
    op.process_watermark(LONG_MAX)
    return sorted((r.key, r.start, r.end, r.result) for r in op.output), op.num_late_records_dropped


def _run(op, k, t, v, batches, start=0):
    prev = start
    for end, wm in batches:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        prev = end
    return prev


@pytest.mark.parametrize("aggs", ["sum_min_max", "avg_count"])
def test_log_layout_checkpoint_continues_exactly(F, aggs):
    """The C4 layout: windows still collecting records are folded (not released) into rows; the restored
    operator folds them back in at the windows' fire together with the records that arrive later.  avg_count:
    raw accumulator words differ from the results (avg keeps (sum, count)), so the fold must emit raw words."""
    rng = np.random.default_rng(5)
    n = 60_000
    k = rng.integers(0, 20_000, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 120_000, n)) + rng.integers(0, 3_000, n)).astype(np.int64)
    v = rng.integers(-500, 500, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 1_500, 1_000)
    if aggs == "sum_min_max":
        oagg = O.MultiAgg([O.SumLongAgg(), O.MinAgg(), O.MaxAgg()])
        agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    else:
        oagg = O.MultiAgg([O.AvgAgg(), O.CountAgg()])
        agg = F.MultiAggregate(F.AverageAggregate(), F.CountAggregate())
    want, late = _oracle_rows(O.TumblingEventTimeWindows(10_000), oagg, k, t, v, b)
    mk = lambda layout: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(10_000), agg, state_layout=layout,
                                            max_parallelism=32768)
    for cut in (len(b) // 3, len(b) // 2 + 3):
        for restore_layout in ("log", "table"):
            a = mk("log")
            prev = _run(a, k, t, v, b[:cut])
            snap = a.snapshot_state()
            assert len(snap["key"]) > 0 and (snap["timer"] == 1).all()
            assert (np.diff(snap["key_group"]) >= 0).all()
            rows, late_a = list(a.output), a.num_late_records_dropped
            a.close()
            c = mk(restore_layout)
            c.restore_state(snap)
            _run(c, k, t, v, b[cut:], start=prev)
            c.end_input()
            assert sorted(rows + list(c.output)) == want
            assert late_a + c.num_late_records_dropped == late
            c.close()


@pytest.mark.parametrize("lateness", [0, 4_000])
def test_session_checkpoint_continues_exactly(F, lateness):
    """Sessions: every in-flight session of every key is a row (merged window, accumulator, pending timer);
    after restore, later records still merge into the restored sessions."""
    k, t, v, _ = G.session_stream(300, 20_000, gap=3_000, lag=1_000, seed=3 + lateness, mean_inner=800,
                                  late_fraction=0.01)
    b = G.punctuated_watermarks(t, 500, 1_000)
    want, late = _oracle_rows(O.EventTimeSessionWindows(3_000), O.SumLongAgg(), k, t, v, b, lateness)
    mk = lambda: F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(3_000), F.SumAggregate(),
                                     allowed_lateness=lateness)
    cut = len(b) // 2
    a = mk()
    prev = _run(a, k, t, v, b[:cut])
    snap = a.snapshot_state()
    assert len(snap["key"]) == a.state_size() > 0
    rows, late_a = list(a.output), a.num_late_records_dropped
    a.close()
    c = mk()
    c.restore_state(snap)
    assert c.state_size() == len(snap["key"])
    _run(c, k, t, v, b[cut:], start=prev)
    c.end_input()
    assert sorted(rows + list(c.output)) == want
    assert late_a + c.num_late_records_dropped == late
    c.close()


def test_checkpoint_rows_are_key_group_ordered(F):
    rng = np.random.default_rng(2)
    k = rng.integers(-(1 << 40), 1 << 40, 5_000).astype(np.int64)
    t = rng.integers(0, 20_000, 5_000).astype(np.int64)
    v = rng.integers(0, 9, 5_000).astype(np.int64)
    for layout in ("table", "log"):
        op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5_000), F.SumAggregate(), state_layout=layout,
                                 max_parallelism=1000)
        op.process_batch(k, t, v)
        snap = op.snapshot_state()
        kg, _ = F.assign_key_groups(snap["key"], 1000)
        assert (snap["key_group"] == kg).all() and (np.diff(kg) >= 0).all()
        assert sorted(zip(snap["key"].tolist(), snap["window_start"].tolist())) == \
            sorted(set(zip(k.tolist(), (t - t % 5_000).tolist())))
        assert (snap["window_end"] - snap["window_start"] == 5_000).all()
        op.close()


def _rescale(F, mk, snaps, nnew, maxp, k, t, v, batches, start):
    """Restore every old subtask's snapshot into nnew subtasks and feed each its keys' records."""
    kg, _ = F.assign_key_groups(k, maxp)
    rows, late = [], 0
    for idx in range(nnew):
        r = F.compute_key_group_range_for_operator_index(maxp, nnew, idx)
        op = mk((r.start_key_group, r.end_key_group))
        op.restore_state(snaps)
        mine = (kg >= r.start_key_group) & (kg <= r.end_key_group)
        p0 = start
        for end, wm in batches:
            sel = np.nonzero(mine[p0:end])[0] + p0
            op.process_batch(k[sel], t[sel], v[sel])
            op.process_watermark(wm)
            p0 = end
        op.end_input()
        rows += list(op.output)
        late += op.num_late_records_dropped
        op.close()
    return rows, late


@pytest.mark.parametrize("layout", ["table", "log"])
def test_rescale_two_to_three_with_unequal_watermarks(F, layout):
    """Two subtasks checkpoint at different watermarks: subtask 1 has already seen a later watermark (one no later
    record is behind, so nothing becomes late) and emitted a window subtask 0 still holds; with allowedLateness 0
    that window's state is gone from subtask 1's checkpoint.  Three restored subtasks continue from the minimum
    watermark; the union of all rows equals the single-operator oracle."""
    rng = np.random.default_rng(11)
    n, maxp, size = 40_000, 128, 4_000
    k = rng.integers(0, 3_000, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 150_000, n)) + rng.integers(0, 2_000, n)).astype(np.int64)
    v = rng.integers(0, 100, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 1_000, 2_500)
    want, _ = _oracle_rows(O.TumblingEventTimeWindows(size), O.SumLongAgg(), k, t, v, b)
    for cut in range(len(b) // 2, len(b) - 2):   # a checkpoint point where a window end lies between the watermarks
        prev, wm0 = b[cut - 1]
        wm1 = int(t[prev:].min()) - 1
        first_end = (wm0 + 2) + ((-(wm0 + 2)) % size)
        if first_end - 1 <= wm1:
            break
    else:
        pytest.fail("no checkpoint point with a window end between the subtasks' watermarks")
    mk = lambda rng_: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(size), F.SumAggregate(), state_layout=layout,
                                          max_parallelism=maxp, key_group_range=rng_)
    kg, _ = F.assign_key_groups(k, maxp)
    snaps, rows = [], []
    for idx in range(2):
        r = F.compute_key_group_range_for_operator_index(maxp, 2, idx)
        op = mk((r.start_key_group, r.end_key_group))
        mine = (kg >= r.start_key_group) & (kg <= r.end_key_group)
        p0 = 0
        for end, wm in b[:cut]:
            sel = np.nonzero(mine[p0:end])[0] + p0
            op.process_batch(k[sel], t[sel], v[sel])
            op.process_watermark(wm)
            p0 = end
        if idx == 1:
            op.process_watermark(wm1)
        snaps.append(op.snapshot_state())
        rows += list(op.output)
        op.close()
    assert snaps[0]["watermark"] == wm0 < wm1 == snaps[1]["watermark"]
    assert any(r[2] == first_end for r in rows)   # subtask 1 emitted the straddled window before the checkpoint
    more, _ = _rescale(F, mk, snaps, 3, maxp, k, t, v, b[cut:], prev)
    assert sorted(rows + more) == want


def test_restore_mixed_timers_and_rejects_mismatched_checkpoints(F):
    """A tumbling window emitted by one subtask but still pending in another (allowedLateness > 0, unequal
    watermarks) restores per key as the reference's timers are per (key, window): the pending key fires at the
    window's maxTimestamp, the emitted keys only re-fire on late records.  Rows with another aggregate layout
    (n_words) are rejected, and a rejected restore leaves the handle fresh: a valid restore afterwards succeeds."""
    from flink_amd import _native as N
    mk = lambda rng_=None, agg=None: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1_000), agg or F.SumAggregate(),
                                                         allowed_lateness=5_000, state_layout="table",
                                                         key_group_range=rng_)
    a = mk()
    a.process_batch(np.array([1, 2]), np.array([100, 200]), np.array([1, 1]))
    a.process_watermark(999)    # window [0, 1000) emitted, kept for late re-fires
    s1 = a.snapshot_state()
    assert (s1["timer"] == 0).all()
    a.close()
    b = mk()
    b.process_batch(np.array([3]), np.array([300]), np.array([1]))
    b.process_watermark(500)    # the same window, still pending
    s2 = b.snapshot_state()
    assert (s2["timer"] == 1).all()
    b.close()
    m = mk()
    m.restore_state([s1, s2])    # at the minimum watermark, 500
    assert m.current_watermark == 500 and m.state_size() == 3
    m.process_watermark(999)
    assert m.output == [(3, 0, 1000, 1)]             # only the pending key's timer fires
    m.process_batch(np.array([1]), np.array([150]), np.array([5]))   # late but allowed: re-fires with the sum
    m.process_watermark(1_000)
    assert m.output == [(3, 0, 1000, 1), (1, 0, 1000, 6)]
    m.close()
    c = mk()
    bad = dict(s1, words=np.zeros((len(s1["key"]), 2), np.int64))
    with pytest.raises(N.GwoError) as e:
        c.restore_state(bad)
    assert e.value.status == N.GWO_ERR_INVALID_ARGUMENT
    c.restore_state(s1)          # still fresh: the valid checkpoint restores
    assert c.state_size() == 2 and c.current_watermark == 999
    c.process_batch(np.array([1]), np.array([150]), np.array([5]))   # late but allowed: re-fires with the sum
    c.process_watermark(1_000)
    assert c.output == [(1, 0, 1000, 6)]
    c.close()


def test_sliding_rescale_straddling_watermarks_rejected(F):
    from flink_amd import _native as N
    mk = lambda: F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3_000, 1_000), F.SumAggregate())
    a, b = mk(), mk()
    a.process_batch(np.array([1]), np.array([500]), np.array([1]))
    b.process_batch(np.array([2]), np.array([500]), np.array([1]))
    a.process_watermark(100)
    b.process_watermark(1_500)   # b emitted window [-2000, 1000), a did not
    sa, sb = a.snapshot_state(), b.snapshot_state()
    a.close()
    b.close()
    c = mk()
    with pytest.raises(N.GwoError):
        c.restore_state([sa, sb])
    c.close()


def test_restored_emitted_key_with_new_records_is_one_entry(F):
    """A tumbling window restored with emitted entries (allowedLateness > 0, restored below maxTimestamp) whose key
    then gets a new record holds that key in two device tables (the pending new records, the restored emitted entry).
    The reference keeps ONE heap entry per (key, window) (CopyOnWriteStateMapSnapshot.java:127-129) -- its accumulator
    the combination, its fire timer pending again (WindowOperator.java:393-410) -- so the snapshot rows, the state size
    and the heap export all show one entry, and a restore of that snapshot fires the combined row."""
    mk = lambda: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1_000),
                                     F.MultiAggregate(F.SumAggregate(), F.MaxAggregate()), allowed_lateness=5_000,
                                     state_layout="table")
    a = mk()
    a.process_batch(np.array([1, 2]), np.array([100, 200]), np.array([1, 4]))
    a.process_watermark(999)    # [0, 1000) emitted (1: 1, 2: 4), kept for late re-fires
    s1 = a.snapshot_state()
    a.close()
    b = mk()
    b.process_batch(np.array([3]), np.array([300]), np.array([7]))
    b.process_watermark(500)    # the same window, pending in this subtask
    s2 = b.snapshot_state()
    b.close()
    m = mk()
    m.restore_state([s1, s2])   # watermark 500: keys 1, 2 emitted, key 3 pending
    m.process_batch(np.array([1]), np.array([150]), np.array([5]))   # key 1 again before maxTimestamp
    assert m.state_size() == 3
    snap = m.snapshot_state()
    rows = sorted(zip(snap["key"].tolist(), snap["window_start"].tolist(), snap["timer"].tolist()))
    assert rows == [(1, 0, 1), (2, 0, 0), (3, 0, 1)]
    w1 = snap["words"][snap["key"].tolist().index(1)]
    assert 6 in w1.tolist() and 5 in w1.tolist()     # sum 1 + 5, max(1, 5): the two entries combined
    # the merged snapshot restores to the same behaviour: key 1 fires with the combined accumulator
    r = mk()
    r.restore_state(snap)
    r.process_watermark(999)
    assert sorted(r.output) == [(1, 0, 1000, (6, 5)), (3, 0, 1000, (7, 7))]
    m.process_watermark(999)
    assert sorted(m.output) == [(1, 0, 1000, (6, 5)), (3, 0, 1000, (7, 7))]
    m.close()
    r.close()
