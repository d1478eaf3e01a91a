"""GPU checkpoint interoperability with the heap state backend (gwo.h gwo_export_heap_state / gwo_import_heap_state).

* The reference's own savepoints (tests/golden/heap_state/, WindowOperatorMigrationTest.java:377-426, 487-535):
  their window contents are transcoded to the GpuAggregates accumulator (a SUM of the tuples' Integer field),
  keys, windows and timers kept as the reference wrote them; restored into the GPU operator, the watermarks of
  the migration test give the migration test's expected output.
* Export: after random streams, the exported key groups hold what the reference's WindowOperator keeps in its
  heap backend at the same point -- the oracle's window contents, merging-window-set and event timers --
  for tumbling (both layouts), sliding (windows built from panes) and sessions, with allowedLateness > 0.
* Import: the oracle's state written in the heap layout and imported into a fresh operator continues exactly
  like the oracle -- sliding windows too (one accumulator per (key, window), WindowOperator.java:385-413, kept per
  window and combined into the window's rows at its fire) on every sliding layout: table panes with the ring and the
  recompute strategy, allowedLateness 0 and > 0, and the sliding log; a 2 -> 3 rescale through exported key groups
  equals one operator.
* The reference's sliding snapshot point (WindowOperatorTest.java:111-184, snapshot at :150-157) replayed through
  the heap layout, imported at Long.MIN_VALUE as a restored WindowOperator's timer service starts.
* Rejections: a purging trigger's session, the reference's session-with-stateful-trigger savepoint (a keyed state
  the operator does not run), a foreign accumulator, truncated bytes, a row that is no sliding window.
Integer aggregates: bit-exact.
"""
import os

import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G
from oracle import heap_keyed_state as H

pytestmark = pytest.mark.gpu

LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1
GOLD = os.path.join(os.path.dirname(__file__), "golden", "heap_state")


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    return flink_amd


def _ref_state(name, list_state):
    with open(os.path.join(GOLD, f"win-op-migration-test-{name}-flink1.11-snapshot"), "rb") as f:
        h = H.read_operator_subtask_state(f.read())["managed_keyed"][0]
    rv = H.list_of(H.read_string_int_tuple) if list_state else H.read_string_int_tuple
    _, st = H.read_key_groups(h, H.window_operator_decoders("string", rv, False))
    s = H.WindowState()
    for _, (w, k, v) in st[H.WINDOW_CONTENTS]:
        s.contents[(k, w)] = (sum(x[1] for x in v) if list_state else v[1], 0)
    s.timers = {e for _, e in st[H.EVENT_TIMERS]}
    return s


@pytest.mark.parametrize("name,list_state", [("reduce-event-time", False), ("apply-event-time", True)])
def test_restore_reference_savepoint(F, name, list_state):
    s = _ref_state(name, list_state)
    buf = H.write_state(s, "string", lambda k: 0, (0, 0))
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(3_000), F.SumAggregate(), key_kind="string",
                             max_parallelism=1)
    op.import_heap_state(buf, 1999)
    assert op.current_watermark == 1999 and op.state_size() == 3
    op.process_watermark(2999)
    assert sorted(op.output) == [("key1", 0, 3000, 3), ("key2", 0, 3000, 3)]
    op.process_watermark(3999)
    op.process_watermark(4999)
    assert len(op.output) == 2
    op.process_watermark(5999)
    assert sorted(op.output)[-1] == ("key2", 3000, 6000, 2) and len(op.output) == 3
    # the restored operator's own export is the state it restored, in the same layout
    op2 = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(3_000), F.SumAggregate(), key_kind="string",
                              max_parallelism=1)
    op2.import_heap_state(buf, 1999)
    out, offs, wm = op2.export_heap_state()
    assert wm == 1999 and list(offs) == [0]
    back = H.parse_export(out, "string", False, (0, 0))
    assert back.contents == s.contents and back.timers == s.timers
    op.close()
    op2.close()


def _streams(kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "session":
        k, t, v, _ = G.session_stream(200, 8_000, gap=3_000, lag=1_000, seed=seed, mean_inner=800,
                                      late_fraction=0.01)
        return k, t, v, G.punctuated_watermarks(t, 400, 1_000)
    n = 20_000
    k = rng.integers(0, 2_000, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 60_000, n)) + rng.integers(0, 2_500, n)).astype(np.int64)
    v = rng.integers(-300, 300, n).astype(np.int64)
    return k, t, v, G.punctuated_watermarks(t, 700, 1_200)


_SL = (lambda F: F.SlidingEventTimeWindows.of(6_000, 2_000), lambda: O.SlidingEventTimeWindows(6_000, 2_000))
CASES = {
    "tumbling_table": (lambda F: F.TumblingEventTimeWindows.of(5_000), lambda: O.TumblingEventTimeWindows(5_000),
                       "table", 2_000),
    "tumbling_log": (lambda F: F.TumblingEventTimeWindows.of(5_000), lambda: O.TumblingEventTimeWindows(5_000),
                     "log", 0),
    "sliding": (*_SL, "auto", 1_500),                      # table panes, recompute (MIN), re-fires
    "sliding_ring": (*_SL, "table", 1_500, "ring"),        # table panes, running total (int64 sums), re-fires
    "sliding_ring_l0": (*_SL, "table", 0, "ring"),
    "sliding_recompute_l0": (*_SL, "table", 0),
    "sliding_log": (*_SL, "log", 0, "ring"),                # logged panes, partitioned running total
    "session": (lambda F: F.EventTimeSessionWindows.withGap(3_000), lambda: O.EventTimeSessionWindows(3_000),
                "auto", 2_000),
}


def _aggs(F, kind="mixed"):
    if kind == "ring":
        return (F.MultiAggregate(F.SumAggregate(), F.CountAggregate(), F.AverageAggregate()),
                O.MultiAgg([O.SumLongAgg(), O.CountAgg(), O.AvgAgg()]))
    return (F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.AverageAggregate()),
            O.MultiAgg([O.SumLongAgg(), O.MinAgg(), O.AvgAgg()]))


def _case(case):
    c = CASES[case]
    return c[0], c[1], c[2], c[3], (c[4] if len(c) > 4 else "mixed")


@pytest.mark.parametrize("case", sorted(CASES))
def test_export_matches_reference_state(F, case):
    ga, oa, layout, lateness, ak = _case(case)
    k, t, v, b = _streams("session" if case == "session" else "win", 7)
    agg, oagg = _aggs(F, ak)
    maxp = 64
    op = F.GpuWindowOperator(ga(F), agg, allowed_lateness=lateness, state_layout=layout, max_parallelism=maxp)
    ref = O.WindowOperatorOracle(oa(), oagg, lateness, max_parallelism=maxp)
    prev = 0
    for end, wm in b[: len(b) // 2]:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        for i in range(prev, end):
            ref.process_element(int(k[i]), int(t[i]), int(v[i]))
        ref.process_watermark(wm)
        prev = end
    buf, offs, wm = op.export_heap_state()
    assert wm == ref.wm
    got = H.parse_export(buf, "long", case == "session", (0, maxp - 1))
    want = H.state_of_oracle(ref)
    assert got.resolved() == want.resolved() and len(want.contents) > 0
    assert got.timers == want.timers
    if case == "session":
        assert set(got.merging) == set(want.merging)
        assert {k: set(m) for k, m in got.merging.items()} == {k: set(m) for k, m in want.merging.items()}
    # key-group offsets: each key group's section starts with its id
    for g, off in enumerate(offs):
        assert int.from_bytes(buf[off:off + 4], "big", signed=True) == g
    op.close()


@pytest.mark.parametrize("case", ["tumbling_table", "tumbling_log", "session", "sliding", "sliding_ring",
                                  "sliding_ring_l0", "sliding_recompute_l0", "sliding_log"])
@pytest.mark.parametrize("key_kind", ["long", "string"])
@pytest.mark.parametrize("restore_at", ["checkpoint", "long_min"])
def test_import_continues_like_reference(F, case, key_kind, restore_at):
    """restore_at long_min: the watermark a restored WindowOperator's timer service starts at (InternalTimerServiceImpl
    .java:78) -- records of windows that already fired before the checkpoint are on time again until the next
    watermark, as in the reference."""
    if key_kind == "string" and case == "sliding_log":
        pytest.skip("the log layouts take Long/Integer keys")
    ga, oa, layout, lateness, ak = _case(case)
    k, t, v, b = _streams("session" if case == "session" else "win", 13)
    kv = (lambda x: f"k{int(x)}") if key_kind == "string" else int
    kh = O.string_hash_code if key_kind == "string" else O.long_hash_code
    agg, oagg = _aggs(F, ak)
    maxp = 32
    ref = O.WindowOperatorOracle(oa(), oagg, lateness, max_parallelism=maxp, key_hash=kh)
    cut = len(b) // 2
    prev = 0
    for end, wm in b[:cut]:
        for i in range(prev, end):
            ref.process_element(kv(k[i]), int(t[i]), int(v[i]))
        ref.process_watermark(wm)
        prev = end
    before, late_before = len(ref.output), ref.num_late_records_dropped
    buf = H.write_state(H.state_of_oracle(ref), key_kind, lambda x: O.assign_to_key_group(kh(x), maxp), (0, maxp - 1))
    op = F.GpuWindowOperator(ga(F), agg, allowed_lateness=lateness, state_layout=layout, max_parallelism=maxp,
                             key_kind=key_kind)
    if restore_at == "long_min":
        ref.wm = LONG_MIN
    op.import_heap_state(buf, ref.wm)
    p0 = prev
    for end, wm in b[cut:]:
        keys = [kv(x) for x in k[p0:end]] if key_kind == "string" else k[p0:end]
        op.process_batch(keys, t[p0:end], v[p0:end])
        op.process_watermark(wm)
        for i in range(p0, end):
            ref.process_element(kv(k[i]), int(t[i]), int(v[i]))
        ref.process_watermark(wm)
        p0 = end
    op.end_input()
    ref.end_input()
    want = sorted((r.key, r.start, r.end, r.result) for r in ref.output[before:])
    got = sorted(op.output)
    assert len(want) > 0
    assert got == want
    assert op.num_late_records_dropped == ref.num_late_records_dropped - late_before
    op.close()


@pytest.mark.parametrize("layout", ["table", "log"])
@pytest.mark.parametrize("restore_at", ["checkpoint", "long_min"])
def test_reference_sliding_snapshot_point_through_heap_layout(F, golden, layout, restore_at):
    """WindowOperatorTest.testSlidingEventTimeWindowsApply's snapshot (WindowOperatorTest.java:150-157, after
    processWatermark(2999)): the reference operator's heap state at that point (the oracle's, per (key, window)), in
    the heap layout, imported into a fresh GPU operator; the rest of the stream then gives the test's expected output."""
    s = next(x for x in golden["operator_streams"] if x["name"] == "sliding_3s_1s")
    a = s["assigner"]
    cut = s["snapshot_after"] + 1
    ref = O.WindowOperatorOracle(O.SlidingEventTimeWindows(a["size"], a["slide"], a["offset"]), O.SumLongAgg(), 0)
    for ev in s["events"][:cut]:
        if ev[0] == "e":
            ref.process_element(ev[1], ev[2], ev[3])
        else:
            ref.process_watermark(ev[1])
    before = [(r.key, r.start, r.end, r.result) for r in ref.output]
    state = H.state_of_oracle(ref)
    assert len(state.contents) > 0
    buf = H.write_state(state, "long", lambda x: O.assign_to_key_group(O.long_hash_code(x), 128), (0, 127))
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(a["size"], a["slide"], a["offset"]), F.SumAggregate(),
                             state_layout=layout)
    op.import_heap_state(buf, LONG_MIN if restore_at == "long_min" else ref.wm)
    assert op.state_size() >= len(state.contents)
    # the restored operator exports what it imported (windows still waiting for their fire timers)
    back = H.parse_export(op.export_heap_state()[0], "long", False, (0, 127))
    assert back.contents == state.contents and back.timers == state.timers
    for ev in s["events"][cut:]:
        if ev[0] == "e":
            op.process_element(ev[1], ev[2], ev[3])
        else:
            op.process_watermark(ev[1])
    op.end_input()
    assert sorted(before + list(op.output)) == sorted(map(tuple, s["expected"]))
    op.close()


def test_rescale_through_heap_layout(F):
    """Two subtasks export their key groups; three restored subtasks (each keeping its own KeyGroupRange from the
    concatenated sections) continue; the union equals one operator."""
    k, t, v, b = _streams("win", 21)
    maxp = 128
    want = O.WindowOperatorOracle(O.TumblingEventTimeWindows(5_000), O.SumLongAgg(), 0, max_parallelism=maxp)
    prev = 0
    for end, wm in b:
        for i in range(prev, end):
            want.process_element(int(k[i]), int(t[i]), int(v[i]))
        want.process_watermark(wm)
        prev = end
    want.end_input()
    kg, _ = F.assign_key_groups(k, maxp)
    cut = len(b) // 2
    mk = lambda r: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5_000), F.SumAggregate(), max_parallelism=maxp,
                                       key_group_range=(r.start_key_group, r.end_key_group))
    parts, rows = [], []
    for idx in range(2):
        r = F.compute_key_group_range_for_operator_index(maxp, 2, idx)
        op = mk(r)
        mine = (kg >= r.start_key_group) & (kg <= r.end_key_group)
        p0 = 0
        for end, wm in b[:cut]:
            sel = np.nonzero(mine[p0:end])[0] + p0
            op.process_batch(k[sel], t[sel], v[sel])
            op.process_watermark(wm)
            p0 = end
        buf, _, wm0 = op.export_heap_state()
        parts.append(buf)
        rows += list(op.output)
        op.close()
    blob = b"".join(parts)
    start = b[cut - 1][0]
    for idx in range(3):
        r = F.compute_key_group_range_for_operator_index(maxp, 3, idx)
        op = mk(r)
        op.import_heap_state(blob, wm0)
        mine = (kg >= r.start_key_group) & (kg <= r.end_key_group)
        p0 = start
        for end, wm in b[cut:]:
            sel = np.nonzero(mine[p0:end])[0] + p0
            op.process_batch(k[sel], t[sel], v[sel])
            op.process_watermark(wm)
            p0 = end
        op.end_input()
        rows += list(op.output)
        op.close()
    assert sorted(rows) == sorted((r.key, r.start, r.end, r.result) for r in want.output)


def test_import_rejections(F):
    from flink_amd import _native as N
    mk = lambda: F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3_000, 1_000), F.SumAggregate(), max_parallelism=1)
    sl = mk()
    sl.import_heap_state(H.write_state(H.WindowState(), "long", lambda k: 0, (0, 0)), 0)   # empty: fine
    sl.close()
    s = H.WindowState()
    s.contents[(5, (500, 3500))] = (4, 0)      # not a window of size 3000 / slide 1000
    s.timers.add((3499, 5, (500, 3500)))
    sl = mk()
    with pytest.raises(N.GwoError) as e:
        sl.import_heap_state(H.write_state(s, "long", lambda k: 0, (0, 0)), 0)
    assert e.value.status == N.GWO_ERR_INVALID_ARGUMENT
    s = H.WindowState()
    s.contents[(5, (0, 3000))] = (4, 0)
    s.timers.add((2999, 5, (0, 3000)))          # a pending fire timer the restore watermark already passed
    with pytest.raises(N.GwoError) as e:
        sl.import_heap_state(H.write_state(s, "long", lambda k: 0, (0, 0)), 5000)
    assert e.value.status == N.GWO_ERR_UNSUPPORTED
    sl.import_heap_state(H.write_state(s, "long", lambda k: 0, (0, 0)), 1000)   # the rejections left it fresh
    with pytest.raises(N.GwoError) as e:        # per-window state has no pane rows: checkpoints go the heap layout
        sl.snapshot_state()
    assert e.value.status == N.GWO_ERR_UNSUPPORTED
    sl.process_watermark(2999)
    assert sl.output == [(5, 0, 3000, 4)]
    sl.close()
    # the reference's session-with-stateful-trigger savepoint: its key groups hold the trigger's "count" state
    with open(os.path.join(GOLD, "win-op-migration-test-session-with-stateful-trigger-flink1.11-snapshot"), "rb") as f:
        h = H.read_operator_subtask_state(f.read())["managed_keyed"][0]
    names = [m[0] for m in H.state_meta(h.data, h.offsets[0])]
    ids = tuple(names.index(x) for x in (H.WINDOW_CONTENTS, H.MERGING_WINDOW_SET, H.EVENT_TIMERS, H.PROCESSING_TIMERS))
    se = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(3_000), F.SumAggregate(), key_kind="string",
                             max_parallelism=1)
    with pytest.raises(N.GwoError) as e:
        se.import_heap_state(h.data[h.offsets[0]:], 0, ids=ids)
    assert e.value.status == N.GWO_ERR_UNSUPPORTED and "trigger" in str(e.value)
    se.close()
    # a purging trigger's session: tracked in the merging-window-set without contents
    s = H.WindowState()
    s.merging["key2"] = {(0, 6500): (0, 3000)}
    s.timers.add((6499, "key2", (0, 6500)))
    se = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(3_000), F.SumAggregate(), key_kind="string",
                             max_parallelism=1)
    with pytest.raises(N.GwoError) as e:
        se.import_heap_state(H.write_state(s, "string", lambda k: 0, (0, 0)), 0)
    assert e.value.status == N.GWO_ERR_UNSUPPORTED
    se.close()
    tu = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1_000), F.SumAggregate(), max_parallelism=1)
    s = H.WindowState()
    s.contents[(5, (0, 1000))] = (1, 0, 2, 0)          # two aggregates' accumulator into a one-aggregate operator
    with pytest.raises(N.GwoError) as e:
        tu.import_heap_state(H.write_state(s, "long", lambda k: 0, (0, 0)), 0)
    assert e.value.status == N.GWO_ERR_INVALID_ARGUMENT
    s.contents[(5, (0, 1000))] = (4, 0)
    s.timers.add((999, 5, (0, 1000)))
    good = H.write_state(s, "long", lambda k: 0, (0, 0))
    with pytest.raises(N.GwoError) as e:
        tu.import_heap_state(good[:-3], 0)
    assert e.value.status == N.GWO_ERR_INVALID_ARGUMENT
    tu.import_heap_state(good, 0)                      # a rejected import left the handle fresh
    tu.process_watermark(999)
    assert tu.output == [(5, 0, 1000, 4)]
    tu.close()
