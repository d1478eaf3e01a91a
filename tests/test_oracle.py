"""CPU: pin the oracle against the reference's own known answers, then cross-check the
vectorised restatement against the record-at-a-time one."""
import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G
from oracle import vectorized as V


def mk_assigner(a):
    if a["kind"] == "tumbling":
        return O.TumblingEventTimeWindows(a["size"], a["offset"])
    if a["kind"] == "sliding":
        return O.SlidingEventTimeWindows(a["size"], a["slide"], a["offset"])
    return O.EventTimeSessionWindows(a["gap"])


def test_key_groups_string_golden(golden):
    g = golden["key_groups_string"]
    got = [O.assign_to_key_group(O.string_hash_code(k), g["max_parallelism"]) for k in g["keys"]]
    assert got == g["groups"]


def test_long_key_groups_restatement():
    # Long.hashCode is a JDK contract no reference test pins ("parity unpinned"); SURVEY.md §8c value.
    assert [O.assign_to_key_group(O.long_hash_code(k), 128) for k in range(10)] == [94, 86, 127, 113, 7, 126, 18, 113, 15, 51]


def test_key_group_ranges():
    # KeyGroupRangeAssignment: ranges tile [0, maxP) and agree with computeOperatorIndexForKeyGroup
    for maxp, p in [(128, 1), (128, 3), (32768, 8), (10, 3), (7, 7)]:
        seen = []
        for i in range(p):
            lo, hi = O.compute_key_group_range_for_operator_index(maxp, p, i)
            seen.extend(range(lo, hi + 1))
            for kg in range(lo, hi + 1):
                assert O.compute_operator_index_for_key_group(maxp, p, kg) == i
        assert seen == list(range(maxp))
    assert O.compute_default_max_parallelism(1) == 128
    assert O.compute_default_max_parallelism(100) == 256
    assert O.compute_default_max_parallelism(30000) == 32768


def test_window_start_golden(golden):
    for ts, off, size, start in golden["window_start_with_offset"]["cases"]:
        assert O.get_window_start_with_offset(ts, off, size) == start


def test_java_rem_quirk():
    # TimeWindow.java:270-272 replicated, not fixed: ts=-7, size=5 -> start -5
    assert O.get_window_start_with_offset(-7, 0, 5) == -5


def test_intersects_golden(golden):
    for a, b, want in golden["intersects"]["cases"]:
        wa, wb = O.TimeWindow(*a), O.TimeWindow(*b)
        assert wa.intersects(wb) == wb.intersects(wa) == want


def test_tumbling_assign_golden(golden):
    for c in golden["tumbling_assign"]["cases"]:
        w = O.TumblingEventTimeWindows(c["size"], c["offset"]).assign_windows(c["ts"])
        assert [(x.start, x.end) for x in w] == [tuple(x) for x in c["windows"]]
    for size, off in golden["tumbling_assign"]["invalid"]:
        with pytest.raises(ValueError, match="abs\\(offset\\) < size"):
            O.TumblingEventTimeWindows(size, off)


def test_sliding_assign_golden(golden):
    for c in golden["sliding_assign"]["cases"]:
        w = O.SlidingEventTimeWindows(c["size"], c["slide"], c["offset"]).assign_windows(c["ts"])
        assert sorted((x.start, x.end) for x in w) == sorted(tuple(x) for x in c["windows"])


def test_session_assign_and_merge_golden(golden):
    for c in golden["session_assign"]["cases"]:
        w = O.EventTimeSessionWindows(c["gap"]).assign_windows(c["ts"])
        assert [(x.start, x.end) for x in w] == [tuple(x) for x in c["windows"]]
    for c in golden["session_merge"]["cases"]:
        calls = []
        O.merge_windows([O.TimeWindow(*w) for w in c["windows"]],
                        lambda group, res: calls.append((sorted((x.start, x.end) for x in group), (res.start, res.end))))
        want = [(sorted(tuple(x) for x in g), tuple(r)) for g, r in c["merges"]]
        assert sorted(calls) == sorted(want)


@pytest.mark.parametrize("idx", range(11))
def test_operator_streams_golden(golden, idx):
    s = golden["operator_streams"][idx]
    op = O.WindowOperatorOracle(mk_assigner(s["assigner"]), O.SumLongAgg(), s["lateness"], s["side_output"])
    O.run_stream(op, s["events"])
    got = O.rows_as_tuples(op.output)
    if "expected" in s:
        assert got == sorted(map(tuple, s["expected"]))
    else:
        assert sorted((r[0], r[1], r[3]) for r in got) == sorted(map(tuple, s["expected_key_start_sum"]))
    assert sorted(op.side_output) == sorted(map(tuple, s.get("side", [])))
    assert op.num_late_records_dropped == s["late"]


def _random_stream(rng, n, nkeys, span, disorder, every, lag):
    keys = rng.integers(0, nkeys, n)
    ts = np.sort(rng.integers(0, span, n)) + rng.integers(0, disorder, n)
    vals = rng.integers(-1000, 1000, n)
    batches = G.punctuated_watermarks(ts, every, lag)
    return keys, ts, vals, batches


def _loop(assigner, agg, keys, ts, vals, batches, lateness=0):
    op = O.WindowOperatorOracle(assigner, agg, lateness)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(keys[i]), int(ts[i]), int(vals[i]))
        op.process_watermark(wm)
        prev = end
    return op


@pytest.mark.parametrize("lag", [0, 300, 2000])
def test_vectorized_matches_loop_tumbling(lag):
    rng = np.random.default_rng(lag + 1)
    keys, ts, vals, batches = _random_stream(rng, 4000, 50, 20000, 1500, 97, lag)
    op = _loop(O.TumblingEventTimeWindows(1000, 100), O.MultiAgg([O.SumLongAgg(), O.MinAgg(), O.MaxAgg(), O.CountAgg()]),
               keys, ts, vals, batches)
    (k, s, e, res), late = V.tumbling_lateness0(keys, ts, vals, batches, 1000, 100, [1, 2, 3, 0])
    want = sorted((r.key, r.start, r.end, r.result) for r in op.output)
    got = sorted(zip(k.tolist(), s.tolist(), e.tolist(), zip(*[x.tolist() for x in res])))
    assert got == want
    assert late == op.num_late_records_dropped


@pytest.mark.parametrize("lag", [0, 700])
def test_vectorized_matches_loop_sliding(lag):
    rng = np.random.default_rng(lag + 7)
    keys, ts, vals, batches = _random_stream(rng, 3000, 40, 20000, 2500, 101, lag)
    op = _loop(O.SlidingEventTimeWindows(3000, 1000, 0), O.AvgAgg(), keys, ts, vals, batches)
    (k, s, e, res), late = V.sliding_lateness0(keys, ts, vals, batches, 3000, 1000, 0, [4])
    want = sorted((r.key, r.start, r.end, r.result) for r in op.output)
    got = sorted(zip(k.tolist(), s.tolist(), e.tolist(), res[0].tolist()))
    assert got == want
    assert late == op.num_late_records_dropped


def test_generator_definition():
    spec = G.GenSpec(seed=42, total_records=1000, num_keys=10, span_ms=60000, disorder_ms=1000)
    k, t, v = G.generate(spec, 1000)
    k2, t2, v2 = G.generate(spec, 500, first=500)
    assert (k[500:] == k2).all() and (t[500:] == t2).all() and (v[500:] == v2).all()
    assert k.min() >= 0 and k.max() < 10 and v.min() >= 0 and v.max() < 1000
    # ts = i*span/N + U[0, disorder)
    base = (np.arange(1000) * 60000) // 1000
    assert ((t - base) >= 0).all() and ((t - base) < 1000).all()
    # first value pinned (guards the cross-language definition)
    z = (42 + 0 * 0xD1B54A32D192ED03 + 1 * 0x9E3779B97F4A7C15) % (1 << 64)
    assert int(k[0]) == O.splitmix64((z - 0x9E3779B97F4A7C15) % (1 << 64)) % 10


class _NonEagerAssigner:
    """The MergingWindowSetTest's misbehaving assigner (MergingWindowSetTest.java:470-536): the windows that start
    inside the earliest-starting window merge into [its start, its end + 1)."""
    merging = True

    def __init__(self, timeout):
        self.timeout = timeout

    def merge_windows(self, windows, callback):
        earliest = None
        for w in windows:
            if earliest is None or w.start < earliest.start:
                earliest = w
        assoc = [w for w in windows if earliest.start <= w.start < earliest.end]
        if len(assoc) > 1:
            callback(set(assoc), O.TimeWindow(earliest.start, earliest.end + 1))


@pytest.mark.parametrize("case", range(9))
def test_merging_window_set_known_answers(case):
    """MergingWindowSetTest.java:71-437 (tests/golden/merging_window_set.json) against the oracle's
    MergingWindowSet restatement -- the session bookkeeping the GPU's per-key session lists follow."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "merging_window_set.json")) as f:
        c = json.load(f)["cases"][case]
    W = lambda x: O.TimeWindow(*x)
    assigner = _NonEagerAssigner(c["timeout"]) if c["assigner"] == "non_eager" else O.EventTimeSessionWindows(c["assigner"])
    ws = O.MergingWindowSet(assigner, {W(a): W(b) for a, b in c.get("initial", [])})
    for op in c["ops"]:
        if op[0] == "add":
            calls = []
            res = ws.add_window(W(op[1]), lambda *a: calls.append(a))
            if op[3] == "any":
                assert ws.get_state_window(res) is not None
                continue
            assert res == W(op[2])
            if op[3] is None:
                assert calls == []
                continue
            assert len(calls) == 1                      # one merge per added window
            target, sources, state_window, merged_state = calls[0]
            m = op[3]
            if "target" in m:
                assert target == W(m["target"])
                assert sorted(sources) == sorted(W(x) for x in m["sources"])
                assert state_window in [W(x) for x in m["state_window"]]
            if "merged_state_windows" in m:
                assert sorted(merged_state) in [sorted(W(x) for x in alt) for alt in m["merged_state_windows"]]
                assert target not in merged_state
        elif op[0] == "state":
            got = ws.get_state_window(W(op[1]))
            assert got is None if op[2] is None else got in [W(x) for x in op[2]]
        elif op[0] == "retire":
            ws.retire_window(W(op[1]))
        elif op[0] == "persist":
            adds = ws.persist()
            if op[1] is None:
                assert adds is None
            else:
                assert sorted(adds) == sorted((W(a), W(b)) for a, b in op[1])
