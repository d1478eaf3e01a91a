"""The heap state backend's savepoint layout (oracle/heap_keyed_state.py), pinned against the reference's own
savepoint files (tests/golden/heap_state/: the data files of flink-streaming-java/src/test/resources written by
WindowOperatorMigrationTest.java's write*Snapshot methods, copied unchanged).

Each file is parsed to its last byte, and the state found is the state the generating test built: the elements it
fed (WindowOperatorMigrationTest.java:349-366, 459-476, 145-151) replayed through the oracle WindowOperator give the
same window contents and timers.  The writer used to build gwo_import_heap_state inputs round-trips through the
reader.  CPU only.
"""
import os

import pytest

from oracle import flink_oracle as O
from oracle import heap_keyed_state as H

GOLD = os.path.join(os.path.dirname(__file__), "golden", "heap_state")


def _handle(name):
    with open(os.path.join(GOLD, f"win-op-migration-test-{name}-flink1.11-snapshot"), "rb") as f:
        st = H.read_operator_subtask_state(f.read())
    assert st["version"] == 3 and st["raw_keyed"] == [] and st["managed_operator"] == []
    assert len(st["managed_keyed"]) == 1
    return st["managed_keyed"][0]


# the generating tests' elements (key, value, timestamp) and watermarks before the snapshot
TUMBLING_ELEMENTS = [("key2", 1, 3999), ("key2", 1, 3000), ("key1", 1, 20), ("key1", 1, 0), ("key1", 1, 999),
                     ("key2", 1, 1998), ("key2", 1, 1999), ("key2", 1, 1000)]
EXPECTED_TIMERS = {(2999, "key1", (0, 3000)), (2999, "key2", (0, 3000)), (5999, "key2", (3000, 6000))}


def _oracle_tumbling():
    op = O.WindowOperatorOracle(O.TumblingEventTimeWindows(3_000), O.SumLongAgg(), key_hash=O.string_hash_code)
    for k, v, ts in TUMBLING_ELEMENTS:
        op.process_element(k, ts, v)
    op.process_watermark(999)
    op.process_watermark(1999)
    assert op.output == []
    return op


def test_reduce_event_time_savepoint():
    """ReducingState<Tuple2<String, Integer>> with SumReducer (WindowOperatorMigrationTest.java:320-375)."""
    h = _handle("reduce-event-time")
    assert h.start_kg == 0 and len(h.offsets) == 1          # the harness's maxParallelism 1
    meta, st = H.read_key_groups(h, H.window_operator_decoders("string", H.read_string_int_tuple, False))
    assert [m[0] for m in meta] == [H.WINDOW_CONTENTS, H.PROCESSING_TIMERS, H.EVENT_TIMERS]
    assert meta[0][2] == "REDUCING"
    contents = {(k, w): v for _, (w, k, v) in st[H.WINDOW_CONTENTS]}
    assert contents == {("key1", (0, 3000)): ("key1", 3), ("key2", (0, 3000)): ("key2", 3),
                        ("key2", (3000, 6000)): ("key2", 2)}
    assert {e for _, e in st[H.EVENT_TIMERS]} == EXPECTED_TIMERS
    assert st[H.PROCESSING_TIMERS] == []
    # the oracle fed the same elements holds the same state
    s = H.state_of_oracle(_oracle_tumbling())
    assert s.contents == {kw: (v[1], 0) for kw, v in contents.items()}
    assert s.timers == EXPECTED_TIMERS


def test_apply_event_time_savepoint():
    """ListState<Tuple2<String, Integer>> (WindowOperatorMigrationTest.java:431-485): the elements themselves."""
    h = _handle("apply-event-time")
    meta, st = H.read_key_groups(h, H.window_operator_decoders("string", H.list_of(H.read_string_int_tuple), False))
    assert meta[0] == (H.WINDOW_CONTENTS, H.KEY_VALUE, "LIST")
    contents = {(k, w): v for _, (w, k, v) in st[H.WINDOW_CONTENTS]}
    assert {kw: sum(x[1] for x in v) for kw, v in contents.items()} == \
        {("key1", (0, 3000)): 3, ("key2", (0, 3000)): 3, ("key2", (3000, 6000)): 2}
    assert all(x[0] == kw[0] for kw, v in contents.items() for x in v)
    assert {e for _, e in st[H.EVENT_TIMERS]} == EXPECTED_TIMERS


def test_session_savepoint_with_merging_window_set():
    """Sessions (gap 3 s) with PurgingTrigger.of(CountTrigger.of(4)) (WindowOperatorMigrationTest.java:119-161):
    the merging-window-set maps each session to its state window; key2's session fired and purged its contents at
    the 4th element but stays tracked with its timer; key1's merged session [10, 4000) keeps its state under the
    first window [10, 3010)."""
    h = _handle("session-with-stateful-trigger")
    extra = {"count": lambda r: (H.read_time_window(r), r.string_value(), r.i64())}
    meta, st = H.read_key_groups(h, H.window_operator_decoders("string", H.list_of(H.read_string_int_tuple), True,
                                                               extra))
    assert [m[0] for m in meta] == ["count", H.WINDOW_CONTENTS, H.MERGING_WINDOW_SET, H.PROCESSING_TIMERS,
                                    H.EVENT_TIMERS]
    assert [e for _, e in st[H.WINDOW_CONTENTS]] == [((10, 3010), "key1", [("key1", 1), ("key1", 2)])]
    assert dict(e for _, e in st[H.MERGING_WINDOW_SET]) == {"key1": [((10, 4000), (10, 3010))],
                                                            "key2": [((0, 6500), (0, 3000))]}
    assert [e for _, e in st["count"]] == [((10, 4000), "key1", 2)]
    assert {e for _, e in st[H.EVENT_TIMERS]} == {(3999, "key1", (10, 4000)), (6499, "key2", (0, 6500))}
    # the oracle (EventTimeTrigger, no purge) keeps the same session windows and state windows for key1
    op = O.WindowOperatorOracle(O.EventTimeSessionWindows(3_000), O.SumLongAgg(), key_hash=O.string_hash_code)
    for k, v, ts in [("key1", 1, 10), ("key1", 2, 1000)]:
        op.process_element(k, ts, v)
    s = H.state_of_oracle(op)
    assert s.merging == {"key1": {(10, 4000): (10, 3010)}}
    assert s.contents == {("key1", (10, 3010)): (3, 0)}
    assert s.timers == {(3999, "key1", (10, 4000))}


def test_mint_session_savepoint_is_empty():
    h = _handle("session-with-stateful-trigger-mint")
    _, st = H.read_key_groups(h, H.window_operator_decoders("string", H.list_of(H.read_string_int_tuple), True))
    assert all(v == [] for v in st.values())


def test_truncated_savepoint_is_rejected():
    with open(os.path.join(GOLD, "win-op-migration-test-reduce-event-time-flink1.11-snapshot"), "rb") as f:
        blob = f.read()
    with pytest.raises(ValueError):
        H.read_operator_subtask_state(blob[:-9])


@pytest.mark.parametrize("key_kind", ["long", "int", "string"])
def test_writer_round_trips(key_kind):
    """write_state -> parse_export over several key groups; sessions carry their state windows."""
    keys = {"long": [-(1 << 40), 7, 123456789], "int": [-5, 0, 2 ** 31 - 1], "string": ["a", "ключ", "\U0001F600x"]}[
        key_kind]
    kh = {"long": O.long_hash_code, "int": O.int_hash_code, "string": O.string_hash_code}[key_kind]
    maxp = 16
    kg = lambda k: O.assign_to_key_group(kh(k), maxp)
    s = H.WindowState()
    for i, k in enumerate(keys):
        s.contents[(k, (100 * i, 100 * i + 50))] = (i, -i, 3, 4)
        s.merging[k] = {(100 * i, 100 * i + 80): (100 * i, 100 * i + 50)}
        s.timers.add((100 * i + 79, k, (100 * i, 100 * i + 80)))
    buf = H.write_state(s, key_kind, kg, (0, maxp - 1))
    back = H.parse_export(buf, key_kind, True, (0, maxp - 1))
    assert back.contents == s.contents and back.merging == s.merging and back.timers == s.timers


def test_gpu_accumulator_layout():
    """GpuAggregates.java:49-100: two longs per aggregate; f64 min/max carry the raw bits and a has-value flag."""
    agg = O.MultiAgg([O.CountAgg(), O.SumLongAgg(), O.MinAgg(is_double=True), O.AvgAgg()])
    acc = agg.create_accumulator()
    for v in (3, -1, 7):
        acc = agg.add(v, acc)
    got = H.gpu_accumulator(agg, acc)
    assert got[:4] == (3, 0, 9, 0)
    assert got[4] == H._bits(-1.0) and got[5] == 1
    assert got[6:] == (9, 3)
