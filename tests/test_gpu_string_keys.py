"""GPU parity for String-keyed streams inside the operator (gwo.h gwo_submit_utf16).

The reference keys a String-keyed stream by the String: its key group is murmur(String.hashCode) over UTF-16
code units (KeyGroupRangeAssignment.java:60-73) and the state is keyed by the String.  The handle interns Strings
into a device dictionary whose ids carry String.hashCode in their high half (gwo_strings.hip).  Checked against the
oracle with the Strings themselves as keys: tumbling on both layouts, sliding, sessions, the key-group range check,
a checkpoint restored into a fresh handle (another dictionary) including rescaling, and dictionary growth.
"""
import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G

pytestmark = pytest.mark.gpu
LONG_MAX = (1 << 63) - 1
ALPHABET = list("abcXYZ019 _-") + ["é", "中", "\U0001F600", "￿", "\ud800"]


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    return flink_amd


def _words(rng, n):
    out = ["", "a", "campaign-42", "\U0001F600" * 3, "Aa", "BB"]   # "Aa" and "BB" share String.hashCode 2112
    while len(out) < n:
        out.append("".join(rng.choice(ALPHABET, rng.integers(1, 12))))
    return list(dict.fromkeys(out))[:n]


def _stream(seed, n, nkeys, span, disorder):
    rng = np.random.default_rng(seed)
    words = _words(rng, nkeys)
    ki = rng.integers(0, len(words), n)
    keys = [words[i] for i in ki]
    t = (np.sort(rng.integers(0, span, n)) + rng.integers(0, disorder, n)).astype(np.int64)
    v = rng.integers(-100, 100, n).astype(np.int64)
    return keys, t, v


def _oracle(assigner, agg, keys, t, v, batches, lateness=0, kg_range=None, maxp=128):
    op = O.WindowOperatorOracle(assigner, agg, lateness, key_group_range=kg_range, max_parallelism=maxp,
                                key_hash=O.string_hash_code)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(keys[i], int(t[i]), int(v[i]))
        op.process_watermark(wm)
        prev = end
    op.process_watermark(LONG_MAX)
    return sorted((r.key, r.start, r.end, r.result) for r in op.output), op.num_late_records_dropped


def _run(op, keys, t, v, batches, start=0):
    prev = start
    for end, wm in batches:
        op.process_batch(keys[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        prev = end
    return prev


@pytest.mark.parametrize("layout", ["table", "log"])
@pytest.mark.parametrize("lateness", [0, 3_000])
def test_string_keys_tumbling(F, layout, lateness):
    keys, t, v = _stream(1 + lateness, 30_000, 2_000, 60_000, 4_000)
    b = G.punctuated_watermarks(t, 2_000, 500)
    want, wl = _oracle(O.TumblingEventTimeWindows(5_000), O.MultiAgg([O.SumLongAgg(), O.CountAgg()]), keys, t, v, b,
                       lateness)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5_000), F.MultiAggregate(F.SumAggregate(), F.CountAggregate()),
                             key_kind="string", state_layout=layout, allowed_lateness=lateness)
    _run(op, keys, t, v, b)
    op.end_input()
    assert sorted(op.output) == want
    assert op.num_late_records_dropped == wl
    op.close()


def test_string_keys_sliding_and_sessions(F):
    keys, t, v = _stream(7, 8_000, 300, 40_000, 2_000)
    b = G.punctuated_watermarks(t, 500, 300)
    for oa, fa in [(O.SlidingEventTimeWindows(4_000, 1_000), F.SlidingEventTimeWindows.of(4_000, 1_000)),
                   (O.EventTimeSessionWindows(700), F.EventTimeSessionWindows.withGap(700))]:
        want, wl = _oracle(oa, O.SumLongAgg(), keys, t, v, b)
        op = F.GpuWindowOperator(fa, F.SumAggregate(), key_kind="string")
        _run(op, keys, t, v, b)
        op.end_input()
        assert sorted(op.output) == want and op.num_late_records_dropped == wl
        op.close()


def test_string_keys_key_group_range(F):
    """Subtasks see only their key groups (murmur of String.hashCode); a foreign key fails the batch."""
    from flink_amd import _native as N
    keys, t, v = _stream(3, 6_000, 500, 30_000, 1_000)
    maxp = 64
    _, kg, _ = F.assign_key_groups_strings(keys, maxp)
    b = [(len(keys), int(t.max()) - 2_000)]
    rows = []
    for idx in range(3):
        r = F.compute_key_group_range_for_operator_index(maxp, 3, idx)
        sel = np.nonzero((kg >= r.start_key_group) & (kg <= r.end_key_group))[0]
        ks = [keys[i] for i in sel]
        want, _ = _oracle(O.TumblingEventTimeWindows(2_000), O.SumLongAgg(), ks, t[sel], v[sel], [(len(sel), b[0][1])],
                          kg_range=(r.start_key_group, r.end_key_group), maxp=maxp)
        op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(2_000), F.SumAggregate(), key_kind="string",
                                 max_parallelism=maxp, key_group_range=(r.start_key_group, r.end_key_group))
        _run(op, ks, t[sel], v[sel], [(len(sel), b[0][1])])
        op.end_input()
        assert sorted(op.output) == want
        rows += op.output
        op.close()
    want_all, _ = _oracle(O.TumblingEventTimeWindows(2_000), O.SumLongAgg(), keys, t, v, b, maxp=maxp)
    assert sorted(rows) == want_all
    r0 = F.compute_key_group_range_for_operator_index(maxp, 3, 0)
    foreign = next(keys[i] for i in range(len(keys)) if kg[i] > r0.end_key_group)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(2_000), F.SumAggregate(), key_kind="string",
                             max_parallelism=maxp, key_group_range=(r0.start_key_group, r0.end_key_group))
    with pytest.raises(N.GwoError) as e:
        op.process_batch([foreign], np.array([5]), np.array([1]))
    assert e.value.status == N.GWO_ERR_KEY_GROUP
    op.close()


@pytest.mark.parametrize("layout", ["table", "log"])
def test_string_keys_checkpoint_restore_and_rescale(F, layout):
    keys, t, v = _stream(9, 20_000, 1_500, 50_000, 3_000)
    b = G.punctuated_watermarks(t, 2_000, 300)
    maxp = 32
    want, wl = _oracle(O.TumblingEventTimeWindows(4_000), O.SumLongAgg(), keys, t, v, b, maxp=maxp)
    mk = lambda rng_=None: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(4_000), F.SumAggregate(), key_kind="string",
                                               state_layout=layout, max_parallelism=maxp, key_group_range=rng_)
    a = mk()
    cut = len(b) // 2
    prev = _run(a, keys, t, v, b[:cut])
    snap = a.snapshot_state()
    assert all(isinstance(k, str) for k in snap["key"])
    rows = list(a.output)
    a.close()
    _, kg, _ = F.assign_key_groups_strings(keys, maxp)
    for idx in range(2):   # 1 -> 2 rescale: each new subtask restores the whole checkpoint, keeps its key groups
        r = F.compute_key_group_range_for_operator_index(maxp, 2, idx)
        c = mk((r.start_key_group, r.end_key_group))
        c.restore_state(snap)
        p0 = prev
        for end, wm in b[cut:]:
            sel = [i for i in range(p0, end) if r.start_key_group <= kg[i] <= r.end_key_group]
            c.process_batch([keys[i] for i in sel], t[sel], v[sel])
            c.process_watermark(wm)
            p0 = end
        c.end_input()
        rows += c.output
        c.close()
    assert sorted(rows) == want


def test_string_dictionary_growth(F):
    """200K distinct Strings over several batches: the dictionary table rehashes and its arena grows."""
    rng = np.random.default_rng(5)
    n = 200_000
    keys = [f"user-{i}-{'x' * int(rng.integers(0, 20))}" for i in rng.permutation(n)]
    t = np.sort(rng.integers(0, 100_000, n)).astype(np.int64)
    v = np.ones(n, np.int64)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(50_000), F.CountAggregate(), key_kind="string")
    for s in range(0, n, 40_000):
        op.process_batch(keys[s:s + 40_000], t[s:s + 40_000], v[s:s + 40_000])
    op.end_input()
    got = sorted(op.output)
    want = sorted((k, (int(ts) // 50_000) * 50_000, (int(ts) // 50_000) * 50_000 + 50_000, 1) for k, ts in zip(keys, t))
    assert got == want
    ids = op.intern_strings(keys[:1000])
    assert op.key_strings(ids) == keys[:1000]
    h, _, _ = F.assign_key_groups_strings(keys[:1000], 128)
    assert ((ids >> 32).astype(np.int32) == h).all()   # the id's high half is String.hashCode
    op.close()


def test_string_offsets_validated_before_any_kernel(F):
    """Interior offsets are checked on the host: one past offsets[n] or a decreasing pair is
    GWO_ERR_INVALID_ARGUMENT (no kernel reads beyond the staged code units), and the handle stays usable."""
    import ctypes as C
    from flink_amd import _native as N
    lib = N.lib()
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1000), F.CountAggregate(), key_kind="string")
    chars = np.frombuffer("abcdef".encode("utf-16-le"), np.uint16).copy()
    ts = np.array([1, 2, 3], np.int64)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    for bad in ([0, 5, 2, 6], [0, 9, 9, 6], [0, 3, 1, 6]):
        off = np.array(bad, np.int64)
        st = lib.gwo_submit_utf16(op.handle, p(chars), p(off), p(ts), None, 3)
        assert N.STATUS_NAMES[st] == "GWO_ERR_INVALID_ARGUMENT", bad
    op.process_batch(["ab", "cd", "ab"], [1, 2, 3])
    op.end_input()
    assert sorted(op.output) == [("ab", 0, 1000, 2), ("cd", 0, 1000, 1)]
    op.close()
