"""GPU parity for sliding windows with allowedLateness > 0: per-element re-fire.

The reference adds a record to each of its windows that is not late (WindowOperator.java:386-427); every such
window whose maxTimestamp the watermark already passed FIREs at once (EventTimeTrigger.java:37-45), so one
row is emitted per (record, fired-but-not-cleaned window) with the window's contents including the record.  The
GPU keeps the panes of a window until its cleanup time and emits those rows from a segmented scan over the
batch's (key, window) pairs in arrival order (gwo_slide.cpp slide_refire_rows).  Checked against the oracle on
the reference's sliding streams replayed with lateness and on random late streams -- ring (invertible) and
recompute (min/max) fire strategies, several records of one key re-firing one window inside a batch, and a
checkpoint taken while fired windows still wait for their cleanup.  Integer aggregates: bit-exact.
"""
import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G

pytestmark = pytest.mark.gpu
LONG_MAX = (1 << 63) - 1


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    return flink_amd


@pytest.mark.parametrize("name", ["sliding_3s_1s", "side_output_lateness_sliding"])
@pytest.mark.parametrize("lateness", [500, 1_000, 2_000, 5_000])
def test_reference_sliding_streams_with_lateness(F, golden, name, lateness):
    """WindowOperatorTest's sliding streams (lateness 0 there) replayed with allowedLateness > 0."""
    s = next(x for x in golden["operator_streams"] if x["name"] == name)
    a = s["assigner"]
    want = O.WindowOperatorOracle(O.SlidingEventTimeWindows(a["size"], a["slide"], a["offset"]), O.SumLongAgg(),
                                  lateness, side_output=s["side_output"])
    got = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(a["size"], a["slide"], a["offset"]), F.SumAggregate(),
                              allowed_lateness=lateness, side_output_late_data=s["side_output"])
    for ev in s["events"]:
        if ev[0] == "e":
            want.process_element(ev[1], ev[2], ev[3])
            got.process_element(ev[1], ev[2], ev[3])
        else:
            want.process_watermark(ev[1])
            got.process_watermark(ev[1])
    want.end_input()
    got.end_input()
    assert sorted(got.output) == sorted((r.key, r.start, r.end, r.result) for r in want.output)
    assert sorted(got.side_output) == sorted(want.side_output)
    assert got.num_late_records_dropped == want.num_late_records_dropped
    got.close()


def _late_stream(seed, n, nkeys, span, disorder):
    rng = np.random.default_rng(seed)
    base = np.sort(rng.integers(0, span, n))
    t = (base + disorder - rng.integers(0, disorder, n) * (rng.random(n) < 0.3)).astype(np.int64)
    k = rng.integers(0, nkeys, n).astype(np.int64)
    v = rng.integers(-100, 100, n).astype(np.int64)
    return k, t, v


def _oracle(assigner, agg, k, t, v, batches, lateness):
    op = O.WindowOperatorOracle(assigner, agg, lateness)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(k[i]), int(t[i]), int(v[i]))
        op.process_watermark(wm)
        prev = end
    op.process_watermark(LONG_MAX)
    return sorted((r.key, r.start, r.end, r.result) for r in op.output), op.num_late_records_dropped


def _gpu(op, k, t, v, batches):
    prev = 0
    for end, wm in batches:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        prev = end
    op.end_input()
    rows, late = sorted(op.output), op.num_late_records_dropped
    op.close()
    return rows, late


CASES = [  # size, slide, offset, lateness, aggregate (ring: sum + count; recompute: min + max)
    (3_000, 1_000, 0, 1_500, "ring"),
    (3_000, 1_000, 0, 7_000, "ring"),
    (4_000, 1_500, -700, 2_500, "ring"),        # panes of 500, windows of 8 panes
    (6_000, 2_000, 300, 3_000, "recompute"),
    (10_000, 1_000, 0, 20_000, "recompute"),     # 10 windows per record, up to 20 fired ones re-fired
]


@pytest.mark.parametrize("size,slide,offset,lateness,kind", CASES)
def test_random_sliding_with_lateness(F, size, slide, offset, lateness, kind):
    k, t, v = _late_stream(size + lateness, 12_000, 40, 120_000, 3 * size)
    b = G.punctuated_watermarks(t, 400, 200)
    if kind == "ring":
        oagg, fagg = O.MultiAgg([O.SumLongAgg(), O.CountAgg()]), F.MultiAggregate(F.SumAggregate(), F.CountAggregate())
    else:
        oagg, fagg = O.MultiAgg([O.MinAgg(), O.MaxAgg()]), F.MultiAggregate(F.MinAggregate(), F.MaxAggregate())
    want, wl = _oracle(O.SlidingEventTimeWindows(size, slide, offset), oagg, k, t, v, b, lateness)
    got, gl = _gpu(F.GpuWindowOperator(F.SlidingEventTimeWindows.of(size, slide, offset), fagg,
                                       allowed_lateness=lateness), k, t, v, b)
    assert gl == wl
    assert len(got) == len(want)
    assert got == want


def test_many_refires_of_one_window_in_one_batch(F):
    """One key, one batch of late records all inside fired windows: each row carries the prefix of the batch's
    records of that window in arrival order."""
    k = np.full(300, 5, np.int64)
    k[::7] = 6
    rng = np.random.default_rng(4)
    t0 = np.arange(0, 12_000, 40, dtype=np.int64)
    v0 = rng.integers(1, 9, len(t0)).astype(np.int64)
    t1 = rng.integers(6_000, 12_000, 300).astype(np.int64)   # late for windows ending by 12 s, not cleaned
    v1 = rng.integers(1, 9, 300).astype(np.int64)
    kk = np.concatenate([np.full(len(t0), 5, np.int64), k])
    tt = np.concatenate([t0, t1])
    vv = np.concatenate([v0, v1])
    b = [(len(t0), 11_999), (len(kk), 12_500)]
    want, wl = _oracle(O.SlidingEventTimeWindows(3_000, 1_000), O.SumLongAgg(), kk, tt, vv, b, 4_000)
    got, gl = _gpu(F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3_000, 1_000), F.SumAggregate(),
                                       allowed_lateness=4_000), kk, tt, vv, b)
    assert got == want and gl == wl
    assert len(got) > 500   # ~14 window fires + two re-fire rows for most of the 300 late records


@pytest.mark.parametrize("kind", ["ring", "recompute"])
def test_sliding_lateness_checkpoint_continues_exactly(F, kind):
    """A checkpoint while fired windows still wait for their cleanup: their panes are rows; after restore,
    late records re-fire them with the restored contents."""
    size, slide, lateness = 4_000, 1_000, 3_000
    k, t, v = _late_stream(11, 10_000, 30, 80_000, 3 * size)
    b = G.punctuated_watermarks(t, 500, 100)
    if kind == "ring":
        oagg, mkagg = O.SumLongAgg(), F.SumAggregate
    else:
        oagg, mkagg = O.MinAgg(), F.MinAggregate
    want, wl = _oracle(O.SlidingEventTimeWindows(size, slide), oagg, k, t, v, b, lateness)
    mk = lambda: F.GpuWindowOperator(F.SlidingEventTimeWindows.of(size, slide), mkagg(), allowed_lateness=lateness)
    cut = len(b) // 2
    a = mk()
    prev = 0
    for end, wm in b[:cut]:
        a.process_batch(k[prev:end], t[prev:end], v[prev:end])
        a.process_watermark(wm)
        prev = end
    snap = a.snapshot_state()
    rows, late = list(a.output), a.num_late_records_dropped
    a.close()
    c = mk()
    c.restore_state(snap)
    for end, wm in b[cut:]:
        c.process_batch(k[prev:end], t[prev:end], v[prev:end])
        c.process_watermark(wm)
        prev = end
    c.end_input()
    assert sorted(rows + list(c.output)) == want
    assert late + c.num_late_records_dropped == wl
    c.close()
