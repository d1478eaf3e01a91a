"""Watermark agreement on the GPU: the operator watermark follows StatusWatermarkValve
(flink-streaming-java/.../runtime/streamstatus/StatusWatermarkValve.java:86-101,163-181) -- a channel
watermark that does not increase is ignored and windows fire only when the min over channels grows --
and the multi-GPU min over ranks runs through RCCL even on one GPU (1-rank communicator rehearsing
P virtual ranks: the count exchange and the ncclMin all-reduce a real rank issues).

Expected outputs come from the oracle run on the same stream with the watermarks made monotone
(running max), which is what the valve forwards.  Integer aggregates: bit-exact.
"""
import ctypes as C
import time

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


def _stream(n=120_000, nkeys=5_000, every=4_000, lag=500, seed=3, disorder=900):
    spec = G.GenSpec(seed=seed, total_records=n, num_keys=nkeys, span_ms=60_000, disorder_ms=disorder,
                     value_range=1000)
    k, t, v = G.generate(spec, n)
    return k, t, v, G.punctuated_watermarks(t, every, lag)


def _regress(batches, rng):
    """Every third watermark moves back by up to 3 s (a channel reporting an older watermark)."""
    out = []
    for i, (end, wm) in enumerate(batches):
        out.append((end, wm - int(rng.integers(1, 3_000)) if i % 3 == 2 else wm))
    return out


def _monotone(batches):
    out, run = [], -(1 << 63)
    for end, wm in batches:
        run = max(run, wm)
        out.append((end, run))
    return out


def _drive(op, k, t, v, batches):
    prev, seen = 0, []
    for end, wm in batches:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        seen.append(op.current_watermark)
        prev = end
    op.end_input()
    return seen


@pytest.mark.parametrize("layout", ["table", "log"])
def test_regressing_watermark_ignored_tumbling(F, layout):
    rng = np.random.default_rng(1)
    k, t, v, b = _stream()
    bad = _regress(b, rng)
    good = _monotone(bad)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000),
                             F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate()), state_layout=layout)
    seen = _drive(op, k, t, v, bad)
    assert seen == [w for _, w in good]          # the operator watermark never moves back
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, good + [(len(k), LONG_MAX)], 5000, 0, [1, 2, 3])
    want = sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[r.tolist() for r in res]))
    assert sorted((a, s, e, *r) for a, s, e, r in op.output) == want
    assert op.num_late_records_dropped == late
    op.close()


def test_regressing_watermark_ignored_sliding(F):
    rng = np.random.default_rng(2)
    k, t, v, b = _stream(seed=5)
    bad = _regress(b, rng)
    good = _monotone(bad)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3000, 1000), F.AverageAggregate())
    _drive(op, k, t, v, bad)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, good + [(len(k), LONG_MAX)], 3000, 1000, 0, [4])
    assert sorted(op.output) == sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), res[0].tolist()))
    assert op.num_late_records_dropped == late
    op.close()


@pytest.mark.parametrize("lateness", [0, 2_000])
def test_regressing_watermark_ignored_sessions(F, lateness):
    rng = np.random.default_rng(3 + lateness)
    n = 15_000
    k = rng.integers(0, 200, n)
    t = np.sort(rng.integers(0, 300_000, n)) + rng.integers(0, 5_000, n)
    v = rng.integers(0, 100, n)
    bad = _regress(G.punctuated_watermarks(t, 500, 1_000), rng)
    good = _monotone(bad)
    ref = O.WindowOperatorOracle(O.EventTimeSessionWindows(2_000), O.SumLongAgg(), lateness)
    prev = 0
    for end, wm in good:
        for i in range(prev, end):
            ref.process_element(int(k[i]), int(t[i]), int(v[i]))
        ref.process_watermark(wm)
        prev = end
    ref.process_watermark(LONG_MAX)
    op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(2_000), F.SumAggregate(), allowed_lateness=lateness)
    _drive(op, k, t, v, bad)
    assert sorted(op.output) == sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    assert op.num_late_records_dropped == ref.num_late_records_dropped
    op.close()


def _virtual(F, op, monkeypatch, P):
    from flink_amd import _native as N
    lib = N.lib()
    uid = (C.c_uint8 * N.COMM_ID_BYTES)()
    N.check(lib.gwo_comm_unique_id(uid))
    monkeypatch.setenv("GWO_COMM_VIRTUAL", str(P))
    N.check(lib.gwo_comm_init(op.handle, uid, 1, 0), op.handle, "gwo_comm_init")
    monkeypatch.delenv("GWO_COMM_VIRTUAL")


def test_virtual_ranks_regressing_watermark(F, monkeypatch):
    """8 virtual ranks: every watermark goes through the ncclMin all-reduce, every batch through the RCCL count
    exchange; regressions are still ignored."""
    rng = np.random.default_rng(9)
    k, t, v, b = _stream(n=200_000, nkeys=20_000, every=20_000, lag=1000)
    bad = _regress(b, rng)
    good = _monotone(bad)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000),
                             F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate()), state_layout="log",
                             max_parallelism=32768)
    _virtual(F, op, monkeypatch, 8)
    seen = _drive(op, k, t, v, bad)
    assert seen == [w for _, w in good]
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, good + [(len(k), LONG_MAX)], 5000, 0, [1, 2, 3])
    want = sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[r.tolist() for r in res]))
    assert sorted((a, s, e, *r) for a, s, e, r in op.output) == want
    assert op.num_late_records_dropped == late
    op.close()


def test_virtual_ranks_after_restore(F, monkeypatch):
    """A subtask restored at watermark W (far from 0) attaches a communicator of 8 virtual ranks: the ranks agree
    on the wire records' timestamp base at gwo_comm_init (all-reduce of the restored watermarks), so the routed
    batches after the restore travel as 20-B records relative to W and decode to the same windows."""
    k, t, v, b = _stream(n=200_000, nkeys=20_000, every=10_000, lag=1000, seed=11)
    t = t + (1 << 40)
    b = G.punctuated_watermarks(t, 10_000, 1000)
    mk = lambda: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000),
                                     F.MultiAggregate(F.SumAggregate(), F.CountAggregate()), state_layout="log",
                                     max_parallelism=32768)
    half = len(b) // 2
    a = mk()
    prev = 0
    for end, wm in b[:half]:
        a.process_batch(k[prev:end], t[prev:end], v[prev:end])
        a.process_watermark(wm)
        prev = end
    snap = a.snapshot_state()
    rows, late = list(a.output), a.num_late_records_dropped
    a.close()
    c = mk()
    c.restore_state(snap)
    assert c.current_watermark == b[half - 1][1] > (1 << 40)
    _virtual(F, c, monkeypatch, 8)
    _drive(c, k[prev:], t[prev:], v[prev:], [(e - prev, w) for e, w in b[half:]])
    (wk, ws, we, res), want_late = V.tumbling_lateness0(k, t, v, b + [(len(k), LONG_MAX)], 5000, 0, [1, 0])
    want = sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[r.tolist() for r in res]))
    assert sorted((a_, s, e, *r) for a_, s, e, r in rows + list(c.output)) == want
    assert late + c.num_late_records_dropped == want_late
    c.close()


@pytest.mark.parametrize("defer", [1, 0])
def test_virtual_ranks_deferred_receives_snapshot(F, monkeypatch, defer):
    """Deferred receives (GWO_COMM_DEFER=1, the default): a routed batch's received records are inserted at the next
    routed batch, or earlier when a watermark may fire their windows or state is observed.  Watermarks every 2,500
    records against 5-s windows, so most watermarks leave the receives pending; a snapshot taken in the middle (with a
    receive pending) must hold them, and the restored subtask (no communicator) continues to the oracle's output.
    defer=0 runs the same stream with every batch's receives inserted inside its gwo_submit."""
    monkeypatch.setenv("GWO_COMM_DEFER", str(defer))
    k, t, v, b = _stream(n=150_000, nkeys=20_000, every=2_500, lag=700, seed=21)
    mk = lambda: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000),
                                     F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.CountAggregate()),
                                     state_layout="log", max_parallelism=32768)
    a = mk()
    _virtual(F, a, monkeypatch, 4)
    half = len(b) // 2
    prev = 0
    for end, wm in b[:half]:
        a.process_batch(k[prev:end], t[prev:end], v[prev:end])
        a.process_watermark(wm)
        prev = end
    a.process_batch(k[prev:b[half][0]], t[prev:b[half][0]], v[prev:b[half][0]])   # pending, no watermark after it
    prev = b[half][0]
    snap = a.snapshot_state()
    rows, late = list(a.output), a.num_late_records_dropped
    a.close()
    c = mk()
    c.restore_state(snap)
    _drive(c, k[prev:], t[prev:], v[prev:], [(e - prev, w) for e, w in b[half:]])
    (wk, ws, we, res), want_late = V.tumbling_lateness0(k, t, v, b + [(len(k), LONG_MAX)], 5000, 0, [1, 2, 0])
    want = sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[r.tolist() for r in res]))
    assert sorted((a_, s, e, *r) for a_, s, e, r in rows + list(c.output)) == want
    assert late + c.num_late_records_dropped == want_late
    c.close()


@pytest.mark.parametrize("async_wm,hold", [(0, 0), (1, 0), (1, 2)])
def test_virtual_ranks_routed_batches_without_host_waits(F, monkeypatch, async_wm, hold):
    """The routed exchange posts each batch's receives one batch behind, from counts the previous batch published to
    host-mapped memory, and the asynchronous watermark agreement applies the min the previous call queued: with the
    host issuing the operator's calls back to back (no pause between batches), a routed batch followed by a watermark
    that fires nothing never waits for its count exchange, and watermarks do not wait per batch.

    gwo_comm_wait_stats counts every host wait and its time, and sets apart flow control -- waits for a result still
    queued behind device work that had not run (a batch's counts behind its routed K1, an agreement behind the
    previous batch's count exchange): the exchange rotates over 3 send/receive slots, so a host more than two routed
    batches ahead of the device must wait before reusing a slot.  What remains is latency, not a round trip per
    batch: a count exchange (or an all-reduce) queued behind a K1 that just finished can still be in flight when the
    host comes back within its few microseconds (the calls are ~tens of us apart here).  Allowed, for counts and for
    asynchronous agreements alike: at most 1 wait in 4 batches and under 25 us of waiting per routed batch on average
    (the synchronous agreement waits for every one: its count is the number of calls).

    Flow control is bounded too: every 8th batch starts with the device caught up (gwo_sync), and such a batch and its
    watermark wait for nothing at all -- no count, watermark or flow-control wait.  Over the whole run the flow-control
    waits are at most one per routed batch each (the slot ring blocks a host at most once per submit).

    hold=2 (GWO_COMM_HOLD_COUNTS): every 4th batch's counts count as missing until 2 more batches were routed, the
    late-count interleaving in which a posted batch's received records would still sit in a receive slot that a later
    exchange reuses (the round-4 advisor's finding): the rows must still be the oracle's, and the held posts happen
    at slot reuse without protocol waits beyond one per held batch.
    The operator's calls are made directly (gwo_submit, gwo_advance_watermark, gwo_wait_fires): gwo_sync would complete
    the exchange on purpose.  60-s windows over a 40-s stream: no window fires before the end of input, which flushes
    the last receives; the output is the oracle's."""
    from flink_amd import _native as N
    lib = N.lib()
    if hold:
        monkeypatch.setenv("GWO_COMM_HOLD_COUNTS", str(hold))
    k, t, v, b = _stream(n=200_000, nkeys=20_000, every=5_000, lag=1000, seed=31)
    t = (t * 2) // 3   # 40-s span
    b = G.punctuated_watermarks(t, 5_000, 1000)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(60_000),
                             F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.CountAggregate()),
                             state_layout="log", max_parallelism=32768)
    _virtual(F, op, monkeypatch, 8)
    N.check(lib.gwo_comm_set_async_watermark(op.handle, async_wm), op.handle, "async watermark")
    h = op.handle
    starts = [0] + [e for e, _ in b[:-1]]
    cols = [tuple(np.ascontiguousarray(x[p0:e]) for x in (k, t, v)) for p0, (e, _) in zip(starts, b)]
    def waits():
        x = N.GwoCommWaits()
        N.check(lib.gwo_comm_wait_stats(h, C.byref(x)), h, "wait stats")
        return x
    caught_up = 0
    for i, (p0, (end, wm), (kk, tt, vv)) in enumerate(zip(starts, b, cols)):   # the operator's calls, rows in place
        if i % 8 == 7:   # the device caught up first: this batch and its watermark wait for nothing
            N.check(lib.gwo_sync(h), h, "sync")
            w0 = waits()
        N.check(lib.gwo_submit(h, kk.ctypes.data, tt.ctypes.data, vv.ctypes.data, end - p0), h, "submit")
        N.check(lib.gwo_advance_watermark(h, wm), h, "watermark")
        N.check(lib.gwo_wait_fires(h), h, "wait fires")
        if i % 8 == 7:
            w1 = waits()
            d = [getattr(w1, f) - getattr(w0, f) for f in ("count_waits", "flow_count_waits")]
            assert d == [0, 0], f"batch {i} after a sync: count / flow-control count waits {d}"
            if async_wm:   # (the synchronous agreement waits for its all-reduce by design)
                d = [getattr(w1, f) - getattr(w0, f) for f in ("wm_waits", "flow_wm_waits")]
                assert d == [0, 0], f"batch {i} after a sync: watermark / flow-control watermark waits {d}"
            caught_up += 1
        n = C.c_int64()
        N.check(lib.gwo_output_count(h, C.byref(n)), h)
        assert n.value == 0
    assert caught_up >= 3
    w = waits()
    print(f"routed {w.routed_batches}: count waits {w.count_waits} ({w.count_wait_ns / 1e3:.1f} us), watermark waits "
          f"{w.wm_waits} ({w.wm_wait_ns / 1e3:.1f} us); flow control {w.flow_count_waits} count, {w.flow_wm_waits} wm "
          f"({w.flow_wait_ns / 1e3:.1f} us)")
    assert w.routed_batches == len(b) and len(b) >= 30
    assert w.flow_count_waits <= len(b) and w.flow_wm_waits <= len(b), "more than one flow-control wait per batch"
    # protocol waits: counts (with their K1 finished) at most 1 in 4 batches (r06 on MI355X: 0, 5 and 2 in 40 for the
    # three variants) and a generous 25 us of waiting per routed batch on average (a shared box's scheduling noise
    # stays inside it)
    assert w.count_waits <= len(b) // 4, f"count waits with their K1 finished: {w.count_waits}"
    assert w.count_wait_ns < 25_000 * len(b), f"{w.count_wait_ns / 1e3:.1f} us waiting for counts"
    if async_wm:
        assert w.wm_waits <= len(b) // 4, f"asynchronous watermark agreements waited for: {w.wm_waits}"
        assert w.wm_wait_ns < 25_000 * len(b), f"{w.wm_wait_ns / 1e3:.1f} us waiting for agreements"
    else:
        assert w.wm_waits + w.flow_wm_waits >= len(b)   # the synchronous agreement waits for each all-reduce
    op.end_input()
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, b + [(len(k), LONG_MAX)], 60_000, 0, [1, 2, 0])
    want = sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[r.tolist() for r in res]))
    assert sorted((a, s, e, *r) for a, s, e, r in op.output) == want
    assert op.num_late_records_dropped == late
    op.close()
