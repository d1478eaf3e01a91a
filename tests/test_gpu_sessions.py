"""GPU parity for session windows with many in-flight sessions per key.

The reference's MergingWindowSet (flink-streaming-java/.../windowing/MergingWindowSet.java:156-225) keeps any
number of in-flight windows per key; the GPU entry holds a few inline and spills the rest into a pool
(gwo_session.hip).  These streams force spills, growth of spilled lists, merges across spilled sessions, re-fires
with allowedLateness, a checkpoint of spilled keys and their restore -- all against the oracle, bit-exact.

A batch's records are grouped by key in per-slot buckets of SESS_BKT_N records (gwo_internal.h SessLists); keys with
more records in one batch go through sess_long_kernel, and while many do the host groups with the radix sort instead.
GWO_SESS_LISTS=0/1 pins either grouping ("auto": the host's choice), read when an operator is created.
"""
import numpy as np
import pytest

from oracle import flink_oracle as O

pytestmark = pytest.mark.gpu
LONG_MAX = (1 << 63) - 1


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    return flink_amd


def _oracle(k, t, v, batches, gap, lateness):
    op = O.WindowOperatorOracle(O.EventTimeSessionWindows(gap), O.MultiAgg([O.SumLongAgg(), O.CountAgg()]), lateness)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(k[i]), int(t[i]), int(v[i]))
        op.process_watermark(wm)
        prev = end
    op.process_watermark(LONG_MAX)
    return sorted((r.key, r.start, r.end, r.result) for r in op.output), op.num_late_records_dropped


def _gpu(F, k, t, v, batches, gap, lateness, snapshot_at=None):
    mk = lambda: F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(gap),
                                     F.MultiAggregate(F.SumAggregate(), F.CountAggregate()), allowed_lateness=lateness)
    op = mk()
    rows, late = [], 0
    prev = 0
    for bi, (end, wm) in enumerate(batches):
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        prev = end
        if snapshot_at is not None and bi == snapshot_at:
            snap = op.snapshot_state()
            assert len(snap["key"]) == op.state_size()
            rows += list(op.output)
            late += op.num_late_records_dropped
            op.close()
            op = mk()
            op.restore_state(snap)
    op.end_input()
    rows += list(op.output)
    late += op.num_late_records_dropped
    op.close()
    return sorted(rows), late


def _hot_stream(rng, nsess, gap, extra_keys=50):
    """Key 7 gets `nsess` disjoint sessions (ts = i * 3 * gap), in shuffled order; other keys a few each."""
    ts_hot = np.arange(nsess, dtype=np.int64) * 3 * gap
    ts_hot = np.concatenate([ts_hot, ts_hot + gap // 2])           # two records per session
    k_hot = np.full(len(ts_hot), 7, np.int64)
    ko = rng.integers(100, 100 + extra_keys, 4 * extra_keys).astype(np.int64)
    to = rng.integers(0, nsess * 3 * gap, len(ko)).astype(np.int64)
    k = np.concatenate([k_hot, ko])
    t = np.concatenate([ts_hot, to])
    perm = rng.permutation(len(k))
    return k[perm], t[perm], rng.integers(-50, 50, len(k)).astype(np.int64)


def _mode(monkeypatch, mode):
    if mode == "auto":
        monkeypatch.delenv("GWO_SESS_LISTS", raising=False)
    else:
        monkeypatch.setenv("GWO_SESS_LISTS", mode)


@pytest.mark.parametrize("mode", ["auto", "0"])
@pytest.mark.parametrize("nsess", [17, 300])
def test_hot_key_many_inflight_sessions_one_batch(F, nsess, mode, monkeypatch):
    _mode(monkeypatch, mode)
    rng = np.random.default_rng(nsess)
    k, t, v = _hot_stream(rng, nsess, 1_000)
    batches = [(len(k), -(1 << 63))]   # every session in flight at once
    want, wl = _oracle(k, t, v, batches, 1_000, 0)
    got, gl = _gpu(F, k, t, v, batches, 1_000, 0)
    assert got == want and gl == wl
    assert sum(1 for r in got if r[0] == 7) == nsess


@pytest.mark.parametrize("mode", ["auto", "0"])
@pytest.mark.parametrize("lateness", [0, 2_500])
def test_spilled_sessions_grow_merge_and_refire(F, lateness, mode, monkeypatch):
    """Sessions of a hot key accumulate over several batches (the spilled list doubles), then bridging records
    merge runs of spilled sessions, and late records re-fire emitted ones."""
    _mode(monkeypatch, mode)
    rng = np.random.default_rng(3 + lateness)
    gap = 1_000
    parts = []
    for b in range(6):   # 6 batches of 40 fresh disjoint sessions of key 7
        base = b * 40 * 3 * gap
        ts = base + np.arange(40, dtype=np.int64) * 3 * gap
        parts.append(ts[rng.permutation(40)])
    # bridging records: ts in the middle of two consecutive sessions' gaps -> merges of 2-3 sessions
    bridge = (np.arange(0, 239, 3, dtype=np.int64) * 3 * gap + gap + gap // 2)[:30]
    parts.append(bridge[rng.permutation(len(bridge))])
    t = np.concatenate(parts)
    k = np.full(len(t), 7, np.int64)
    k[::11] = 9   # another key in between
    v = rng.integers(0, 100, len(t)).astype(np.int64)
    ends = np.cumsum([len(p) for p in parts])
    wms = [-(1 << 63)] * 6 + [int(t.max()) // 2]
    batches = list(zip(ends.tolist(), wms))
    # late records after the watermark: some re-fire (lateness > 0), some are dropped
    tl = np.array([100, 5 * 3 * gap + 10, int(t.max()) // 4], dtype=np.int64)
    k = np.concatenate([k, np.full(3, 7, np.int64)])
    t = np.concatenate([t, tl])
    v = np.concatenate([v, np.array([1, 2, 3], np.int64)])
    batches.append((len(k), int(t.max()) // 2 + 10))
    want, wl = _oracle(k, t, v, batches, gap, lateness)
    got, gl = _gpu(F, k, t, v, batches, gap, lateness)
    assert got == want and gl == wl


def test_spilled_sessions_checkpoint_and_restore(F):
    rng = np.random.default_rng(9)
    k, t, v = _hot_stream(rng, 120, 1_000)
    order = np.argsort(t, kind="stable")
    k, t, v = k[order], t[order], v[order]
    n = len(k)
    batches = [(n // 4, -(1 << 63)), (n // 2, int(t[n // 2 - 1]) - 5_000), (3 * n // 4, int(t[3 * n // 4 - 1]) - 5_000),
               (n, int(t[-1]) - 5_000)]
    want, wl = _oracle(k, t, v, batches, 1_000, 0)
    got, gl = _gpu(F, k, t, v, batches, 1_000, 0, snapshot_at=0)   # key 7 holds ~30+ in-flight sessions here
    assert got == want and gl == wl


@pytest.mark.parametrize("mode", ["auto", "0", "1"])
@pytest.mark.parametrize("lateness", [0, 3_000])
def test_overflowing_buckets_switch_grouping(F, mode, lateness, monkeypatch):
    """Batches where hundreds of keys bring more records than a bucket holds (the host switches to the sort after the
    first), then thin batches (back to the buckets), with watermarks between them: every grouping bit-exact."""
    _mode(monkeypatch, mode)
    rng = np.random.default_rng(11 + lateness)
    gap, ks, ts, batches, t0 = 1_000, [], [], [], 0
    for b in range(7):
        heavy = b < 3
        nkeys, per = (200, 24) if heavy else (3_000, 1)
        k = np.repeat(rng.integers(0, 5_000, nkeys), per).astype(np.int64)
        t = t0 + rng.integers(0, 8_000, len(k)).astype(np.int64)
        perm = rng.permutation(len(k))
        ks.append(k[perm])
        ts.append(t[perm])
        t0 += 6_000
        batches.append((sum(len(x) for x in ks), t0 - 4_000))
    k, t = np.concatenate(ks), np.concatenate(ts)
    v = rng.integers(-100, 100, len(k)).astype(np.int64)
    want, wl = _oracle(k, t, v, batches, gap, lateness)
    got, gl = _gpu(F, k, t, v, batches, gap, lateness)
    assert got == want and gl == wl
