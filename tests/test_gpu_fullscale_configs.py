"""GPU parity at the stated sizes of configs C2, C3 and C5 (BASELINE.json configs[1], [2], [4]).

The checkers are the C restatements of WindowOperator (oracle/window_oracle.c for tumbling,
oracle/window_oracle_sw.c for sliding and sessions), pinned against the record-at-a-time Python oracle in
tests/test_oracle_c.py and tests/test_oracle_c_sw.py.  Every watermark step is compared: the GPU's rows drained
after gwo_advance_watermark against the oracle's rows of that step -- per step the row count and an
order-independent checksum over every row's words (key, start, end, result bits), and row for row (sorted) on the
steps that hold the complete windows.  Integer results bit-exact; the C3 average is the double
(double)sum / count on both sides, compared bit for bit.

* C3: sliding 60 s / 1 s AverageAggregate over 10M keys, the whole stream of 200M records over 120 s, watermark
  every second (lag 1 s), then endInput: windows fill, slide and retire for another minute -- 10M-key pane tables,
  rehashes, window steps of ~10M rows each.
* C5: event-time sessions (30 s gap) over 100K keys and 10M records in bursts, arrival order ts + U[0, 5 s),
  watermark maxTs - 5 s - 1 every 10 s of event time; and the late variant (0.1 % of the events delayed a further
  [5 s, 15 s) + 30 s, so many of them are dropped and counted).
* C2: YSB-shaped 10 s tumbling count per campaign (10K ad ids -> 1K campaigns, key_mode 1 generator), 100M events
  in 1M-record batches with a watermark each (lag 1 s): the combine path's full regime (245 tiles per batch,
  speculative merge, multi-workgroup merge runs).
"""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import cbaseline

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
THREADS = 16


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    if not cbaseline.available():
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return flink_amd


def _gen(N, n, nkeys, span, disorder, key_mode=0, total=None, seed=42):
    import torch
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    v = torch.empty(n, dtype=torch.int64, device="cuda")
    spec = N.GwoGenSpec(seed, 0, total or n, nkeys, span, disorder, 0, 1000, N.DTYPE_INT64, key_mode)
    N.check(N.lib().gwo_generate(C.byref(spec), n, k.data_ptr(), t.data_ptr(), v.data_ptr(), None, 0))
    torch.cuda.synchronize()
    return k, t, v


def _drain(N, h, naggs):
    """Every pending row of h into fresh device int64 columns (float64 results as their bits)."""
    import torch
    N.check(N.lib().gwo_sync(h), h)
    cnt = C.c_int64()
    N.check(N.lib().gwo_output_count(h, C.byref(cnt)), h)
    m = cnt.value
    cols = [torch.empty(max(m, 1), dtype=torch.int64, device="cuda") for _ in range(3 + naggs)]
    if m:
        o = N.GwoOut()
        o.key, o.start, o.end = cols[0].data_ptr(), cols[1].data_ptr(), cols[2].data_ptr()
        for i in range(naggs):
            o.result[i] = cols[3 + i].data_ptr()
        got = C.c_int64()
        N.check(N.lib().gwo_drain(h, C.byref(o), m, C.byref(got)), h, "gwo_drain")
        assert got.value == m
    return [c[:m] for c in cols]


def _checksum(cols):
    """cbaseline.rows_checksum on the GPU: wrapping FNV-1a over each row's words, summed (int64 wraps like uint64)."""
    import torch
    if cols[0].numel() == 0:
        return 0
    h = torch.full_like(cols[0], 1469598103934665603)
    prime = 1099511628211
    for c in cols:
        h = torch.bitwise_xor(h, c) * prime
    return int(h.sum().item()) & ((1 << 64) - 1)


def _sorted(cols):
    import torch
    o1 = torch.argsort(cols[1], stable=True)
    o2 = torch.argsort(cols[0][o1], stable=True)
    idx = o1[o2]
    return [c[idx] for c in cols]


def _event_watermarks(ts_host, every, lag):
    """One watermark per `every` ms of the running max timestamp (a periodic BoundedOutOfOrderness generator)."""
    rm = np.maximum.accumulate(ts_host)
    cuts = np.flatnonzero(np.diff(rm // every)) + 1
    edges = [0] + cuts.tolist() + [len(ts_host)]
    return [(b, int(rm[b - 1]) - lag - 1) for a, b in zip(edges[:-1], edges[1:]) if b > a]


def _run_steps(N, h, key, ts, val, batches, naggs, keep):
    """Submit each batch, advance its watermark, drain; per step (count, checksum) and the rows of kept steps."""
    lib = N.lib()
    counts, sums, kept = [], [], {}
    prev = 0
    for b, (end, wm) in enumerate(batches):
        if end > prev:
            N.check(lib.gwo_submit(h, C.c_void_p(key.data_ptr() + 8 * prev), C.c_void_p(ts.data_ptr() + 8 * prev),
                                   C.c_void_p(val.data_ptr() + 8 * prev), end - prev), h, "submit")
        N.check(lib.gwo_advance_watermark(h, wm), h, "watermark")
        cols = _drain(N, h, naggs)
        counts.append(cols[0].numel())
        sums.append(_checksum(cols))
        if b in keep:
            kept[b] = cols
        prev = end
    return counts, sums, kept


def _compare(counts, sums, kept, want_rows, want_cs, rows, naggs):
    import torch
    nb = len(counts)
    assert counts == want_rows[:nb].tolist()
    assert want_rows[nb] == 0   # no records after the final watermark
    assert sums == [int(x) for x in want_cs[:nb]]
    for b, cols in kept.items():
        sel = rows[rows[:, -1] == b]
        want = _sorted([torch.from_numpy(np.ascontiguousarray(sel[:, c])).cuda() for c in range(3 + naggs)])
        got = _sorted(cols)
        for c in range(3 + naggs):
            assert torch.equal(got[c], want[c]), f"step {b} column {c}"


@pytest.mark.parametrize("layout", ["table", "log"])
def test_c3_sliding_10m_keys_full_scale(F, layout):
    import torch
    from flink_amd import _native as N
    R, span, nkeys = 200_000_000, 120_000, 10_000_000
    per = R * 1000 // span
    steps = span // 1000   # the whole 120-s stream: windows fill, slide and retire for another minute
    n = per * steps
    key, ts, val = _gen(N, n, nkeys, span, 1000, total=R)
    th = ts.cpu().numpy()
    wms, mx = [], -(1 << 63)
    for s in range(steps):
        mx = max(mx, int(th[s * per:(s + 1) * per].max()))
        wms.append(mx - 1000 - 1)
    batches = [((s + 1) * per, wms[s]) for s in range(steps)] + [(n, LONG_MAX)]
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(60_000, 1000), F.AverageAggregate(), max_parallelism=128,
                             state_layout=layout, expected_keys=nkeys if layout == "log" else 0)
    keep = {59, 60, 61, 119}   # watermark steps firing windows [-1 s, 59 s), [0, 60 s), [1 s, 61 s) and [59 s, 119 s)
    counts, sums, kept = _run_steps(N, op.handle, key, ts, val, batches, 1, keep)
    late_gpu = op.num_late_records_dropped
    op.close()
    kh, vh = key.cpu().numpy(), val.cpu().numpy()
    del key, ts, val
    torch.cuda.empty_cache()
    rows, srows, scs, late = cbaseline.run_sliding(kh, th, vh, batches, 60_000, 1000, 0, 0, ["avg"], THREADS, 128,
                                                   keep_steps=keep)
    assert late_gpu == late
    assert sum(counts) > 500_000_000 and max(counts[55:]) > 9_000_000   # ~10M rows per slide once windows fill
    _compare(counts, sums, kept, srows, scs, rows, 1)


@pytest.mark.parametrize("variant", ["ontime", "late"])
def test_c5_sessions_100k_keys_10m_records(F, variant):
    import torch
    from flink_amd import _native as N
    from oracle import gen as G
    late_fraction, extra = (0.0, 0) if variant == "ontime" else (0.001, 30_000)
    k, t, v, _ = G.session_stream(100_000, 10_000_000, gap=30_000, lag=5_000, seed=42, late_fraction=late_fraction,
                                  late_extra=extra)
    batches = _event_watermarks(t, 10_000, 5_000) + [(len(k), LONG_MAX)]
    key, ts, val = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v))
    agg = F.MultiAggregate(F.SumAggregate(), F.CountAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(30_000), agg, max_parallelism=128,
                             expected_keys=100_000)
    nb = len(batches)
    counts, sums, kept = _run_steps(N, op.handle, key, ts, val, batches, 4, set(range(nb)))
    late_gpu = op.num_late_records_dropped
    op.close()
    rows, srows, scs, late = cbaseline.run_sessions(k, t, v, batches, 30_000, 0, ["sum", "count", "min", "max"],
                                                    THREADS, 128, keep_steps=range(nb + 1))
    assert late_gpu == late
    if variant == "late":
        assert late > 1000
    assert sum(counts) > 800_000
    assert int(rows[:, 4].sum()) == len(k) - late   # every accepted record is in exactly one session row
    _compare(counts, sums, kept, srows, scs, rows, 4)


def test_sessions_600k_keys_multi_round_sweep(F):
    """A session table of 2^21 slots (600K keys): the watermark sweep's persistent grid (256 workgroups x 256 threads
    x 8 slots = 2^19 slots per round) takes four rounds per watermark, each with its own due-slot compaction and row
    reservation -- C5's 100K keys fit one round.  Rows per watermark and the final rows against the C restatement
    (MergingWindowSet.java:156-225, WindowOperator.java:430-473)."""
    import torch
    from flink_amd import _native as N
    from oracle import gen as G
    k, t, v, _ = G.session_stream(600_000, 6_000_000, gap=30_000, lag=5_000, seed=7)
    batches = _event_watermarks(t, 10_000, 5_000) + [(len(k), LONG_MAX)]
    key, ts, val = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v))
    agg = F.MultiAggregate(F.SumAggregate(), F.CountAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(30_000), agg, max_parallelism=128,
                             expected_keys=600_000)
    nb = len(batches)
    counts, sums, kept = _run_steps(N, op.handle, key, ts, val, batches, 4, set(range(nb)))
    late_gpu = op.num_late_records_dropped
    op.close()
    rows, srows, scs, late = cbaseline.run_sessions(k, t, v, batches, 30_000, 0, ["sum", "count", "min", "max"],
                                                    THREADS, 128, keep_steps=range(nb + 1))
    assert late_gpu == late
    assert int(rows[:, 4].sum()) == len(k) - late
    _compare(counts, sums, kept, srows, scs, rows, 4)


@pytest.mark.parametrize("pipelined", [False, True])
def test_c2_ysb_campaign_count_1m_batches(F, pipelined):
    """pipelined: gwo_set_pipelined_submit -- each batch's gather and speculative merge queue before the previous
    batch's readback is read (the bench's mode for C2); window crossings turn the chained verdicts down and both
    batches are redone in order."""
    import torch
    from flink_amd import _native as N
    n, every, span = 100_000_000, 1_000_000, 100_000
    key, ts, val = _gen(N, n, 1_000, span, 1000, key_mode=1)
    th = ts.cpu().numpy()
    batches, mx = [], -(1 << 63)
    for s in range(0, n, every):
        mx = max(mx, int(th[s:s + every].max()))
        batches.append((s + every, mx - 1000 - 1))
    batches.append((n, LONG_MAX))
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(10_000), F.CountAggregate(), max_parallelism=128,
                             expected_keys=1000)
    if pipelined:
        N.check(N.lib().gwo_set_pipelined_submit(op.handle, 1), op.handle)
    nb = len(batches)
    counts, sums, kept = _run_steps(N, op.handle, key, ts, val, batches, 1, set(range(nb)))
    late_gpu = op.num_late_records_dropped
    op.close()
    kh = key.cpu().numpy()
    del key, ts, val
    torch.cuda.empty_cache()
    # the tumbling C twin: rows (key, start, end, sum, min, max, count) of the whole stream, tagged per step below
    rows7, _, late = cbaseline.run_tumbling(kh, th, None, batches, 10_000, threads=THREADS, max_par=128)
    assert late_gpu == late
    got = _sorted([torch.cat([kept[b][c] for b in range(nb)]) for c in range(4)])
    want = _sorted([torch.from_numpy(np.ascontiguousarray(rows7[:, c])).cuda() for c in (0, 1, 2, 6)])
    assert got[0].numel() == want[0].numel() >= 9_000   # 1K campaigns x 10 windows
    for c in range(4):
        assert torch.equal(got[c], want[c])
    assert int(want[3].sum().item()) == n - late
    # per step: a window fires in the step whose watermark first reaches its end - 1
    wm = np.array([w for _, w in batches])
    ends = want[2].cpu().numpy()
    step_of = np.searchsorted(np.maximum.accumulate(wm), ends - 1, side="left")
    assert counts == np.bincount(step_of, minlength=nb).tolist()


@pytest.mark.parametrize("layout", ["table", "log"])
def test_c3_sliding_export_import_continue(F, layout):
    """C3's shape (sliding 60 s / 1 s AverageAggregate, a watermark every second, lag 1 s) through a checkpoint in the
    heap backend's layout: an operator runs 62 s of a 120-s stream, its state is exported (one accumulator per
    (key, window): WindowOperator's window-contents and timers), a fresh operator imports it at the checkpoint's
    watermark and runs the rest.  Every step's rows -- before and after the restore -- equal the uninterrupted C
    twin's (count and checksum per step, row for row on the steps that fire the first restored windows).  100K keys
    (the export holds ~60 entries per key: 6M window entries, the heap backend's own size for this state)."""
    import torch
    from flink_amd import _native as N
    R, span, nkeys = 12_000_000, 120_000, 100_000
    per = R * 1000 // span
    steps = span // 1000
    n = per * steps
    key, ts, val = _gen(N, n, nkeys, span, 1000, total=R, seed=7)
    th = ts.cpu().numpy()
    wms, mx = [], -(1 << 63)
    for s in range(steps):
        mx = max(mx, int(th[s * per:(s + 1) * per].max()))
        wms.append(mx - 1000 - 1)
    batches = [((s + 1) * per, wms[s]) for s in range(steps)] + [(n, LONG_MAX)]
    cut = 62
    mk = lambda: F.GpuWindowOperator(F.SlidingEventTimeWindows.of(60_000, 1000), F.AverageAggregate(),
                                     max_parallelism=128, state_layout=layout,
                                     expected_keys=nkeys if layout == "log" else 0)
    a = mk()
    keep_a, keep_b = {59, 60, 61}, {62, 63, 119}
    c1, s1, k1 = _run_steps(N, a.handle, key, ts, val, batches[:cut], 1, keep_a)
    blob, _, wm = a.export_heap_state()
    late_a = a.num_late_records_dropped
    a.close()
    assert wm == batches[cut - 1][1]
    b = mk()
    b.import_heap_state(blob, wm)
    assert b.state_size() > 50 * nkeys   # every key in (nearly) every open window
    del blob
    rest = [(e - batches[cut - 1][0], w) for e, w in batches[cut:]]
    off = batches[cut - 1][0]
    c2, s2, k2 = _run_steps(N, b.handle, key[off:], ts[off:], val[off:], rest, 1, {x - cut for x in keep_b})
    late_b = b.num_late_records_dropped
    b.close()
    kh, vh = key.cpu().numpy(), val.cpu().numpy()
    del key, ts, val
    torch.cuda.empty_cache()
    rows, srows, scs, late = cbaseline.run_sliding(kh, th, vh, batches, 60_000, 1000, 0, 0, ["avg"], THREADS, 128,
                                                   keep_steps=keep_a | keep_b)
    assert late_a + late_b == late
    kept = dict(k1)
    kept.update({x + cut: cols for x, cols in k2.items()})
    _compare(c1 + c2, s1 + s2, kept, srows, scs, rows, 1)
