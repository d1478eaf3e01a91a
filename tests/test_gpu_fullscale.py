"""GPU parity at the headline scale and across key-group shards.

* One full C4 window (BASELINE.json configs[3]: 100M keys, maxParallelism 32768, tumbling 10 s
  sum/min/max over int64, 16.7M records per 1-s watermark step) through the LOG layout, compared row for
  row with the C restatement of WindowOperator (oracle/window_oracle.c, 16 threads sharded by key group;
  pinned against the Python oracle in tests/test_oracle_c.py); and the whole 60-s C4 stream (six windows
  retire) against the C twin's output hash.
* Key-group sharding on one GPU: N = 2, 4, 8 handles, each owning
  KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex(32768, N, i)
  (flink-runtime/.../state/KeyGroupRangeAssignment.java:88-101), fed by gwo_partition_by_operator (the
  batch form of KeyGroupStreamPartitioner.selectChannel, KeyGroupStreamPartitioner.java:51-58).  The union
  of their outputs must equal the single-operator oracle -- the multi-GPU contract of SURVEY.md §8e
  without the RCCL transport.

Integer aggregates: bit-exact.
"""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import cbaseline
from oracle import vectorized as V

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    if not cbaseline.available():
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return flink_amd


def _gen(N, seed, first, total, nkeys, span, n, disorder=1000, vrange=1000):
    import torch
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    v = torch.empty(n, dtype=torch.int64, device="cuda")
    spec = N.GwoGenSpec(seed, first, total, nkeys, span, disorder, 0, vrange, N.DTYPE_INT64, 0)
    N.check(N.lib().gwo_generate(C.byref(spec), n, k.data_ptr(), t.data_ptr(), v.data_ptr(), None, 0))
    torch.cuda.synchronize()
    return k, t, v


def _watermarks(ts, bounds, lag):
    wms, run = [], -(1 << 63)
    for s, e in bounds:
        run = max(run, int(ts[s:e].max().item()))
        wms.append(run - lag - 1)
    return wms


def _drain_device(N, h, naggs):
    """Every pending row of handle h into fresh device tensors (gwo_drain into device columns)."""
    import torch
    n = C.c_int64()
    N.check(N.lib().gwo_rows_emitted(h, C.byref(n)), h)
    cnt = C.c_int64()
    N.check(N.lib().gwo_output_count(h, C.byref(cnt)), h)
    m = cnt.value
    cols = [torch.empty(max(m, 1), dtype=torch.int64, device="cuda") for _ in range(3 + naggs)]
    o = N.GwoOut()
    o.key, o.start, o.end = cols[0].data_ptr(), cols[1].data_ptr(), cols[2].data_ptr()
    for i in range(naggs):
        o.result[i] = cols[3 + i].data_ptr()
    got = C.c_int64()
    if m:
        N.check(N.lib().gwo_drain(h, C.byref(o), m, C.byref(got)), h, "gwo_drain")
        assert got.value == m
    return [c[:m] for c in cols]


def _sorted_rows(cols):
    """Rows ordered by (start, key): two stable sorts (keys are unique within a window)."""
    import torch
    key, start = cols[0], cols[1]
    o1 = torch.argsort(key, stable=True)
    o2 = torch.argsort(start[o1], stable=True)
    idx = o1[o2]
    return [c[idx] for c in cols]


def test_c4_full_window_log_layout_vs_c_twin(F):
    """Headline config at full scale: 11 watermark steps of 16,666,666 records (window [0, 10 s) complete,
    window [10 s, 20 s) partial), then endInput; every one of the ~87M rows equals the C twin's."""
    import torch
    from flink_amd import _native as N
    R, span, window, lag, maxp, nkeys = 1_000_000_000, 60_000, 10_000, 1_000, 32768, 100_000_000
    per = R * 1000 // span
    steps = 11
    n = per * steps
    key, ts, val = _gen(N, 42, 0, R, nkeys, span, n)
    bounds = [(i * per, (i + 1) * per) for i in range(steps)]
    wms = _watermarks(ts, bounds, lag)
    rec_per_window = R * window // span
    exp_keys = int(nkeys * (1.0 - np.exp(-rec_per_window / nkeys)))
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(window), agg, max_parallelism=maxp,
                             expected_keys=exp_keys)
    assert op.cfg.state_layout == N.STATE_AUTO
    lib, h = N.lib(), op.handle
    for (s, e), wm in zip(bounds, wms):
        N.check(lib.gwo_submit(h, C.c_void_p(key.data_ptr() + 8 * s), C.c_void_p(ts.data_ptr() + 8 * s),
                               C.c_void_p(val.data_ptr() + 8 * s), e - s), h, "submit")
        N.check(lib.gwo_advance_watermark(h, wm), h, "watermark")
    N.check(lib.gwo_end_input(h), h)
    late = C.c_int64()
    N.check(lib.gwo_late_dropped(h, C.byref(late)), h)
    got = _sorted_rows(_drain_device(N, h, 3))
    op.close()

    kh, th, vh = key.cpu().numpy(), ts.cpu().numpy(), val.cpu().numpy()
    del key, ts, val
    batches = [(e, w) for (_, e), w in zip(bounds, wms)] + [(n, LONG_MAX)]
    rows, _, want_late = cbaseline.run_tumbling(kh, th, vh, batches, window, threads=16, max_par=maxp)
    del kh, th, vh
    assert late.value == want_late
    assert got[0].numel() == rows.shape[0]
    assert rows.shape[0] > 80_000_000            # a full 100M-key window: ~81M distinct keys, plus window 1
    assert int(rows[:, 6].sum()) == n - want_late   # every accepted record is in exactly one row
    want = _sorted_rows([torch.from_numpy(np.ascontiguousarray(rows[:, c])).cuda() for c in range(6)])
    # per-key-group row counts over all 32768 key groups (KeyGroupRangeAssignment.java:60-73)
    kg, _ = V.key_groups(rows[:, 0], maxp)
    assert np.count_nonzero(np.bincount(kg, minlength=maxp)) == maxp
    for c, name in enumerate(["key", "start", "end", "sum", "min", "max"]):
        assert torch.equal(got[c], want[c]), f"column {name} differs"


def _gpu_row_checksum(cols):
    """cbaseline.row_checksum on the device: wrapping sum over rows of an FNV-1a-style hash of the row's words."""
    import torch
    h = torch.full_like(cols[0], 1469598103934665603)
    for c in cols:
        h = (h ^ c) * 1099511628211   # int64 arithmetic wraps like the C twin's uint64
    return int(h.sum().item()) % (1 << 64)


def test_c4_whole_stream_six_windows_vs_c_twin(F):
    """The whole C4 stream: 1e9 records over 60 s of event time in 60 watermark steps, so six 10-s windows fill,
    fire and retire through the LOG layout (the chunk pool recycled five times) plus the end-of-input fire.  Every
    step's rows (key, start, end, sum, min, max, count) are drained and hashed on the device; the sum of the row
    hashes over the stream and the late count equal the C twin's (window_oracle.c emit(): the same hash).  The
    row-for-row comparison of one full window is test_c4_full_window_log_layout_vs_c_twin."""
    import torch
    from flink_amd import _native as N
    R, span, window, lag, maxp, nkeys = 1_000_000_000, 60_000, 10_000, 1_000, 32768, 100_000_000
    per = R * 1000 // span
    steps = span // 1000
    n = per * steps
    key, ts, val = _gen(N, 42, 0, R, nkeys, span, n)
    bounds = [(i * per, (i + 1) * per) for i in range(steps)]
    wms = _watermarks(ts, bounds, lag)
    rec_per_window = R * window // span
    exp_keys = int(nkeys * (1.0 - np.exp(-rec_per_window / nkeys)))
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate(), F.CountAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(window), agg, max_parallelism=maxp,
                             expected_keys=exp_keys)
    lib, h = N.lib(), op.handle
    cs, rows, fires = 0, 0, 0
    for (s, e), wm in zip(bounds, wms):
        N.check(lib.gwo_submit(h, C.c_void_p(key.data_ptr() + 8 * s), C.c_void_p(ts.data_ptr() + 8 * s),
                               C.c_void_p(val.data_ptr() + 8 * s), e - s), h, "submit")
        N.check(lib.gwo_advance_watermark(h, wm), h, "watermark")
        cols = _drain_device(N, h, 4)
        if cols[0].numel():
            fires += 1
            rows += cols[0].numel()
            cs = (cs + _gpu_row_checksum(cols)) % (1 << 64)
        del cols
    N.check(lib.gwo_end_input(h), h)
    cols = _drain_device(N, h, 4)
    rows += cols[0].numel()
    cs = (cs + _gpu_row_checksum(cols)) % (1 << 64)
    del cols
    late = C.c_int64()
    N.check(lib.gwo_late_dropped(h, C.byref(late)), h)
    op.close()
    kh, th, vh = key.cpu().numpy(), ts.cpu().numpy(), val.cpu().numpy()
    del key, ts, val
    torch.cuda.empty_cache()
    batches = [(e, w) for (_, e), w in zip(bounds, wms)] + [(n, LONG_MAX)]
    _, want_cs, want_late = cbaseline.run_tumbling(kh, th, vh, batches, window, threads=16, max_par=maxp, rows=False)
    assert fires == 5                      # windows [0, 10 s) .. [40 s, 50 s) fire at watermark steps; the sixth at end
    assert rows > 5 * 80_000_000
    assert late.value == want_late
    assert cs == want_cs


@pytest.mark.parametrize("layout", ["log", "table"])
@pytest.mark.parametrize("nshards", [2, 4, 8])
def test_sharded_union_single_gpu(F, nshards, layout):
    """N key-group shards on one GPU, records routed by gwo_partition_by_operator: union == oracle."""
    import torch
    from flink_amd import _native as N
    total, nkeys, span, window, lag, maxp = 6_000_000, 2_000_000, 30_000, 5_000, 1_000, 32768
    per = 500_000
    key, ts, val = _gen(N, 7 + nshards, 0, total, nkeys, span, total)
    bounds = [(i, min(i + per, total)) for i in range(0, total, per)]
    wms = _watermarks(ts, bounds, lag)
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    ops = []
    for i in range(nshards):
        r = F.compute_key_group_range_for_operator_index(maxp, nshards, i)
        ops.append(F.GpuWindowOperator(F.TumblingEventTimeWindows.of(window), agg, max_parallelism=maxp,
                                       key_group_range=(r.start_key_group, r.end_key_group),
                                       expected_keys=nkeys // nshards, state_layout=layout))
    lib = N.lib()
    cap = per
    routed = torch.empty(nshards * cap * 3, dtype=torch.int64, device="cuda")
    counts = np.zeros(nshards, np.int64)
    for (s, e), wm in zip(bounds, wms):
        m = e - s
        N.check(lib.gwo_partition_by_operator(C.c_void_p(key.data_ptr() + 8 * s), C.c_void_p(ts.data_ptr() + 8 * s),
                                              C.c_void_p(val.data_ptr() + 8 * s), m, N.KEY_LONG, maxp, nshards,
                                              C.c_void_p(routed.data_ptr()), cap,
                                              counts.ctypes.data_as(C.c_void_p), 0), None, "partition")
        assert counts.sum() == m and (counts <= cap).all()
        reg = routed.view(nshards, cap, 3)
        for i, op in enumerate(ops):
            c = int(counts[i])
            if c:
                # the columns are produced on torch's stream and may still be in flight: process_device_batch names
                # that stream to gwo_wait_stream (gwo.h "Device-input readiness") and keeps the tensors alive until
                # the operator's next call returns (the borrow).  r05 failed here once (4 rows short, late counts
                # equal) when K1 on the handle's non-blocking stream could read the columns before the copies --
                # test_device_input_waits_for_producer_stream shows that race deterministically.
                cols = [reg[i, :c, j].contiguous() for j in range(3)]
                op.process_device_batch(*(x.data_ptr() for x in cols), c, keep=cols)
        for op in ops:
            N.check(lib.gwo_advance_watermark(op.handle, wm), op.handle)
    parts, late = [], 0
    for op in ops:
        N.check(lib.gwo_end_input(op.handle), op.handle)
        parts.append([c.cpu().numpy() for c in _drain_device(N, op.handle, 3)])
        late += op.num_late_records_dropped
        op.close()
    got = np.stack([np.concatenate([p[c] for p in parts]) for c in range(6)], axis=1)
    kh, th, vh = key.cpu().numpy(), ts.cpu().numpy(), val.cpu().numpy()
    batches = [(e, w) for (_, e), w in zip(bounds, wms)] + [(total, LONG_MAX)]
    rows, _, want_late = cbaseline.run_tumbling(kh, th, vh, batches, window, threads=8, max_par=maxp)
    assert late == want_late
    want = rows[:, :6]
    order = lambda a: a[np.lexsort((a[:, 0], a[:, 1]))]
    assert got.shape == want.shape
    assert (order(got) == order(want)).all()
    # every shard only emitted keys of its own key-group range
    for i, p in enumerate(parts):
        r = F.compute_key_group_range_for_operator_index(maxp, nshards, i)
        kg, _ = V.key_groups(p[0], maxp)
        assert ((kg >= r.start_key_group) & (kg <= r.end_key_group)).all()
