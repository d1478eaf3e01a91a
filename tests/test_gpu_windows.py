"""GPU parity: libgwo.so's HIP kernels against the oracle (bit-exact for integers, 1e-6 relative
for float64 sums/averages -- the tolerance BASELINE.json's north_star states)."""
import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G
from oracle import vectorized as V

pytestmark = pytest.mark.gpu

LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1
FLOAT_RTOL = 1e-6
# tumbling windows run on both device state layouts: per-window hash tables, and the
# per-window partitioned record log folded in LDS at fire -- results must be identical
LAYOUTS = pytest.mark.parametrize("layout", ["table", "log"])


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    return flink_amd


def mk(F, a):
    if a["kind"] == "tumbling":
        return F.TumblingEventTimeWindows.of(a["size"], a["offset"])
    if a["kind"] == "sliding":
        return F.SlidingEventTimeWindows.of(a["size"], a["slide"], a["offset"])
    return F.EventTimeSessionWindows.withGap(a["gap"])


# ---- stateless kernels ---------------------------------------------------------------------------
def test_key_group_kernel_bit_exact(F):
    rng = np.random.default_rng(0)
    keys = np.concatenate([np.arange(-1000, 1000), rng.integers(LONG_MIN, LONG_MAX, 20000, dtype=np.int64),
                           np.array([LONG_MIN, LONG_MAX, 0, -1, 1 << 32, (1 << 32) - 1], dtype=np.int64)])
    for maxp, par in [(128, 1), (32768, 8), (10, 3), (1000, 7)]:
        kg, op = F.assign_key_groups(keys, maxp, par)
        want = np.array([O.assign_to_key_group(O.long_hash_code(int(k)), maxp) for k in keys])
        assert (kg == want).all()
        assert (op == want * par // maxp).all()
    kg, _ = F.assign_key_groups(np.arange(10), 128)
    assert kg.tolist() == [94, 86, 127, 113, 7, 126, 18, 113, 15, 51]


def test_key_group_kernel_string_keys(F, golden):
    """String keys: JDK String.hashCode over UTF-16 code units (surrogate pairs count as two units) ->
    murmur -> key group, pinned by the reference's own String-key vectors
    (RocksIncrementalCheckpointRescalingTest.java:55-92) and checked against the restatement."""
    g = golden["key_groups_string"]
    _, kg, op = F.assign_key_groups_strings(g["keys"], g["max_parallelism"], 1)
    assert kg.tolist() == g["groups"] and op.tolist() == [0] * len(g["keys"])
    rng = np.random.default_rng(1)
    alphabet = list("abcXYZ019 _-") + ["\u00e9", "\u4e2d", "\U0001F600", "\uffff"]
    keys = ["", "a", "campaign-42", "\U0001F600" * 3] + \
        ["".join(rng.choice(alphabet, rng.integers(0, 40))) for _ in range(3000)]
    for maxp, par in [(128, 1), (32768, 8), (10, 3)]:
        h, kg, op = F.assign_key_groups_strings(keys, maxp, par)
        want_h = [O.string_hash_code(k) for k in keys]
        want = np.array([O.assign_to_key_group(x, maxp) for x in want_h])
        assert h.tolist() == want_h
        assert (kg == want).all() and (op == want * par // maxp).all()


def test_key_group_kernel_int_keys(F):
    keys = np.arange(-5000, 5000)
    kg, _ = F.assign_key_groups(keys, 128, 1, key_kind="int")
    want = [O.assign_to_key_group(O.int_hash_code(int(k)), 128) for k in keys]
    assert kg.tolist() == want


def test_window_start_kernel(F, golden):
    cases = golden["window_start_with_offset"]["cases"]
    for ts, off, size, start in cases:
        assert F.window_starts(np.array([ts]), off, size)[0] == start
    rng = np.random.default_rng(1)
    ts = np.concatenate([rng.integers(-10**12, 10**12, 5000), np.arange(-50, 50)])
    for off, size in [(0, 7), (3, 7), (-2, 7), (0, 5000), (-100, 5000)]:
        got = F.window_starts(ts, off, size)
        want = [O.get_window_start_with_offset(int(t), off, size) for t in ts]
        assert got.tolist() == want


def test_generator_kernel_matches_numpy(F):
    import ctypes as C
    import torch
    from flink_amd import _native as N
    spec = G.GenSpec(seed=7, first_index=123, total_records=10**6, num_keys=5000, span_ms=60000,
                     disorder_ms=1000, value_range=1000)
    n = 100_000
    for vdt in ("int64", "float64"):
        spec.value_dtype = vdt
        k = torch.empty(n, dtype=torch.int64, device="cuda")
        t = torch.empty(n, dtype=torch.int64, device="cuda")
        v = torch.empty(n, dtype=torch.int64, device="cuda")
        gs = N.GwoGenSpec(spec.seed, spec.first_index, spec.total_records, spec.num_keys, spec.span_ms,
                          spec.disorder_ms, spec.t0, spec.value_range,
                          N.DTYPE_FLOAT64 if vdt == "float64" else N.DTYPE_INT64, 0)
        N.check(N.lib().gwo_generate(C.byref(gs), n, k.data_ptr(), t.data_ptr(), v.data_ptr(), None, 0))
        wk, wt, wv = G.generate(spec, n)
        assert (k.cpu().numpy() == wk).all() and (t.cpu().numpy() == wt).all()
        got_v = v.cpu().numpy().view(np.float64) if vdt == "float64" else v.cpu().numpy()
        assert (got_v == wv).all()


# ---- the reference's operator streams (WindowOperatorTest / examples) ----------------------------
def _run_stream(F, s, agg=None, layout="auto"):
    op = F.GpuWindowOperator(mk(F, s["assigner"]), agg or F.SumAggregate(), allowed_lateness=s["lateness"],
                             side_output_late_data=s["side_output"], state_layout=layout)
    for ev in s["events"]:
        if ev[0] == "e":
            op.process_element(ev[1], ev[2], ev[3])
        else:
            op.process_watermark(ev[1])
    return op


def _golden_streams(golden, kinds):
    return [s for s in golden["operator_streams"] if s["assigner"]["kind"] in kinds]


@pytest.mark.parametrize("name", ["sliding_3s_1s", "tumbling_3s", "side_output_lateness_tumbling",
                                  "side_output_lateness_sliding", "cleanup_time_overflow"])
def test_reference_operator_streams(F, golden, name):
    s = next(x for x in golden["operator_streams"] if x["name"] == name)
    op = _run_stream(F, s)
    assert sorted(op.output) == sorted(map(tuple, s["expected"]))
    assert sorted(op.side_output) == sorted(map(tuple, s.get("side", [])))
    assert op.num_late_records_dropped == s["late"]
    op.close()


@pytest.mark.parametrize("name", ["tumbling_3s", "side_output_lateness_tumbling", "cleanup_time_overflow"])
def test_reference_tumbling_streams_log_layout(F, golden, name):
    s = next(x for x in golden["operator_streams"] if x["name"] == name)
    if s["assigner"]["kind"] != "tumbling":
        pytest.skip("log layout serves tumbling windows")
    op = _run_stream(F, s, layout="log")
    assert sorted(op.output) == sorted(map(tuple, s["expected"]))
    assert sorted(op.side_output) == sorted(map(tuple, s.get("side", [])))
    assert op.num_late_records_dropped == s["late"]
    op.close()


def test_log_layout_multi_round_partitions(F):
    """One window fed by many small batches: the window's partitions (sized from its first batch)
    end up holding ~10x the LDS table, so the fire kernel folds them in hash rounds."""
    k, t, v, b = _c1(n=1_000_000, nkeys=200_000, every=10_000, lag=100, disorder=50)
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(60000), agg, state_layout="log")
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 60000, 0, [1, 2, 3])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


def test_log_layout_hot_key(F):
    """Half the records on one key: its partition is huge but holds one distinct key."""
    k, t, v, b = _c1(n=400_000, nkeys=20_000, every=20_000)
    k = k.copy()
    k[::2] = 7
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), F.MultiAggregate(F.SumAggregate(), F.CountAggregate()),
                             state_layout="log")
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), _ = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1, 0])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    op.close()


@pytest.mark.parametrize("vdt", ["int64", "float64"])
def test_table_layout_hot_keys_wave_prereduction(F, vdt):
    """Combine path (low cardinality): 3/4 of the records on two hot keys, so most waves fold runs of lanes of
    one key into one lane (ballot + masked wave reduction) before the LDS table; the workgroups' tables then
    fold into the batch's delta tables and the merge.  int64 bit-exact, float64 sums/avg within 1e-6."""
    k, t, v, b = _c1(n=600_000, nkeys=800, every=50_000, vdt=vdt, seed=7)
    k = k.copy()
    k[0::4] = 7
    k[1::4] = -3
    k[2::4] = 7
    agg = F.MultiAggregate(F.SumAggregate(vdt), F.AverageAggregate(vdt), F.MinAggregate(vdt), F.MaxAggregate(vdt))
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), agg, state_layout="table", expected_keys=1000)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1, 4, 2, 3],
                                                   value_is_f64=vdt == "float64")
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    want = _want(wk, ws, we, res)
    assert [g[:3] for g in got] == [w[:3] for w in want]
    gs = np.array([g[3:] for g in got])
    ws_ = np.array([w[3:] for w in want])
    if vdt == "int64":
        assert (gs[:, [0, 2, 3]] == ws_[:, [0, 2, 3]]).all()   # sum, min, max bit-exact
    else:
        np.testing.assert_allclose(gs[:, 0], ws_[:, 0], rtol=FLOAT_RTOL)
        assert (gs[:, 2:] == ws_[:, 2:]).all()
    np.testing.assert_allclose(gs[:, 1], ws_[:, 1], rtol=FLOAT_RTOL)   # avg
    assert op.num_late_records_dropped == late
    op.close()


def test_log_layout_rejected_for_sliding_min_and_sessions(F):
    """Sliding windows take the log layout only with invertible (int64 sum) aggregates (tests/test_gpu_sliding_log.py);
    sessions never."""
    from flink_amd import _native as N
    with pytest.raises(N.GwoError) as ei:
        F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3000, 1000), F.MinAggregate(), state_layout="log")
    assert ei.value.status_name == "GWO_ERR_UNSUPPORTED"
    with pytest.raises(N.GwoError) as ei:
        F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(3000), F.SumAggregate(), state_layout="log")
    assert ei.value.status_name == "GWO_ERR_UNSUPPORTED"


# ---- randomized parity against the oracle -------------------------------------------------------
def _c1(n=1_000_000, nkeys=10_000, every=10_000, lag=1000, vdt="int64", seed=42, disorder=1000):
    spec = G.GenSpec(seed=seed, total_records=n, num_keys=nkeys, span_ms=60000, disorder_ms=disorder,
                     value_range=1000, value_dtype=vdt)
    k, t, v = G.generate(spec, n)
    return k, t, v, G.punctuated_watermarks(t, every, lag)


def _run_batches(op, k, t, v, batches):
    prev = 0
    for end, wm in batches:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end] if v is not None else None)
        op.process_watermark(wm)
        prev = end
    op.end_input()


def _rows(op):
    return sorted(op.output)


def _want(k, s, e, res):
    cols = [x.tolist() for x in res]
    return sorted(zip(k.tolist(), s.tolist(), e.tolist(), *cols)) if len(cols) > 1 else \
        sorted(zip(k.tolist(), s.tolist(), e.tolist(), cols[0]))


def _final(batches):
    return batches + [(batches[-1][0], LONG_MAX)]


@LAYOUTS
def test_c1_tumbling_sum_bit_exact(F, layout):
    """Config 1: 1M records, 10K Long keys, 5 s tumbling sum, watermark every 10K records."""
    k, t, v, b = _c1()
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), F.SumAggregate(), state_layout=layout)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1])
    got = _rows(op)
    assert len(got) == len(wk) > 100_000
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


@pytest.mark.parametrize("lag", [0, 200])
@LAYOUTS
def test_tumbling_multi_agg_with_late_records(F, lag, layout):
    """sum/min/max/count with disorder larger than the lag: late drops must match exactly."""
    k, t, v, b = _c1(n=300_000, nkeys=50_000, every=3_000, lag=lag, disorder=1500, seed=3)
    v = v - 500
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(2000, 300),
                             F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate(), F.CountAggregate()), state_layout=layout)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 2000, 300, [1, 2, 3, 0])
    assert late > 0
    assert op.num_late_records_dropped == late
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    op.close()


@LAYOUTS
def test_tumbling_avg_int_bit_exact(F, layout):
    k, t, v, b = _c1(n=200_000, nkeys=3_000, every=5_000)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(10000), F.AverageAggregate(), state_layout=layout)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), _ = V.tumbling_lateness0(k, t, v, _final(b), 10000, 0, [4])
    assert _rows(op) == _want(wk, ws, we, res)   # (double)sum/count is exactly rounded on both sides
    op.close()


@LAYOUTS
def test_tumbling_float64_sum_avg_min_max(F, layout):
    k, t, v, b = _c1(n=200_000, nkeys=2_000, every=5_000, vdt="float64")
    agg = F.MultiAggregate(F.SumAggregate("float64"), F.AverageAggregate("float64"), F.MinAggregate("float64"),
                           F.MaxAggregate("float64"))
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), agg, state_layout=layout)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), _ = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1, 4, 2, 3], value_is_f64=True)
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    want = _want(wk, ws, we, res)
    assert [g[:3] for g in got] == [w[:3] for w in want]
    gs = np.array([g[3:] for g in got])
    ws_ = np.array([w[3:] for w in want])
    np.testing.assert_allclose(gs[:, :2], ws_[:, :2], rtol=FLOAT_RTOL)   # order-dependent float sums
    assert (gs[:, 2:] == ws_[:, 2:]).all()                                # min/max are exact
    op.close()


@LAYOUTS
def test_high_cardinality_growth_and_rehash(F, layout):
    """1M distinct keys in few windows: tables start small and must grow (rehash) mid-stream."""
    k, t, v, b = _c1(n=2_000_000, nkeys=1_000_000, every=400_000)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(20000), F.MultiAggregate(F.SumAggregate(), F.MaxAggregate()), state_layout=layout)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 20000, 0, [1, 3])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    op.close()


@LAYOUTS
def test_count_only_without_value_column(F, layout):
    k, t, _, b = _c1(n=100_000, nkeys=1000, every=10_000)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(10000), F.CountAggregate(), state_layout=layout)
    prev = 0
    for end, wm in b:
        op.process_batch(k[prev:end], t[prev:end], None)
        op.process_watermark(wm)
        prev = end
    op.end_input()
    (wk, ws, we, res), _ = V.tumbling_lateness0(k, t, None, _final(b), 10000, 0, [0])
    assert _rows(op) == _want(wk, ws, we, res)
    op.close()


@LAYOUTS
def test_extreme_keys_and_timestamps(F, layout):
    """Long.MIN_VALUE as a key (the table's EMPTY sentinel) and negative timestamps (Java '%')."""
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5), F.SumAggregate(), state_layout=layout)
    ref = O.WindowOperatorOracle(O.TumblingEventTimeWindows(5), O.SumLongAgg())
    events = [(LONG_MIN, -7, 1), (LONG_MIN, -6, 2), (LONG_MAX, -7, 3), (0, -12, 4), (-1, 3, 5), (LONG_MIN, 4, 6)]
    for key, ts, val in events:
        op.process_element(key, ts, val)
        ref.process_element(key, ts, val)
    op.end_input()
    ref.end_input()
    assert sorted(op.output) == O.rows_as_tuples(ref.output)
    op.close()


@LAYOUTS
def test_key_group_violation_fails_like_the_task(F, layout):
    from flink_amd import _native as N
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1000), F.SumAggregate(), max_parallelism=128,
                             key_group_range=(0, 63), state_layout=layout)
    keys = np.arange(100)
    kg = np.array([O.assign_to_key_group(O.long_hash_code(int(x)), 128) for x in keys])
    with pytest.raises(N.GwoError) as ei:
        op.process_batch(keys, np.full(100, 5), np.ones(100))
    assert ei.value.status_name == "GWO_ERR_KEY_GROUP" and (kg > 63).any()
    op.close()


@LAYOUTS
def test_no_timestamp_fails(F, layout):
    from flink_amd import _native as N
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1000), F.SumAggregate(), state_layout=layout)
    with pytest.raises(N.GwoError) as ei:
        op.process_batch(np.array([1, 2]), np.array([5, LONG_MIN]), np.array([1, 1]))
    assert ei.value.status_name == "GWO_ERR_NO_TIMESTAMP"
    op.close()


@LAYOUTS
def test_batch_boundaries_do_not_change_results(F, layout):
    """Same stream, different batch splits between the same watermarks -> identical output."""
    k, t, v, b = _c1(n=120_000, nkeys=5_000, every=6_000, lag=300, disorder=900)
    outs = []
    for split in (1, 7):
        op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(3000), F.SumAggregate(), state_layout=layout)
        prev = 0
        for end, wm in b:
            edges = np.linspace(prev, end, split + 1).astype(int)
            for a, c in zip(edges[:-1], edges[1:]):
                op.process_batch(k[a:c], t[a:c], v[a:c])
            op.process_watermark(wm)
            prev = end
        op.end_input()
        outs.append((_rows(op), op.num_late_records_dropped))
        op.close()
    assert outs[0] == outs[1]


# ---- sliding windows (panes; ring for invertible aggregates, recompute otherwise) ----------------
@pytest.mark.parametrize("size,slide,offset", [(60000, 1000, 0), (3000, 1000, 0), (3000, 2000, 500), (5000, 5000, 0),
                                               (7000, 3000, -1000)])
def test_sliding_avg_ring_bit_exact(F, size, slide, offset):
    """Config 3 shape (AverageAggregate over int64, exact int64 accumulators, double result)."""
    k, t, v, b = _c1(n=150_000, nkeys=20_000, every=5_000, lag=500, disorder=900, seed=5)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(size, slide, offset), F.AverageAggregate())
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), size, slide, offset, [4])
    got = _rows(op)
    assert len(got) == len(wk)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


def test_sliding_sum_count_ring(F):
    k, t, v, b = _c1(n=100_000, nkeys=3_000, every=2_000, lag=0, disorder=4500, seed=9)
    agg = F.MultiAggregate(F.SumAggregate(), F.CountAggregate())
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(4000, 1000), agg)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 4000, 1000, 0, [1, 0])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late > 0
    op.close()


def test_sliding_min_max_recompute(F):
    k, t, v, b = _c1(n=100_000, nkeys=5_000, every=4_000, lag=200, disorder=800, seed=11)
    agg = F.MultiAggregate(F.MinAggregate(), F.MaxAggregate(), F.SumAggregate())
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(6000, 2000, 0), agg)
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 6000, 2000, 0, [2, 3, 1])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


def test_sliding_float64_avg_recompute(F):
    k, t, v, b = _c1(n=80_000, nkeys=2_000, every=4_000, vdt="float64", seed=13)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(10000, 5000), F.AverageAggregate("float64"))
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), _ = V.sliding_lateness0(k, t, v, _final(b), 10000, 5000, 0, [4], value_is_f64=True)
    got = _rows(op)
    want = _want(wk, ws, we, res)
    assert [g[:3] for g in got] == [w[:3] for w in want]
    np.testing.assert_allclose([g[3] for g in got], [w[3] for w in want], rtol=FLOAT_RTOL)
    op.close()


def test_sliding_gap_in_stream(F):
    """Event time with a hole of many windows: empty windows are skipped, the ring re-anchors."""
    k1, t1, v1, _ = _c1(n=20_000, nkeys=500, seed=21)
    t2 = t1 + 10_000_000
    k = np.concatenate([k1, k1])
    t = np.concatenate([t1, t2])
    v = np.concatenate([v1, v1])
    b = G.punctuated_watermarks(t, 2_000, 1000)
    op = F.GpuWindowOperator(F.SlidingEventTimeWindows.of(3000, 1000), F.SumAggregate())
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.sliding_lateness0(k, t, v, _final(b), 3000, 1000, 0, [1])
    assert _rows(op) == _want(wk, ws, we, res)
    op.close()


# ---- session windows ----------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["session_reduce_3s", "session_list_3s", "side_output_lateness_session_zero",
                                  "session_lateness_10", "session_lateness_10000"])
def test_reference_session_streams(F, golden, name):
    s = next(x for x in golden["operator_streams"] if x["name"] == name)
    op = _run_stream(F, s)
    assert sorted(op.output) == sorted(map(tuple, s["expected"]))
    assert sorted(op.side_output) == sorted(map(tuple, s.get("side", [])))
    op.close()


def test_session_windowing_example(F, golden):
    s = next(x for x in golden["operator_streams"] if x["name"] == "session_windowing_example")
    op = _run_stream(F, s)
    assert sorted((k, st, r) for k, st, e, r in op.output) == sorted(map(tuple, s["expected_key_start_sum"]))
    op.close()


def _session_oracle(k, t, v, batches, gap, lateness=0, agg=None):
    op = O.WindowOperatorOracle(O.EventTimeSessionWindows(gap), agg or O.SumLongAgg(), lateness)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(k[i]), int(t[i]), int(v[i]))
        op.process_watermark(wm)
        prev = end
    op.process_watermark(LONG_MAX)
    return op


@pytest.mark.parametrize("late_fraction", [0.0, 0.01])
def test_c5_sessions_vs_oracle(F, late_fraction):
    """Config 5 shape: bursty sessions, 30 s gap, disorder < lag (plus a late variant)."""
    k, t, v, _ = G.session_stream(2_000, 60_000, late_fraction=late_fraction, seed=17, late_extra=30_000)
    b = G.punctuated_watermarks(t, 100, 5_000)
    ref = _session_oracle(k, t, v, b, 30_000, agg=O.MultiAgg([O.SumLongAgg(), O.CountAgg(), O.MaxAgg()]))
    op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(30_000),
                             F.MultiAggregate(F.SumAggregate(), F.CountAggregate(), F.MaxAggregate()))
    _run_batches(op, k, t, v, b)
    got = sorted(op.output)
    want = sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    assert len(got) == len(want) > 1000
    assert got == want
    assert op.num_late_records_dropped == ref.num_late_records_dropped
    if late_fraction:
        assert ref.num_late_records_dropped > 0
    op.close()


@pytest.mark.parametrize("lateness", [0, 3_000])
def test_sessions_out_of_order_with_lateness(F, lateness):
    """Heavy disorder relative to the lag, small gap: merges, bridging, late drops and (with
    allowedLateness) per-element re-fires, all in arrival order per key."""
    rng = np.random.default_rng(lateness + 3)
    n = 20_000
    k = rng.integers(0, 300, n)
    t = np.sort(rng.integers(0, 400_000, n)) + rng.integers(0, 6_000, n)
    v = rng.integers(0, 100, n)
    b = G.punctuated_watermarks(t, 500, 1_000)
    ref = _session_oracle(k, t, v, b, 2_000, lateness)
    op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(2_000), F.SumAggregate(), allowed_lateness=lateness)
    _run_batches(op, k, t, v, b)
    assert sorted(op.output) == sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    assert op.num_late_records_dropped == ref.num_late_records_dropped
    if lateness == 0:
        assert ref.num_late_records_dropped > 0
    op.close()


@pytest.mark.parametrize("split", [1, 3])
def test_sessions_pipelined_submit_matches_oracle(F, split):
    """Pipelined submission on sessions: a batch's readback is read at the next watermark, right after that
    watermark's sweep is queued (sized for every unread record opening a session), or at the next call; the sweep
    of the previous watermark stays running while the next batch queues.  Several batches between watermarks, merges,
    bridging and late drops, as the oracle sees them."""
    import ctypes as C
    import torch
    from flink_amd import _native as N
    lib = N.lib()
    rng = np.random.default_rng(17)
    n = 30_000
    k = rng.integers(0, 400, n)
    t = np.sort(rng.integers(0, 400_000, n)) + rng.integers(0, 6_000, n)
    v = rng.integers(0, 100, n)
    b = G.punctuated_watermarks(t, 600, 1_000)
    ref = _session_oracle(k, t, v, b, 2_000, 0)
    dk, dt, dv = (torch.from_numpy(np.ascontiguousarray(x, dtype=np.int64)).cuda() for x in (k, t, v))
    op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(2_000), F.SumAggregate())
    h = op.handle
    N.check(lib.gwo_set_pipelined_submit(h, 1), h)
    prev = 0
    for end, wm in b:
        edges = np.linspace(prev, end, split + 1).astype(int)
        for a, c in zip(edges[:-1].tolist(), edges[1:].tolist()):
            if c > a:
                N.check(lib.gwo_submit(h, C.c_void_p(dk.data_ptr() + 8 * a), C.c_void_p(dt.data_ptr() + 8 * a),
                                       C.c_void_p(dv.data_ptr() + 8 * a), int(c - a)), h)
        N.check(lib.gwo_advance_watermark(h, wm), h)
        prev = end
    assert prev == n
    N.check(lib.gwo_end_input(h), h)
    op._collect()
    assert sorted(op.output) == sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    assert op.num_late_records_dropped == ref.num_late_records_dropped > 0
    op.close()


def test_sessions_pipelined_columns_released_at_the_watermark_with_table_growth(F):
    """Pipelined sessions with every batch staged in ONE device buffer that is overwritten with garbage as soon as
    gwo_advance_watermark returns: the watermark waits for the batch's input-release word instead of its readback, and
    the next gwo_submit reads that readback after queueing its slot pass (gwo_session.cpp fire_session, insert_session).
    New keys keep arriving into a table sized for 64, so it grows several times with a batch pending: sizing runs on
    the readback's exact occupancy and, for the unread batch, the 0.9 safety bound (sess_ensure)."""
    import ctypes as C
    import torch
    from flink_amd import _native as N
    lib = N.lib()
    rng = np.random.default_rng(29)
    n = 40_000
    k = (np.arange(n) * 6_000 // n + rng.integers(0, 80, n)).astype(np.int64)   # the key range widens over time
    t = np.sort(rng.integers(0, 400_000, n)) + rng.integers(0, 6_000, n)
    v = rng.integers(0, 100, n)
    b = G.punctuated_watermarks(t, 700, 1_000)
    ref = _session_oracle(k, t, v, b, 2_000, 0)
    op = F.GpuWindowOperator(F.EventTimeSessionWindows.withGap(2_000), F.SumAggregate(), expected_keys=64)
    h = op.handle
    N.check(lib.gwo_set_pipelined_submit(h, 1), h)
    cap = max(e - s for (e, _), s in zip(b, [0] + [e for e, _ in b[:-1]]))
    dk, dt, dv = (torch.empty(cap, dtype=torch.int64, device="cuda") for _ in range(3))
    prev = 0
    for end, wm in b:
        m = end - prev
        if m:
            for d, x in ((dk, k), (dt, t), (dv, v)):
                d[:m].copy_(torch.from_numpy(np.ascontiguousarray(x[prev:end], dtype=np.int64)))
            torch.cuda.synchronize()   # complete before the call (gwo.h device-input readiness)
            N.check(lib.gwo_submit(h, C.c_void_p(dk.data_ptr()), C.c_void_p(dt.data_ptr()), C.c_void_p(dv.data_ptr()),
                                   int(m)), h)
        N.check(lib.gwo_advance_watermark(h, wm), h)
        for d in (dk, dt, dv):   # released: the batch's kernels no longer read these columns
            d.fill_(LONG_MIN)
        torch.cuda.synchronize()
        prev = end
    N.check(lib.gwo_end_input(h), h)
    op._collect()
    assert sorted(op.output) == sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    assert op.num_late_records_dropped == ref.num_late_records_dropped
    op.close()


def test_fast_division_full_int64_range(F):
    """window_start_f/fdiv_floor (double reciprocal + exact corrections) against Java semantics over
    the whole int64 range, including the extremes and sizes from 1 to Long.MAX_VALUE."""
    rng = np.random.default_rng(11)
    ts = np.concatenate([rng.integers(LONG_MIN, LONG_MAX, 20000, dtype=np.int64),
                         np.array([LONG_MIN + 1, LONG_MAX, LONG_MAX - 1, 0, -1, 1, -(1 << 62), 1 << 62],
                                  dtype=np.int64)])
    for size in [1, 2, 3, 7, 1000, 86_400_000, (1 << 40) + 7, (1 << 62) + 3, LONG_MAX]:
        for off in sorted({0, size // 3, -(size // 5)}):
            got = F.window_starts(ts, off, size)
            want = [O.get_window_start_with_offset(int(t), off, size) for t in ts]
            assert got.tolist() == want, (size, off)


# ---- multi-GPU path (RCCL keyBy shuffle), one rank on the box's one GPU -----------------------------
@LAYOUTS
def test_comm_single_rank_matches_oracle(F, layout):
    """gwo_comm_init with one rank: every batch goes through the partition kernels, the RCCL count and
    record exchange (send/recv to self) and the min-watermark all-reduce before the local insert."""
    import ctypes as C
    from flink_amd import _native as N
    lib = N.lib()
    k, t, v, b = _c1(n=300_000, nkeys=20_000, every=20_000)
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), agg, state_layout=layout)
    uid = (C.c_uint8 * N.COMM_ID_BYTES)()
    N.check(lib.gwo_comm_unique_id(uid))
    N.check(lib.gwo_comm_init(op.handle, uid, 1, 0), op.handle, "gwo_comm_init")
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1, 2, 3])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


@pytest.mark.parametrize("vranks,maxp,hot", [(2, 128, False), (3, 32768, False), (8, 32768, False), (8, 128, True),
                                              (8, 32768, "wide")])
def test_comm_virtual_ranks_log_route_matches_oracle(F, monkeypatch, vranks, maxp, hot):
    """The log layout's routed K1 (keyBy routing fused into the partition kernel): GWO_COMM_VIRTUAL=P makes a
    1-rank communicator route as GPU 0 of P -- the other GPUs' records leave through RCCL (to this rank itself)
    and come back as received records, so every record takes a rank's real multi-GPU data path once.  hot: one
    key carries half the records, overflowing its destination's send region (exact re-route).  wide: timestamps
    near 2^40 ms, so before the first watermark (timestamp base 0) every record exceeds the 20-B wire format's
    int32 range and travels as a 24-B wide record (its regions overflow: route-only re-run), and 1 % of the
    records sit 2^33 ms before the stream (wide records next to narrow ones, late drops)."""
    import ctypes as C
    from flink_amd import _native as N
    lib = N.lib()
    k, t, v, b = _c1(n=300_000, nkeys=20_000, every=20_000)
    if hot is True:
        k = k.copy()
        k[::2] = 12345
    if hot == "wide":   # watermarks from the in-range stream; then the far-past outliers (wide and late)
        t = t + (1 << 40)
        b = G.punctuated_watermarks(t, 20_000, 1000)
        t = t.copy()
        t[20_000::100] -= 1 << 33   # (after the first watermark: late)
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), agg, state_layout="log", max_parallelism=maxp)
    uid = (C.c_uint8 * N.COMM_ID_BYTES)()
    N.check(lib.gwo_comm_unique_id(uid))
    monkeypatch.setenv("GWO_COMM_VIRTUAL", str(vranks))
    N.check(lib.gwo_comm_init(op.handle, uid, 1, 0), op.handle, "gwo_comm_init")
    monkeypatch.delenv("GWO_COMM_VIRTUAL")
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1, 2, 3])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


def test_log_layout_far_future_records(F):
    """1 % of the records 2^33 ms (~100 days) after the stream: windows far beyond the batch's range fire at the
    final watermark; the log layout must not walk the empty windows in between."""
    k, t, v, b = _c1(n=200_000, nkeys=20_000, every=20_000)
    t = t.copy()
    t[50::100] += 1 << 33
    agg = F.MultiAggregate(F.SumAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), agg, state_layout="log")
    _run_batches(op, k, t, v, b)
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1, 3])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()


def test_comm_rejects_wrong_key_group_range(F):
    """With a communicator the handle's range must be its rank's computeKeyGroupRangeForOperatorIndex."""
    import ctypes as C
    from flink_amd import _native as N
    lib = N.lib()
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), F.SumAggregate(), max_parallelism=128,
                             key_group_range=(0, 63))
    uid = (C.c_uint8 * N.COMM_ID_BYTES)()
    N.check(lib.gwo_comm_unique_id(uid))
    st = lib.gwo_comm_init(op.handle, uid, 1, 0)   # rank 0 of 1 owns [0, 127], not [0, 63]
    assert st == N.GWO_ERR_INVALID_ARGUMENT
    op.close()


@pytest.mark.parametrize("par,maxp", [(8, 32768), (3, 128), (1, 128), (256, 32768)])
def test_partition_by_operator_routes_like_the_partitioner(F, par, maxp):
    """The exchange's route kernel: every record lands in the region of
    computeOperatorIndexForKeyGroup(assignToKeyGroup(key)) with its ts and value, none lost or duplicated."""
    import ctypes as C
    from flink_amd import _native as N
    rng = np.random.default_rng(par)
    n = 200_003
    k = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64)
    k[:1000] = 42   # a hot key: one destination gets far more than its share
    t = rng.integers(0, 1 << 40, n, dtype=np.int64)
    v = rng.integers(-1000, 1000, n, dtype=np.int64)
    _, dest = V.key_groups(k, maxp, par)
    cap = int(np.bincount(dest, minlength=par).max())
    out = np.zeros((par, cap, 3), np.int64)
    counts = np.zeros(par, np.int64)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    N.check(N.lib().gwo_partition_by_operator(p(k), p(t), p(v), n, N.KEY_LONG, maxp, par, p(out), cap, p(counts), 0))
    assert counts.tolist() == np.bincount(dest, minlength=par).tolist()
    for d in range(par):
        got = out[d, :counts[d]]
        want = np.stack([k[dest == d], t[dest == d], v[dest == d]], 1)
        assert sorted(map(tuple, got.tolist())) == sorted(map(tuple, want.tolist()))
    # a too-small region reports the true count and writes only `cap` records
    small = max(1, cap // 4)
    out2 = np.zeros((par, small, 3), np.int64)
    N.check(N.lib().gwo_partition_by_operator(p(k), p(t), p(v), n, N.KEY_LONG, maxp, par, p(out2), small, p(counts), 0))
    assert counts.tolist() == np.bincount(dest, minlength=par).tolist()


def test_log_layout_async_fire_overlaps_later_batches(F):
    """Fires run on their own stream while later batches are partitioned; the rows only become visible
    at drain.  Many windows, several fires in flight across batches, no host sync in between -- the
    results must still equal the oracle's, and discarding during a running fire drops its rows."""
    import ctypes as C
    from flink_amd import _native as N
    lib = N.lib()
    k, t, v, b = _c1(n=2_000_000, nkeys=300_000, every=50_000, lag=500, disorder=400)
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(2000), agg, state_layout="log", expected_keys=300_000)
    h = op.handle
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    prev = 0
    for end, wm in b:
        N.check(lib.gwo_submit(h, P(k[prev:end]), P(t[prev:end]), P(v[prev:end]), end - prev), h)
        N.check(lib.gwo_advance_watermark(h, wm), h)
        n = C.c_int64()
        N.check(lib.gwo_output_count(h, C.byref(n)), h)   # non-blocking: may not include a running fire
        prev = end
    N.check(lib.gwo_end_input(h), h)
    op._collect()
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 2000, 0, [1, 2, 3])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == _want(wk, ws, we, res)
    tot = C.c_int64()
    N.check(lib.gwo_rows_emitted(h, C.byref(tot)), h)
    assert tot.value == len(got)
    op.close()
    # discard while a fire may be running: none of those rows reach the output
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(2000), agg, state_layout="log", expected_keys=300_000)
    h = op.handle
    half = len(b) // 2
    prev = 0
    for end, wm in b[:half]:
        N.check(lib.gwo_submit(h, P(k[prev:end]), P(t[prev:end]), P(v[prev:end]), end - prev), h)
        N.check(lib.gwo_advance_watermark(h, wm), h)
        prev = end
    N.check(lib.gwo_discard_output(h), h)
    n = C.c_int64()
    N.check(lib.gwo_sync(h), h)
    N.check(lib.gwo_output_count(h, C.byref(n)), h)
    assert n.value == 0
    N.check(lib.gwo_rows_emitted(h, C.byref(tot)), h)
    assert tot.value > 0
    op.close()


def _pipelined_run(F, k, t, v, b, agg, size, offset=0, split=1, expected_keys=0, layout="log"):
    """Drives gwo_submit in pipelined mode with caller-owned DEVICE columns (the bench's mode): each
    watermark interval is cut into `split` batches, so K1 launches queue ahead of the previous batch's
    resolution; the watermark flushes only when the pending batch may hold a window it fires."""
    import ctypes as C
    import torch
    from flink_amd import _native as N
    lib = N.lib()
    dk, dt, dv = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v))
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(size, offset), agg, state_layout=layout,
                             expected_keys=expected_keys)
    h = op.handle
    N.check(lib.gwo_set_pipelined_submit(h, 1), h)
    prev = 0
    for end, wm in b:
        edges = np.linspace(prev, end, split + 1).astype(int)
        for a, c in zip(edges[:-1].tolist(), edges[1:].tolist()):
            if c > a:
                N.check(lib.gwo_submit(h, C.c_void_p(dk.data_ptr() + 8 * a), C.c_void_p(dt.data_ptr() + 8 * a),
                                       C.c_void_p(dv.data_ptr() + 8 * a), int(c - a)), h)
        N.check(lib.gwo_advance_watermark(h, wm), h)
        prev = end
    N.check(lib.gwo_end_input(h), h)
    op._collect()
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    late = op.num_late_records_dropped
    op.close()
    return got, late


@pytest.mark.parametrize("split", [1, 3])
def test_log_layout_pipelined_submit_matches_oracle(F, split):
    """Pipelined submission (K1 of batch i queued before batch i-1 is resolved) gives exactly the
    oracle's rows and late count, with late records and several batches between watermarks."""
    k, t, v, b = _c1(n=600_000, nkeys=200_000, every=20_000, lag=200, disorder=1500, seed=11)
    v = v - 500
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate(), F.CountAggregate())
    got, late = _pipelined_run(F, k, t, v, b, agg, 2000, 300, split=split, expected_keys=200_000)
    (wk, ws, we, res), want_late = V.tumbling_lateness0(k, t, v, _final(b), 2000, 300, [1, 2, 3, 0])
    assert want_late > 0 and late == want_late
    assert got == _want(wk, ws, we, res)


@pytest.mark.parametrize("split", [1, 3])
def test_combine_pipelined_submit_matches_oracle(F, split):
    """Pipelined submission on the combine path (table layout, few keys: gather + speculative merge): batch i's
    kernels queue before batch i-1's readback is read.  2-s windows with 20K-record watermark intervals cross a
    window every few batches, so chained verdicts are turned down and redone in order; late records are counted."""
    k, t, v, b = _c1(n=600_000, nkeys=1_000, every=20_000, lag=200, disorder=1500, seed=13)
    v = v - 500
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate(), F.CountAggregate())
    got, late = _pipelined_run(F, k, t, v, b, agg, 2000, 300, split=split, expected_keys=1_000, layout="table")
    (wk, ws, we, res), want_late = V.tumbling_lateness0(k, t, v, _final(b), 2000, 300, [1, 2, 3, 0])
    assert want_late > 0 and late == want_late
    assert got == _want(wk, ws, we, res)


def test_combine_pipelined_snapshot_and_error(F):
    """Pipelined combine path: a snapshot taken while a batch is still queued holds that batch (restored into a fresh
    operator, the rest of the stream gives the oracle's rows); a batch carrying a Long.MIN_VALUE timestamp is reported
    by the next call as GWO_ERR_NO_TIMESTAMP and fails the handle."""
    import ctypes as C
    import torch
    from flink_amd import _native as N
    lib = N.lib()
    k, t, v, b = _c1(n=200_000, nkeys=500, every=20_000, lag=200, disorder=1500, seed=23)
    dk, dt, dv = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (k, t, v))
    agg = lambda: F.MultiAggregate(F.SumAggregate(), F.CountAggregate())
    mk = lambda: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(2000), agg(), state_layout="table",
                                     expected_keys=500)
    sub = lambda h, a, c: N.check(lib.gwo_submit(h, C.c_void_p(dk.data_ptr() + 8 * a), C.c_void_p(dt.data_ptr() + 8 * a),
                                                 C.c_void_p(dv.data_ptr() + 8 * a), int(c - a)), h)
    op = mk()
    N.check(lib.gwo_set_pipelined_submit(op.handle, 1), op.handle)
    half = len(b) // 2
    prev = 0
    for end, wm in b[:half]:
        sub(op.handle, prev, end)
        N.check(lib.gwo_advance_watermark(op.handle, wm), op.handle)
        prev = end
    sub(op.handle, prev, b[half][0])   # queued, its readback unread: the snapshot completes it
    prev = b[half][0]
    snap = op.snapshot_state()
    op._collect()
    rows, late = list(op.output), op.num_late_records_dropped
    op.close()
    c = mk()
    c.restore_state(snap)
    h = c.handle
    N.check(lib.gwo_set_pipelined_submit(h, 1), h)
    for end, wm in [(b[half][0], b[half][1])] + b[half + 1:]:
        if end > prev:
            sub(h, prev, end)
        N.check(lib.gwo_advance_watermark(h, wm), h)
        prev = end
    N.check(lib.gwo_end_input(h), h)
    c._collect()
    (wk, ws, we, res), want_late = V.tumbling_lateness0(k, t, v, _final(b), 2000, 0, [1, 0])
    got = sorted((a_, s_, e_, *r) for a_, s_, e_, r in rows + list(c.output))
    assert got == _want(wk, ws, we, res)
    assert late + c.num_late_records_dropped == want_late
    c.close()
    # a bad timestamp in a pipelined batch: the next call reports it
    bad = t[:20_000].copy()
    bad[777] = LONG_MIN
    tb = torch.from_numpy(bad).cuda()
    e = mk()
    h = e.handle
    N.check(lib.gwo_set_pipelined_submit(h, 1), h)
    sub(h, 0, 20_000)
    st = lib.gwo_submit(h, C.c_void_p(dk.data_ptr()), C.c_void_p(tb.data_ptr()), C.c_void_p(dv.data_ptr()), 20_000)
    if st == 0:
        st = lib.gwo_sync(h)
    assert st == 2   # GWO_ERR_NO_TIMESTAMP
    assert lib.gwo_advance_watermark(h, 10_000) == 2   # the handle stays failed
    e.close()


def test_log_layout_pipelined_window_jumps_and_wide_batches(F):
    """Event time jumps many windows between batches (the pipelined K1's window-range guess is wrong and
    must be re-run) and batches spanning more windows than one K1 covers (multi-range resolution)."""
    rng = np.random.default_rng(5)
    parts = []
    t0 = 0
    for i in range(12):
        n = 20_000
        width = 50_000 if i % 3 == 0 else 3_000          # every third batch spans ~25 windows
        ts = t0 + np.sort(rng.integers(0, width, n))
        parts.append(ts)
        t0 = int(ts[-1]) + (40_000 if i % 4 == 1 else 500)   # jumps of 20 windows
    t = np.concatenate(parts).astype(np.int64)
    n = len(t)
    k = rng.integers(0, 30_000, n).astype(np.int64)
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    ends = np.cumsum([len(p) for p in parts])
    b = [(int(e), int(t[:e].max()) - 100 - 1) for e in ends]
    agg = F.MultiAggregate(F.SumAggregate(), F.MaxAggregate())
    got, late = _pipelined_run(F, k, t, v, b, agg, 2000, expected_keys=30_000)
    (wk, ws, we, res), want_late = V.tumbling_lateness0(k, t, v, _final(b), 2000, 0, [1, 3])
    assert late == want_late
    assert got == _want(wk, ws, we, res)


def test_log_layout_pipelined_error_reported_by_next_call(F):
    """A pipelined batch's Long.MIN_VALUE timestamp is reported by the next call on the handle, and the
    handle stays failed (gwo.h: gwo_set_pipelined_submit)."""
    import ctypes as C
    import torch
    from flink_amd import _native as N
    lib = N.lib()
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1000), F.SumAggregate(), state_layout="log")
    h = op.handle
    N.check(lib.gwo_set_pipelined_submit(h, 1), h)
    good = [torch.tensor(x, dtype=torch.int64, device="cuda") for x in ([1, 2], [5, 6], [1, 1])]
    bad = [torch.tensor(x, dtype=torch.int64, device="cuda") for x in ([1, 2], [5, LONG_MIN], [1, 1])]
    P = lambda x: C.c_void_p(x.data_ptr())
    assert lib.gwo_submit(h, *map(P, good), 2) == 0
    assert lib.gwo_submit(h, *map(P, bad), 2) == 0          # queued; resolved by the next call
    st = lib.gwo_sync(h)
    assert N.STATUS_NAMES.get(st) == "GWO_ERR_NO_TIMESTAMP"
    assert lib.gwo_submit(h, *map(P, good), 2) == st         # the handle stays failed
    op.close()


def _tumbling_oracle(k, t, v, batches, size, offset, lateness, agg, side_output=False):
    op = O.WindowOperatorOracle(O.TumblingEventTimeWindows(size, offset), agg, lateness, side_output=side_output)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(k[i]), int(t[i]), v[i].item())
        op.process_watermark(wm)
        prev = end
    op.process_watermark(LONG_MAX)
    return op


@pytest.mark.parametrize("side", [False, True])
@pytest.mark.parametrize("layout", ["table", "auto"])
@pytest.mark.parametrize("lateness", [1_500, 7_000])
def test_tumbling_per_element_refire_with_lateness(F, lateness, layout, side):
    """allowedLateness > 0: a record landing in an already-fired window (before its cleanup time) is
    added and EventTimeTrigger.onElement FIREs at once -- one row per such record with the window's
    contents including it, in arrival order (WindowOperator.java:393-406).  Heavy disorder relative to
    the lag, several records per (key, window) per batch, windows first created after the watermark
    passed their end, and late drops beyond the lateness -- all exactly as the loop restatement."""
    rng = np.random.default_rng(lateness)
    n = 12_000
    k = rng.integers(0, 60, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 200_000, n)) + rng.integers(0, 9_000, n)).astype(np.int64)
    v = rng.integers(-50, 100, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 400, 500)
    ref = _tumbling_oracle(k, t, v, b, 2_000, 300, lateness,
                           O.MultiAgg([O.SumLongAgg(), O.CountAgg(), O.MaxAgg(), O.MinAgg()]), side_output=side)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(2_000, 300),
                             F.MultiAggregate(F.SumAggregate(), F.CountAggregate(), F.MaxAggregate(), F.MinAggregate()),
                             allowed_lateness=lateness, state_layout=layout, side_output_late_data=side,
                             expected_keys=2_000_000 if layout == "auto" else 0)
    _run_batches(op, k, t, v, b)
    got = sorted(op.output)
    want = sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    # re-fires make duplicate (key, window) rows with growing contents: compare multisets
    assert len(got) == len(want)
    assert got == want
    n_windows = len({(r.key, r.start) for r in ref.output})
    assert len(want) > n_windows + 500          # many per-element re-fire rows
    if side:   # late records beyond the lateness go to the side output instead of being counted
        assert sorted(op.side_output) == sorted((r[0], r[1], r[2]) for r in ref.side_output) and op.side_output
        assert op.num_late_records_dropped == ref.num_late_records_dropped == 0
    else:
        assert op.num_late_records_dropped == ref.num_late_records_dropped > 0
    op.close()


def test_tumbling_refire_avg_and_float_sum(F):
    """Re-fire rows for AVG ((double) sum / count of an exact int64 accumulator: bit-exact) and a float64
    sum (order-dependent: within FLOAT_RTOL)."""
    rng = np.random.default_rng(9)
    n = 8_000
    k = rng.integers(0, 40, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 120_000, n)) + rng.integers(0, 6_000, n)).astype(np.int64)
    vi = rng.integers(0, 1000, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 300, 300)
    ref = _tumbling_oracle(k, t, vi, b, 3_000, 0, 4_000, O.AvgAgg())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(3_000), F.AverageAggregate(), allowed_lateness=4_000)
    _run_batches(op, k, t, vi, b)
    assert sorted(op.output) == sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    op.close()
    vf = rng.random(n) * 10.0
    ref = _tumbling_oracle(k, t, vf, b, 3_000, 0, 4_000, O.SumDoubleAgg())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(3_000), F.SumAggregate("float64"), allowed_lateness=4_000)
    _run_batches(op, k, t, vf, b)
    got = sorted(op.output, key=lambda r: (r[0], r[1], r[3]))
    want = sorted(((r.key, r.start, r.end, r.result) for r in ref.output), key=lambda r: (r[0], r[1], r[3]))
    assert [g[:3] for g in got] == [w[:3] for w in want]
    np.testing.assert_allclose([g[3] for g in got], [w[3] for w in want], rtol=FLOAT_RTOL)
    op.close()


@pytest.mark.parametrize("lateness", [0, 3_000])
def test_snapshot_restore_continues_exactly(F, lateness):
    """Checkpoint mid-stream (raw accumulators + watermark), restore into a fresh operator, continue:
    the rows before the checkpoint plus the restored operator's rows equal the uninterrupted oracle
    run (no window lost, none emitted twice; with allowedLateness the restored windows still re-fire)."""
    rng = np.random.default_rng(21 + lateness)
    n = 40_000
    k = rng.integers(0, 500, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 300_000, n)) + rng.integers(0, 4_000, n)).astype(np.int64)
    v = rng.integers(-100, 100, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 1_000, 1_000)
    agg_o = O.MultiAgg([O.SumLongAgg(), O.CountAgg(), O.MaxAgg()])
    ref = _tumbling_oracle(k, t, v, b, 5_000, 0, lateness, agg_o)
    mk_op = lambda: F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5_000),
                                        F.MultiAggregate(F.SumAggregate(), F.CountAggregate(), F.MaxAggregate()),
                                        allowed_lateness=lateness, state_layout="table")
    half = len(b) // 2
    a = mk_op()
    prev = 0
    for end, wm in b[:half]:
        a.process_batch(k[prev:end], t[prev:end], v[prev:end])
        a.process_watermark(wm)
        prev = end
    snap = a.snapshot_state()
    assert len(snap["key"]) == a.state_size() > 0 and snap["watermark"] == b[half - 1][1]
    rows, late = list(a.output), a.num_late_records_dropped
    a.close()
    c = mk_op()
    c.restore_state(snap)
    assert c.state_size() == len(snap["key"]) and c.current_watermark == snap["watermark"]
    _run_batches(c, k[prev:], t[prev:], v[prev:], [(e - prev, w) for e, w in b[half:]])
    got = sorted(rows + list(c.output))
    assert got == sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    assert late + c.num_late_records_dropped == ref.num_late_records_dropped
    c.close()


def test_snapshot_restore_rescales_by_key_group(F):
    """Rescale 1 -> 2 subtasks: both new subtasks restore the same snapshot and keep only their
    KeyGroupRange (computeKeyGroupRangeForOperatorIndex); each then receives its keys' records (as the
    keyBy partitioner routes them).  The union of outputs equals the single-operator oracle."""
    rng = np.random.default_rng(4)
    n = 30_000
    k = rng.integers(0, 2_000, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 200_000, n)) + rng.integers(0, 2_000, n)).astype(np.int64)
    v = rng.integers(0, 50, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 1_000, 2_000)
    ref = _tumbling_oracle(k, t, v, b, 4_000, 0, 0, O.SumLongAgg())
    half = len(b) // 2
    a = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(4_000), F.SumAggregate(), state_layout="table",
                            max_parallelism=128)
    prev = 0
    for end, wm in b[:half]:
        a.process_batch(k[prev:end], t[prev:end], v[prev:end])
        a.process_watermark(wm)
        prev = end
    snap = a.snapshot_state()
    rows = list(a.output)
    a.close()
    kg, _ = F.assign_key_groups(k, 128, 1)
    restored = 0
    for idx in range(2):
        r = F.compute_key_group_range_for_operator_index(128, 2, idx)
        op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(4_000), F.SumAggregate(), state_layout="table",
                                 max_parallelism=128, key_group_range=(r.start_key_group, r.end_key_group))
        op.restore_state([snap])
        restored += op.state_size()
        mine = (kg >= r.start_key_group) & (kg <= r.end_key_group)
        p0 = prev
        for end, wm in b[half:]:
            sel = np.nonzero(mine[p0:end])[0] + p0
            op.process_batch(k[sel], t[sel], v[sel])
            op.process_watermark(wm)
            p0 = end
        op.end_input()
        rows += list(op.output)
        op.close()
    assert restored == len(snap["key"])
    assert sorted(rows) == sorted((r.key, r.start, r.end, r.result) for r in ref.output)


@pytest.mark.parametrize("ring", [True, False])
def test_snapshot_restore_sliding_panes(F, ring):
    """Sliding windows checkpoint their panes; the restored operator anchors the next window to fire
    at the restored watermark and rebuilds the running ring total (invertible aggregates) from the panes."""
    rng = np.random.default_rng(8)
    n = 30_000
    k = rng.integers(0, 300, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 120_000, n)) + rng.integers(0, 1_500, n)).astype(np.int64)
    v = rng.integers(0, 1_000, n).astype(np.int64)
    b = G.punctuated_watermarks(t, 700, 1_500)
    agg_o = O.AvgAgg() if ring else O.MultiAgg([O.MinAgg(), O.MaxAgg()])
    mk = lambda: F.GpuWindowOperator(F.SlidingEventTimeWindows.of(6_000, 2_000),
                                     F.AverageAggregate() if ring else F.MultiAggregate(F.MinAggregate(), F.MaxAggregate()))
    ref = O.WindowOperatorOracle(O.SlidingEventTimeWindows(6_000, 2_000), agg_o)
    prev = 0
    for end, wm in b:
        for i in range(prev, end):
            ref.process_element(int(k[i]), int(t[i]), int(v[i]))
        ref.process_watermark(wm)
        prev = end
    ref.process_watermark(LONG_MAX)
    half = len(b) // 2
    a = mk()
    prev = 0
    for end, wm in b[:half]:
        a.process_batch(k[prev:end], t[prev:end], v[prev:end])
        a.process_watermark(wm)
        prev = end
    snap = a.snapshot_state()
    rows = list(a.output)
    a.close()
    c = mk()
    c.restore_state(snap)
    _run_batches(c, k[prev:], t[prev:], v[prev:], [(e - prev, w) for e, w in b[half:]])
    assert sorted(rows + list(c.output)) == sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    c.close()


def test_device_and_host_batches_alternate_after_free(F):
    """Batches alternate between device columns (freed after their call) and host columns: each call learns its
    own device ranges (Handle::known_device), so host columns -- possibly at addresses a freed device buffer had --
    are always staged, and every row equals the oracle's."""
    import torch
    k, t, v, b = _c1(n=200_000, nkeys=2_000, every=20_000)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), F.SumAggregate())
    prev = 0
    for i, (end, wm) in enumerate(b):
        if i % 2 == 0:
            dk, dt, dv = (torch.from_numpy(np.ascontiguousarray(x[prev:end])).cuda() for x in (k, t, v))
            op.process_device_batch(dk.data_ptr(), dt.data_ptr(), dv.data_ptr(), end - prev)
            torch.cuda.synchronize()
            del dk, dt, dv
            torch.cuda.empty_cache()
        else:
            op.process_batch(k[prev:end].copy(), t[prev:end].copy(), v[prev:end].copy())
        op.process_watermark(wm)
        prev = end
    op.end_input()
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, _final(b), 5000, 0, [1])
    assert _rows(op) == _want(wk, ws, we, res)
    assert op.num_late_records_dropped == late
    op.close()
