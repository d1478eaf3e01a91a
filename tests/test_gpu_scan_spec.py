"""GPU: the speculative two-pass insert of the table layout (gwo_runtime.cpp insert_speculative; the scan's last
workgroup decides whether the direct insert queued behind it runs).  Pre-aggregation off (GWO_PREAGG=0) sends
every tumbling batch down this path.  Each case checks the verdict's fallbacks against the oracle: batches moving
to new windows (no hint table yet), tables that must grow, late records with and without the side output, a
key-group violation after accepted batches (the batch is rejected, the state stays), re-fires with
allowedLateness > 0, and -- at the end -- that the fast path really ran (GWO_SCAN_SPEC=0 gives the same rows).
"""
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


def _stream(n, nkeys, every, lag, disorder, seed=7):
    spec = G.GenSpec(seed=seed, total_records=n, num_keys=nkeys, span_ms=60000, disorder_ms=disorder,
                     value_range=1000)
    k, t, v = G.generate(spec, n)
    return k, t, v, G.punctuated_watermarks(t, every, lag)


def _timed_kernels(op, F):
    from flink_amd import _native as N
    import ctypes as C
    la, ms, it = C.c_int64(), C.c_double(), C.c_int64()
    op._lib.gwo_kernel_stats(op.handle, N.KERNEL_SCAN, C.byref(la), C.byref(ms), C.byref(it))
    return la.value


@pytest.mark.parametrize("spec", ["1", "0"])
def test_small_batches_match_oracle(F, monkeypatch, spec):
    """C1's shape (10K-record batches over 10K keys, 5 s windows) with growth: 50K keys, tables start small."""
    monkeypatch.setenv("GWO_PREAGG", "0")
    monkeypatch.setenv("GWO_SCAN_SPEC", spec)
    k, t, v, b = _stream(300_000, 50_000, 3_000, 200, 1500)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5000), F.MultiAggregate(F.SumAggregate(), F.MaxAggregate()))
    prev = 0
    for end, wm in b:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        prev = end
    op.end_input()
    (wk, ws, we, res), late = V.tumbling_lateness0(k, t, v, b + [(b[-1][0], LONG_MAX)], 5000, 0, [1, 3])
    got = sorted((a, s, e, *r) for a, s, e, r in op.output)
    assert got == sorted(zip(wk.tolist(), ws.tolist(), we.tolist(), *[x.tolist() for x in res]))
    assert op.num_late_records_dropped == late > 0
    op.close()


@pytest.mark.parametrize("side", [False, True])
def test_late_records_and_refires(F, monkeypatch, side):
    """allowedLateness 1 s: re-fire batches turn the verdict down (the host path emits them per element); late
    records go to the side output or are counted, never twice across a turned-down speculation."""
    monkeypatch.setenv("GWO_PREAGG", "0")
    k, t, v, b = _stream(120_000, 3_000, 4_000, 300, 3000, seed=11)
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(3000), F.SumAggregate(), allowed_lateness=1000,
                             side_output_late_data=side)
    ref = O.WindowOperatorOracle(O.TumblingEventTimeWindows(3000), O.SumLongAgg(), 1000, side_output=side)
    prev = 0
    for end, wm in b:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        for i in range(prev, end):
            ref.process_element(int(k[i]), int(t[i]), int(v[i]))
        ref.process_watermark(wm)
        prev = end
    op.end_input()
    ref.end_input()
    assert sorted(op.output) == O.rows_as_tuples(ref.output)
    if side:
        assert sorted(op.side_output) == sorted(ref.side_output) and len(ref.side_output) > 0
    else:
        assert op.num_late_records_dropped == ref.num_late_records_dropped > 0
    op.close()


def test_key_group_violation_after_speculated_batches(F, monkeypatch):
    """Accepted batches first (the fast path), then a batch with a key outside the subtask's KeyGroupRange: the
    verdict is no, the host path rejects the batch with GWO_ERR_KEY_GROUP."""
    from flink_amd import _native as N
    monkeypatch.setenv("GWO_PREAGG", "0")
    maxp = 128
    keys = np.arange(20_000, dtype=np.int64)
    kg = np.array([O.assign_to_key_group(O.long_hash_code(int(x)), maxp) for x in keys])
    mine, other = keys[kg <= 63], keys[kg > 63]
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(1000), F.SumAggregate(), max_parallelism=maxp,
                             key_group_range=(0, 63))
    for i in range(4):
        op.process_batch(mine[:5000], np.full(5000, 100 + i), np.ones(5000))
    bad = np.concatenate([mine[:100], other[:1]])
    with pytest.raises(N.GwoError) as ei:
        op.process_batch(bad, np.full(len(bad), 200), np.ones(len(bad)))
    assert ei.value.status_name == "GWO_ERR_KEY_GROUP"
    op.close()


def test_fast_path_runs(F, monkeypatch):
    """The speculation is taken: one scan per batch (a turned-down speculation would scan twice)."""
    monkeypatch.setenv("GWO_PREAGG", "0")
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(60_000), F.SumAggregate())
    op._lib.gwo_set_profiling(op.handle, 1)
    rng = np.random.default_rng(1)
    op.process_batch(rng.integers(0, 1000, 5000), np.full(5000, 10), np.ones(5000))   # creates the table
    op._lib.gwo_reset_stats(op.handle)
    for i in range(10):
        op.process_batch(rng.integers(0, 1000, 5000), np.full(5000, 20 + i), np.ones(5000))
    op._lib.gwo_sync(op.handle)
    assert _timed_kernels(op, F) == 10
    op.end_input()
    assert sum(r[3] for r in op.output) == 55_000 and len(op.output) == 1000
    op.close()
