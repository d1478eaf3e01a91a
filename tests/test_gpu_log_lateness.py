"""GPU parity for allowedLateness > 0 on the log-structured tumbling layout (the C4 layout).

A log window that fires with allowedLateness > 0 must keep its state until its cleanup time and re-fire for every
late record that reaches it (EventTimeTrigger.java:37-45, WindowOperator.java:393-406, cleanup :639-646).  The
log layout hands such a window to a hash table at its fire (gwo_log.cpp log_migrate); the batch's re-fire
records go through a table pass (refire_only) while its accepted records stay in the log.  Checked against the
oracle on the reference's tumbling streams replayed with lateness, random late streams (with and without the
late-data side output), and a checkpoint holding both collecting log windows and fired tables.  Integer
aggregates: bit-exact; both layouts must agree.
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


@pytest.mark.parametrize("name", ["tumbling_3s", "side_output_lateness_tumbling", "cleanup_time_overflow"])
@pytest.mark.parametrize("lateness", [1_000, 2_500])
@pytest.mark.parametrize("layout", ["log", "table"])
def test_reference_tumbling_streams_with_lateness(F, golden, name, lateness, layout):
    s = next(x for x in golden["operator_streams"] if x["name"] == name)
    a = s["assigner"]
    want = O.WindowOperatorOracle(O.TumblingEventTimeWindows(a["size"], a["offset"]), O.SumLongAgg(), lateness,
                                  side_output=s["side_output"])
    got = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(a["size"], a["offset"]), F.SumAggregate(),
                              allowed_lateness=lateness, side_output_late_data=s["side_output"], state_layout=layout)
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


def _late_stream(seed, n, nkeys, span, disorder, frac=0.2):
    rng = np.random.default_rng(seed)
    base = np.sort(rng.integers(0, span, n))
    t = (base + disorder - rng.integers(0, disorder, n) * (rng.random(n) < frac)).astype(np.int64)
    k = rng.integers(0, nkeys, n).astype(np.int64)
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    return k, t, v


def _oracle(k, t, v, batches, size, lateness, side):
    op = O.WindowOperatorOracle(O.TumblingEventTimeWindows(size), O.MultiAgg([O.SumLongAgg(), O.MinAgg(), O.MaxAgg()]),
                                lateness, side_output=side)
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            op.process_element(int(k[i]), int(t[i]), int(v[i]))
        op.process_watermark(wm)
        prev = end
    op.process_watermark(LONG_MAX)
    return (sorted((r.key, r.start, r.end, r.result) for r in op.output), op.num_late_records_dropped,
            sorted(op.side_output))


def _mk(F, size, lateness, layout, side=False):
    return F.GpuWindowOperator(F.TumblingEventTimeWindows.of(size),
                               F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate()),
                               allowed_lateness=lateness, side_output_late_data=side, state_layout=layout,
                               max_parallelism=32768)


@pytest.mark.parametrize("lateness,side", [(3_000, False), (12_000, False), (3_000, True)])
@pytest.mark.parametrize("layout", ["log", "table"])
def test_random_tumbling_with_lateness(F, lateness, side, layout):
    size = 5_000
    k, t, v = _late_stream(lateness + side, 40_000, 3_000, 100_000, 4 * size)
    b = G.punctuated_watermarks(t, 1_000, 300)
    want, wl, wside = _oracle(k, t, v, b, size, lateness, side)
    op = _mk(F, size, lateness, layout, side)
    prev = 0
    for end, wm in b:
        op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        op.process_watermark(wm)
        prev = end
    op.end_input()
    got = sorted(op.output)
    assert op.num_late_records_dropped == wl
    assert sorted(op.side_output) == wside
    assert len(got) == len(want) and got == want
    op.close()


@pytest.mark.parametrize("restore_layout", ["log", "table"])
def test_log_lateness_checkpoint_continues_exactly(F, restore_layout):
    """The checkpoint holds collecting log windows (timer pending) and fired windows kept for lateness (timer
    0); after restore late records still re-fire the fired ones."""
    size, lateness = 5_000, 8_000
    k, t, v = _late_stream(21, 30_000, 2_000, 80_000, 3 * size)
    b = G.punctuated_watermarks(t, 1_000, 200)
    want, wl, _ = _oracle(k, t, v, b, size, lateness, False)
    a = _mk(F, size, lateness, "log")
    cut = len(b) // 2
    prev = 0
    for end, wm in b[:cut]:
        a.process_batch(k[prev:end], t[prev:end], v[prev:end])
        a.process_watermark(wm)
        prev = end
    snap = a.snapshot_state()
    assert (snap["timer"] == 0).any() and (snap["timer"] == 1).any()
    assert len(snap["key"]) <= a.state_size()
    rows, late = list(a.output), a.num_late_records_dropped
    a.close()
    c = _mk(F, size, lateness, restore_layout)
    c.restore_state(snap)
    for end, wm in b[cut:]:
        c.process_batch(k[prev:end], t[prev:end], v[prev:end])
        c.process_watermark(wm)
        prev = end
    c.end_input()
    assert sorted(rows + list(c.output)) == want
    assert late + c.num_late_records_dropped == wl
    c.close()


def test_migration_and_refires_of_a_window_with_more_partitions_than_the_grid(F):
    """A window of 1.5M records: more log partitions than the fold's persistent grid (2 workgroups per CU), so each
    workgroup folds several partitions in turn.  Its fire with allowedLateness > 0 migrates it to a hash table through
    the slow-only fold (gwo_log.cpp log_migrate); late records then re-fire rows from that table.  Checked row for row
    against the C restatement of WindowOperator (oracle/window_oracle.c; WindowOperator.java:393-406 re-fires)."""
    import ctypes as C
    from flink_amd import _native as N
    from oracle import cbaseline
    if not cbaseline.available():
        import os
        import subprocess
        subprocess.run(["make", "-C", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "oracle")], check=True, capture_output=True)
    rng = np.random.default_rng(11)
    n1, n2, size, lateness = 1_500_000, 200_000, 10_000, 5_000
    k = rng.integers(0, 1_000_000, n1 + n2).astype(np.int64)
    t = np.concatenate([rng.integers(0, size, n1), rng.integers(0, size, n2)]).astype(np.int64)
    v = rng.integers(-10**6, 10**6, n1 + n2).astype(np.int64)
    batches = [(n1, size), (n1 + n2, size + 2_000)]
    rows, _, late = cbaseline.run_tumbling(k, t, v, batches, size, lateness=lateness, threads=8, max_par=128)
    want = rows[:, :6]
    op = _mk(F, size, lateness, "log")
    lib = N.lib()
    got = []
    prev = 0
    for end, wm in batches + [(n1 + n2, LONG_MAX)]:
        if end > prev:
            op.process_batch(k[prev:end], t[prev:end], v[prev:end])
        prev = end
        N.check(lib.gwo_advance_watermark(op.handle, wm), op.handle, "gwo_advance_watermark")
        N.check(lib.gwo_wait_fires(op.handle), op.handle, "gwo_wait_fires")
        key, start, end_, res = op.drain_arrays()
        got.append(np.stack([key, start, end_, *res], axis=1))
    assert op.num_late_records_dropped == late
    op.close()
    got = np.concatenate(got)
    order = lambda a: a[np.lexsort(a.T[::-1])]
    assert got.shape == want.shape
    assert (order(got) == order(want)).all()
