"""Device-input readiness at the C-ABI boundary (gwo.h "Device-input readiness", gwo_wait_stream).

A device-resident caller -- a GPU source, or a test building columns with torch -- produces a batch's columns on
its own stream.  The handle runs K1 on a non-blocking stream, so without an ordering the kernel may read the columns
before the producer has written them.  That is how `test_sharded_union_single_gpu[8-log]` lost 4 rows once in round
5 (the test built its columns with `.contiguous()` on torch's stream and submitted at once).  Here the producer is
held back by a delay kernel so the race is deterministic:

* unordered (log layout): the handle processes what the columns held BEFORE the producer's copy (batch A);
* ordered (gwo_wait_stream, what `GpuWindowOperator.process_device_batch` does by default): exactly batch B,
  row for row against the C restatement of WindowOperator (oracle/window_oracle.c).

Reference: WindowOperator.processElement / onEventTime (WindowOperator.java:294-427, 430-473) -- every record of
the batch is aggregated, every fired (key, window) emitted.  Integer aggregates: bit-exact.
"""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import cbaseline

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


def _batch(seed, n, nkeys):
    rng = np.random.default_rng(seed)
    return (rng.integers(0, nkeys, n).astype(np.int64), rng.integers(0, 20_000, n).astype(np.int64),
            rng.integers(-1000, 1000, n).astype(np.int64))


def _want(cols):
    k, t, v = cols
    rows, _, late = cbaseline.run_tumbling(k, t, v, [(len(k), LONG_MAX)], 5_000, threads=4, max_par=128)
    assert late == 0
    return rows[:, :6]


def _run(F, layout, a_host, b_host, ordered):
    """Columns hold batch A (complete); a producer stream sleeps, then overwrites them with batch B; the batch is
    submitted right away.  Returns the handle's rows and how long the producer's delay measured (ms)."""
    import torch
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    op = F.GpuWindowOperator(F.TumblingEventTimeWindows.of(5_000), agg, state_layout=layout,
                             expected_keys=1 << 20 if layout == "log" else 50_000)
    cols = [torch.from_numpy(x).cuda() for x in a_host]      # H2D + stream sync: batch A is complete
    src = [torch.from_numpy(x).cuda() for x in b_host]
    torch.cuda.synchronize()
    producer = torch.cuda.Stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(producer):
        e0.record()
        torch.cuda._sleep(400_000_000)                        # hundreds of ms of GPU time before the copies
        e1.record()
        for d, s in zip(cols, src):
            d.copy_(s)
    op.process_device_batch(*(c.data_ptr() for c in cols), len(b_host[0]),
                            producer_stream=producer.cuda_stream if ordered else None, keep=cols)
    op.end_input()
    torch.cuda.synchronize()
    delay_ms = e0.elapsed_time(e1)
    got = np.array([(k, s, e, *r) for k, s, e, r in op.output], dtype=np.int64).reshape(-1, 6)
    op.close()
    return got, delay_ms


def _order(a):
    return a[np.lexsort((a[:, 0], a[:, 1]))]


@pytest.mark.parametrize("layout", ["log", "table"])
def test_device_input_waits_for_producer_stream(F, layout):
    import torch
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep (the delay kernel) is not available")
    n, nkeys = 200_000, 50_000
    a_host, b_host = _batch(1, n, nkeys), _batch(2, n, nkeys)
    want_a, want_b = _want(a_host), _want(b_host)
    assert want_a.shape != want_b.shape or (_order(want_a) != _order(want_b)).any()

    # ordered: the handle's stream waits for the producer on the device -- exactly batch B
    got, delay = _run(F, layout, a_host, b_host, ordered=True)
    assert delay > 20.0, f"the delay kernel ran {delay:.1f} ms: no race window to test"
    assert got.shape == want_b.shape
    assert (_order(got) == want_b[np.lexsort((want_b[:, 0], want_b[:, 1]))]).all()

    # unordered (the r05 test's pattern), on the log layout -- the layout that lost rows in round 5: K1 runs while the
    # producer still sleeps and reads batch A, exactly A's rows come out.  The mechanism of the round-5 row loss, shown
    # deterministically.  (A fresh table-layout handle allocates its first window tables before its first kernel;
    # hipMalloc synchronises the device, which happens to order it after the producer here -- not a guarantee.)
    if layout == "log":
        got_u, delay_u = _run(F, layout, a_host, b_host, ordered=False)
        if delay_u > 20.0:
            assert got_u.shape == want_a.shape and (_order(got_u) == _order(want_a)).all()
