"""Copies between the handle and caller memory (gwo_xfer.cpp): pageable host columns go through the library's pinned
bounce buffer in 4 MiB chunks, pinned host and device columns are copied directly.

Rows drained, snapshotted and restored through numpy (pageable), pinned torch tensors and device tensors must be the
same rows, bit for bit, and equal the C restatement of WindowOperator (oracle/window_oracle.c) -- at sizes that take
several bounce chunks and a partial last chunk (columns of 8-24 MiB), for the submit (host -> device) and the drain,
snapshot and restore (device -> host) directions.

Reference: WindowOperator.processElement / onEventTime (WindowOperator.java:294-427, 430-473) for the rows; the
heap backend's snapshot / restore (HeapSnapshotStrategy.java:97-222, HeapRestoreOperation) for the state rows.
"""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import cbaseline

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZE = 10_000


@pytest.fixture(scope="module")
def F():
    import flink_amd
    from flink_amd import _native
    _native.lib()
    if not cbaseline.available():
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return flink_amd


@pytest.fixture(scope="module")
def stream():
    # 3M records (24 MiB per column: 5 full bounce chunks + a partial one), ~1.5M (key, window) rows
    rng = np.random.default_rng(7)
    n = 3_000_001
    k = rng.integers(0, 1_000_000, n).astype(np.int64)
    t = rng.integers(0, 2 * SIZE, n).astype(np.int64)
    v = rng.integers(-10**6, 10**6, n).astype(np.int64)
    rows, _, late = cbaseline.run_tumbling(k, t, v, [(n, LONG_MAX)], SIZE, threads=8, max_par=128)
    assert late == 0
    want = rows[:, :6]
    return k, t, v, want[np.lexsort((want[:, 0], want[:, 1]))]


def _op(F, layout):
    agg = F.MultiAggregate(F.SumAggregate(), F.MinAggregate(), F.MaxAggregate())
    return F.GpuWindowOperator(F.TumblingEventTimeWindows.of(SIZE), agg, state_layout=layout,
                               expected_keys=1 << 21)


def _fire_all(F, op):
    from flink_amd import _native as N
    lib = N.lib()
    N.check(lib.gwo_advance_watermark(op.handle, LONG_MAX), op.handle, "gwo_advance_watermark")
    N.check(lib.gwo_wait_fires(op.handle), op.handle, "gwo_wait_fires")
    n = C.c_int64()
    N.check(lib.gwo_output_count(op.handle, C.byref(n)), op.handle)
    return n.value


def _drain_into(F, op, m, cols):
    """gwo_drain into caller-provided columns (key, start, end, r0, r1, r2): data pointers."""
    from flink_amd import _native as N
    o = N.GwoOut()
    o.key, o.start, o.end = cols[0], cols[1], cols[2]
    for i in range(3):
        o.result[i] = cols[3 + i]
    got = C.c_int64()
    N.check(N.lib().gwo_drain(op.handle, C.byref(o), m, C.byref(got)), op.handle, "gwo_drain")
    return got.value


def _sorted(a):
    return a[np.lexsort((a[:, 0], a[:, 1]))]


@pytest.mark.parametrize("layout", ["log", "table"])
def test_pageable_submit_and_drain_match_the_c_twin(F, stream, layout):
    k, t, v, want = stream
    op = _op(F, layout)
    op.process_batch(k, t, v)                  # pageable numpy columns in: bounced
    m = _fire_all(F, op)
    assert m == len(want)
    key, start, end, res = op.drain_arrays()   # pageable numpy columns out: bounced
    got = np.stack([key, start, end, *res], axis=1)
    op.close()
    assert (_sorted(got) == want).all()


def test_pinned_and_device_drains_equal_the_pageable_one(F, stream):
    import torch
    k, t, v, want = stream
    kinds = {}
    for kind in ("pageable", "pinned", "device"):
        op = _op(F, "log")
        op.process_batch(k, t, v)
        m = _fire_all(F, op)
        if kind == "pageable":
            cols = [np.empty(m, np.int64) for _ in range(6)]
            ptrs = [c.ctypes.data for c in cols]
        elif kind == "pinned":
            cols = [torch.empty(m, dtype=torch.int64).pin_memory() for _ in range(6)]
            ptrs = [c.data_ptr() for c in cols]
        else:
            cols = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in range(6)]
            ptrs = [c.data_ptr() for c in cols]
        # two drains: a first part, then the rest (the rest is shifted to the front of the output columns)
        half = m // 2 + 12345
        got1 = _drain_into(F, op, half, ptrs)
        rest = [np.empty(m - got1, np.int64) for _ in range(6)]
        got2 = _drain_into(F, op, m, [r.ctypes.data for r in rest])
        assert (got1, got2) == (half, m - half)
        if kind == "device":
            torch.cuda.synchronize()
        first = np.stack([c.cpu().numpy()[:half] if hasattr(c, "cpu") else c[:half] for c in cols], axis=1)
        kinds[kind] = np.concatenate([first, np.stack(rest, axis=1)])
        op.close()
    for kind in ("pageable", "pinned", "device"):   # (the log fire's row order is not deterministic)
        assert (_sorted(kinds[kind]) == want).all(), kind


@pytest.mark.parametrize("layout", ["log", "table"])
def test_snapshot_and_restore_through_pageable_rows(F, stream, layout):
    k, t, v, want = stream
    op = _op(F, layout)
    op.process_batch(k, t, v)
    snap = op.snapshot_state()                 # state rows out through numpy: bounced
    op.close()
    assert len(snap["key"]) >= len(want)
    op2 = _op(F, layout)
    op2.restore_state(snap)                    # state rows in from numpy: read by the CPU
    m = _fire_all(F, op2)
    key, start, end, res = op2.drain_arrays()
    op2.close()
    assert m == len(want)
    assert (_sorted(np.stack([key, start, end, *res], axis=1)) == want).all()
