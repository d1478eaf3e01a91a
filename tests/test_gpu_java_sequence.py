"""The Java drop-in's call sequence, replayed through ctypes on the GPU.

There is no JDK here or on the GPU box, so GpuWindowOperator.java cannot run.  `JavaSequence`
below issues the same libgwo calls, in the same order and with the same arguments, as the Java operator and
its JNI shim (java/.../gpu/GpuWindowOperator.java, jni/gwo_jni.c):

* initializeState: gwo_create with the subtask's KeyGroupRange and maxParallelism = the task's number of key
  groups (getRuntimeContext().getMaxNumberOfParallelSubtasks(), StreamTaskStateInitializerImpl.java:290-306);
  when restored, the managed-state import below;
* processElement: records appended to columns, gwo_submit every `batch` records;
* processWatermark / endInput: flush, gwo_advance_watermark, emitFired -- gwo_wait_fires (JNI `waitFires`), then
  gwo_output_count / gwo_drain in chunks of `batch` rows until none is left, the side output the same way,
  gwo_late_dropped -- then the watermark is forwarded (rows before the watermark, AbstractStreamOperator.java:
  566-571);
* snapshotState: flush, gwo_export_heap_state_begin, per key group gwo_export_heap_state_read and the section
  parsed into WindowOperator's managed keyed states ("window-contents", "merging-window-set", the "window-timers"
  timer service), gwo_export_heap_state_end;
* initializeState of a restored subtask: the backend's entries of its key groups (enumerated through the timers,
  sessions through the merging window set) written as key-group sections into one gwo_import_heap_state;
* the mirror's lifetime (clearMirror): the backend's copy -- a checkpoint's, or a restore's -- is dropped at the
  first record, watermark or end of input after it, or at notifyCheckpointComplete / notifyCheckpointAborted.
  `JavaSequence.backend` models the keyed backend's live window states, so the tests assert that between
  checkpoints it holds no window entry (the GPU is the only copy).

Sessions fire asynchronously (gwo_session.cpp fire_session): without the sync in emitFired the drain loop would
miss rows and forward the watermark first (the round-2 advisor's finding); the session case covers it.
The expected results are the loop oracle's (oracle/flink_oracle.py, WindowOperator restated).  Integers
bit-exact; float64 within 1e-6 relative.
"""
import ctypes as C
import struct

import numpy as np
import pytest

from oracle import flink_oracle as O
from oracle import gen as G
from oracle import heap_keyed_state as H

pytestmark = pytest.mark.gpu

LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1


@pytest.fixture(scope="module")
def N():
    from flink_amd import _native
    _native.lib()
    return _native


def _p(a):
    return a.ctypes.data_as(C.c_void_p).value


class Output:
    """The operator's Output: records and watermarks in emission order."""

    def __init__(self):
        self.events = []

    def collect(self, row):
        self.events.append(("r", row))

    def side(self, rec):
        self.events.append(("s", rec))

    def watermark(self, wm):
        self.events.append(("w", wm))

    def rows(self):
        return [e[1] for e in self.events if e[0] == "r"]


_OPEN = []   # JavaSequence objects not closed yet (a failing test's are closed by the fixture below)


@pytest.fixture(autouse=True)
def _close_sequences():
    yield
    while _OPEN:   # (their pinned numpy columns must not stay registered once Python frees them)
        _OPEN.pop().close()


class JavaSequence:
    """GpuWindowOperator.java, call for call (Long keys)."""

    def __init__(self, N, spec, key_group_range, max_par, batch, out, side_output=False, restore_sections=None):
        self.N, self.lib, self.batch, self.out = N, N.lib(), batch, out
        cfg = N.GwoConfig()
        self.lib.gwo_config_init(C.byref(cfg))
        cfg.assigner, cfg.size, cfg.slide, cfg.offset, cfg.gap = (spec["assigner"], spec.get("size", 0),
                                                                  spec.get("slide", 0), 0, spec.get("gap", 0))
        cfg.allowed_lateness = spec.get("lateness", 0)
        cfg.num_aggs = len(spec["aggs"])
        for i, a in enumerate(spec["aggs"]):
            cfg.aggs[i] = a
        cfg.value_dtype = spec.get("dtype", N.DTYPE_INT64)
        cfg.key_kind = N.KEY_LONG
        cfg.max_parallelism = max_par
        cfg.key_group_start, cfg.key_group_end = key_group_range
        cfg.side_output = 1 if side_output else 0
        cfg.state_layout = spec.get("layout", N.STATE_AUTO)
        h = C.c_void_p()
        N.check(self.lib.gwo_create(C.byref(cfg), C.byref(h)), None, "create")
        self.h = h
        self.f64 = cfg.value_dtype == N.DTYPE_FLOAT64
        self.side_enabled = side_output
        self.range = key_group_range
        self.max_par = max_par
        self.merging = spec["assigner"] == N.ASSIGNER_SESSION
        self.backend = H.WindowState()   # the keyed backend's live "window-contents" / "merging-window-set" / timers
        self.mirrored = False
        if restore_sections is not None:
            self._restore(restore_sections)
        # open(): the columns and the drain buffers, allocated once
        self.keys = np.zeros(batch, np.int64)
        self.ts = np.zeros(batch, np.int64)
        self.vals = np.zeros(batch, np.float64 if self.f64 else np.int64)
        self.ok, self.os_, self.oe = (np.zeros(batch, np.int64) for _ in range(3))
        self.dt = []
        for a in range(cfg.num_aggs):
            d = C.c_int32()
            N.check(self.lib.gwo_result_dtype(h, a, C.byref(d)), h)
            self.dt.append(np.float64 if d.value == N.DTYPE_FLOAT64 else np.int64)
        self.ores = [np.zeros(batch, d) for d in self.dt]
        # open(): every column and drain buffer is pinned once (GwoNative.hostRegister -> gwo_host_register)
        self.pinned = [self.keys, self.ts, self.vals, self.ok, self.os_, self.oe] + self.ores
        for b in self.pinned:
            N.check(self.lib.gwo_host_register(_p(b), b.nbytes), None, "host register")
        self.n = 0
        self.late_reported = 0
        self.late_metric = 0
        _OPEN.append(self)

    def close(self):
        if self in _OPEN:
            _OPEN.remove(self)
        for b in self.pinned:   # close(): unpinned, then the handle destroyed
            self.N.check(self.lib.gwo_host_unregister(_p(b)), None, "host unregister")
        self.lib.gwo_destroy(self.h)

    def mirror_entries(self):
        """Window entries + timers + merging sets the keyed backend holds now."""
        return len(self.backend.contents) + len(self.backend.timers) + len(self.backend.merging)

    def clear_mirror(self):   # clearMirror: every mirrored state and timer removed from the backend
        if self.mirrored:
            self.backend = H.WindowState()
            self.mirrored = False

    def notify_checkpoint_complete(self, checkpoint_id):
        self.clear_mirror()

    notify_checkpoint_aborted = notify_checkpoint_complete

    # processElement
    def process_element(self, key, ts, value):
        if self.mirrored:
            self.clear_mirror()
        i = self.n
        self.keys[i], self.ts[i], self.vals[i] = key, ts, value
        self.n += 1
        if self.n == self.batch:
            self.flush()

    def flush(self):
        if self.n == 0:
            return
        self.N.check(self.lib.gwo_submit(self.h, _p(self.keys), _p(self.ts), _p(self.vals), self.n), self.h, "submit")
        self.n = 0

    def process_watermark(self, wm):
        if self.mirrored:
            self.clear_mirror()
        self.flush()
        self.N.check(self.lib.gwo_advance_watermark(self.h, wm), self.h, "advanceWatermark")
        self.emit_fired()
        self.out.watermark(wm)

    def end_input(self):
        if self.mirrored:
            self.clear_mirror()
        self.flush()
        self.N.check(self.lib.gwo_advance_watermark(self.h, LONG_MAX), self.h, "advanceWatermark")
        self.emit_fired()

    def emit_fired(self):
        N, lib, h = self.N, self.lib, self.h
        N.check(lib.gwo_wait_fires(h), h, "waitFires")
        n = C.c_int64()
        while True:
            N.check(lib.gwo_output_count(h, C.byref(n)), h)
            rows = n.value
            if rows <= 0:
                break
            cap = min(rows, self.batch)
            o = N.GwoOut()
            o.key, o.start, o.end = _p(self.ok), _p(self.os_), _p(self.oe)
            for a, r in enumerate(self.ores):
                o.result[a] = _p(r)
            got = C.c_int64()
            N.check(lib.gwo_drain(h, C.byref(o), cap, C.byref(got)), h, "drain")
            assert got.value > 0
            for i in range(got.value):
                res = tuple(r[i].item() for r in self.ores)
                self.out.collect((int(self.ok[i]), int(self.os_[i]), int(self.oe[i]), res[0] if len(res) == 1 else res))
        while self.side_enabled:
            N.check(lib.gwo_side_output_count(h, C.byref(n)), h)
            if n.value <= 0:
                break
            cap = min(n.value, self.batch)
            k, t = np.zeros(cap, np.int64), np.zeros(cap, np.int64)
            v = np.zeros(cap, np.float64 if self.f64 else np.int64)
            so = N.GwoSideOut(_p(k), _p(t), _p(v))
            got = C.c_int64()
            N.check(lib.gwo_drain_side_output(h, C.byref(so), cap, C.byref(got)), h)
            for i in range(got.value):
                self.out.side((int(k[i]), int(t[i]), v[i].item()))
        late = C.c_int64()
        N.check(lib.gwo_late_dropped(h, C.byref(late)), h)
        self.late_metric += late.value - self.late_reported
        self.late_reported = late.value

    # snapshotState: the GPU state into WindowOperator's managed keyed states, key group by key group
    # (gwo_export_heap_state_begin, one gwo_export_heap_state_read per key group, gwo_export_heap_state_end; each
    # section parsed into the backend).  Returns the backend's copy (a WindowState: what the heap backend snapshots).
    def snapshot_state(self, key_group_list):
        N, lib, h = self.N, self.lib, self.h
        self.flush()
        self.clear_mirror()   # a mirror still held (no record or watermark since the last checkpoint) is replaced
        groups = list(key_group_list)
        ids = N.GwoHeapStateIds(0, 1 if self.merging else -1, 2, 3)
        offs = np.zeros(len(groups), np.int64)
        total, wm = C.c_int64(), C.c_int64()
        N.check(lib.gwo_export_heap_state_begin(h, C.byref(ids), C.byref(total),
                                                offs.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(wm)), h, "begin")
        backend = H.WindowState()
        try:
            for i, g in enumerate(groups):
                end = int(offs[i + 1]) if i + 1 < len(groups) else total.value
                n = end - int(offs[i])
                buf = (C.c_uint8 * max(n, 1))()
                N.check(lib.gwo_export_heap_state_read(h, int(offs[i]), buf, n), h, "read")
                part = H.parse_export(bytes(buf)[:n], "long", self.merging, (g, g))
                backend.contents.update(part.contents)
                backend.merging.update(part.merging)
                backend.timers |= part.timers
        finally:
            N.check(lib.gwo_export_heap_state_end(h), h, "end")
        self.backend, self.mirrored = backend, True
        # the checkpoint: the backend's synchronous snapshot (copy-on-write maps, a copy of the timer queue)
        snap = H.WindowState()
        snap.contents.update(backend.contents)
        snap.merging.update({k: dict(m) for k, m in backend.merging.items()})
        snap.timers |= backend.timers
        return snap

    # initializeState of a restored subtask (importMirror): the backend's entries of this subtask's key groups,
    # enumerated through the timers, sessions resolved through the merging window set, written as sections (each
    # window its own state window) into one gwo_import_heap_state at Long.MIN_VALUE
    def _restore(self, backend):
        kg_of = lambda key: O.assign_to_key_group(O.long_hash_code(int(key)), self.max_par)
        timers = {t for t in backend.timers if self.range[0] <= kg_of(t[1]) <= self.range[1]}
        if not timers:
            return
        s = H.WindowState()
        s.timers = timers
        for ts, key, w in sorted(timers):
            if (key, w) in s.contents:
                continue
            sw = backend.merging.get(key, {}).get(w, w) if self.merging else w
            acc = backend.contents.get((key, sw))
            if acc is not None:
                s.contents[(key, w)] = acc
                if self.merging:
                    s.merging.setdefault(key, {})[w] = w
        buf = H.write_state(s, "long", kg_of, self.range)
        ids = self.N.GwoHeapStateIds(0, 1 if self.merging else -1, 2, 3)
        arr = (C.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf + b"\0")
        self.N.check(self.lib.gwo_import_heap_state(self.h, C.byref(ids), arr, len(buf), LONG_MIN), self.h, "import")
        # the restored keyed states stay in the backend until the first record / watermark (importMirror: mirrored)
        self.backend, self.mirrored = s, True


def _oracle_run(assigner, agg, lateness, k, t, v, batches, side=False, restore_after=None):
    """The loop oracle over the stream; also returns, per watermark (by index), the rows its timers emitted.
    restore_after=i: a restore from a checkpoint after watermark i -- the keyed state and timers carry over, the
    watermark starts again at Long.MIN_VALUE (WindowOperator keeps no watermark in its state: a restored subtask's
    timer service starts at Long.MIN_VALUE, InternalTimerServiceImpl.java:78)."""
    op = O.WindowOperatorOracle(assigner, agg, lateness, side_output=side)
    prev, fired = 0, []
    for bi, (end, wm) in enumerate(batches):
        if restore_after is not None and bi == restore_after + 1:
            op.wm = LONG_MIN
        for i in range(prev, end):
            op.process_element(int(k[i]), int(t[i]), v[i].item())
        before = len(op.output)
        op.process_watermark(wm)
        fired.append({(r.key, r.start, r.end) for r in op.output[before:]})
        prev = end
    op.end_input()
    return op, fired


def _events(k, t, v, batches):
    prev = 0
    for end, wm in batches:
        for i in range(prev, end):
            yield ("e", int(k[i]), int(t[i]), v[i].item())
        yield ("w", wm)
        prev = end


def _events_from(k, t, v, batches, first):
    """The events of batches[first:] (records after batches[first - 1]'s end, then each watermark)."""
    prev = batches[first - 1][0] if first else 0
    for end, wm in batches[first:]:
        for i in range(prev, end):
            yield ("e", int(k[i]), int(t[i]), v[i].item())
        yield ("w", wm)
        prev = end


def _drive(seq, events):
    for ev in events:
        if ev[0] == "e":
            seq.process_element(ev[1], ev[2], ev[3])
        else:
            seq.process_watermark(ev[1])


def _rows_before_watermarks(out, fired):
    """Rows a watermark fires are collected before that watermark is forwarded (AbstractStreamOperator.java:
    566-571): for the i-th forwarded watermark, every row the oracle's timers emitted at watermark i is already in
    the output."""
    seen, i = set(), 0
    for ev in out.events:
        if ev[0] == "r":
            seen.add(ev[1][:3])
        elif ev[0] == "w":
            missing = fired[i] - seen
            assert not missing, f"{len(missing)} rows of watermark {ev[1]} came after it"
            i += 1
    assert i == len(fired)


def _cases(N):
    return {
        "tumbling_log": dict(assigner=N.ASSIGNER_TUMBLING, size=5000, aggs=[N.AGG_SUM, N.AGG_MIN, N.AGG_MAX],
                             layout=N.STATE_LOG, o=lambda: (O.TumblingEventTimeWindows(5000),
                                                            O.MultiAgg([O.SumLongAgg(), O.MinAgg(), O.MaxAgg()]))),
        "tumbling_table_lateness": dict(assigner=N.ASSIGNER_TUMBLING, size=5000, aggs=[N.AGG_SUM, N.AGG_COUNT],
                                        lateness=2000, layout=N.STATE_TABLE,
                                        o=lambda: (O.TumblingEventTimeWindows(5000),
                                                   O.MultiAgg([O.SumLongAgg(), O.CountAgg()]))),
        "sliding_avg": dict(assigner=N.ASSIGNER_SLIDING, size=3000, slide=1000, aggs=[N.AGG_AVG],
                            o=lambda: (O.SlidingEventTimeWindows(3000, 1000), O.AvgAgg())),
        "sessions": dict(assigner=N.ASSIGNER_SESSION, gap=2000, aggs=[N.AGG_SUM, N.AGG_COUNT, N.AGG_MAX],
                         o=lambda: (O.EventTimeSessionWindows(2000),
                                    O.MultiAgg([O.SumLongAgg(), O.CountAgg(), O.MaxAgg()]))),
        "sessions_lateness_side": dict(assigner=N.ASSIGNER_SESSION, gap=2000, aggs=[N.AGG_SUM], lateness=1500,
                                       side=True, o=lambda: (O.EventTimeSessionWindows(2000), O.SumLongAgg())),
    }


def _stream(seed, n=12_000, nkeys=300):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, nkeys, n).astype(np.int64)
    t = (np.sort(rng.integers(0, 200_000, n)) + rng.integers(0, 4_000, n)).astype(np.int64)
    v = rng.integers(-50, 1000, n).astype(np.int64)
    return k, t, v, G.punctuated_watermarks(t, 600, 1_000)


@pytest.mark.parametrize("case", ["tumbling_log", "tumbling_table_lateness", "sliding_avg", "sessions",
                                  "sessions_lateness_side"])
def test_java_call_sequence_matches_oracle(N, case):
    spec = _cases(N)[case]
    k, t, v, b = _stream(hash(case) % 1000)
    out = Output()
    seq = JavaSequence(N, spec, (0, 127), 128, batch=1000, out=out, side_output=spec.get("side", False))
    half = len(b) // 2
    _drive(seq, _events(k, t, v, b[:half]))
    # a checkpoint mid-stream: the mirror exists only until the next record or watermark, and exporting does not
    # change the GPU state (the rows below still equal the uninterrupted oracle run)
    snap = seq.snapshot_state(range(0, 128))
    assert seq.mirror_entries() == len(snap.contents) + len(snap.timers) + len(snap.merging) > 0
    _drive(seq, _events_from(k, t, v, b, half))
    assert seq.mirror_entries() == 0   # between checkpoints the backend holds no window entry
    seq.end_input()
    a, agg = spec["o"]()
    ref, fired = _oracle_run(a, agg, spec.get("lateness", 0), k, t, v, b, side=spec.get("side", False))
    want = sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    got = sorted(out.rows())
    if case == "sliding_avg":
        assert [g[:3] for g in got] == [w[:3] for w in want]
        np.testing.assert_allclose([g[3] for g in got], [w[3] for w in want], rtol=1e-6)
    else:
        assert got == want
    assert sorted(e[1] for e in out.events if e[0] == "s") == sorted(ref.side_output)
    assert seq.late_metric == ref.num_late_records_dropped
    _rows_before_watermarks(out, fired)
    seq.close()


@pytest.mark.parametrize("case", ["tumbling_log", "tumbling_table_lateness", "sliding_avg", "sessions"])
def test_java_snapshot_sections_rescale_2_to_3(N, case):
    """Two subtasks (KeyGroupRange of operator i of 2) checkpoint into WindowOperator's managed keyed states; three
    new subtasks each import the entries of ITS key groups (the managed keyed state Flink hands a rescaled subtask)
    and continue.  The union of all rows equals the uninterrupted single-operator oracle run."""
    maxp = 128
    spec = _cases(N)[case]
    k, t, v, b = _stream(7 + len(case))
    kg = np.array([O.assign_to_key_group(O.long_hash_code(int(x)), maxp) for x in k])
    half = len(b) // 2
    cut = b[half - 1][0]
    out_before, out_after = Output(), Output()
    backend = H.WindowState()   # the keyed state backends' snapshots, by key (redistributed by key group)
    for p in range(2):
        r = O.compute_key_group_range_for_operator_index(maxp, 2, p)
        own = (kg >= r[0]) & (kg <= r[1])
        seq = JavaSequence(N, spec, r, maxp, batch=700, out=out_before)
        prev = 0
        for end, wm in b[:half]:
            for i in np.flatnonzero(own[prev:end]) + prev:
                seq.process_element(int(k[i]), int(t[i]), int(v[i]))
            seq.process_watermark(wm)
            prev = end
        part = seq.snapshot_state(range(r[0], r[1] + 1))
        assert seq.mirror_entries() > 0
        seq.notify_checkpoint_complete(1)
        assert seq.mirror_entries() == 0   # dropped once the checkpoint is complete
        backend.contents.update(part.contents)
        backend.merging.update(part.merging)
        backend.timers |= part.timers
        seq.close()
    late = 0
    for p in range(3):
        r = O.compute_key_group_range_for_operator_index(maxp, 3, p)
        own = (kg >= r[0]) & (kg <= r[1])
        seq = JavaSequence(N, spec, r, maxp, batch=700, out=out_after, restore_sections=backend)
        restored = seq.mirror_entries()
        prev = cut
        for end, wm in b[half:]:
            for i in np.flatnonzero(own[prev:end]) + prev:
                seq.process_element(int(k[i]), int(t[i]), int(v[i]))
            seq.process_watermark(wm)
            assert seq.mirror_entries() == 0   # the restored copy is gone after the first record / watermark
            prev = end
        assert restored > 0
        seq.end_input()
        late += seq.late_metric
        seq.close()
    a, agg = spec["o"]()
    ref, _ = _oracle_run(a, agg, spec.get("lateness", 0), k, t, v, b, restore_after=half - 1)
    got = sorted(out_before.rows() + out_after.rows())
    want = sorted((r.key, r.start, r.end, r.result) for r in ref.output)
    if case == "sliding_avg":   # float64 avg: within 1e-6 relative (the (key, window) set exactly)
        assert [g[:3] for g in got] == [w[:3] for w in want]
        np.testing.assert_allclose([g[3] for g in got], [w[3] for w in want], rtol=1e-6)
    else:
        assert got == want


def test_host_register_contract(N):
    """gwo_host_register pins host memory (idempotent), gwo_host_unregister releases it; unregistering memory that is
    not registered, a null pointer or a non-positive size is GWO_ERR_INVALID_ARGUMENT."""
    lib = N.lib()
    a = np.zeros(1 << 16, np.int64)
    assert lib.gwo_host_register(_p(a), a.nbytes) == 0
    assert lib.gwo_host_register(_p(a), a.nbytes) == 0          # already registered: fine
    assert lib.gwo_host_unregister(_p(a)) == 0
    assert lib.gwo_host_unregister(_p(a)) == 1   # GWO_ERR_INVALID_ARGUMENT
    assert lib.gwo_host_register(None, 64) == 1   # GWO_ERR_INVALID_ARGUMENT
    assert lib.gwo_host_register(_p(a), 0) == 1   # GWO_ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("case", ["tumbling_log", "sessions"])
def test_staged_export_equals_export(N, case):
    """gwo_export_heap_state_begin/_read/_end stage exactly gwo_export_heap_state's image (same bytes, key-group
    offsets and watermark), reading past the image is GWO_ERR_INVALID_ARGUMENT, and _end releases it (a read after it
    is GWO_ERR_STATE)."""
    spec = _cases(N)[case]
    k, t, v, b = _stream(5)
    seq = JavaSequence(N, spec, (0, 127), 128, batch=1000, out=Output())
    _drive(seq, _events(k, t, v, b[: len(b) // 2]))
    seq.flush()
    lib, h = seq.lib, seq.h
    ids = N.GwoHeapStateIds(0, 1 if seq.merging else -1, 2, 3)
    need, wm = C.c_int64(), C.c_int64()
    o1 = np.zeros(128, np.int64)
    N.check(lib.gwo_export_heap_state(h, C.byref(ids), None, 0, C.byref(need), None, None), h)
    ref = (C.c_uint8 * max(need.value, 1))()
    N.check(lib.gwo_export_heap_state(h, C.byref(ids), ref, need.value, C.byref(need), _p(o1), C.byref(wm)), h)
    total, wm2 = C.c_int64(), C.c_int64()
    o2 = np.zeros(128, np.int64)
    N.check(lib.gwo_export_heap_state_begin(h, C.byref(ids), C.byref(total), o2.ctypes.data_as(C.POINTER(C.c_int64)),
                                            C.byref(wm2)), h)
    assert total.value == need.value > 0 and wm2.value == wm.value
    assert (o1 == o2).all()
    got = (C.c_uint8 * total.value)()
    half = total.value // 2
    N.check(lib.gwo_export_heap_state_read(h, 0, got, half), h)
    tail = (C.c_uint8 * (total.value - half))()
    N.check(lib.gwo_export_heap_state_read(h, half, tail, total.value - half), h)
    staged = bytes(got)[:half] + bytes(tail)
    # the same entries (a key group's entries may come in another order from another snapshot of the device state)
    a_ = H.parse_export(staged, "long", seq.merging, (0, 127))
    b_ = H.parse_export(bytes(ref)[: need.value], "long", seq.merging, (0, 127))
    assert a_.contents == b_.contents and a_.merging == b_.merging and a_.timers == b_.timers and a_.contents
    assert lib.gwo_export_heap_state_read(h, 1, got, total.value) == 1   # GWO_ERR_INVALID_ARGUMENT: past the image
    N.check(lib.gwo_export_heap_state_end(h), h)
    assert lib.gwo_export_heap_state_read(h, 0, got, 1) != 0   # released
    seq.close()
