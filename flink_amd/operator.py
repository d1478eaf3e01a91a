"""``GpuWindowOperator`` -- the host-side mirror of the Java drop-in operator.

Mirrors the interface the task runtime drives (``OneInputStreamOperator``, ``BoundedOneInput``;
SJ/api/operators/OneInputStreamOperator.java:35-51, BoundedOneInput.java:26-31) and the window
operator's observable behaviour (WindowOperator.java:294-653): ``process_element`` buffers into
columnar batches (the mailbox batching the Java operator does), and every ``process_watermark``
first flushes the pending batch, then fires -- results are emitted before the watermark is
forwarded (AbstractStreamOperator.java:566-571).  All state lives in HBM behind libgwo.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .keygroups import decode_utf16, encode_utf16
from .windowing import AggregateFunction, WindowAssigner

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _torch_current_stream(device: int = 0):
    """torch's current stream on `device` as a raw hipStream_t (0 = the null stream), or None when torch has not
    initialised the GPU (then nothing of torch's can still be producing device columns)."""
    import sys
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return None
    return int(torch.cuda.current_stream(device).cuda_stream)


class GpuWindowOperator:
    """One subtask of ``keyBy(...).window(assigner).aggregate(fn)`` on one MI355X."""

    def __init__(self, assigner: WindowAssigner, aggregate: AggregateFunction, allowed_lateness: int = 0,
                 side_output_late_data: bool = False, max_parallelism: int = 128, key_group_range=None,
                 key_kind: str = "long", device: int = 0, batch_size: int = 1 << 20, expected_keys: int = 0,
                 stream=None, state_layout: str = "auto"):
        if allowed_lateness < 0:
            raise ValueError("The allowed lateness cannot be negative.")
        self._lib = N.lib()
        cfg = N.GwoConfig()
        self._lib.gwo_config_init(C.byref(cfg))
        cfg.assigner = assigner.kind
        cfg.size = getattr(assigner, "size", 0)
        cfg.slide = getattr(assigner, "slide", 0)
        cfg.offset = getattr(assigner, "offset", 0)
        cfg.gap = getattr(assigner, "gap", 0)
        cfg.allowed_lateness = allowed_lateness
        kinds, vdt = aggregate.descriptor
        cfg.num_aggs = len(kinds)
        for i, k in enumerate(kinds):
            cfg.aggs[i] = k
        cfg.value_dtype = vdt
        kinds_ = {"long": N.KEY_LONG, "int": N.KEY_INT, "string": N.KEY_STRING}
        if key_kind not in kinds_:
            raise ValueError(f"key_kind must be one of {sorted(kinds_)}")
        cfg.key_kind = kinds_[key_kind]
        # String keys (KeyGroupRangeAssignment over String.hashCode): the handle interns them into its device
        # dictionary; rows come back keyed by the Strings (gwo.h gwo_submit_utf16 / gwo_key_strings)
        self._strings = key_kind == "string"
        cfg.max_parallelism = max_parallelism
        lo, hi = key_group_range if key_group_range is not None else (0, max_parallelism - 1)
        cfg.key_group_start, cfg.key_group_end = lo, hi
        cfg.device = device
        cfg.side_output = 1 if side_output_late_data else 0
        cfg.expected_keys = expected_keys
        layouts = {"auto": N.STATE_AUTO, "table": N.STATE_TABLE, "log": N.STATE_LOG}
        if state_layout not in layouts:
            raise ValueError(f"state_layout must be one of {sorted(layouts)}")
        cfg.state_layout = layouts[state_layout]
        cfg.stream = stream
        h = C.c_void_p()
        st = self._lib.gwo_create(C.byref(cfg), C.byref(h))
        N.check(st, None, "gwo_create")
        self._h = h
        self.cfg = cfg
        self.assigner = assigner
        self.aggregate = aggregate
        self.value_dtype = np.float64 if vdt == N.DTYPE_FLOAT64 else np.int64
        self.batch_size = batch_size
        self._borrowed = None   # device columns of the last process_device_batch (gwo.h: borrowed until the next call)
        self._pk, self._pt, self._pv = [], [], []
        self.output: list[tuple] = []
        self.side_output: list[tuple] = []
        self._result_dtypes = []
        for i in range(len(kinds)):
            d = C.c_int32()
            N.check(self._lib.gwo_result_dtype(h, i, C.byref(d)), h)
            self._result_dtypes.append(np.float64 if d.value == N.DTYPE_FLOAT64 else np.int64)

    # -- lifecycle ---------------------------------------------------------------------------
    def open(self):
        return self

    def close(self):
        if self._h:
            self._lib.gwo_destroy(self._h)
            self._h = None
        self._borrowed = None

    dispose = close

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- OneInputStreamOperator --------------------------------------------------------------
    def process_element(self, key: int, timestamp: int, value=0):
        self._pk.append(key)
        self._pt.append(timestamp)
        self._pv.append(value)
        if len(self._pk) >= self.batch_size:
            self.flush()

    def process_batch(self, keys, timestamps, values=None):
        """Columnar batch in arrival order (numpy arrays; host memory; String keys: a sequence of str)."""
        self.flush()
        k = list(keys) if self._strings else np.ascontiguousarray(keys, dtype=np.int64)
        t = np.ascontiguousarray(timestamps, dtype=np.int64)
        v = None if values is None else np.ascontiguousarray(values, dtype=self.value_dtype)
        self._submit(k, t, v)

    def process_device_batch(self, key_ptr: int, ts_ptr: int, val_ptr, n: int, producer_stream="current",
                             keep=None):
        """Columnar batch already resident in HBM (device pointers).

        The columns may still be in flight on the stream that produced them: ``producer_stream`` (a raw
        hipStream_t as int, 0 = the null stream; default "current" = torch's current stream of this device when
        torch has initialised the GPU) is named to gwo_wait_stream, so the handle's stream waits for it on the
        device (gwo.h "Device-input readiness").  ``None``: the caller guarantees the columns are complete.
        ``keep`` (e.g. the tensors owning the columns) is held until the next call on this operator returns --
        the borrow gwo.h states for device input."""
        self.flush()
        if producer_stream == "current":
            producer_stream = _torch_current_stream(self.cfg.device)
        if producer_stream is not None:
            N.check(self._lib.gwo_wait_stream(self._h, C.c_void_p(producer_stream or None)), self._h,
                    "gwo_wait_stream")
        st = self._lib.gwo_submit(self._h, C.c_void_p(key_ptr), C.c_void_p(ts_ptr),
                                  C.c_void_p(val_ptr) if val_ptr else None, n)
        self._borrowed = keep   # the previous batch's columns are released only now (this call has returned)
        N.check(st, self._h, "gwo_submit")

    def _submit(self, k, t, v):
        if len(k) == 0:
            return
        if self._strings:
            chars, offsets = encode_utf16(k)
            st = self._lib.gwo_submit_utf16(self._h, _ptr(chars), _ptr(offsets), _ptr(t), _ptr(v), len(k))
            N.check(st, self._h, "gwo_submit_utf16")
            return
        st = self._lib.gwo_submit(self._h, _ptr(k), _ptr(t), _ptr(v), len(k))
        N.check(st, self._h, "gwo_submit")

    def key_strings(self, ids):
        """Dictionary ids (output / side-output / checkpoint key column of a String-keyed handle) -> Strings."""
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        n = len(ids)
        off = np.empty(n + 1, np.int64)
        need = C.c_int64()
        N.check(self._lib.gwo_key_strings(self._h, _ptr(ids), n, _ptr(off), None, 0, C.byref(need)), self._h)
        chars = np.empty(max(need.value, 1), np.uint16)
        N.check(self._lib.gwo_key_strings(self._h, _ptr(ids), n, _ptr(off), _ptr(chars), need.value, C.byref(need)),
                self._h)
        return decode_utf16(chars, off)

    def intern_strings(self, keys):
        """Strings -> this handle's dictionary ids."""
        chars, offsets = encode_utf16(keys)
        ids = np.empty(max(len(keys), 1), np.int64)
        N.check(self._lib.gwo_intern_utf16(self._h, _ptr(chars), _ptr(offsets), len(keys), _ptr(ids)), self._h,
                "gwo_intern_utf16")
        return ids[:len(keys)]

    def flush(self):
        if not self._pk:
            return
        k = list(self._pk) if self._strings else np.array(self._pk, dtype=np.int64)
        t = np.array(self._pt, dtype=np.int64)
        v = np.array(self._pv, dtype=self.value_dtype)
        self._pk, self._pt, self._pv = [], [], []
        self._submit(k, t, v)

    def process_watermark(self, watermark: int):
        self.flush()
        N.check(self._lib.gwo_advance_watermark(self._h, int(watermark)), self._h, "gwo_advance_watermark")
        self._collect()

    def prepare_snapshot_pre_barrier(self, checkpoint_id: int = 0):
        self.flush()

    def end_input(self):
        """BoundedOneInput.endInput: the source's final Long.MAX_VALUE watermark."""
        self.process_watermark(LONG_MAX)

    # -- results -----------------------------------------------------------------------------
    def _collect(self):
        # processWatermark emits the fired rows before it returns (AbstractStreamOperator.java:566-571):
        # wait for an asynchronous fire (log layout, sessions) to complete -- only the fires: batches and the
        # multi-GPU exchange stay in flight
        N.check(self._lib.gwo_wait_fires(self._h), self._h, "gwo_wait_fires")
        n = C.c_int64()
        N.check(self._lib.gwo_output_count(self._h, C.byref(n)), self._h)
        if n.value:
            cols = self.drain_arrays()
            keys, starts, ends, res = cols
            ks = self.key_strings(keys) if self._strings else [int(x) for x in keys]
            for i in range(len(keys)):
                r = tuple(x[i].item() for x in res)
                self.output.append((ks[i], int(starts[i]), int(ends[i]), r[0] if len(r) == 1 else r))
        sn = C.c_int64()
        N.check(self._lib.gwo_side_output_count(self._h, C.byref(sn)), self._h)
        if sn.value:
            m = sn.value
            k = np.empty(m, np.int64)
            t = np.empty(m, np.int64)
            v = np.empty(m, self.value_dtype)
            so = N.GwoSideOut(_ptr(k).value, _ptr(t).value, _ptr(v).value)
            got = C.c_int64()
            N.check(self._lib.gwo_drain_side_output(self._h, C.byref(so), m, C.byref(got)), self._h)
            ks = self.key_strings(k[:got.value]) if self._strings else [int(x) for x in k[:got.value]]
            for i in range(got.value):
                self.side_output.append((ks[i], int(t[i]), v[i].item()))

    def drain_arrays(self):
        """Drain pending fired rows into numpy columns: (key, start, end, [results...])."""
        n = C.c_int64()
        N.check(self._lib.gwo_output_count(self._h, C.byref(n)), self._h)
        m = n.value
        key = np.empty(m, np.int64)
        start = np.empty(m, np.int64)
        end = np.empty(m, np.int64)
        res = [np.empty(m, dt) for dt in self._result_dtypes]
        o = N.GwoOut()
        o.key, o.start, o.end = _ptr(key).value, _ptr(start).value, _ptr(end).value
        for i, r in enumerate(res):
            o.result[i] = _ptr(r).value
        got = C.c_int64()
        if m:
            N.check(self._lib.gwo_drain(self._h, C.byref(o), m, C.byref(got)), self._h, "gwo_drain")
        return key, start, end, res

    @property
    def num_late_records_dropped(self) -> int:
        n = C.c_int64()
        N.check(self._lib.gwo_late_dropped(self._h, C.byref(n)), self._h)
        return n.value

    @property
    def current_watermark(self) -> int:
        n = C.c_int64()
        N.check(self._lib.gwo_current_watermark(self._h, C.byref(n)), self._h)
        return n.value

    def snapshot_state(self):
        """Checkpoint of the keyed window state (every assigner and layout; gwo.h gwo_snapshot): numpy columns
        key, window_start, window_end, words[n, n_words], key_group, timer (rows grouped by key group, the
        heap backend's per-key-group (namespace, key, state) entries with their window timers) and the
        watermark."""
        self.flush()
        n, nw = C.c_int64(), C.c_int32()
        N.check(self._lib.gwo_snapshot_rows(self._h, C.byref(n), C.byref(nw)), self._h, "gwo_snapshot_rows")
        m = max(n.value, 1)
        cols = {"key": np.empty(m, np.int64), "window_start": np.empty(m, np.int64), "window_end": np.empty(m, np.int64),
                "words": np.empty((m, nw.value), np.int64), "key_group": np.empty(m, np.int32),
                "timer": np.empty(m, np.int32)}
        rows = N.GwoStateRows(*[_ptr(cols[c]).value for c in ("key", "window_start", "window_end", "words", "key_group",
                                                              "timer")])
        got, wm = C.c_int64(), C.c_int64()
        N.check(self._lib.gwo_snapshot(self._h, C.byref(rows), n.value, C.byref(got), C.byref(wm)), self._h,
                "gwo_snapshot")
        g = got.value
        out = {c: v[:g] for c, v in cols.items()}
        if self._strings:   # checkpoints carry the Strings: dictionary ids are private to a handle
            out["key"] = np.array(self.key_strings(out["key"]), dtype=object)
        out["watermark"] = wm.value
        return out

    def restore_state(self, snap):
        """initializeState from one or more snapshots.  A list restores a rescaled job: every subtask's rows are
        offered and only this subtask's KeyGroupRange is kept.  The restored watermark is the minimum of the
        snapshots'; each row's timer says whether its window was already emitted.  Sliding windows checkpoint
        panes, whose emitted windows follow from the watermark alone, so snapshots whose watermarks straddle a
        window end are rejected rather than restored ambiguously."""
        snaps = snap if isinstance(snap, (list, tuple)) else [snap]
        wms = [x["watermark"] for x in snaps]
        wm = min(wms)
        if self.cfg.assigner == N.ASSIGNER_SLIDING and max(wms) != wm:
            size, slide, off = self.cfg.size, self.cfg.slide, self.cfg.offset
            # the first window end e (e = off + k * slide + size) still pending at the minimum watermark: e - 1 > wm
            first_end = (wm + 2) + ((off + size - (wm + 2)) % slide)
            if first_end - 1 <= max(wms):
                raise N.GwoError(N.GWO_ERR_UNSUPPORTED, "sliding-window snapshots taken at watermarks that straddle a "
                                 "window end cannot be restored together")
        cat = lambda c, dt: np.ascontiguousarray(np.concatenate([x[c] for x in snaps]), dtype=dt)
        if self._strings:
            key = self.intern_strings([k for x in snaps for k in x["key"]])
        else:
            key = cat("key", np.int64)
        start, end = cat("window_start", np.int64), cat("window_end", np.int64)
        timer = cat("timer", np.int32)
        words = np.ascontiguousarray(np.concatenate([x["words"] for x in snaps]), dtype=np.int64)
        nw = words.shape[1] if words.ndim == 2 else 0
        n = len(key)
        if n == 0:
            key = start = end = np.zeros(1, np.int64)
            timer = np.zeros(1, np.int32)
            words = np.zeros((1, max(nw, 1)), np.int64)
        rows = N.GwoStateRows(_ptr(key).value, _ptr(start).value, _ptr(end).value, _ptr(words).value, None,
                              _ptr(timer).value)
        N.check(self._lib.gwo_restore(self._h, C.byref(rows), nw, n, wm), self._h, "gwo_restore")

    HEAP_STATE_IDS = (0, 1, 2, 3)   # window-contents, merging-window-set, event timers, processing timers

    def export_heap_state(self, ids=HEAP_STATE_IDS):
        """The keyed state in the heap state backend's per-key-group savepoint layout (gwo.h gwo_export_heap_state;
        HeapSnapshotStrategy.java:175-193): (bytes, key-group offsets into them, watermark)."""
        self.flush()
        sid = N.GwoHeapStateIds(*ids)
        need = C.c_int64()
        N.check(self._lib.gwo_export_heap_state(self._h, C.byref(sid), None, 0, C.byref(need), None, None), self._h,
                "gwo_export_heap_state")
        buf = np.zeros(max(need.value, 1), np.uint8)
        nkg = self.cfg.key_group_end - self.cfg.key_group_start + 1
        offs = np.zeros(nkg, np.int64)
        got, wm = C.c_int64(), C.c_int64()
        N.check(self._lib.gwo_export_heap_state(self._h, C.byref(sid), _ptr(buf), buf.size, C.byref(got), _ptr(offs),
                                                C.byref(wm)), self._h, "gwo_export_heap_state")
        return buf[:got.value].tobytes(), offs, wm.value

    def import_heap_state(self, data: bytes, watermark: int, ids=HEAP_STATE_IDS):
        """initializeState from heap-layout key groups (gwo.h gwo_import_heap_state): only this subtask's
        KeyGroupRange is kept; the watermark is the restored operator watermark."""
        sid = N.GwoHeapStateIds(*ids)
        buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
        buf = np.ascontiguousarray(buf)
        N.check(self._lib.gwo_import_heap_state(self._h, C.byref(sid), _ptr(buf), len(data), watermark), self._h,
                "gwo_import_heap_state")

    def state_size(self) -> int:
        n = C.c_int64()
        N.check(self._lib.gwo_state_size(self._h, C.byref(n)), self._h)
        return n.value

    @property
    def handle(self):
        return self._h
