"""CPU restatement of the heap keyed state backend's savepoint layout for WindowOperator's state.

TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline): nothing on the product path imports this module.
It is the checker of gwo_export_heap_state / gwo_import_heap_state (include/gwo.h, flink_amd/csrc/gwo_heapstate.cpp).

Pinned against the reference's own savepoint fixtures (tests/golden/heap_state/, copied data files of
flink-streaming-java/src/test/resources/win-op-migration-test-*-flink1.11-snapshot, written by
WindowOperatorMigrationTest.java:320-375/431-485/119-161): the parser reads them to their last byte and finds the
state the generating test put in, see tests/test_heap_state_format.py.

What is restated, with the reference file it follows:
* OperatorSnapshotUtil.java:122-190 -- the test-harness file: version, a null stream handle, raw/managed operator
  handles, raw/managed keyed handles, then the channel-state collections.
* MetadataV2V3SerializerBase.java:298-352 (KEY_GROUPS_HANDLE = 3: start key group, count, offsets, delegate) and
  :472-499 (BYTE_STREAM_STATE_HANDLE = 1: handle name, byte length, bytes); :380-410 operator handles.
* KeyedBackendSerializationProxy.java:114-128 + StateMetaInfoSnapshotReadersWriters.java:163-186 -- the keyed
  backend's metadata: its state names, in the order of their ids (HeapSnapshotStrategy.java:246-263).
* HeapSnapshotStrategy.java:175-193 -- per key group: int key group, then per state (any order) short state id and
  the state's entries.
* CopyOnWriteStateMapSnapshot.java:113-131 -- a key/value state: int count, (namespace, key, value) per entry.
* KeyGroupPartitioner.java:251-264 + TimerSerializer.java:158-162 -- a timer queue: int count, (flipSignBit(ts),
  key, namespace) per timer.
* TimeWindow.Serializer (start, end longs), StringValue.writeString (7-bit varint of length+1, then one varint per
  UTF-16 unit), IntSerializer / LongSerializer (big-endian), VoidNamespaceSerializer (one zero byte),
  ListSerializer (int size + elements), TupleSerializer (fields back to back), LongPrimitiveArraySerializer (int
  length + longs: the GpuAggregates accumulator).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

NULL_HANDLE, BYTE_STREAM_STATE_HANDLE, KEY_GROUPS_HANDLE, PARTITIONABLE_OPERATOR_STATE_HANDLE = 0, 1, 3, 4
KEY_VALUE, PRIORITY_QUEUE = 0, 3          # StateMetaInfoSnapshot.BackendStateType ordinals
FLIP = 1 << 63

WINDOW_CONTENTS = "window-contents"
MERGING_WINDOW_SET = "merging-window-set"
EVENT_TIMERS = "_timer_state/event_window-timers"
PROCESSING_TIMERS = "_timer_state/processing_window-timers"


class Reader:
    """DataInputView (big-endian)."""

    def __init__(self, data: bytes, pos: int = 0, end: int | None = None):
        self.d, self.p = data, pos
        self.end = len(data) if end is None else end

    def take(self, n: int) -> bytes:
        if self.p + n > self.end:
            raise ValueError(f"truncated: {n} bytes at {self.p}, region ends at {self.end}")
        b = self.d[self.p:self.p + n]
        self.p += n
        return b

    def u8(self): return self.take(1)[0]
    def i16(self): return struct.unpack(">h", self.take(2))[0]
    def i32(self): return struct.unpack(">i", self.take(4))[0]
    def i64(self): return struct.unpack(">q", self.take(8))[0]
    def boolean(self): return self.u8() != 0

    def utf(self) -> str:                  # DataOutput.writeUTF (the names here are ASCII)
        return self.take(struct.unpack(">H", self.take(2))[0]).decode("utf-8", "surrogatepass")

    def varint(self) -> int:
        v = self.u8()
        if v < 0x80:
            return v
        v &= 0x7F
        shift = 7
        while True:
            c = self.u8()
            if c < 0x80:
                return v | (c << shift)
            v |= (c & 0x7F) << shift
            shift += 7

    def string_value(self):                # StringValue.readString
        n = self.varint()
        if n == 0:
            return None
        units = [self.varint() for _ in range(n - 1)]
        return struct.pack(f"<{len(units)}H", *units).decode("utf-16-le", "surrogatepass")


class Writer:
    """DataOutputView (big-endian)."""

    def __init__(self):
        self.b = bytearray()

    def u8(self, v): self.b.append(v & 0xFF)
    def i16(self, v): self.b += struct.pack(">h", v)
    def i32(self, v): self.b += struct.pack(">i", v)
    def i64(self, v): self.b += struct.pack(">q", v)

    def varint(self, v: int):
        while v >= 0x80:
            self.u8(v | 0x80)
            v >>= 7
        self.u8(v)

    def string_value(self, s: str):        # StringValue.writeString
        units = struct.unpack(f"<{len(s.encode('utf-16-le', 'surrogatepass')) // 2}H",
                              s.encode("utf-16-le", "surrogatepass"))
        self.varint(len(units) + 1)
        for u in units:
            self.varint(u)

    def bytes(self) -> bytes:
        return bytes(self.b)


# ---- serializers ---------------------------------------------------------------------------------------------------

def key_codec(kind: str):
    """(read, write) of a key serializer: "long" LongSerializer, "int" IntSerializer, "string" StringSerializer."""
    if kind == "long":
        return (lambda r: r.i64()), (lambda w, k: w.i64(k))
    if kind == "int":
        return (lambda r: r.i32()), (lambda w, k: w.i32(k))
    if kind == "string":
        return (lambda r: r.string_value()), (lambda w, k: w.string_value(k))
    raise ValueError(kind)


def read_time_window(r: Reader):
    return (r.i64(), r.i64())


def read_long_array(r: Reader):            # LongPrimitiveArraySerializer
    return tuple(r.i64() for _ in range(r.i32()))


def read_string_int_tuple(r: Reader):      # TupleSerializer<Tuple2<String, Integer>>
    return (r.string_value(), r.i32())


def list_of(read_elem):                    # ListSerializer
    return lambda r: [read_elem(r) for _ in range(r.i32())]


def read_window_pair(r: Reader):           # MergingWindowSet's Tuple2<TimeWindow, TimeWindow>
    return (read_time_window(r), read_time_window(r))


# ---- the harness file and its handles -----------------------------------------------------------------------------

@dataclass
class KeyGroupsHandle:
    start_kg: int
    offsets: list
    name: str
    data: bytes


def _stream_handle(r: Reader):
    t = r.u8()
    if t == NULL_HANDLE:
        return None
    if t != BYTE_STREAM_STATE_HANDLE:
        raise ValueError(f"stream handle type {t} (only in-memory byte streams are read here)")
    name = r.utf()
    return name, r.take(r.i32())


def _operator_handle(r: Reader):
    t = r.u8()
    if t == NULL_HANDLE:
        return None
    if t != PARTITIONABLE_OPERATOR_STATE_HANDLE:
        raise ValueError(f"operator handle type {t}")
    parts = {}
    for _ in range(r.i32()):
        name = r.utf()
        mode = r.u8()
        parts[name] = (mode, [r.i64() for _ in range(r.i32())])
    return parts, _stream_handle(r)


def _keyed_handle(r: Reader):
    t = r.u8()
    if t == NULL_HANDLE:
        return None
    if t != KEY_GROUPS_HANDLE:
        raise ValueError(f"keyed handle type {t} (incremental handles are not heap snapshots)")
    start, n = r.i32(), r.i32()
    offsets = [r.i64() for _ in range(n)]
    name, data = _stream_handle(r)
    return KeyGroupsHandle(start, offsets, name, data)


def read_operator_subtask_state(blob: bytes) -> dict:
    """OperatorSnapshotUtil.readStateHandle: every collection, the file consumed to its last byte."""
    r = Reader(blob)
    out = {"version": r.i32()}
    if _stream_handle(r) is not None:
        raise ValueError("expected the null compatibility handle")
    for part, fn in (("raw_operator", _operator_handle), ("managed_operator", _operator_handle),
                     ("raw_keyed", _keyed_handle), ("managed_keyed", _keyed_handle)):
        n = r.i32()
        out[part] = None if n < 0 else [fn(r) for _ in range(n)]
    if out["version"] == 3:
        out["input_channel"], out["result_subpartition"] = r.i32(), r.i32()
        if out["input_channel"] or out["result_subpartition"]:
            raise ValueError("channel state is not part of a window operator savepoint here")
    if r.p != len(blob):
        raise ValueError(f"{len(blob) - r.p} trailing bytes")
    return out


def state_meta(data: bytes, end: int):
    """The keyed backend's state names in id order, with their backend state type and KEYED_STATE_TYPE option.

    The metadata (KeyedBackendSerializationProxy.write) holds Java serializer snapshots, which cannot be skipped
    without their classes; every state's entry starts with writeUTF(name), writeInt(type), writeInt(#options) and
    either the KEYED_STATE_TYPE option (key/value states) or the VALUE_SERIALIZER entry (priority queues), which is
    what is matched here.  The proxy header is checked: version 6, key groups uncompressed."""
    r = Reader(data, 0, end)
    version = r.i32()
    if version != 6:
        raise ValueError(f"serialization proxy version {version}")
    if r.boolean():
        raise ValueError("compressed key groups (snappy) are not read here")
    found = []
    p = r.p
    while p + 2 < end:
        L = struct.unpack_from(">H", data, p)[0]
        q = p + 2 + L
        if 0 < L < 256 and q + 8 <= end and all(32 <= c < 127 for c in data[p + 2:q]):
            typ, nopt = struct.unpack_from(">ii", data, q)
            try:
                nxt = Reader(data, q + 8, end)
                if typ == KEY_VALUE and 1 <= nopt <= 8:
                    if nxt.utf() == "KEYED_STATE_TYPE":
                        found.append((data[p + 2:q].decode(), typ, nxt.utf()))
                elif typ == PRIORITY_QUEUE and nopt == 0:
                    if nxt.i32() >= 1 and nxt.utf() == "VALUE_SERIALIZER":
                        found.append((data[p + 2:q].decode(), typ, None))
            except (ValueError, UnicodeDecodeError):
                pass
        p += 1
    return found


def read_key_groups(h: KeyGroupsHandle, decoders: dict) -> tuple[list, dict]:
    """Every key group of a heap snapshot: {state name: [(key group, entry), ...]}.

    ``decoders`` maps a state name to a function reading ONE entry of that state (namespace, key, value / timer);
    each key group's region must be consumed exactly."""
    meta = state_meta(h.data, h.offsets[0] if h.offsets else len(h.data))
    names = [m[0] for m in meta]
    out = {n: [] for n in names}
    for i, off in enumerate(h.offsets):
        end = h.offsets[i + 1] if i + 1 < len(h.offsets) else len(h.data)
        r = Reader(h.data, off, end)
        kg = r.i32()
        if kg != h.start_kg + i:
            raise ValueError(f"key group {kg} at position {i}")
        seen = set()
        for _ in names:
            sid = r.i16()
            if not 0 <= sid < len(names) or sid in seen:
                raise ValueError(f"state id {sid}")
            seen.add(sid)
            dec = decoders[names[sid]]
            for _ in range(r.i32()):
                out[names[sid]].append((kg, dec(r)))
        if r.p != end:
            raise ValueError(f"key group {kg}: {end - r.p} unread bytes")
    return meta, out


def window_operator_decoders(key_kind: str, value_reader, merging: bool, extra: dict | None = None):
    """Entry readers of WindowOperator's states (WindowOperator.java:251-276, InternalTimerServiceImpl)."""
    rk, _ = key_codec(key_kind)
    def timer(r):
        return _signed(r.i64() ^ FLIP), rk(r), read_time_window(r)

    dec = {
        WINDOW_CONTENTS: lambda r: (read_time_window(r), rk(r), value_reader(r)),
        EVENT_TIMERS: timer,
        PROCESSING_TIMERS: timer,
    }
    if merging:
        def mws(r):
            if r.u8() != 0:
                raise ValueError("VoidNamespace byte")
            return rk(r), list_of(read_window_pair)(r)
        dec[MERGING_WINDOW_SET] = mws
    dec.update(extra or {})
    return dec


def _signed(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= 1 << 63 else x


# ---- the GPU operator's state in this layout (the export's expected content, the import's input) ------------------

DEFAULT_IDS = {WINDOW_CONTENTS: 0, MERGING_WINDOW_SET: 1, EVENT_TIMERS: 2, PROCESSING_TIMERS: 3}


def _bits(x: float) -> int:
    return struct.unpack(">q", struct.pack(">d", x))[0]


def gpu_accumulator(agg, acc) -> tuple:
    """An oracle accumulator as GpuAggregates' long[] (GpuAggregates.java:49-100): two longs per aggregate."""
    aggs = getattr(agg, "aggs", None)
    if aggs is None:
        aggs, acc = [agg], (acc,)
    out = []
    for a, x in zip(aggs, acc):
        if a.name == "count":
            out += [x, 0]
        elif a.name == "sum":
            out += [_bits(x) if a.is_double else x, 0]
        elif a.name in ("min", "max"):
            out += [_bits(x), 1] if a.is_double else [x, 0]
        elif a.name == "avg":
            out += [_bits(x[0]) if a.is_double else x[0], x[1]]
        else:
            raise ValueError(a.name)
    return tuple(out)


@dataclass
class WindowState:
    """WindowOperator's keyed state, resolved: contents {(key, window): long[]}, merging sets {key: {window: state
    window}}, event timers {(ts, key, window)}."""
    contents: dict = field(default_factory=dict)
    merging: dict = field(default_factory=dict)
    timers: set = field(default_factory=set)

    def resolved(self):
        """(key, window) -> accumulator as the windows see it (sessions: through their state windows)."""
        if not self.merging:
            return dict(self.contents)
        out = {}
        for key, m in self.merging.items():
            for w, sw in m.items():
                if (key, sw) in self.contents:
                    out[(key, w)] = self.contents[(key, sw)]
        return out


def state_of_oracle(op) -> WindowState:
    """The oracle WindowOperator's state (oracle/flink_oracle.py WindowOperatorOracle) as heap-backend content."""
    s = WindowState()
    for (key, w), acc in op.state.items():
        if acc is not None:
            s.contents[(key, (w.start, w.end))] = gpu_accumulator(op.agg, acc)
    for key, m in op.merging_sets.items():
        s.merging[key] = {(w.start, w.end): (sw.start, sw.end) for w, sw in m.items()}
    for ts, key, w in op.timers:
        s.timers.add((ts, key, (w.start, w.end)))
    return s


def parse_export(buf: bytes, key_kind: str, merging: bool, kg_range, ids=None) -> WindowState:
    """gwo_export_heap_state's bytes (key groups back to back, no metadata) -> WindowState."""
    ids = dict(DEFAULT_IDS if ids is None else ids)
    if not merging:
        ids.pop(MERGING_WINDOW_SET, None)
    by_id = {v: k for k, v in ids.items()}
    dec = window_operator_decoders(key_kind, read_long_array, merging)
    s = WindowState()
    r = Reader(buf)
    for kg in range(kg_range[0], kg_range[1] + 1):
        if r.i32() != kg:
            raise ValueError(f"expected key group {kg}")
        for _ in range(len(ids)):
            name = by_id[r.i16()]
            for _ in range(r.i32()):
                e = dec[name](r)
                if name == WINDOW_CONTENTS:
                    s.contents[(e[1], e[0])] = e[2]
                elif name == MERGING_WINDOW_SET:
                    s.merging[e[0]] = {w: sw for w, sw in e[1]}
                elif name == EVENT_TIMERS:
                    s.timers.add(e)
                else:
                    raise ValueError("processing-time timer in an event-time window operator")
    if r.p != len(buf):
        raise ValueError(f"{len(buf) - r.p} trailing bytes")
    return s


def write_state(s: WindowState, key_kind: str, key_group_of, kg_range, ids=None) -> bytes:
    """WindowState -> the key-group sections gwo_import_heap_state reads (HeapSnapshotStrategy.java:175-193)."""
    ids = dict(DEFAULT_IDS if ids is None else ids)
    merging = bool(s.merging)
    if not merging:
        ids.pop(MERGING_WINDOW_SET, None)
    _, wk = key_codec(key_kind)
    w = Writer()
    for kg in range(kg_range[0], kg_range[1] + 1):
        w.i32(kg)
        for name, sid in sorted(ids.items(), key=lambda kv: kv[1]):
            w.i16(sid)
            if name == WINDOW_CONTENTS:
                es = [(k, win, acc) for (k, win), acc in s.contents.items() if key_group_of(k) == kg]
                w.i32(len(es))
                for k, win, acc in es:
                    w.i64(win[0]); w.i64(win[1]); wk(w, k)
                    w.i32(len(acc))
                    for x in acc:
                        w.i64(x)
            elif name == MERGING_WINDOW_SET:
                ks = [k for k in s.merging if key_group_of(k) == kg]
                w.i32(len(ks))
                for k in ks:
                    w.u8(0); wk(w, k)
                    w.i32(len(s.merging[k]))
                    for win, sw in s.merging[k].items():
                        w.i64(win[0]); w.i64(win[1]); w.i64(sw[0]); w.i64(sw[1])
            elif name == EVENT_TIMERS:
                ts = [t for t in s.timers if key_group_of(t[1]) == kg]
                w.i32(len(ts))
                for t, k, win in ts:
                    w.i64(_signed(t ^ FLIP)); wk(w, k); w.i64(win[0]); w.i64(win[1])
            else:
                w.i32(0)
    return w.bytes()
