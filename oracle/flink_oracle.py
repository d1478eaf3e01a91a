"""CPU restatement of Flink 1.12's event-time keyed window path -- TEST INFRASTRUCTURE ONLY.

This module is the parity *oracle*.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker.  The product path
(``flink_amd``) never imports it and fails loudly when the HIP library is missing.

Pinning: the pure functions here are checked against every known-answer vector the reference's
own tests hold for this path (``tests/golden/reference_vectors.json``, transcribed from the
files cited there), and the operator restatement against the end-to-end expected outputs of
``WindowOperatorTest`` and the ``SessionWindowing`` example.  ``Long.hashCode`` is a JDK
contract that no reference test pins numerically ("parity unpinned" for that one function; it
is ``(int)(v ^ (v >>> 32))``).

Every function cites the reference file:line it restates.  Paths are relative to
``/root/reference``; ``SJ/`` = ``flink-streaming-java/src/main/java/org/apache/flink/streaming/``,
``RT/`` = ``flink-runtime/src/main/java/org/apache/flink/runtime/``, ``CO/`` =
``flink-core/src/main/java/org/apache/flink/``.
"""
from __future__ import annotations

import heapq
import math
import struct
from dataclasses import dataclass, field

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1
INT_MIN = -(1 << 31)


# ----------------------------------------------------------------------------------------------
# Java integer arithmetic
# ----------------------------------------------------------------------------------------------

def i32(x: int) -> int:
    """Wrap to a Java ``int``."""
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def i64(x: int) -> int:
    """Wrap to a Java ``long``."""
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x & 0x8000000000000000 else x


def java_rem(a: int, b: int) -> int:
    """Java ``%`` on longs: truncating division, remainder takes the dividend's sign."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def urshift32(x: int, n: int) -> int:
    return (x & 0xFFFFFFFF) >> n


def urshift64(x: int, n: int) -> int:
    return (x & 0xFFFFFFFFFFFFFFFF) >> n


def rotl32(x: int, n: int) -> int:
    x &= 0xFFFFFFFF
    return i32((x << n) | (x >> (32 - n)))


# ----------------------------------------------------------------------------------------------
# Key hashing and key groups
# ----------------------------------------------------------------------------------------------

def long_hash_code(v: int) -> int:
    """JDK ``Long.hashCode(long)``: ``(int)(value ^ (value >>> 32))`` (parity unpinned: JDK)."""
    v = i64(v)
    return i32(v ^ urshift64(v, 32))


def int_hash_code(v: int) -> int:
    """JDK ``Integer.hashCode(int)``: the value itself."""
    return i32(v)


def string_hash_code(s: str) -> int:
    """JDK ``String.hashCode``: ``h = 31*h + c`` over UTF-16 code units."""
    h = 0
    data = s.encode("utf-16-le", "surrogatepass")   # Java Strings may hold lone surrogates
    for i in range(0, len(data), 2):
        c = data[i] | (data[i + 1] << 8)
        h = i32(31 * h + c)
    return h


def tuple_hash_code(*field_hashes: int) -> int:
    """``TupleN.hashCode``: CO/api/java/tuple/Tuple1.java:143-146, Tuple2.java:166-169."""
    h = 0
    for i, fh in enumerate(field_hashes):
        h = fh if i == 0 else i32(31 * h + fh)
    return h


def bit_mix(x: int) -> int:
    """``MathUtils.bitMix`` (Murmur3 fmix32), CO/util/MathUtils.java:191-198."""
    x = i32(x)
    x ^= urshift32(x, 16)
    x = i32(x * 0x85EBCA6B)
    x ^= urshift32(x, 13)
    x = i32(x * 0xC2B2AE35)
    x ^= urshift32(x, 16)
    return i32(x)


def murmur_hash(code: int) -> int:
    """``MathUtils.murmurHash(int)``, CO/util/MathUtils.java:134-154."""
    code = i32(code * 0xCC9E2D51)
    code = rotl32(code, 15)
    code = i32(code * 0x1B873593)
    code = rotl32(code, 13)
    code = i32(code * 5 + 0xE6546B64)
    code = i32(code ^ 4)
    code = bit_mix(code)
    if code >= 0:
        return code
    if code != INT_MIN:
        return -code
    return 0


def compute_key_group_for_key_hash(key_hash: int, max_parallelism: int) -> int:
    """RT/state/KeyGroupRangeAssignment.java:72-73."""
    return murmur_hash(key_hash) % max_parallelism


def assign_to_key_group(key_hash: int, max_parallelism: int) -> int:
    """RT/state/KeyGroupRangeAssignment.java:60-62 (takes the key's ``hashCode()``)."""
    return compute_key_group_for_key_hash(key_hash, max_parallelism)


def compute_operator_index_for_key_group(max_parallelism: int, parallelism: int, kg: int) -> int:
    """RT/state/KeyGroupRangeAssignment.java:118-119."""
    return kg * parallelism // max_parallelism


def assign_key_to_parallel_operator(key_hash: int, max_parallelism: int, parallelism: int) -> int:
    """RT/state/KeyGroupRangeAssignment.java:48-51."""
    return compute_operator_index_for_key_group(
        max_parallelism, parallelism, assign_to_key_group(key_hash, max_parallelism))


def compute_key_group_range_for_operator_index(max_parallelism: int, parallelism: int, index: int):
    """RT/state/KeyGroupRangeAssignment.java:88-101 -> inclusive (start, end)."""
    if not (0 < parallelism <= max_parallelism):
        raise ValueError("Maximum parallelism must not be smaller than parallelism.")
    start = (index * max_parallelism + parallelism - 1) // parallelism
    end = ((index + 1) * max_parallelism - 1) // parallelism
    return start, end


def round_up_to_power_of_two(x: int) -> int:
    """CO/util/MathUtils.java roundUpToPowerOfTwo."""
    x = i32(x - 1)
    for s in (1, 2, 4, 8, 16):
        x |= x >> s
    return i32(x + 1)


def compute_default_max_parallelism(parallelism: int) -> int:
    """RT/state/KeyGroupRangeAssignment.java:129-137 (lower bound 128, upper 1<<15)."""
    return min(max(round_up_to_power_of_two(parallelism + parallelism // 2), 128), 1 << 15)


# ----------------------------------------------------------------------------------------------
# Time windows and assigners
# ----------------------------------------------------------------------------------------------

@dataclass(frozen=True, order=True)
class TimeWindow:
    """SJ/api/windowing/windows/TimeWindow.java."""
    start: int
    end: int

    def max_timestamp(self) -> int:
        """TimeWindow.java:85-87."""
        return i64(self.end - 1)

    def intersects(self, other: "TimeWindow") -> bool:
        """TimeWindow.java:120-122 (inclusive: [10,20) intersects [20,30))."""
        return self.start <= other.end and self.end >= other.start

    def cover(self, other: "TimeWindow") -> "TimeWindow":
        """TimeWindow.java:127-129."""
        return TimeWindow(min(self.start, other.start), max(self.end, other.end))


def get_window_start_with_offset(timestamp: int, offset: int, window_size: int) -> int:
    """TimeWindow.java:270-272 -- Java truncating ``%`` replicated, including its negative-ts quirk."""
    return i64(timestamp - java_rem(i64(timestamp - offset + window_size), window_size))


def merge_windows(windows, callback):
    """TimeWindow.java:217-262: sort by start, sweep-merge intersecting windows.

    ``callback(to_be_merged: set, merge_result)`` is invoked for every group of size > 1.
    Java's ``Collections.sort`` is stable, so ties in ``start`` keep input order.
    """
    sorted_windows = sorted(windows, key=lambda w: w.start)
    merged = []
    current = None
    for cand in sorted_windows:
        if current is None:
            current = [cand, {cand}]
        elif current[0].intersects(cand):
            current[0] = current[0].cover(cand)
            current[1].add(cand)
        else:
            merged.append(current)
            current = [cand, {cand}]
    if current is not None:
        merged.append(current)
    for res, group in merged:
        if len(group) > 1:
            callback(group, res)


class NoTimestampError(RuntimeError):
    """TumblingEventTimeWindows.java:76-79: ``Record has Long.MIN_VALUE timestamp``."""


class TumblingEventTimeWindows:
    """SJ/api/windowing/assigners/TumblingEventTimeWindows.java:57-81 (stagger ALIGNED)."""
    merging = False

    def __init__(self, size: int, offset: int = 0):
        if abs(offset) >= size:
            raise ValueError("TumblingEventTimeWindows parameters must satisfy abs(offset) < size")
        self.size = size
        self.offset = offset

    def assign_windows(self, timestamp: int):
        if timestamp <= LONG_MIN:
            raise NoTimestampError("Record has Long.MIN_VALUE timestamp (= no timestamp marker).")
        # (globalOffset + staggerOffset) % size with ALIGNED stagger = 0 (WindowStagger.java:34-40)
        off = java_rem(self.offset + 0, self.size)
        start = get_window_start_with_offset(timestamp, off, self.size)
        return [TimeWindow(start, i64(start + self.size))]


class SlidingEventTimeWindows:
    """SJ/api/windowing/assigners/SlidingEventTimeWindows.java:56-82."""
    merging = False

    def __init__(self, size: int, slide: int, offset: int = 0):
        if abs(offset) >= slide or size <= 0:
            raise ValueError("SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0")
        self.size = size
        self.slide = slide
        self.offset = offset

    def assign_windows(self, timestamp: int):
        if timestamp <= LONG_MIN:
            raise NoTimestampError("Record has Long.MIN_VALUE timestamp (= no timestamp marker).")
        out = []
        start = get_window_start_with_offset(timestamp, self.offset, self.slide)
        while start > timestamp - self.size:
            out.append(TimeWindow(start, i64(start + self.size)))
            start -= self.slide
        return out


class EventTimeSessionWindows:
    """SJ/api/windowing/assigners/EventTimeSessionWindows.java:50-112."""
    merging = True

    def __init__(self, gap: int):
        if gap <= 0:
            raise ValueError("EventTimeSessionWindows parameters must satisfy 0 < size")
        self.gap = gap

    def assign_windows(self, timestamp: int):
        return [TimeWindow(timestamp, i64(timestamp + self.gap))]

    def merge_windows(self, windows, callback):
        merge_windows(windows, callback)


class MergingWindowSet:
    """SJ/runtime/operators/windowing/MergingWindowSet.java:81-225 (mapping in-flight -> state window)."""

    def __init__(self, assigner, mapping: dict):
        self.assigner = assigner
        self.mapping = mapping          # the persisted dict is mutated in place (persist() is implicit)
        self.initial = dict(mapping)    # MergingWindowSet.java:81-96: the mapping as restored

    def persist(self):
        """MergingWindowSet.java:102-109: rewrite the list state only if the mapping changed; returns the
        (window, state window) entries added to the state (None: the state is left untouched)."""
        if self.mapping == self.initial:
            return None
        return list(self.mapping.items())

    def get_state_window(self, w):
        return self.mapping.get(w)

    def retire_window(self, w):
        if self.mapping.pop(w, None) is None:
            raise RuntimeError(f"Window {w} is not in in-flight window set.")

    def add_window(self, new_window, merge_function):
        windows = list(self.mapping.keys()) + [new_window]
        merge_results = {}

        def cb(to_be_merged, merge_result):
            merge_results[merge_result] = set(to_be_merged)

        self.assigner.merge_windows(windows, cb)
        result_window = new_window
        merged_new_window = False
        for merge_result, merged_windows in merge_results.items():
            if new_window in merged_windows:
                merged_windows.discard(new_window)
                merged_new_window = True
                result_window = merge_result
            # "pick any of the merged windows": the survivors are all pre-existing in-flight
            # windows; the choice only names the state namespace and never changes results.
            first = min(merged_windows)
            merged_state_window = self.mapping.get(first)
            merged_state_windows = []
            for mw in sorted(merged_windows):
                res = self.mapping.pop(mw, None)
                if res is not None:
                    merged_state_windows.append(res)
            self.mapping[merge_result] = merged_state_window
            if merged_state_window in merged_state_windows:
                merged_state_windows.remove(merged_state_window)
            if not (merge_result in merged_windows and len(merged_windows) == 1):
                merge_function(merge_result, merged_windows, self.mapping.get(merge_result),
                               merged_state_windows)
        if not merge_results or (result_window == new_window and not merged_new_window):
            self.mapping[result_window] = result_window
        return result_window


# ----------------------------------------------------------------------------------------------
# Aggregate functions (CO/api/common/functions/AggregateFunction.java:115-164 contract)
# ----------------------------------------------------------------------------------------------

def _double_sort_key(x: float) -> int:
    """``Double.compareTo`` total order via ``doubleToLongBits`` (NaN canonical, -0.0 < 0.0)."""
    if math.isnan(x):
        bits = 0x7FF8000000000000
    else:
        bits = struct.unpack("<q", struct.pack("<d", x))[0]
    return bits if bits >= 0 else bits ^ 0x7FFFFFFFFFFFFFFF


class Agg:
    """Base: mirrors ``AggregateFunction<IN, ACC, OUT>``; ``add`` returns the new accumulator."""
    name = "agg"
    is_double = False

    def create_accumulator(self):
        raise NotImplementedError

    def add(self, value, acc):
        raise NotImplementedError

    def get_result(self, acc):
        return acc

    def merge(self, a, b):
        raise NotImplementedError


class CountAgg(Agg):
    name = "count"

    def create_accumulator(self):
        return 0

    def add(self, value, acc):
        return i64(acc + 1)

    def merge(self, a, b):
        return i64(a + b)


class SumLongAgg(Agg):
    """``SumFunction.LongSum``: Java wrap-around ``long + long`` (SumFunction.java:63-68)."""
    name = "sum"

    def create_accumulator(self):
        return 0

    def add(self, value, acc):
        return i64(acc + value)

    def merge(self, a, b):
        return i64(a + b)


class SumDoubleAgg(Agg):
    """``SumFunction.DoubleSum`` (SumFunction.java:72-78)."""
    name = "sum"
    is_double = True

    def create_accumulator(self):
        return 0.0

    def add(self, value, acc):
        return acc + float(value)

    def merge(self, a, b):
        return a + b


class MinAgg(Agg):
    """``ComparableAggregator`` MIN (ComparableAggregator.java:72-94, Comparator.java:99-107)."""
    name = "min"

    def __init__(self, is_double=False):
        self.is_double = is_double

    def create_accumulator(self):
        return None

    def add(self, value, acc):
        if acc is None:
            return value
        if self.is_double:
            return acc if _double_sort_key(acc) < _double_sort_key(value) else value
        return acc if acc < value else value

    def merge(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        return self.add(b, a)


class MaxAgg(MinAgg):
    """``ComparableAggregator`` MAX (Comparator.java:50-58)."""
    name = "max"

    def add(self, value, acc):
        if acc is None:
            return value
        if self.is_double:
            return acc if _double_sort_key(acc) > _double_sort_key(value) else value
        return acc if acc > value else value


class AvgAgg(Agg):
    """``AverageAggregate`` of docs/dev/stream/operators/windows.md:493-514: acc (sum, count)."""
    name = "avg"
    result_is_double = True

    def __init__(self, is_double=False):
        self.is_double = is_double

    def create_accumulator(self):
        return (0.0 if self.is_double else 0, 0)

    def add(self, value, acc):
        s, c = acc
        return ((s + float(value)) if self.is_double else i64(s + value), c + 1)

    def get_result(self, acc):
        s, c = acc
        return float(s) / c

    def merge(self, a, b):
        s = a[0] + b[0] if self.is_double else i64(a[0] + b[0])
        return (s, a[1] + b[1])


class MultiAgg(Agg):
    """Several aggregates over the same value in one accumulator (C4: sum/min/max)."""

    def __init__(self, aggs):
        self.aggs = list(aggs)
        self.name = "+".join(a.name for a in self.aggs)

    def create_accumulator(self):
        return tuple(a.create_accumulator() for a in self.aggs)

    def add(self, value, acc):
        return tuple(a.add(value, x) for a, x in zip(self.aggs, acc))

    def get_result(self, acc):
        return tuple(a.get_result(x) for a, x in zip(self.aggs, acc))

    def merge(self, a, b):
        return tuple(f.merge(x, y) for f, x, y in zip(self.aggs, a, b))


# ----------------------------------------------------------------------------------------------
# WindowOperator (event time, EventTimeTrigger, AggregatingState)
# ----------------------------------------------------------------------------------------------

@dataclass
class OutputRow:
    key: int
    start: int
    end: int
    result: object
    timestamp: int          # record timestamp = window.maxTimestamp() (WindowOperator.java:547)


class WindowOperatorOracle:
    """Restates SJ/runtime/operators/windowing/WindowOperator.java:294-653 for one subtask.

    Trigger = EventTimeTrigger (SJ/api/windowing/triggers/EventTimeTrigger.java:37-81).
    Timers = InternalTimerServiceImpl (SJ/api/operators/InternalTimerServiceImpl.java:216-278):
    a set deduplicated on (timestamp, key, window), fired in timestamp order.
    """

    def __init__(self, assigner, agg: Agg, allowed_lateness: int = 0, side_output: bool = False,
                 key_group_range=None, max_parallelism: int = 128, key_hash=long_hash_code):
        if allowed_lateness < 0:
            raise ValueError("The allowed lateness cannot be negative.")
        self.assigner = assigner
        self.agg = agg
        self.lateness = allowed_lateness
        self.side_output_enabled = side_output
        self.key_group_range = key_group_range
        self.max_parallelism = max_parallelism
        self.key_hash = key_hash
        self.wm = LONG_MIN                       # InternalTimerServiceImpl.currentWatermark
        self.state = {}                          # (key, window) -> acc   ("window-contents")
        self.merging_sets = {}                   # key -> {in-flight window: state window}
        self.timers = set()                      # (ts, key, window)
        self.heap = []
        self.output: list[OutputRow] = []
        self.side_output: list[tuple] = []
        self.num_late_records_dropped = 0

    # -- helpers ------------------------------------------------------------------------------
    def _cleanup_time(self, w: TimeWindow) -> int:
        """WindowOperator.java:639-646 (overflow -> Long.MAX_VALUE)."""
        ct = w.max_timestamp() + self.lateness
        return ct if ct <= LONG_MAX and ct >= w.max_timestamp() else LONG_MAX

    def _is_window_late(self, w) -> bool:
        """WindowOperator.java:578-580."""
        return self._cleanup_time(w) <= self.wm

    def _is_element_late(self, ts) -> bool:
        """WindowOperator.java:588-591 (Java long arithmetic)."""
        return i64(ts + self.lateness) <= self.wm

    def _register_timer(self, ts, key, w):
        t = (ts, key, w)
        if t not in self.timers:
            self.timers.add(t)
            heapq.heappush(self.heap, t)

    def _delete_timer(self, ts, key, w):
        self.timers.discard((ts, key, w))

    def _register_cleanup_timer(self, key, w):
        """WindowOperator.java:598-610."""
        ct = self._cleanup_time(w)
        if ct == LONG_MAX:
            return
        self._register_timer(ct, key, w)

    def _delete_cleanup_timer(self, key, w):
        """WindowOperator.java:617-628."""
        ct = self._cleanup_time(w)
        if ct == LONG_MAX:
            return
        self._delete_timer(ct, key, w)

    def _emit(self, key, w, acc):
        """WindowOperator.java:546-550 via InternalSingleValueWindowFunction."""
        self.output.append(OutputRow(key, w.start, w.end, self.agg.get_result(acc), w.max_timestamp()))

    def _check_key(self, key):
        if self.key_group_range is None:
            return
        kg = assign_to_key_group(self.key_hash(key), self.max_parallelism)
        lo, hi = self.key_group_range
        if not (lo <= kg <= hi):
            raise ValueError(f"Key group {kg} is not in KeyGroupRange{{startKeyGroup={lo}, endKeyGroup={hi}}}.")

    # -- OneInputStreamOperator ---------------------------------------------------------------
    def process_element(self, key, ts, value):
        """WindowOperator.java:294-427."""
        self._check_key(key)
        windows = self.assigner.assign_windows(ts)
        skipped = True
        if self.assigner.merging:
            mapping = self.merging_sets.setdefault(key, {})
            mws = MergingWindowSet(self.assigner, mapping)
            for window in windows:
                def merge_fn(merge_result, merged_windows, state_window_result, merged_state_windows):
                    if merge_result.max_timestamp() + self.lateness <= self.wm:
                        raise RuntimeError(
                            "The end timestamp of an event-time window cannot become earlier than "
                            "the current watermark by merging.")
                    # EventTimeTrigger.onMerge (EventTimeTrigger.java:72-81)
                    if merge_result.max_timestamp() > self.wm:
                        self._register_timer(merge_result.max_timestamp(), key, merge_result)
                    for m in merged_windows:
                        self._delete_timer(m.max_timestamp(), key, m)     # trigger.clear
                        self._delete_cleanup_timer(key, m)
                    # AbstractHeapMergingState.mergeNamespaces (RT/state/heap/AbstractHeapMergingState.java:67-90)
                    merged = None
                    for src in merged_state_windows:
                        s = self.state.pop((key, src), None)
                        if merged is not None and s is not None:
                            merged = self.agg.merge(merged, s)
                        elif merged is None:
                            merged = s
                    if merged is not None:
                        tgt = self.state.get((key, state_window_result))
                        self.state[(key, state_window_result)] = (
                            merged if tgt is None else self.agg.merge(tgt, merged))

                actual = mws.add_window(window, merge_fn)
                if self._is_window_late(actual):
                    mws.retire_window(actual)
                    continue
                skipped = False
                state_window = mws.get_state_window(actual)
                if state_window is None:
                    raise RuntimeError(f"Window {window} is not in in-flight window set.")
                self._add_and_trigger(key, actual, state_window, value)
            if not mapping:
                self.merging_sets.pop(key, None)
        else:
            for window in windows:
                if self._is_window_late(window):
                    continue
                skipped = False
                self._add_and_trigger(key, window, window, value)
        if skipped and self._is_element_late(ts):
            if self.side_output_enabled:
                self.side_output.append((key, ts, value))
            else:
                self.num_late_records_dropped += 1

    def _add_and_trigger(self, key, window, state_window, value):
        sk = (key, state_window)
        acc = self.state.get(sk)
        if acc is None:
            acc = self.agg.create_accumulator()
        self.state[sk] = self.agg.add(value, acc)          # HeapAggregatingState.add :96-109
        # EventTimeTrigger.onElement (EventTimeTrigger.java:37-45)
        if window.max_timestamp() <= self.wm:
            contents = self.state.get(sk)
            if contents is not None:
                self._emit(key, window, contents)
        else:
            self._register_timer(window.max_timestamp(), key, window)
        self._register_cleanup_timer(key, window)

    def process_watermark(self, wm):
        """AbstractStreamOperator.processWatermark (:566-571) -> advanceWatermark (:268-278)."""
        self.wm = wm
        while self.heap and self.heap[0][0] <= wm:
            t = heapq.heappop(self.heap)
            if t not in self.timers:
                continue                                # deleted timer
            self.timers.discard(t)
            self._on_event_time(*t)

    def _on_event_time(self, time, key, window):
        """WindowOperator.java:430-473."""
        mapping = None
        if self.assigner.merging:
            mapping = self.merging_sets.get(key, {})
            state_window = mapping.get(window)
            if state_window is None:
                return
        else:
            state_window = window
        sk = (key, state_window)
        if time == window.max_timestamp():                  # EventTimeTrigger.onEventTime :48-52
            contents = self.state.get(sk)
            if contents is not None:
                self._emit(key, window, contents)
        if time == self._cleanup_time(window):              # isCleanupTime :651-653
            self.state.pop(sk, None)                        # clearAllState :528-540
            self._delete_timer(window.max_timestamp(), key, window)
            if mapping is not None:
                mapping.pop(window, None)
                if not mapping:
                    self.merging_sets.pop(key, None)

    def end_input(self):
        """A bounded source ends with Watermark.MAX_WATERMARK (SJ/api/operators/StreamSource.java:122)."""
        self.process_watermark(LONG_MAX)


# ----------------------------------------------------------------------------------------------
# Stream drivers used by tests
# ----------------------------------------------------------------------------------------------

def run_stream(op: WindowOperatorOracle, events):
    """``events``: iterable of ('e', key, ts, value) / ('w', wm) tuples."""
    for ev in events:
        if ev[0] == "e":
            op.process_element(ev[1], ev[2], ev[3])
        else:
            op.process_watermark(ev[1])
    return op


def rows_as_tuples(rows):
    return sorted((r.key, r.start, r.end, r.result) for r in rows)


# ----------------------------------------------------------------------------------------------
# splitmix64 synthetic generators -- shared definition with the HIP generator
# ----------------------------------------------------------------------------------------------

MASK64 = 0xFFFFFFFFFFFFFFFF


def splitmix64(x: int) -> int:
    """splitmix64 finaliser applied to ``x`` (a counter-based generator: value i = mix(seed + i*gamma))."""
    z = (x + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)
