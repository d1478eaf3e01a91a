"""Window assigners and aggregate functions of the GPU window path -- Flink API mirrors.

Names, argument meaning and error behaviour follow the reference:
``TumblingEventTimeWindows.of(size[, offset])`` (SJ/api/windowing/assigners/TumblingEventTimeWindows.java:57-60,
107-131), ``SlidingEventTimeWindows.of(size, slide[, offset])`` (SlidingEventTimeWindows.java:56-60, 110-132),
``EventTimeSessionWindows.withGap(gap)`` (EventTimeSessionWindows.java:50-55, 82-85) and the
GPU-describable ``AggregateFunction`` subset (CO/api/common/functions/AggregateFunction.java:115-164).
Times are milliseconds (Flink's ``Time.milliseconds``).
"""
from __future__ import annotations

from dataclasses import dataclass

from . import _native as N


class Time:
    """``org.apache.flink.streaming.api.windowing.time.Time`` (milliseconds)."""

    @staticmethod
    def milliseconds(x: int) -> int:
        return int(x)

    @staticmethod
    def seconds(x: int) -> int:
        return int(x) * 1000

    @staticmethod
    def minutes(x: int) -> int:
        return int(x) * 60_000

    @staticmethod
    def hours(x: int) -> int:
        return int(x) * 3_600_000


@dataclass(frozen=True)
class TimeWindow:
    start: int
    end: int

    def max_timestamp(self) -> int:
        return self.end - 1


class WindowAssigner:
    kind = -1
    merging = False

    def is_event_time(self) -> bool:
        return True


class TumblingEventTimeWindows(WindowAssigner):
    kind = N.ASSIGNER_TUMBLING

    def __init__(self, size: int, offset: int = 0):
        if abs(offset) >= size:
            raise ValueError("TumblingEventTimeWindows parameters must satisfy abs(offset) < size")
        self.size, self.offset = int(size), int(offset)

    @staticmethod
    def of(size: int, offset: int = 0) -> "TumblingEventTimeWindows":
        return TumblingEventTimeWindows(size, offset)

    def __repr__(self):
        return f"TumblingEventTimeWindows({self.size})"


class SlidingEventTimeWindows(WindowAssigner):
    kind = N.ASSIGNER_SLIDING

    def __init__(self, size: int, slide: int, offset: int = 0):
        if abs(offset) >= slide or size <= 0:
            raise ValueError("SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0")
        self.size, self.slide, self.offset = int(size), int(slide), int(offset)

    @staticmethod
    def of(size: int, slide: int, offset: int = 0) -> "SlidingEventTimeWindows":
        return SlidingEventTimeWindows(size, slide, offset)

    def __repr__(self):
        return f"SlidingEventTimeWindows({self.size}, {self.slide})"


class EventTimeSessionWindows(WindowAssigner):
    kind = N.ASSIGNER_SESSION
    merging = True

    def __init__(self, gap: int):
        if gap <= 0:
            raise ValueError("EventTimeSessionWindows parameters must satisfy 0 < size")
        self.gap = int(gap)

    @staticmethod
    def withGap(gap: int) -> "EventTimeSessionWindows":  # noqa: N802 (Flink name)
        return EventTimeSessionWindows(gap)

    with_gap = withGap

    def __repr__(self):
        return f"EventTimeSessionWindows({self.gap})"


# ------------------------------------------------------------------------------------------------
# GPU-describable AggregateFunctions.  Each carries its descriptor (kind, value dtype); the same
# objects also implement Flink's createAccumulator/add/getResult/merge contract so a CPU harness
# can run them unchanged, which is how parity is stated.
# ------------------------------------------------------------------------------------------------
class AggregateFunction:
    kinds: tuple = ()
    value_dtype = N.DTYPE_INT64

    @property
    def descriptor(self):
        return list(self.kinds), self.value_dtype


class _Simple(AggregateFunction):
    kind = -1

    def __init__(self, value_dtype: str = "int64"):
        if value_dtype not in ("int64", "float64"):
            raise ValueError(f"unsupported value dtype {value_dtype!r}")
        self.value_dtype = N.DTYPE_FLOAT64 if value_dtype == "float64" else N.DTYPE_INT64
        self.kinds = (self.kind,)


class CountAggregate(_Simple):
    """COUNT(*) per window: ``acc + 1``."""
    kind = N.AGG_COUNT


class SumAggregate(_Simple):
    """``SumFunction`` semantics (SJ/api/functions/aggregation/SumFunction.java:63-78)."""
    kind = N.AGG_SUM


class MinAggregate(_Simple):
    """``ComparableAggregator`` MIN (ComparableAggregator.java:72-94)."""
    kind = N.AGG_MIN


class MaxAggregate(_Simple):
    kind = N.AGG_MAX


class AverageAggregate(_Simple):
    """The ``AverageAggregate`` of docs/dev/stream/operators/windows.md:493-514: acc (sum, count),
    result ``(double) sum / count``."""
    kind = N.AGG_AVG


class MultiAggregate(AggregateFunction):
    """Several aggregates of one value column in one accumulator (e.g. sum/min/max)."""

    def __init__(self, *aggs: _Simple):
        if not 1 <= len(aggs) <= N.GWO_MAX_AGGS:
            raise ValueError("1..4 aggregates")
        dts = {a.value_dtype for a in aggs if a.kind != N.AGG_COUNT}
        if len(dts) > 1:
            raise ValueError("all aggregates must share the value dtype")
        self.value_dtype = dts.pop() if dts else N.DTYPE_INT64
        self.kinds = tuple(a.kind for a in aggs)
