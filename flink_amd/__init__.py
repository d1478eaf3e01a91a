"""flink_amd -- MI355X-native keyed event-time window aggregation (drop-in GpuWindowOperator).

The compute path is libgwo.so (hand-written gfx950 HIP kernels behind the C ABI in include/gwo.h);
this package is the host-side mirror of Flink's operator API over it.
"""
from .windowing import (AggregateFunction, AverageAggregate, CountAggregate, EventTimeSessionWindows,
                        MaxAggregate, MinAggregate, MultiAggregate, SlidingEventTimeWindows, SumAggregate,
                        Time, TimeWindow, TumblingEventTimeWindows)
from .keygroups import (KeyGroupRange, assign_key_groups, assign_key_groups_strings, compute_default_max_parallelism,
                        compute_key_group_range_for_operator_index, window_starts)

__all__ = [
    "AggregateFunction", "AverageAggregate", "CountAggregate", "EventTimeSessionWindows", "MaxAggregate",
    "MinAggregate", "MultiAggregate", "SlidingEventTimeWindows", "SumAggregate", "Time", "TimeWindow",
    "TumblingEventTimeWindows", "KeyGroupRange", "assign_key_groups", "assign_key_groups_strings", "compute_default_max_parallelism",
    "compute_key_group_range_for_operator_index", "window_starts", "GpuWindowOperator",
]


def __getattr__(name):
    if name == "GpuWindowOperator":
        from .operator import GpuWindowOperator
        return GpuWindowOperator
    raise AttributeError(name)
