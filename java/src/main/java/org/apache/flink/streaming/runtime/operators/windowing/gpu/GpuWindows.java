/*
 * Builds the GPU operator for keyBy(selector).window(assigner).aggregate(fn) -- the transformation
 * WindowedStream.aggregate installs (WindowedStream.java:792-850) -- keeping the keyed stream, so the
 * KeyGroupStreamPartitioner and the key-group ranges of the subtasks stay the reference's.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.java.functions.KeySelector;
import org.apache.flink.streaming.api.datastream.KeyedStream;
import org.apache.flink.streaming.api.datastream.SingleOutputStreamOperator;
import org.apache.flink.streaming.api.windowing.assigners.EventTimeSessionWindows;
import org.apache.flink.streaming.api.windowing.assigners.SlidingEventTimeWindows;
import org.apache.flink.streaming.api.windowing.assigners.TumblingEventTimeWindows;
import org.apache.flink.streaming.api.windowing.assigners.WindowAssigner;
import org.apache.flink.util.OutputTag;

public final class GpuWindows {
    private GpuWindows() {}

    public static <IN, K> SingleOutputStreamOperator<GpuWindowResult<K>> aggregate(
            KeyedStream<IN, K> keyed, WindowAssigner<? super IN, ?> assigner, GpuAggregates.Descriptor<IN> fn,
            long allowedLateness, OutputTag<GpuLateRecord<K>> lateTag, int gpuIndex) {
        GpuWindowSpec spec = new GpuWindowSpec();
        if (assigner instanceof TumblingEventTimeWindows) {
            TumblingEventTimeWindows a = (TumblingEventTimeWindows) assigner;
            spec.assigner = GwoNative.ASSIGNER_TUMBLING;
            spec.size = a.getSize();
            spec.offset = a.getOffset();
        } else if (assigner instanceof SlidingEventTimeWindows) {
            SlidingEventTimeWindows a = (SlidingEventTimeWindows) assigner;
            spec.assigner = GwoNative.ASSIGNER_SLIDING;
            spec.size = a.getSize();
            spec.slide = a.getSlide();
            spec.offset = a.getOffset();
        } else if (assigner instanceof EventTimeSessionWindows) {
            spec.assigner = GwoNative.ASSIGNER_SESSION;
            spec.gap = ((EventTimeSessionWindows) assigner).getGap();
        } else {
            throw new UnsupportedOperationException("no GPU form for window assigner " + assigner);
        }
        spec.allowedLateness = allowedLateness;
        spec.aggs = fn.aggs;
        spec.valueDtype = fn.valueDtype;
        Class<?> keyClass = keyed.getKeyType().getTypeClass();
        spec.keyKind = keyClass == String.class ? GwoNative.KEY_STRING
                : keyClass == Integer.class ? GwoNative.KEY_INT : GwoNative.KEY_LONG;
        if (keyClass != String.class && keyClass != Integer.class && keyClass != Long.class) {
            throw new UnsupportedOperationException("GPU keys are Long, Integer or String, not " + keyClass);
        }
        // the number of key groups is the subtask's: GpuWindowOperator reads it from its runtime context at
        // initializeState (a per-operator setMaxParallelism or computeDefaultMaxParallelism included)
        spec.maxParallelism = 0;
        spec.device = gpuIndex;
        KeySelector<IN, K> selector = keyed.getKeySelector();
        @SuppressWarnings({"unchecked", "rawtypes"})
        TypeInformation<GpuWindowResult<K>> outType = (TypeInformation) TypeInformation.of(GpuWindowResult.class);
        return keyed.transform("GpuWindowOperator", outType,
                new GpuWindowOperator<>(spec, selector, fn, lateTag, 1 << 20));
    }
}
