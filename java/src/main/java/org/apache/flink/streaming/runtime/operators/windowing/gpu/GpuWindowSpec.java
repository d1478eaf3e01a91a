/*
 * The GPU-describable part of a keyBy().window(assigner).aggregate(fn) transformation: the gwo_config fields
 * (include/gwo.h) a GpuWindowOperator creates its handle from.  Built by GpuWindows from the reference's own
 * assigner objects (TumblingEventTimeWindows / SlidingEventTimeWindows / EventTimeSessionWindows); anything
 * else is rejected when the transformation is built -- there is no fallback operator.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import java.io.Serializable;

public final class GpuWindowSpec implements Serializable {
    private static final long serialVersionUID = 1L;

    int assigner;
    long size, slide, offset, gap, allowedLateness;
    int[] aggs;
    int valueDtype;
    int keyKind;
    int maxParallelism;
    int device;
    int stateLayout = GwoNative.STATE_AUTO;
    long expectedKeys;

    GpuWindowSpec() {}
}
