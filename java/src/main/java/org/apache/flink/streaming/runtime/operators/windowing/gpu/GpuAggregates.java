/*
 * Aggregates the GPU operator evaluates: count / sum / min / max / avg of one value column, alone or several at
 * once (gwo_agg_kind).  Each is an ordinary AggregateFunction as well -- it runs unchanged inside the reference
 * WindowOperator, which is how the two are compared -- carrying the descriptor the GPU operator reads.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.common.functions.AggregateFunction;

import java.io.Serializable;

public final class GpuAggregates {
    private GpuAggregates() {}

    /** The value column of a record: int64 or float64. */
    public interface ValueExtractor<IN> extends Serializable {
        long longValue(IN in);

        default double doubleValue(IN in) {
            return longValue(in);
        }
    }

    /** AggregateFunction whose GPU form is {aggs[], value dtype}. */
    public abstract static class Descriptor<IN> implements AggregateFunction<IN, long[], Object[]> {
        private static final long serialVersionUID = 1L;
        final int[] aggs;
        final ValueExtractor<IN> value;

        Descriptor(ValueExtractor<IN> value, int... aggs) {
            this.value = value;
            this.aggs = aggs;
        }

        // host-side restatement (the reference operator's accumulator): one slot per aggregate, AVG as sum+count
        @Override
        public long[] createAccumulator() {
            long[] acc = new long[aggs.length * 2];
            for (int a = 0; a < aggs.length; a++) {
                acc[2 * a] = aggs[a] == GwoNative.AGG_MIN ? Long.MAX_VALUE
                        : aggs[a] == GwoNative.AGG_MAX ? Long.MIN_VALUE : 0L;
            }
            return acc;
        }

        @Override
        public long[] add(IN in, long[] acc) {
            final long v = value.longValue(in);
            for (int a = 0; a < aggs.length; a++) {
                switch (aggs[a]) {
                    case GwoNative.AGG_COUNT: acc[2 * a]++; break;
                    case GwoNative.AGG_MIN: acc[2 * a] = Math.min(acc[2 * a], v); break;
                    case GwoNative.AGG_MAX: acc[2 * a] = Math.max(acc[2 * a], v); break;
                    case GwoNative.AGG_AVG: acc[2 * a] += v; acc[2 * a + 1]++; break;
                    default: acc[2 * a] += v; break;
                }
            }
            return acc;
        }

        @Override
        public Object[] getResult(long[] acc) {
            Object[] r = new Object[aggs.length];
            for (int a = 0; a < aggs.length; a++) {
                r[a] = aggs[a] == GwoNative.AGG_AVG ? (Object) ((double) acc[2 * a] / acc[2 * a + 1]) : (Object) acc[2 * a];
            }
            return r;
        }

        @Override
        public long[] merge(long[] x, long[] y) {
            for (int a = 0; a < aggs.length; a++) {
                switch (aggs[a]) {
                    case GwoNative.AGG_MIN: x[2 * a] = Math.min(x[2 * a], y[2 * a]); break;
                    case GwoNative.AGG_MAX: x[2 * a] = Math.max(x[2 * a], y[2 * a]); break;
                    default: x[2 * a] += y[2 * a]; x[2 * a + 1] += y[2 * a + 1]; break;
                }
            }
            return x;
        }
    }

    public static <IN> Descriptor<IN> of(ValueExtractor<IN> value, int... aggs) {
        return new Descriptor<IN>(value, aggs) {
            private static final long serialVersionUID = 1L;
        };
    }

    public static <IN> Descriptor<IN> count() {
        return of(in -> 0L, GwoNative.AGG_COUNT);
    }

    public static <IN> Descriptor<IN> sum(ValueExtractor<IN> v) {
        return of(v, GwoNative.AGG_SUM);
    }

    public static <IN> Descriptor<IN> sumMinMax(ValueExtractor<IN> v) {
        return of(v, GwoNative.AGG_SUM, GwoNative.AGG_MIN, GwoNative.AGG_MAX);
    }

    public static <IN> Descriptor<IN> avg(ValueExtractor<IN> v) {
        return of(v, GwoNative.AGG_AVG);
    }
}
