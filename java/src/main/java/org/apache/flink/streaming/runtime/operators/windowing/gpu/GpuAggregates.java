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

    /**
     * AggregateFunction whose GPU form is {aggs[], value dtype}.  The accumulator holds one or two 64-bit words per
     * aggregate, exactly the words the GPU keeps (gwo_internal.h AccPlan): int64 values as longs, float64 values as
     * their raw bits (sum as a double, min/max ordered by Double.compare like ComparableAggregator), counts as longs.
     */
    public abstract static class Descriptor<IN> implements AggregateFunction<IN, long[], Object[]> {
        private static final long serialVersionUID = 1L;
        final int[] aggs;
        final ValueExtractor<IN> value;
        final int valueDtype;   // GwoNative.DTYPE_INT64 or DTYPE_FLOAT64

        Descriptor(ValueExtractor<IN> value, int valueDtype, int... aggs) {
            if (valueDtype != GwoNative.DTYPE_INT64 && valueDtype != GwoNative.DTYPE_FLOAT64) {
                throw new IllegalArgumentException("value dtype " + valueDtype);
            }
            this.value = value;
            this.aggs = aggs;
            this.valueDtype = valueDtype;
        }

        private boolean f64() {
            return valueDtype == GwoNative.DTYPE_FLOAT64;
        }

        @Override
        public long[] createAccumulator() {
            long[] acc = new long[aggs.length * 2];
            for (int a = 0; a < aggs.length; a++) {
                if (aggs[a] == GwoNative.AGG_MIN) {
                    acc[2 * a] = f64() ? Double.doubleToRawLongBits(Double.POSITIVE_INFINITY) : Long.MAX_VALUE;
                } else if (aggs[a] == GwoNative.AGG_MAX) {
                    acc[2 * a] = f64() ? Double.doubleToRawLongBits(Double.NEGATIVE_INFINITY) : Long.MIN_VALUE;
                } else if (f64() && aggs[a] != GwoNative.AGG_COUNT) {
                    acc[2 * a] = Double.doubleToRawLongBits(0.0);
                }
                acc[2 * a + 1] = 0L;   // AVG: count; otherwise "has a value" (min/max of an empty window are never read)
            }
            return acc;
        }

        @Override
        public long[] add(IN in, long[] acc) {
            if (f64()) {
                final double v = value.doubleValue(in);
                for (int a = 0; a < aggs.length; a++) {
                    final double cur = Double.longBitsToDouble(acc[2 * a]);
                    switch (aggs[a]) {
                        case GwoNative.AGG_COUNT: acc[2 * a]++; break;
                        case GwoNative.AGG_MIN:
                            if (acc[2 * a + 1] == 0 || Double.compare(v, cur) < 0) {
                                acc[2 * a] = Double.doubleToRawLongBits(v);
                            }
                            acc[2 * a + 1] = 1;
                            break;
                        case GwoNative.AGG_MAX:
                            if (acc[2 * a + 1] == 0 || Double.compare(v, cur) > 0) {
                                acc[2 * a] = Double.doubleToRawLongBits(v);
                            }
                            acc[2 * a + 1] = 1;
                            break;
                        case GwoNative.AGG_AVG: acc[2 * a] = Double.doubleToRawLongBits(cur + v); acc[2 * a + 1]++; break;
                        default: acc[2 * a] = Double.doubleToRawLongBits(cur + v); break;
                    }
                }
                return acc;
            }
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
                final long w = acc[2 * a];
                if (aggs[a] == GwoNative.AGG_COUNT) {
                    r[a] = w;
                } else if (aggs[a] == GwoNative.AGG_AVG) {
                    r[a] = (f64() ? Double.longBitsToDouble(w) : (double) w) / acc[2 * a + 1];
                } else {
                    r[a] = f64() ? (Object) Double.longBitsToDouble(w) : (Object) w;
                }
            }
            return r;
        }

        @Override
        public long[] merge(long[] x, long[] y) {
            for (int a = 0; a < aggs.length; a++) {
                final int k = aggs[a];
                if (k == GwoNative.AGG_COUNT) {
                    x[2 * a] += y[2 * a];
                } else if (k == GwoNative.AGG_MIN || k == GwoNative.AGG_MAX) {
                    if (y[2 * a + 1] == 0 && f64()) {
                        continue;
                    }
                    final int c = f64() ? Double.compare(Double.longBitsToDouble(y[2 * a]), Double.longBitsToDouble(x[2 * a]))
                            : Long.compare(y[2 * a], x[2 * a]);
                    if ((k == GwoNative.AGG_MIN && c < 0) || (k == GwoNative.AGG_MAX && c > 0) || x[2 * a + 1] == 0) {
                        x[2 * a] = y[2 * a];
                    }
                    x[2 * a + 1] |= y[2 * a + 1];
                } else if (f64()) {
                    x[2 * a] = Double.doubleToRawLongBits(Double.longBitsToDouble(x[2 * a]) + Double.longBitsToDouble(y[2 * a]));
                    x[2 * a + 1] += y[2 * a + 1];
                } else {
                    x[2 * a] += y[2 * a];
                    x[2 * a + 1] += y[2 * a + 1];
                }
            }
            return x;
        }
    }

    public static <IN> Descriptor<IN> of(ValueExtractor<IN> value, int valueDtype, int... aggs) {
        return new Descriptor<IN>(value, valueDtype, aggs) {
            private static final long serialVersionUID = 1L;
        };
    }

    public static <IN> Descriptor<IN> count() {
        return of(in -> 0L, GwoNative.DTYPE_INT64, GwoNative.AGG_COUNT);
    }

    public static <IN> Descriptor<IN> sum(ValueExtractor<IN> v) {
        return of(v, GwoNative.DTYPE_INT64, GwoNative.AGG_SUM);
    }

    public static <IN> Descriptor<IN> sumMinMax(ValueExtractor<IN> v) {
        return of(v, GwoNative.DTYPE_INT64, GwoNative.AGG_SUM, GwoNative.AGG_MIN, GwoNative.AGG_MAX);
    }

    public static <IN> Descriptor<IN> avg(ValueExtractor<IN> v) {
        return of(v, GwoNative.DTYPE_INT64, GwoNative.AGG_AVG);
    }

    /** float64 value column (SumFunction over a double field, SumFunction.java:78; AverageAggregate over doubles). */
    public static <IN> Descriptor<IN> sumDouble(ValueExtractor<IN> v) {
        return of(v, GwoNative.DTYPE_FLOAT64, GwoNative.AGG_SUM);
    }

    public static <IN> Descriptor<IN> avgDouble(ValueExtractor<IN> v) {
        return of(v, GwoNative.DTYPE_FLOAT64, GwoNative.AGG_AVG);
    }

    public static <IN> Descriptor<IN> sumMinMaxDouble(ValueExtractor<IN> v) {
        return of(v, GwoNative.DTYPE_FLOAT64, GwoNative.AGG_SUM, GwoNative.AGG_MIN, GwoNative.AGG_MAX);
    }
}
