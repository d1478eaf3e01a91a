/*
 * One fired (key, window) row: TimeWindow{start, end} and one result per aggregate (Long or Double), emitted
 * with timestamp end - 1 (window.maxTimestamp(), WindowOperator.java:546-550).
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import java.util.Arrays;
import java.util.Objects;

public final class GpuWindowResult<K> {
    public final K key;
    public final long start;
    public final long end;
    public final Object[] results;

    public GpuWindowResult(K key, long start, long end, Object[] results) {
        this.key = key;
        this.start = start;
        this.end = end;
        this.results = results;
    }

    @Override
    public boolean equals(Object o) {
        if (!(o instanceof GpuWindowResult)) {
            return false;
        }
        GpuWindowResult<?> r = (GpuWindowResult<?>) o;
        return start == r.start && end == r.end && Objects.equals(key, r.key) && Arrays.equals(results, r.results);
    }

    @Override
    public int hashCode() {
        return Objects.hash(key, start, end, Arrays.hashCode(results));
    }

    @Override
    public String toString() {
        return "(" + key + ", [" + start + ", " + end + "), " + Arrays.toString(results) + ")";
    }
}
