/*
 * A record routed to the late-data side output (sideOutputLateData, WindowOperator.java:420-423,560-562): the
 * GPU operator hands back the columns it received -- key, timestamp, value.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

public final class GpuLateRecord<K> {
    public final K key;
    public final long timestamp;
    public final Object value;

    public GpuLateRecord(K key, long timestamp, Object value) {
        this.key = key;
        this.timestamp = timestamp;
        this.value = value;
    }

    @Override
    public String toString() {
        return "(" + key + ", " + timestamp + ", " + value + ")";
    }
}
