/*
 * GpuWindowOperator -- the drop-in for WindowOperator on keyBy().window(assigner).aggregate(fn) whose window
 * state and per-record work live on one MI355X (libgwo.so through jni/gwo_jni.c).
 *
 * Reference interfaces: WindowOperator.java:294-473 (processElement, onEventTime), OneInputStreamTask.java:
 * 158-168 (records and watermarks arrive on the mailbox thread), AbstractStreamOperator.java:566-571 (fired
 * rows are emitted before the watermark is forwarded), HeapSnapshotStrategy.java:97-222 (keyed state written
 * per key group) and StateInitializationContext.getRawKeyedStateInputs (restore of the subtask's key groups).
 *
 * Records are batched into direct (pinned-able) columnar buffers; every watermark flushes the batch, advances
 * the GPU watermark, drains the fired rows and forwards the watermark.  Keys are Long, Integer or String
 * (String keys are interned into the handle's device dictionary, gwo.h gwo_submit_utf16).  Checkpoints write the
 * handle's rows (key, window, raw accumulator words, fire-timer flag) into the raw keyed state stream, one
 * section per key group, so rescaling hands every key group to its new owner.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.java.functions.KeySelector;
import org.apache.flink.core.memory.DataInputView;
import org.apache.flink.core.memory.DataInputViewStreamWrapper;
import org.apache.flink.core.memory.DataOutputView;
import org.apache.flink.core.memory.DataOutputViewStreamWrapper;
import org.apache.flink.metrics.Counter;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.KeyGroupStatePartitionStreamProvider;
import org.apache.flink.runtime.state.KeyedStateCheckpointOutputStream;
import org.apache.flink.runtime.state.StateInitializationContext;
import org.apache.flink.runtime.state.StateSnapshotContext;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.BoundedOneInput;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.util.OutputTag;

import java.io.InputStream;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.List;

public class GpuWindowOperator<IN, K> extends AbstractStreamOperator<GpuWindowResult<K>>
        implements OneInputStreamOperator<IN, GpuWindowResult<K>>, BoundedOneInput {

    private static final long serialVersionUID = 1L;
    private static final long LONG_MIN = Long.MIN_VALUE;

    private final GpuWindowSpec spec;
    private final KeySelector<IN, K> keySelector;
    private final GpuAggregates.ValueExtractor<IN> valueOf;
    private final OutputTag<GpuLateRecord<K>> lateTag;   // null: late records are counted and dropped
    private final int batch;

    private transient long handle;
    private transient ByteBuffer keys, timestamps, values, chars, offsets;
    private transient List<String> pendingStrings;
    private transient int n;
    private transient long lateReported;
    private transient Counter numLateRecordsDropped;   // WindowOperator.java:141,221,424
    private transient int[] resultDtypes;

    public GpuWindowOperator(GpuWindowSpec spec, KeySelector<IN, K> keySelector,
                             GpuAggregates.ValueExtractor<IN> valueOf, OutputTag<GpuLateRecord<K>> lateTag,
                             int batch) {
        this.spec = spec;
        this.keySelector = keySelector;
        this.valueOf = valueOf;
        this.lateTag = lateTag;
        this.batch = batch;
    }

    // ---- lifecycle ------------------------------------------------------------------------------------------
    @Override
    public void initializeState(StateInitializationContext context) throws Exception {
        super.initializeState(context);
        GwoNative.load();
        KeyGroupRange range = getKeyedStateBackend().getKeyGroupRange();
        handle = GwoNative.create(spec.assigner, spec.size, spec.slide, spec.offset, spec.gap, spec.allowedLateness,
                spec.aggs, spec.valueDtype, spec.keyKind, spec.maxParallelism, range.getStartKeyGroup(),
                range.getEndKeyGroup(), spec.device, lateTag != null, spec.stateLayout, spec.expectedKeys);
        if (context.isRestored()) {
            restoreRows(context);
        }
    }

    @Override
    public void open() throws Exception {
        super.open();
        keys = direct(batch * 8L);
        timestamps = direct(batch * 8L);
        values = direct(batch * 8L);
        if (spec.keyKind == GwoNative.KEY_STRING) {
            pendingStrings = new ArrayList<>(batch);
            offsets = direct((batch + 1) * 8L);
        }
        numLateRecordsDropped = metrics.counter("numLateRecordsDropped");
        resultDtypes = new int[spec.aggs.length];
        for (int a = 0; a < spec.aggs.length; a++) {
            resultDtypes[a] = GwoNative.resultDtype(handle, a);
        }
    }

    @Override
    public void close() throws Exception {
        super.close();
        if (handle != 0) {
            GwoNative.destroy(handle);
            handle = 0;
        }
    }

    // ---- OneInputStreamOperator ------------------------------------------------------------------------------
    @Override
    public void processElement(StreamRecord<IN> element) throws Exception {
        final IN v = element.getValue();
        final K key = keySelector.getKey(v);
        final int i = n;
        if (spec.keyKind == GwoNative.KEY_STRING) {
            pendingStrings.add((String) key);
        } else {
            keys.putLong(i * 8, ((Number) key).longValue());
        }
        // a record without a timestamp carries Long.MIN_VALUE: the GPU rejects the batch like the assigner does
        timestamps.putLong(i * 8, element.hasTimestamp() ? element.getTimestamp() : LONG_MIN);
        if (spec.valueDtype == GwoNative.DTYPE_FLOAT64) {
            values.putDouble(i * 8, valueOf.doubleValue(v));
        } else {
            values.putLong(i * 8, valueOf.longValue(v));
        }
        if (++n == batch) {
            flush();
        }
    }

    @Override
    public void processWatermark(Watermark mark) throws Exception {
        flush();   // the pending records precede the watermark
        GwoNative.advanceWatermark(handle, mark.getTimestamp());
        emitFired();
        super.processWatermark(mark);
    }

    @Override
    public void endInput() throws Exception {
        flush();
        GwoNative.advanceWatermark(handle, Long.MAX_VALUE);   // StreamSource.java:122
        emitFired();
    }

    private void flush() {
        if (n == 0) {
            return;
        }
        if (spec.keyKind == GwoNative.KEY_STRING) {
            int units = 0;
            for (String s : pendingStrings) {
                units += s.length();
            }
            if (chars == null || chars.capacity() < units * 2) {
                chars = direct(Math.max(units * 2L, 1L << 16));
            }
            int at = 0;
            offsets.putLong(0, 0);
            for (int i = 0; i < n; i++) {
                String s = pendingStrings.get(i);
                for (int c = 0; c < s.length(); c++) {
                    chars.putChar((at + c) * 2, s.charAt(c));   // UTF-16 code units, as String.hashCode sees them
                }
                at += s.length();
                offsets.putLong((i + 1) * 8, at);
            }
            GwoNative.submitUtf16(handle, chars, offsets, timestamps, values, n);
            pendingStrings.clear();
        } else {
            GwoNative.submit(handle, keys, timestamps, values, n);
        }
        n = 0;
    }

    // ---- results (TimestampedCollector.collect, WindowOperator.java:546-550) --------------------------------
    @SuppressWarnings("unchecked")
    private void emitFired() {
        long rows = GwoNative.outputCount(handle);
        while (rows > 0) {
            final int cap = (int) Math.min(rows, batch);
            ByteBuffer k = direct(cap * 8L), s = direct(cap * 8L), e = direct(cap * 8L);
            ByteBuffer[] r = new ByteBuffer[spec.aggs.length];
            for (int a = 0; a < r.length; a++) {
                r[a] = direct(cap * 8L);
            }
            final int got = (int) GwoNative.drain(handle, k, s, e, r, cap);
            final String[] names = spec.keyKind == GwoNative.KEY_STRING ? GwoNative.keyStrings(handle, k, got) : null;
            for (int i = 0; i < got; i++) {
                Object[] res = new Object[r.length];
                for (int a = 0; a < r.length; a++) {
                    res[a] = resultDtypes[a] == GwoNative.DTYPE_FLOAT64 ? (Object) r[a].getDouble(i * 8)
                            : (Object) r[a].getLong(i * 8);
                }
                K key = (K) (names != null ? names[i] : boxKey(k.getLong(i * 8)));
                long end = e.getLong(i * 8);
                output.collect(new StreamRecord<>(new GpuWindowResult<>(key, s.getLong(i * 8), end, res), end - 1));
            }
            rows -= got;
        }
        long side = GwoNative.sideOutputCount(handle);
        if (side > 0 && lateTag != null) {
            ByteBuffer k = direct(side * 8), t = direct(side * 8), v = direct(side * 8);
            final int got = (int) GwoNative.drainSideOutput(handle, k, t, v, side);
            final String[] names = spec.keyKind == GwoNative.KEY_STRING ? GwoNative.keyStrings(handle, k, got) : null;
            for (int i = 0; i < got; i++) {
                K key = (K) (names != null ? names[i] : boxKey(k.getLong(i * 8)));
                Object value = spec.valueDtype == GwoNative.DTYPE_FLOAT64 ? (Object) v.getDouble(i * 8)
                        : (Object) v.getLong(i * 8);
                output.collect(lateTag, new StreamRecord<>(new GpuLateRecord<>(key, t.getLong(i * 8), value),
                        t.getLong(i * 8)));
            }
        }
        final long late = GwoNative.lateDropped(handle);
        numLateRecordsDropped.inc(late - lateReported);
        lateReported = late;
    }

    private Object boxKey(long k) {
        return spec.keyKind == GwoNative.KEY_INT ? (Object) (int) k : (Object) k;
    }

    // ---- checkpoints: rows per key group in the raw keyed state stream ---------------------------------------
    @Override
    public void snapshotState(StateSnapshotContext context) throws Exception {
        super.snapshotState(context);
        flush();   // prepareSnapshotPreBarrier semantics: the batch is part of the state
        final long[] bound = GwoNative.snapshotRows(handle);
        final long cap = Math.max(bound[0], 1);
        final int words = (int) bound[1];
        ByteBuffer k = direct(cap * 8), s = direct(cap * 8), e = direct(cap * 8), w = direct(cap * 8 * words),
                kg = direct(cap * 4), tm = direct(cap * 4);
        final long[] got = GwoNative.snapshot(handle, k, s, e, w, kg, tm, cap);
        final int rows = (int) got[0];
        final String[] names = spec.keyKind == GwoNative.KEY_STRING ? GwoNative.keyStrings(handle, k, rows) : null;
        KeyedStateCheckpointOutputStream out = context.getRawKeyedOperatorStateOutput();
        DataOutputView view = new DataOutputViewStreamWrapper(out);
        int i = 0;
        for (int group : out.getKeyGroupList()) {   // the rows arrive grouped by ascending key group
            out.startNewKeyGroup(group);
            int j = i;
            while (j < rows && kg.getInt(j * 4) == group) {
                j++;
            }
            view.writeLong(got[1]);   // watermark
            view.writeInt(words);
            view.writeInt(j - i);
            for (int r = i; r < j; r++) {
                if (names != null) {
                    byte[] utf = names[r].getBytes(StandardCharsets.UTF_16LE);
                    view.writeInt(utf.length);
                    view.write(utf);
                } else {
                    view.writeLong(k.getLong(r * 8));
                }
                view.writeLong(s.getLong(r * 8));
                view.writeLong(e.getLong(r * 8));
                view.writeInt(tm.getInt(r * 4));
                for (int x = 0; x < words; x++) {
                    view.writeLong(w.getLong((r * words + x) * 8));
                }
            }
            i = j;
        }
    }

    private void restoreRows(StateInitializationContext context) throws Exception {
        List<Object> key = new ArrayList<>();
        List<long[]> rows = new ArrayList<>();   // start, end, timer, words...
        long watermark = Long.MAX_VALUE;
        int words = -1;
        for (KeyGroupStatePartitionStreamProvider p : context.getRawKeyedStateInputs()) {
            try (InputStream in = p.getStream()) {
                DataInputView view = new DataInputViewStreamWrapper(in);
                watermark = Math.min(watermark, view.readLong());
                words = view.readInt();
                final int m = view.readInt();
                for (int r = 0; r < m; r++) {
                    if (spec.keyKind == GwoNative.KEY_STRING) {
                        byte[] utf = new byte[view.readInt()];
                        view.readFully(utf);
                        key.add(new String(utf, StandardCharsets.UTF_16LE));
                    } else {
                        key.add(view.readLong());
                    }
                    long[] row = new long[3 + words];
                    row[0] = view.readLong();
                    row[1] = view.readLong();
                    row[2] = view.readInt();
                    for (int x = 0; x < words; x++) {
                        row[3 + x] = view.readLong();
                    }
                    rows.add(row);
                }
            }
        }
        if (words < 0) {
            return;   // no key group of this subtask held state
        }
        final int m = rows.size();
        ByteBuffer k = direct(Math.max(m, 1) * 8L), s = direct(Math.max(m, 1) * 8L), e = direct(Math.max(m, 1) * 8L),
                w = direct(Math.max(m, 1) * 8L * Math.max(words, 1)), tm = direct(Math.max(m, 1) * 4L);
        if (spec.keyKind == GwoNative.KEY_STRING) {   // re-key by this handle's dictionary
            int units = 0;
            for (Object o : key) {
                units += ((String) o).length();
            }
            ByteBuffer c = direct(Math.max(units, 1) * 2L), off = direct((m + 1) * 8L);
            int at = 0;
            for (int r = 0; r < m; r++) {
                String str = (String) key.get(r);
                for (int x = 0; x < str.length(); x++) {
                    c.putChar((at + x) * 2, str.charAt(x));
                }
                off.putLong(r * 8, at);
                at += str.length();
            }
            off.putLong(m * 8, at);
            GwoNative.internUtf16(handle, c, off, m, k);
        } else {
            for (int r = 0; r < m; r++) {
                k.putLong(r * 8, (Long) key.get(r));
            }
        }
        for (int r = 0; r < m; r++) {
            long[] row = rows.get(r);
            s.putLong(r * 8, row[0]);
            e.putLong(r * 8, row[1]);
            tm.putInt(r * 4, (int) row[2]);
            for (int x = 0; x < words; x++) {
                w.putLong((r * words + x) * 8, row[3 + x]);
            }
        }
        GwoNative.restore(handle, k, s, e, w, tm, words, m, watermark);
    }

    private static ByteBuffer direct(long bytes) {
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }
}
