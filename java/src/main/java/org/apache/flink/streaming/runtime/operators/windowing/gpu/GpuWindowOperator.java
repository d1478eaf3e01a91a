/*
 * GpuWindowOperator -- the drop-in for WindowOperator on keyBy().window(assigner).aggregate(fn) whose window
 * state and per-record work live on one MI355X (libgwo.so through jni/gwo_jni.c).
 *
 * Reference interfaces: WindowOperator.java:294-473 (processElement, onEventTime), OneInputStreamTask.java:
 * 158-168 (records and watermarks arrive on the mailbox thread), AbstractStreamOperator.java:566-571 (fired
 * rows are emitted before the watermark is forwarded), HeapSnapshotStrategy.java:97-222 (keyed state written
 * per key group) and StateInitializationContext.getRawKeyedStateInputs (restore of the subtask's key groups).
 *
 * Records are batched into direct columnar buffers pinned once in open() (gwo_host_register); every watermark
 * flushes the batch, advances the GPU watermark, drains the fired rows and forwards the watermark.  Keys are Long, Integer or String
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
    // drain buffers, allocated once at open() (batch rows; the side output's grow on demand)
    private transient ByteBuffer outKeys, outStarts, outEnds, sideKeys, sideTs, sideValues;
    private transient ByteBuffer[] outResults;
    private transient List<ByteBuffer> pinned;   // direct buffers registered with gwo_host_register in open()
    private transient long[] idScratch;
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
        // the number of key groups of this operator: the keyed backend is created with the task's max parallelism
        // (StreamTaskStateInitializerImpl.java:290-306), which is what getMaxNumberOfParallelSubtasks returns --
        // per-operator setMaxParallelism and KeyGroupRangeAssignment.computeDefaultMaxParallelism included
        final int maxParallelism = getRuntimeContext().getMaxNumberOfParallelSubtasks();
        handle = GwoNative.create(spec.assigner, spec.size, spec.slide, spec.offset, spec.gap, spec.allowedLateness,
                spec.aggs, spec.valueDtype, spec.keyKind, maxParallelism, range.getStartKeyGroup(),
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
        outKeys = direct(batch * 8L);
        outStarts = direct(batch * 8L);
        outEnds = direct(batch * 8L);
        outResults = new ByteBuffer[spec.aggs.length];
        for (int a = 0; a < outResults.length; a++) {
            outResults[a] = direct(batch * 8L);
        }
        // the mailbox batches into pinned columns: registered once, so every gwo_submit (and every drain) moves them
        // by DMA (gwo.h gwo_host_register)
        pinned = new ArrayList<>();
        pin(keys);
        pin(timestamps);
        pin(values);
        if (offsets != null) {
            pin(offsets);
        }
        pin(outKeys);
        pin(outStarts);
        pin(outEnds);
        for (ByteBuffer r : outResults) {
            pin(r);
        }
        idScratch = new long[batch];
        numLateRecordsDropped = metrics.counter("numLateRecordsDropped");
        resultDtypes = new int[spec.aggs.length];
        for (int a = 0; a < spec.aggs.length; a++) {
            resultDtypes[a] = GwoNative.resultDtype(handle, a);
        }
    }

    private void pin(ByteBuffer b) {
        GwoNative.hostRegister(b);
        pinned.add(b);
    }

    @Override
    public void close() throws Exception {
        super.close();
        if (pinned != null) {
            for (ByteBuffer b : pinned) {
                GwoNative.hostUnregister(b);
            }
            pinned = null;
        }
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
            long units = 0;
            for (String s : pendingStrings) {
                units += s.length();
            }
            if (chars == null || chars.capacity() < units * 2) {
                if (chars != null) {
                    GwoNative.hostUnregister(chars);
                    pinned.remove(chars);
                }
                chars = direct(Math.max(units * 2L, 1L << 16));
                pin(chars);
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
    // Called after advanceWatermark and before the watermark is forwarded (AbstractStreamOperator.java:566-571):
    // gwo_wait_fires first completes a fire that runs asynchronously (sessions, log layout), then the rows are
    // drained in chunks of `batch` rows through the buffers allocated at open() until none is left.  Submitted
    // batches and the multi-GPU exchange stay in flight.
    @SuppressWarnings("unchecked")
    private void emitFired() {
        GwoNative.waitFires(handle);
        long rows;
        while ((rows = GwoNative.outputCount(handle)) > 0) {
            final int cap = (int) Math.min(rows, batch);
            final int got = (int) GwoNative.drain(handle, outKeys, outStarts, outEnds, outResults, cap);
            final String[] names = spec.keyKind == GwoNative.KEY_STRING ? keyStrings(outKeys, got) : null;
            for (int i = 0; i < got; i++) {
                Object[] res = new Object[outResults.length];
                for (int a = 0; a < outResults.length; a++) {
                    res[a] = resultDtypes[a] == GwoNative.DTYPE_FLOAT64 ? (Object) outResults[a].getDouble(i * 8)
                            : (Object) outResults[a].getLong(i * 8);
                }
                K key = (K) (names != null ? names[i] : boxKey(outKeys.getLong(i * 8)));
                long end = outEnds.getLong(i * 8);
                output.collect(new StreamRecord<>(new GpuWindowResult<>(key, outStarts.getLong(i * 8), end, res),
                        end - 1));
            }
            if (got == 0) {
                throw new IllegalStateException("gwo_drain returned no rows while " + rows + " are pending");
            }
        }
        long side;
        while (lateTag != null && (side = GwoNative.sideOutputCount(handle)) > 0) {
            final int cap = (int) Math.min(side, batch);
            if (sideKeys == null) {
                sideKeys = direct(batch * 8L);
                sideTs = direct(batch * 8L);
                sideValues = direct(batch * 8L);
                pin(sideKeys);
                pin(sideTs);
                pin(sideValues);
            }
            final int got = (int) GwoNative.drainSideOutput(handle, sideKeys, sideTs, sideValues, cap);
            final String[] names = spec.keyKind == GwoNative.KEY_STRING ? keyStrings(sideKeys, got) : null;
            for (int i = 0; i < got; i++) {
                K key = (K) (names != null ? names[i] : boxKey(sideKeys.getLong(i * 8)));
                Object value = spec.valueDtype == GwoNative.DTYPE_FLOAT64 ? (Object) sideValues.getDouble(i * 8)
                        : (Object) sideValues.getLong(i * 8);
                output.collect(lateTag, new StreamRecord<>(new GpuLateRecord<>(key, sideTs.getLong(i * 8), value),
                        sideTs.getLong(i * 8)));
            }
            if (got == 0) {
                throw new IllegalStateException("side output drain returned no rows while " + side + " are pending");
            }
        }
        final long late = GwoNative.lateDropped(handle);
        numLateRecordsDropped.inc(late - lateReported);
        lateReported = late;
    }

    private String[] keyStrings(ByteBuffer ids, int n) {
        for (int i = 0; i < n; i++) {
            idScratch[i] = ids.getLong(i * 8);
        }
        return GwoNative.keyStrings(handle, idScratch, n);
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
        final int words = (int) bound[1];
        final long capL = Math.max(bound[0], 1);
        if (capL * Math.max(words, 1) > Integer.MAX_VALUE - 8) {
            throw new IllegalStateException("GPU window state of " + bound[0] + " rows x " + words
                    + " words exceeds one Java array; checkpoint it with more subtasks");
        }
        final int cap = (int) capL;
        final long[] k = new long[cap], s = new long[cap], e = new long[cap], w = new long[cap * Math.max(words, 1)];
        final int[] kg = new int[cap], tm = new int[cap];
        final long[] got = GwoNative.snapshot(handle, k, s, e, w, kg, tm, words, cap);
        final int rows = (int) got[0];
        final String[] names = spec.keyKind == GwoNative.KEY_STRING ? GwoNative.keyStrings(handle, k, rows) : null;
        KeyedStateCheckpointOutputStream out = context.getRawKeyedOperatorStateOutput();
        DataOutputView view = new DataOutputViewStreamWrapper(out);
        int i = 0;
        for (int group : out.getKeyGroupList()) {   // the rows arrive grouped by ascending key group
            out.startNewKeyGroup(group);
            int j = i;
            while (j < rows && kg[j] == group) {
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
                    view.writeLong(k[r]);
                }
                view.writeLong(s[r]);
                view.writeLong(e[r]);
                view.writeInt(tm[r]);
                for (int x = 0; x < words; x++) {
                    view.writeLong(w[r * words + x]);
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
        if ((long) m * Math.max(words, 1) > Integer.MAX_VALUE - 8) {
            throw new IllegalStateException("restored GPU window state exceeds one Java array");
        }
        final long[] k = new long[Math.max(m, 1)], s = new long[Math.max(m, 1)], e = new long[Math.max(m, 1)],
                w = new long[Math.max(m, 1) * Math.max(words, 1)];
        final int[] tm = new int[Math.max(m, 1)];
        if (spec.keyKind == GwoNative.KEY_STRING) {   // re-key by this handle's dictionary
            long units = 0;
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
                k[r] = (Long) key.get(r);
            }
        }
        for (int r = 0; r < m; r++) {
            long[] row = rows.get(r);
            s[r] = row[0];
            e[r] = row[1];
            tm[r] = (int) row[2];
            System.arraycopy(row, 3, w, r * words, words);
        }
        GwoNative.restore(handle, k, s, e, w, tm, words, m, watermark);
    }

    private static ByteBuffer direct(long bytes) {
        if (bytes > Integer.MAX_VALUE) {   // a direct ByteBuffer holds at most 2^31 - 1 bytes
            throw new IllegalArgumentException("direct buffer of " + bytes + " bytes");
        }
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }
}
