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
 * GPU state into WindowOperator's own managed keyed states ("window-contents", "merging-window-set", the
 * "window-timers" timer service), key group by key group, so a savepoint moves between WindowOperator and this
 * operator in both directions, and rescaling hands every key group to its new owner.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.common.state.AggregatingStateDescriptor;
import org.apache.flink.api.common.state.ListStateDescriptor;
import org.apache.flink.api.common.typeutils.TypeSerializer;
import org.apache.flink.api.common.typeutils.base.array.LongPrimitiveArraySerializer;
import org.apache.flink.api.java.functions.KeySelector;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.typeutils.runtime.TupleSerializer;
import org.apache.flink.core.memory.DataInputDeserializer;
import org.apache.flink.core.memory.DataInputView;
import org.apache.flink.core.memory.DataInputViewStreamWrapper;
import org.apache.flink.core.memory.DataOutputSerializer;
import org.apache.flink.core.memory.DataOutputView;
import org.apache.flink.metrics.Counter;
import org.apache.flink.runtime.state.AbstractKeyedStateBackend;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.KeyGroupRangeAssignment;
import org.apache.flink.runtime.state.KeyGroupStatePartitionStreamProvider;
import org.apache.flink.runtime.state.StateInitializationContext;
import org.apache.flink.runtime.state.StateSnapshotContext;
import org.apache.flink.runtime.state.VoidNamespace;
import org.apache.flink.runtime.state.VoidNamespaceSerializer;
import org.apache.flink.runtime.state.internal.InternalAppendingState;
import org.apache.flink.runtime.state.internal.InternalListState;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.BoundedOneInput;
import org.apache.flink.streaming.api.operators.InternalTimer;
import org.apache.flink.streaming.api.operators.InternalTimerService;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.operators.Triggerable;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.types.StringValue;
import org.apache.flink.util.OutputTag;

import java.io.InputStream;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.HashSet;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.Set;
import java.util.TreeMap;
import java.util.TreeSet;

public class GpuWindowOperator<IN, K> extends AbstractStreamOperator<GpuWindowResult<K>>
        implements OneInputStreamOperator<IN, GpuWindowResult<K>>, BoundedOneInput, Triggerable<K, TimeWindow> {

    private static final long serialVersionUID = 1L;
    private static final long LONG_MIN = Long.MIN_VALUE;

    private final GpuWindowSpec spec;
    private final KeySelector<IN, K> keySelector;
    private final GpuAggregates.ValueExtractor<IN> valueOf;
    private final GpuAggregates.Descriptor<IN> fn;   // window-contents' AggregateFunction (its long[] accumulator)
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
    // WindowOperator's keyed states, holding a checkpoint's copy of the GPU state (see snapshotState)
    private transient InternalAppendingState<K, TimeWindow, IN, long[], Object[]> windowState;
    private transient InternalListState<K, VoidNamespace, Tuple2<TimeWindow, TimeWindow>> mergingSets;
    private transient InternalTimerService<TimeWindow> timers;
    private transient boolean mirrored;

    public GpuWindowOperator(GpuWindowSpec spec, KeySelector<IN, K> keySelector, GpuAggregates.Descriptor<IN> fn,
                             OutputTag<GpuLateRecord<K>> lateTag, int batch) {
        this.spec = spec;
        this.keySelector = keySelector;
        this.fn = fn;
        this.valueOf = fn.value;
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
        // The checkpoint mirror (snapshotState) registers its window timers while the operator snapshots; a backend
        // that snapshots timers synchronously into raw keyed state (RocksDB with the HEAP timer service) writes them
        // BEFORE operator.snapshotState runs (InternalTimeServiceManager.java:160-170, StreamOperatorStateHandler
        // .java:183-186), so its checkpoint would hold the previous mirror's timers: refuse it up front
        if (getKeyedStateBackend() instanceof AbstractKeyedStateBackend
                && ((AbstractKeyedStateBackend<?>) getKeyedStateBackend()).requiresLegacySynchronousTimerSnapshots()) {
            throw new UnsupportedOperationException("GpuWindowOperator checkpoints its windows through the keyed state "
                    + "backend's timer service; this backend snapshots timers synchronously before the operator (RocksDB "
                    + "with state.backend.rocksdb.timer-service.factory=HEAP): use the ROCKSDB timer service or a heap "
                    + "state backend");
        }
        handle = GwoNative.create(spec.assigner, spec.size, spec.slide, spec.offset, spec.gap, spec.allowedLateness,
                spec.aggs, spec.valueDtype, spec.keyKind, maxParallelism, range.getStartKeyGroup(),
                range.getEndKeyGroup(), spec.device, lateTag != null, spec.stateLayout, spec.expectedKeys);
        registerWindowStates();
        if (context.isRestored() && !importMirror()) {
            restoreRows(context);   // (a savepoint of an earlier version: raw keyed state rows only, no timers)
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
        try {
            super.close();
        } finally {
            try {
                if (pinned != null) {
                    for (ByteBuffer b : pinned) {
                        try {   // (a buffer that shared a page with one pinned earlier was never registered itself)
                            GwoNative.hostUnregister(b);
                        } catch (IllegalArgumentException notRegistered) {
                            // nothing to release
                        }
                    }
                    pinned = null;
                }
            } finally {
                if (handle != 0) {   // the device state is released whatever happened before
                    GwoNative.destroy(handle);
                    handle = 0;
                }
            }
        }
    }

    // ---- OneInputStreamOperator ------------------------------------------------------------------------------
    @Override
    public void processElement(StreamRecord<IN> element) throws Exception {
        if (mirrored) {   // the last checkpoint's (or restore's) copy in the keyed backend: dropped before any record
            clearMirror();
        }
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
        if (mirrored) {
            clearMirror();
        }
        flush();   // the pending records precede the watermark
        GwoNative.advanceWatermark(handle, mark.getTimestamp());
        emitFired();
        // forwarded without advancing the "window-timers" service (AbstractStreamOperator.processWatermark would): the
        // service only ever holds a checkpoint's mirror, which is gone before any watermark gets here (clearMirror)
        output.emitWatermark(mark);
    }

    @Override
    public void endInput() throws Exception {
        if (mirrored) {
            clearMirror();
        }
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

    // ---- checkpoints: the window state as WindowOperator's managed keyed state --------------------------------
    // WindowOperator keeps its state in the keyed state backend (WindowOperator.java:224-271): "window-contents" (the
    // AggregateFunction's accumulator per (key, TimeWindow)), "merging-window-set" (sessions: per key, window -> state
    // window) and the "window-timers" timer service.  This operator registers the same states with the same
    // serializers.  At a checkpoint it writes the GPU state into them, one key group at a time from the image
    // gwo_export_heap_state_begin stages in native memory (the heap backend's section layout, parsed here), so the
    // backend's snapshot -- taken right after snapshotState (StreamOperatorStateHandler.java:186-198) -- is a savepoint
    // WindowOperator restores, and a WindowOperator savepoint restores here (initializeState reads the states back
    // into one gwo_import_heap_state).  The mirror lives only from the operator's snapshot to the first of: the next
    // record, watermark or end of input, notifyCheckpointComplete / notifyCheckpointAborted (or the backend's disposal
    // with the operator).  The keyed backend's snapshot is taken synchronously right after snapshotState
    // (StreamOperatorStateHandler.java:183-198: copy-on-write state maps and a copy of the timer queue on the heap
    // backend, a native snapshot on RocksDB), so clearing the states afterwards does not touch the checkpoint.
    // Between checkpoints the backend holds no window entries: the GPU is the only copy of the state.
    private static final short SID_CONTENTS = 0, SID_MERGING = 1, SID_EVENT_TIMERS = 2, SID_PROCESSING_TIMERS = 3;

    private int[] stateIds() {   // gwo_heap_state_ids: this operator's own numbering of the sections it parses
        final boolean merging = spec.assigner == GwoNative.ASSIGNER_SESSION;
        return new int[] {SID_CONTENTS, merging ? SID_MERGING : -1, SID_EVENT_TIMERS, SID_PROCESSING_TIMERS};
    }

    @SuppressWarnings("unchecked")
    private void registerWindowStates() throws Exception {
        final TimeWindow.Serializer ws = new TimeWindow.Serializer();
        windowState = (InternalAppendingState<K, TimeWindow, IN, long[], Object[]>) getOrCreateKeyedState(ws,
                new AggregatingStateDescriptor<>("window-contents", fn, LongPrimitiveArraySerializer.INSTANCE));
        if (spec.assigner == GwoNative.ASSIGNER_SESSION) {   // WindowOperator.java:261-271
            final TupleSerializer<Tuple2<TimeWindow, TimeWindow>> pairs = new TupleSerializer<>(
                    (Class<Tuple2<TimeWindow, TimeWindow>>) (Class<?>) Tuple2.class, new TypeSerializer[] {ws, ws});
            mergingSets = (InternalListState<K, VoidNamespace, Tuple2<TimeWindow, TimeWindow>>) getOrCreateKeyedState(
                    VoidNamespaceSerializer.INSTANCE, new ListStateDescriptor<>("merging-window-set", pairs));
        }
        timers = getInternalTimerService("window-timers", ws, this);
    }

    // The mirror's timers never fire: the mirror is cleared before any watermark, and the watermark never advances the
    // timer service (processWatermark).
    @Override
    public void onEventTime(InternalTimer<K, TimeWindow> timer) {}

    @Override
    public void onProcessingTime(InternalTimer<K, TimeWindow> timer) {}

    @Override
    public void snapshotState(StateSnapshotContext context) throws Exception {
        super.snapshotState(context);
        flush();   // prepareSnapshotPreBarrier semantics: the batch is part of the state
        // a mirror still in the backend (two checkpoints with no record or watermark between them) is replaced
        clearMirror();
        final KeyGroupRange range = getKeyedStateBackend().getKeyGroupRange();
        final int groups = range.getNumberOfKeyGroups();
        final long[] offsets = new long[groups];
        final long[] watermark = new long[1];
        final long total = GwoNative.exportHeapStateBegin(handle, stateIds(), offsets, watermark);
        try {
            byte[] buf = new byte[1 << 16];
            for (int g = 0; g < groups; g++) {   // key group by key group: one section in Java memory at a time
                final long len = (g + 1 < groups ? offsets[g + 1] : total) - offsets[g];
                if (len > Integer.MAX_VALUE - 8) {
                    throw new IllegalStateException("key group " + (range.getStartKeyGroup() + g) + " holds " + len
                            + " bytes of window state; checkpoint it with a larger maxParallelism");
                }
                if (buf.length < len) {
                    buf = new byte[(int) Math.max(len, Math.min(2L * buf.length, Integer.MAX_VALUE - 8))];
                }
                GwoNative.exportHeapStateRead(handle, offsets[g], buf, (int) len);
                mirrorKeyGroup(new DataInputDeserializer(buf, 0, (int) len), range.getStartKeyGroup() + g);
            }
        } finally {
            GwoNative.exportHeapStateEnd(handle);
        }
        mirrored = true;
    }

    // One key group's section (include/gwo.h, gwo_export_heap_state) into the backend's states.
    private void mirrorKeyGroup(DataInputView in, int group) throws Exception {
        if (in.readInt() != group) {
            throw new IllegalStateException("heap-state image out of key-group order at " + group);
        }
        final int states = spec.assigner == GwoNative.ASSIGNER_SESSION ? 4 : 3;
        for (int st = 0; st < states; st++) {
            final short id = in.readShort();
            final int n = in.readInt();
            for (int e = 0; e < n; e++) {
                if (id == SID_CONTENTS) {   // TimeWindow namespace, key, accumulator
                    final TimeWindow w = readWindow(in);
                    setCurrentKey(readKey(in));
                    windowState.setCurrentNamespace(w);
                    windowState.updateInternal(readAccumulator(in));
                } else if (id == SID_MERGING) {   // VoidNamespace, key, (window, state window) pairs
                    in.readByte();
                    setCurrentKey(readKey(in));
                    final int m = in.readInt();
                    final List<Tuple2<TimeWindow, TimeWindow>> pairs = new ArrayList<>(m);
                    for (int x = 0; x < m; x++) {
                        pairs.add(new Tuple2<>(readWindow(in), readWindow(in)));
                    }
                    mergingSets.setCurrentNamespace(VoidNamespace.INSTANCE);
                    mergingSets.update(pairs);
                } else if (id == SID_EVENT_TIMERS) {   // timestamp (sign bit flipped), key, window
                    final long ts = in.readLong() ^ Long.MIN_VALUE;
                    setCurrentKey(readKey(in));
                    timers.registerEventTimeTimer(readWindow(in), ts);
                } else {
                    throw new IllegalStateException("processing-time timer in an event-time window operator");
                }
            }
        }
    }

    // The backend's window states -> one gwo_import_heap_state (a WindowOperator savepoint, or this operator's).
    // Every window with state has a timer (its fire timer, or with allowedLateness its cleanup timer), so the timers
    // enumerate the (key, window) entries; sessions read their accumulator through the merging window set.
    @SuppressWarnings("unchecked")
    private boolean importMirror() throws Exception {
        final Map<Integer, List<Object[]>> entries = new TreeMap<>();   // key group -> {key, window, accumulator}
        final Map<Integer, List<Object[]>> timerList = new TreeMap<>(); // key group -> {timestamp, key, window}
        final Set<Tuple2<Object, TimeWindow>> seen = new HashSet<>();
        final int maxParallelism = getRuntimeContext().getMaxNumberOfParallelSubtasks();
        timers.forEachEventTimeTimer((w, ts) -> {
            final Object key = getCurrentKey();
            final int group = KeyGroupRangeAssignment.assignToKeyGroup(key, maxParallelism);
            timerList.computeIfAbsent(group, x -> new ArrayList<>()).add(new Object[] {ts, key, w});
            if (!seen.add(new Tuple2<>(key, w))) {
                return;
            }
            TimeWindow stateWindow = w;
            if (mergingSets != null) {
                mergingSets.setCurrentNamespace(VoidNamespace.INSTANCE);
                final Iterable<Tuple2<TimeWindow, TimeWindow>> pairs = mergingSets.get();
                if (pairs != null) {
                    for (Tuple2<TimeWindow, TimeWindow> pr : pairs) {
                        if (pr.f0.equals(w)) {
                            stateWindow = pr.f1;
                        }
                    }
                }
            }
            windowState.setCurrentNamespace(stateWindow);
            final long[] acc = windowState.getInternal();
            if (acc != null) {
                entries.computeIfAbsent(group, x -> new ArrayList<>()).add(new Object[] {key, w, acc});
            }
        });
        if (timerList.isEmpty()) {
            return false;
        }
        final DataOutputSerializer out = new DataOutputSerializer(1 << 16);
        final Set<Integer> groups = new TreeSet<>(entries.keySet());
        groups.addAll(timerList.keySet());
        for (int group : groups) {   // sections in the layout mirrorKeyGroup parses, each window its own state window
            final List<Object[]> es = entries.getOrDefault(group, new ArrayList<>());
            final List<Object[]> ts = timerList.getOrDefault(group, new ArrayList<>());
            out.writeInt(group);
            out.writeShort(SID_CONTENTS);
            out.writeInt(es.size());
            for (Object[] e : es) {
                writeWindow(out, (TimeWindow) e[1]);
                writeKey(out, e[0]);
                final long[] acc = (long[]) e[2];
                out.writeInt(acc.length);
                for (long x : acc) {
                    out.writeLong(x);
                }
            }
            if (mergingSets != null) {
                final Map<Object, List<TimeWindow>> byKey = new LinkedHashMap<>();
                for (Object[] e : es) {
                    byKey.computeIfAbsent(e[0], x -> new ArrayList<>()).add((TimeWindow) e[1]);
                }
                out.writeShort(SID_MERGING);
                out.writeInt(byKey.size());
                for (Map.Entry<Object, List<TimeWindow>> kv : byKey.entrySet()) {
                    out.writeByte(0);
                    writeKey(out, kv.getKey());
                    out.writeInt(kv.getValue().size());
                    for (TimeWindow w : kv.getValue()) {
                        writeWindow(out, w);
                        writeWindow(out, w);
                    }
                }
            }
            out.writeShort(SID_EVENT_TIMERS);
            out.writeInt(ts.size());
            for (Object[] t : ts) {
                out.writeLong((Long) t[0] ^ Long.MIN_VALUE);
                writeKey(out, t[1]);
                writeWindow(out, (TimeWindow) t[2]);
            }
            out.writeShort(SID_PROCESSING_TIMERS);
            out.writeInt(0);
        }
        // no watermark is part of WindowOperator's state: the restored operator starts at Long.MIN_VALUE like it
        GwoNative.importHeapState(handle, stateIds(), out.getCopyOfBuffer(), Long.MIN_VALUE);
        mirrored = true;   // the restored copy is dropped at the first record, watermark or checkpoint notification
        return true;
    }

    @Override
    public void notifyCheckpointComplete(long checkpointId) throws Exception {
        super.notifyCheckpointComplete(checkpointId);
        clearMirror();   // (the checkpoint holds its own copy since the synchronous snapshot)
    }

    @Override
    public void notifyCheckpointAborted(long checkpointId) throws Exception {
        super.notifyCheckpointAborted(checkpointId);
        clearMirror();
    }

    // Drops the backend copy (the GPU holds the state): every window state, merging set and timer of the mirror,
    // enumerated through the mirror's timers (every mirrored window has one; they never fire, see processWatermark).
    // Sessions: a window's accumulator lives at its state window (a restored WindowOperator savepoint's merged sessions
    // map windows to other state windows), resolved through the merging set before that is cleared.
    private void clearMirror() throws Exception {
        if (!mirrored) {
            return;
        }
        final List<Object[]> all = new ArrayList<>();
        timers.forEachEventTimeTimer((w, ts) -> all.add(new Object[] {getCurrentKey(), w, ts}));
        for (Object[] t : all) {
            setCurrentKey(t[0]);
            final TimeWindow w = (TimeWindow) t[1];
            timers.deleteEventTimeTimer(w, (Long) t[2]);
            windowState.setCurrentNamespace(w);
            windowState.clear();
            if (mergingSets != null) {
                mergingSets.setCurrentNamespace(VoidNamespace.INSTANCE);
                final Iterable<Tuple2<TimeWindow, TimeWindow>> pairs = mergingSets.get();
                if (pairs != null) {
                    for (Tuple2<TimeWindow, TimeWindow> pr : pairs) {
                        windowState.setCurrentNamespace(pr.f1);
                        windowState.clear();
                    }
                }
                mergingSets.setCurrentNamespace(VoidNamespace.INSTANCE);
                mergingSets.clear();
            }
        }
        mirrored = false;
    }

    private Object readKey(DataInputView in) throws Exception {
        switch (spec.keyKind) {
            case GwoNative.KEY_STRING: return StringValue.readString(in);
            case GwoNative.KEY_INT: return in.readInt();
            default: return in.readLong();
        }
    }

    private void writeKey(DataOutputView out, Object key) throws Exception {
        switch (spec.keyKind) {
            case GwoNative.KEY_STRING: StringValue.writeString((String) key, out); break;
            case GwoNative.KEY_INT: out.writeInt((Integer) key); break;
            default: out.writeLong((Long) key); break;
        }
    }

    private static TimeWindow readWindow(DataInputView in) throws Exception {
        final long start = in.readLong();
        return new TimeWindow(start, in.readLong());
    }

    private static void writeWindow(DataOutputView out, TimeWindow w) throws Exception {
        out.writeLong(w.getStart());
        out.writeLong(w.getEnd());
    }

    private static long[] readAccumulator(DataInputView in) throws Exception {   // LongPrimitiveArraySerializer
        final long[] acc = new long[in.readInt()];
        for (int i = 0; i < acc.length; i++) {
            acc[i] = in.readLong();
        }
        return acc;
    }

    // Raw keyed state rows of a savepoint taken by an earlier version of this operator (before the managed mirror):
    // per key group, watermark, words, count, then per row key, start, end, timer, words.
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
