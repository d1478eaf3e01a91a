/*
 * JNI binding of include/gwo.h (libgwo.so + the shim jni/gwo_jni.c, built by `make jni` where a JDK is present).
 *
 * One static native per C entry point the operator uses; columns travel as direct ByteBuffers in native byte
 * order (no copies across the boundary).  A non-zero gwo_status becomes an exception thrown by the shim:
 * IllegalArgumentException (GWO_ERR_INVALID_ARGUMENT), UnsupportedOperationException (GWO_ERR_UNSUPPORTED,
 * GWO_ERR_MERGE_LATE -- the reference's own exception for a merge into a late window,
 * WindowOperator.java:318-323), RuntimeException otherwise, with gwo_last_error's message.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import java.nio.ByteBuffer;

final class GwoNative {
    static final int ABI_VERSION = 4;

    // gwo_assigner_kind, gwo_agg_kind, gwo_dtype, gwo_key_kind, gwo_state_layout
    static final int ASSIGNER_TUMBLING = 0, ASSIGNER_SLIDING = 1, ASSIGNER_SESSION = 2;
    static final int AGG_COUNT = 0, AGG_SUM = 1, AGG_MIN = 2, AGG_MAX = 3, AGG_AVG = 4;
    static final int DTYPE_INT64 = 0, DTYPE_FLOAT64 = 1;
    static final int KEY_LONG = 0, KEY_INT = 1, KEY_STRING = 2;
    static final int STATE_AUTO = 0, STATE_TABLE = 1, STATE_LOG = 2;

    private static volatile boolean loaded;

    static void load() {
        if (loaded) {
            return;
        }
        synchronized (GwoNative.class) {
            if (!loaded) {
                // gwo_jni links libgwo.so; both are found on java.library.path (no CPU fallback exists)
                System.loadLibrary("gwo_jni");
                if (abiVersion() != ABI_VERSION) {
                    throw new IllegalStateException("libgwo ABI " + abiVersion() + ", binding expects " + ABI_VERSION);
                }
                loaded = true;
            }
        }
    }

    private GwoNative() {}

    static native int abiVersion();

    /** gwo_create; returns the handle. */
    static native long create(int assigner, long size, long slide, long offset, long gap, long allowedLateness,
                              int[] aggs, int valueDtype, int keyKind, int maxParallelism, int keyGroupStart,
                              int keyGroupEnd, int device, boolean sideOutput, int stateLayout, long expectedKeys);

    static native void destroy(long handle);

    /** gwo_host_register: pins a direct buffer's memory (hipHostRegister) so its batches move to the GPU by DMA. */
    static native void hostRegister(ByteBuffer buffer);

    /** gwo_host_unregister: releases the pinning of hostRegister. */
    static native void hostUnregister(ByteBuffer buffer);

    /** gwo_submit: n records; keys, timestamps, values as int64 (values: int64 or float64 bits). */
    static native void submit(long handle, ByteBuffer keys, ByteBuffer timestamps, ByteBuffer values, int n);

    /** gwo_submit_utf16: String keys as UTF-16 code units plus n + 1 int64 offsets. */
    static native void submitUtf16(long handle, ByteBuffer chars, ByteBuffer offsets, ByteBuffer timestamps,
                                   ByteBuffer values, int n);

    static native void advanceWatermark(long handle, long watermark);

    /** gwo_sync: completes every submitted batch, exchange and fire (snapshots, close). */
    static native void sync(long handle);

    /** gwo_wait_fires: completes a fire still running (sessions, log layout) so outputCount sees all of its rows. */
    static native void waitFires(long handle);

    static native long outputCount(long handle);

    /** gwo_drain into key/start/end columns and one column per aggregate; returns the rows copied. */
    static native long drain(long handle, ByteBuffer keys, ByteBuffer starts, ByteBuffer ends, ByteBuffer[] results,
                             long capacity);

    static native int resultDtype(long handle, int aggregate);

    static native long lateDropped(long handle);

    static native long sideOutputCount(long handle);

    static native long drainSideOutput(long handle, ByteBuffer keys, ByteBuffer timestamps, ByteBuffer values,
                                       long capacity);

    static native long currentWatermark(long handle);

    static native long stateSize(long handle);

    /** gwo_snapshot_rows: {row bound, accumulator words per row}. */
    static native long[] snapshotRows(long handle);

    /**
     * gwo_snapshot into heap arrays of capacity `capacity` rows (words: capacity * nWords); returns {rows,
     * watermark}.  The shim checks every array's length.
     */
    static native long[] snapshot(long handle, long[] keys, long[] starts, long[] ends, long[] words, int[] keyGroups,
                                  int[] timers, int nWords, long capacity);

    static native void restore(long handle, long[] keys, long[] starts, long[] ends, long[] words, int[] timers,
                               int nWords, long n, long watermark);

    /**
     * gwo_export_heap_state: the keyed state as the heap state backend writes WindowOperator's state, one section
     * per key group of the handle (HeapSnapshotStrategy.java:175-193).  ids: state ids of {window-contents,
     * merging-window-set (-1: none), event timers, processing timers}; keyGroupOffsets receives each key group's
     * byte offset, watermarkOut[0] the watermark.
     */
    static native byte[] exportHeapState(long handle, int[] ids, long[] keyGroupOffsets, long[] watermarkOut);

    /**
     * gwo_export_heap_state_begin: stages that image in native memory; returns its length (keyGroupOffsets and
     * watermarkOut as for exportHeapState).  exportHeapStateRead copies [offset, offset + len) of it into dst;
     * exportHeapStateEnd releases it.
     */
    static native long exportHeapStateBegin(long handle, int[] ids, long[] keyGroupOffsets, long[] watermarkOut);

    static native void exportHeapStateRead(long handle, long offset, byte[] dst, int len);

    static native void exportHeapStateEnd(long handle);

    /** gwo_import_heap_state: key-group sections of that layout; only the handle's KeyGroupRange is kept. */
    static native void importHeapState(long handle, int[] ids, byte[] data, long watermark);

    /** gwo_key_strings: dictionary ids of a String-keyed handle back to Strings. */
    static native String[] keyStrings(long handle, long[] ids, int n);

    /** gwo_intern_utf16: Strings (UTF-16 code units + offsets) to this handle's ids. */
    static native void internUtf16(long handle, ByteBuffer chars, ByteBuffer offsets, int n, long[] idsOut);
}
