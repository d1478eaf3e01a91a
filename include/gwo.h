/*
 * gwo.h -- C ABI of the MI355X-native keyed event-time window operator ("GPU window operator").
 *
 * This is the drop-in boundary for Flink's `keyBy().window(WindowAssigner).aggregate(...)` path.
 * A Java `GpuWindowOperator` binds these entry points through a thin JNI
 * shim; the C++ and Python harnesses in this repository bind them directly.  No torch or HIP
 * types appear in any signature: plain pointers, sizes and integer status codes.
 *
 * Reference interfaces each entry point replaces (paths relative to the Flink source tree,
 * SJ/ = flink-streaming-java/src/main/java/org/apache/flink/streaming/):
 *
 *   gwo_create            WindowOperator ctor + open()          SJ/runtime/operators/windowing/WindowOperator.java:182-273
 *                         (assigner/trigger/lateness/state descriptor built by WindowedStream.aggregate,
 *                          SJ/api/datastream/WindowedStream.java:792-850)
 *   gwo_submit            OneInputStreamOperator.processElement, batched
 *                                                               SJ/api/operators/OneInputStreamOperator.java:35-41,
 *                                                               WindowOperator.java:294-427 (via OneInputStreamTask.java:158-162)
 *   gwo_advance_watermark OneInputStreamOperator.processWatermark -> InternalTimerServiceImpl.advanceWatermark
 *                                                               SJ/api/operators/AbstractStreamOperator.java:566-571,
 *                                                               InternalTimerServiceImpl.java:268-278, WindowOperator.java:430-473
 *   gwo_drain             TimestampedCollector.collect of emitted window results
 *                                                               SJ/api/operators/TimestampedCollector.java:52-64,
 *                                                               WindowOperator.java:546-550
 *   gwo_late_dropped      metric numLateRecordsDropped          WindowOperator.java:141,221,424
 *   gwo_drain_side_output late-data side output (sideOutputLateData)   WindowOperator.java:420-423,560-562
 *   gwo_destroy           StreamOperator.close/dispose          SJ/api/operators/StreamOperator.java:96-110
 *   gwo_assign_key_groups KeyGroupRangeAssignment.assignToKeyGroup / computeOperatorIndexForKeyGroup
 *                                                               flink-runtime/.../state/KeyGroupRangeAssignment.java:48-73,118-119
 *   gwo_assign_key_groups_utf16  the same for String keys (JDK String.hashCode over UTF-16 code units)
 *   gwo_comm_*            keyBy shuffle (KeyGroupStreamPartitioner + network stack) across the GPUs of a node
 *   gwo_partition_by_operator  KeyGroupStreamPartitioner.selectChannel over a batch (route step of the shuffle)
 *                                                               SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:51-58
 *
 * Error convention: every call returns a gwo_status; nothing is thrown across the ABI.  A failing
 * gwo_submit rejects the WHOLE batch before any state changes (Flink would have failed the task at
 * the first offending record).  gwo_last_error() gives a message for the last failure on a handle.
 *
 * Threading: one handle = one operator subtask = one thread at a time (Flink's mailbox model,
 * SJ/runtime/tasks/mailbox/TaskMailboxImpl.java:98-110).  Distinct handles may be driven
 * concurrently from different threads.
 *
 * Buffers: input columns may be host or device pointers (detected per call).  Device input is
 * borrowed until the next call on the handle returns (the caller must neither free nor overwrite it
 * before then); host input is copied before gwo_submit returns.  Output columns given to gwo_drain
 * may be host or device pointers.
 *
 * Device-input readiness: the handle runs on its own non-blocking stream (or gwo_config.stream), which is
 * NOT ordered after work the caller queued on other streams.  Device columns must therefore be complete
 * as seen from the handle's stream when gwo_submit / gwo_submit_utf16 / gwo_intern_utf16 / gwo_restore
 * is called: the caller either synchronises its producer first, produces on the handle's stream
 * (gwo_config.stream, gwo_get_stream), or calls gwo_wait_stream(h, producer_stream) before the call --
 * the handle's stream then waits on the device for everything queued on the producer so far, with no
 * host wait.  The stateless helpers (gwo_assign_key_groups*, gwo_window_starts,
 * gwo_partition_by_operator) run on a blocking stream, ordered behind the device's null stream.
 */
#ifndef GWO_H
#define GWO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GWO_ABI_VERSION 4
#define GWO_MAX_AGGS 4

typedef enum {
    GWO_OK = 0,
    GWO_ERR_INVALID_ARGUMENT = 1, /* bad config (mirrors the assigners' IllegalArgumentException) */
    GWO_ERR_NO_TIMESTAMP = 2,     /* a record carries Long.MIN_VALUE (TumblingEventTimeWindows.java:76-79) */
    GWO_ERR_KEY_GROUP = 3,        /* key outside this subtask's KeyGroupRange (HeapKeyedStateBackend) */
    GWO_ERR_OUT_OF_MEMORY = 4,
    GWO_ERR_HIP = 5,              /* HIP runtime failure */
    GWO_ERR_UNSUPPORTED = 6,      /* configuration outside the GPU-describable subset: rejected, never faked */
    GWO_ERR_MERGE_LATE = 7,       /* UnsupportedOperationException of WindowOperator.java:318-323 */
    GWO_ERR_COMM = 8,             /* RCCL failure */
    GWO_ERR_STATE = 9,            /* call out of order (e.g. submit after destroy) */
    GWO_ERR_CAPACITY = 10         /* caller buffer too small */
} gwo_status;

typedef enum {
    GWO_ASSIGNER_TUMBLING = 0,    /* TumblingEventTimeWindows.of(size, offset), stagger ALIGNED */
    GWO_ASSIGNER_SLIDING = 1,     /* SlidingEventTimeWindows.of(size, slide, offset) */
    GWO_ASSIGNER_SESSION = 2      /* EventTimeSessionWindows.withGap(gap) */
} gwo_assigner_kind;

typedef enum {
    GWO_AGG_COUNT = 0,            /* result int64 */
    GWO_AGG_SUM = 1,              /* int64 (Java wrap-around) or float64, per value_dtype */
    GWO_AGG_MIN = 2,              /* Comparable min (Double.compareTo order for float64) */
    GWO_AGG_MAX = 3,
    GWO_AGG_AVG = 4               /* (sum, count) accumulator, result float64 = (double)sum / count */
} gwo_agg_kind;

typedef enum { GWO_DTYPE_INT64 = 0, GWO_DTYPE_FLOAT64 = 1 } gwo_dtype;

/* Device layout of the keyed window state.  Both give identical results. */
typedef enum {
    GWO_STATE_AUTO = 0,           /* tumbling: LOG when expected_keys >= 2^20, else TABLE; others TABLE */
    GWO_STATE_TABLE = 1,          /* open-addressed HBM hash table per window/pane, updated per batch */
    GWO_STATE_LOG = 2             /* tumbling only: per-window partitioned record log, folded in LDS at fire */
} gwo_state_layout;

typedef enum {
    GWO_KEY_LONG = 0,             /* key.hashCode() = Long.hashCode: (int)(v ^ (v >>> 32)) */
    GWO_KEY_INT = 1,              /* key.hashCode() = Integer.hashCode: (int)v; key must fit in int32 */
    GWO_KEY_STRING = 2            /* java.lang.String keys: gwo_submit_utf16; inside the handle a key is its
                                     dictionary id, (int64)String.hashCode << 32 | sequence number */
} gwo_key_kind;

typedef struct {
    int32_t abi_version;          /* must be GWO_ABI_VERSION */
    int32_t assigner;             /* gwo_assigner_kind */
    int64_t size;                 /* tumbling/sliding window size, ms */
    int64_t slide;                /* sliding slide, ms */
    int64_t offset;               /* tumbling/sliding offset, ms */
    int64_t gap;                  /* session gap, ms */
    int64_t allowed_lateness;     /* WindowedStream.allowedLateness, ms (>= 0) */
    int32_t num_aggs;             /* 1..GWO_MAX_AGGS aggregates over the same value column */
    int32_t aggs[GWO_MAX_AGGS];   /* gwo_agg_kind */
    int32_t value_dtype;          /* gwo_dtype of the value column */
    int32_t key_kind;             /* gwo_key_kind */
    int32_t max_parallelism;      /* number of key groups (1 .. 32768) */
    int32_t key_group_start;      /* inclusive KeyGroupRange owned by this subtask */
    int32_t key_group_end;
    int32_t device;               /* HIP device ordinal */
    int32_t side_output;          /* 1: late records go to the side output instead of being counted */
    int32_t state_layout;         /* gwo_state_layout */
    int64_t expected_keys;        /* sizing hint: distinct keys per window (0 = grow on demand) */
    void *stream;                 /* hipStream_t to run on; NULL: the handle creates its own */
} gwo_config;

typedef struct gwo_handle gwo_handle;

/* Output rows: one per fired (key, window); result[i] is int64 or float64 per gwo_result_dtype. */
typedef struct {
    int64_t *key;
    int64_t *start;
    int64_t *end;
    void *result[GWO_MAX_AGGS];
} gwo_out;

/* Late records routed to the side output (WindowOperator.sideOutput). */
typedef struct {
    int64_t *key;
    int64_t *ts;
    void *value;
} gwo_side_out;

void gwo_config_init(gwo_config *cfg);
gwo_status gwo_create(const gwo_config *cfg, gwo_handle **out);
gwo_status gwo_destroy(gwo_handle *h);

/* processElement for n records in arrival order; value may be NULL when every aggregate is COUNT.  Columns are device
 * pointers (read in place; complete as seen from the handle's stream and borrowed until the next call on the handle
 * returns -- see "Device-input readiness" above) or host pointers (copied to HBM on the handle's stream -- pinned
 * memory, see gwo_host_register, is copied by DMA directly). */
gwo_status gwo_submit(gwo_handle *h, const int64_t *key, const int64_t *ts, const void *value, int64_t n);
/* Orders the handle's stream after the work queued so far on `producer` (a hipStream_t; NULL = the device's null
 * stream): device columns written there are complete before any later call of this handle reads them.  One
 * hipEventRecord + hipStreamWaitEvent, no host wait.  The caller names its producer before each gwo_submit of
 * device columns it produced on another stream (the one-shot form keeps the ordering explicit per batch). */
gwo_status gwo_wait_stream(gwo_handle *h, void *producer);
/* Pins (page-locks) host memory for the GPUs (hipHostRegister), so gwo_submit / gwo_drain move it by DMA without a
 * pageable staging bounce: the Java operator registers its direct ByteBuffer columns once in open() (the mailbox
 * batching into pinned columnar buffers) and unregisters them in close().  Process-wide, not per handle. */
gwo_status gwo_host_register(void *ptr, int64_t bytes);
gwo_status gwo_host_unregister(void *ptr);
/* processWatermark: fire every window whose timers are <= wm, then adopt wm as current watermark. */
gwo_status gwo_advance_watermark(gwo_handle *h, int64_t wm);
/* processWatermark(Long.MAX_VALUE) -- a bounded source's end (StreamSource.java:122). */
gwo_status gwo_end_input(gwo_handle *h);

/* Rows available now.  Non-blocking: with the log layout a fire runs asynchronously (overlapping later
 * batches) and its rows count once it has completed; gwo_drain / gwo_output_view / gwo_sync wait for it. */
gwo_status gwo_output_count(gwo_handle *h, int64_t *n);
/* Total rows emitted since creation, including discarded ones (waits for a running fire). */
gwo_status gwo_rows_emitted(gwo_handle *h, int64_t *n);
/* Copies up to cap rows into cols (host or device buffers) and removes them from the handle. */
gwo_status gwo_drain(gwo_handle *h, const gwo_out *cols, int64_t cap, int64_t *n_out);
/* Library-owned device columns of the pending output (valid until the next call); n_out rows. */
gwo_status gwo_output_view(gwo_handle *h, gwo_out *cols, int64_t *n_out);
/* Drops every row emitted so far, including those of a fire still running (non-blocking). */
gwo_status gwo_discard_output(gwo_handle *h);
gwo_status gwo_result_dtype(const gwo_handle *h, int32_t agg_index, int32_t *dtype);

gwo_status gwo_late_dropped(gwo_handle *h, int64_t *count);
gwo_status gwo_side_output_count(gwo_handle *h, int64_t *n);
gwo_status gwo_drain_side_output(gwo_handle *h, const gwo_side_out *cols, int64_t cap, int64_t *n_out);
gwo_status gwo_current_watermark(gwo_handle *h, int64_t *wm);
/* The configuration the handle runs with (gwo_create's, defaults applied), e.g. its KeyGroupRange. */
gwo_status gwo_get_config(const gwo_handle *h, gwo_config *out);
/* Number of (key, window) entries currently held (device-resident state). */
gwo_status gwo_state_size(gwo_handle *h, int64_t *entries);

/* Checkpoint / restore of the keyed window state, every assigner and state layout.  A row is the heap backend's
 * (namespace, key, state) entry (CopyOnWriteStateMapSnapshot.java:127-129) plus that entry's window timer
 * (InternalTimeServiceManager.java:160-198): key, TimeWindow{window_start, window_end}, the raw accumulator words
 * (n_words per row, row-major) and timer = 1 while the window's event-time fire timer is pending (0: already
 * emitted, kept for allowedLateness re-fires).  Sliding windows checkpoint their panes ([start, end) = the pane);
 * session windows one row per in-flight session.  gwo_snapshot writes rows grouped by key group in ascending
 * order (key_group[i] = KeyGroupRangeAssignment.assignToKeyGroup of key[i]; the per-key-group layout of
 * HeapSnapshotStrategy.java:97-222) and the current watermark; key_group and timer may be NULL.
 * gwo_snapshot_rows gives an upper bound of the rows (exact except for the log layout, whose records are folded
 * only by the snapshot) and the words per row.  gwo_restore on a fresh handle of the same configuration
 * (n_words must match: GWO_ERR_INVALID_ARGUMENT) re-creates the rows whose key group lies in ITS KeyGroupRange
 * (rows of other key groups are skipped, so the union of the old subtasks' checkpoints restores a rescaled job)
 * and adopts `watermark`; with timer == NULL a window counts as emitted iff the watermark passed its end.  A
 * tumbling window whose rows disagree on their timer (subtasks checkpointed at different watermarks, lateness >
 * 0) is GWO_ERR_UNSUPPORTED.  Nothing changes on a failed validation.  Buffers may be host or device memory. */
typedef struct {
    int64_t *key;
    int64_t *window_start;
    int64_t *window_end;
    int64_t *words;
    int32_t *key_group;
    int32_t *timer;
} gwo_state_rows;
gwo_status gwo_snapshot_rows(gwo_handle *h, int64_t *n_rows, int32_t *n_words);
gwo_status gwo_snapshot(gwo_handle *h, const gwo_state_rows *rows, int64_t cap, int64_t *n_out, int64_t *watermark);
gwo_status gwo_restore(gwo_handle *h, const gwo_state_rows *rows, int32_t n_words, int64_t n, int64_t watermark);

/* ---- The keyed window state in the heap state backend's savepoint layout ------------------------------------
 * The data part of a HeapKeyedStateBackend snapshot as WindowOperator's state leaves it (HeapSnapshotStrategy.java:
 * 172-193): for every key group of the handle's KeyGroupRange, in ascending order, int32 key group, then for every
 * state int16 state id (the caller's KeyedBackendSerializationProxy numbering) and the state's entries of that key
 * group, all big-endian:
 *   window-contents      int32 n, n x {TimeWindow namespace: int64 start, int64 end; key; accumulator}
 *                        (CopyOnWriteStateMapSnapshot.java:113-131, TimeWindow.java:167-170)
 *   merging-window-set   sessions only: int32 n, n x {VoidNamespace: one byte 0; key; int32 m, m x {window,
 *                        state window}} (WindowOperator.java:265-271, MergingWindowSet.java:102-108)
 *   event timers         "_timer_state/event_window-timers": int32 n, n x {int64 timestamp with its sign bit flipped;
 *                        key; window} (KeyGroupPartitioner.java:251-264, TimerSerializer.java:158-162) -- a window's
 *                        fire timer at maxTimestamp and, with allowedLateness > 0, its cleanup timer
 *                        (WindowOperator.java:598-610)
 *   processing timers    "_timer_state/processing_window-timers": int32 0
 * Keys: Long (int64), Integer (int32) or String (StringValue.writeString: length + 1 and UTF-16 units, 7-bit varints).
 * The accumulator is GpuAggregates.Descriptor's long[] (LongPrimitiveArraySerializer: int32 length, int64 words; two
 * words per aggregate: COUNT {n, 0}, SUM {sum, 0}, MIN/MAX {value, 0} -- float64 {double bits, 1} --, AVG {sum, count}),
 * so a savepoint of the reference WindowOperator running that same AggregateFunction restores here and vice versa.
 * Sliding windows export one entry per (key, window) from their panes.  Their import restores each (key, window)
 * entry as its own restored window -- pending windows fire as the watermark passes them (the ring and recompute
 * tables and the log layout's running total alike), emitted ones re-fire their late records while allowedLateness
 * keeps them; a pending window the import watermark already passed, an emitted window on the log layout, or a
 * gwo_snapshot / gwo_snapshot_rows of a handle that still holds restored sliding windows is GWO_ERR_UNSUPPORTED
 * (export works).  A state id outside `ids` (a stateful trigger's or user keyed state) is GWO_ERR_UNSUPPORTED with
 * the id named in the message.
 * gwo_export_heap_state with buf == NULL sets *len to the bytes needed; kg_offsets (may be NULL) receives each key
 * group's offset in buf (KeyGroupRangeOffsets).  gwo_import_heap_state reads a concatenation of key-group sections
 * (several old subtasks' for a rescale), keeps ITS key groups and restores them as gwo_restore does (fresh handle;
 * every state id in the data must be one of `ids`). */
typedef struct {
    int16_t window_contents;
    int16_t merging_window_set;   /* -1: not written (non-merging assigners) */
    int16_t event_timers;
    int16_t processing_timers;
} gwo_heap_state_ids;
gwo_status gwo_export_heap_state(gwo_handle *h, const gwo_heap_state_ids *ids, uint8_t *buf, int64_t cap, int64_t *len,
                                 int64_t *kg_offsets, int64_t *watermark);
gwo_status gwo_import_heap_state(gwo_handle *h, const gwo_heap_state_ids *ids, const uint8_t *buf, int64_t len,
                                 int64_t watermark);
/* The same image, staged for a host that streams it key group by key group (the Java operator writes each group
 * into its keyed state backend): _begin builds it in host memory the handle owns and returns its length, each key
 * group's offset (kg_offsets: one per key group of the range) and the watermark; _read copies [offset, offset + len)
 * of it; _end releases it (also implied by gwo_destroy).  The device state is not changed. */
gwo_status gwo_export_heap_state_begin(gwo_handle *h, const gwo_heap_state_ids *ids, int64_t *len, int64_t *kg_offsets,
                                       int64_t *watermark);
gwo_status gwo_export_heap_state_read(gwo_handle *h, int64_t offset, uint8_t *buf, int64_t len);
gwo_status gwo_export_heap_state_end(gwo_handle *h);

gwo_status gwo_sync(gwo_handle *h);
/* Waits for the fires queued so far only (the log layout and sessions fire asynchronously): afterwards
 * gwo_output_count counts every row of the watermarks applied -- what WindowOperator emits before it forwards a
 * watermark (AbstractStreamOperator.java:566-571).  Unlike gwo_sync it leaves submitted batches and the multi-GPU
 * exchange in flight (a watermark already completed whatever a window it fired could hold). */
gwo_status gwo_wait_fires(gwo_handle *h);
gwo_status gwo_get_stream(gwo_handle *h, void **stream);
const char *gwo_last_error(const gwo_handle *h);
const char *gwo_status_string(gwo_status s);

/* ---- String keys (key_kind GWO_KEY_STRING) -------------------------------------------------------------------
 * The reference keys a String-keyed stream by the String itself: its key group is murmur(String.hashCode)
 * (KeyGroupRangeAssignment.java:60-73) and the window state is keyed by the String.  Here every distinct String
 * a handle sees is interned into a device-resident dictionary and the state is keyed by its id, whose high 32 bits
 * are the JDK String.hashCode (so every key-group computation is the reference's) and whose low 32 bits number the
 * handle's distinct keys.  Key i of a batch is the UTF-16 code units chars[offsets[i] .. offsets[i + 1]).
 * Output rows, side-output rows and checkpoint rows carry ids; gwo_key_strings turns ids back into Strings (a
 * checkpoint restored into another handle is re-keyed by interning its Strings there).  Host or device pointers.
 * Interning is exact: two distinct Strings never share an id (a 64-bit fingerprint match is verified code unit by
 * code unit; a true fingerprint collision rejects the batch with GWO_ERR_UNSUPPORTED). */
gwo_status gwo_submit_utf16(gwo_handle *h, const uint16_t *chars, const int64_t *offsets, const int64_t *ts,
                            const void *value, int64_t n);
gwo_status gwo_intern_utf16(gwo_handle *h, const uint16_t *chars, const int64_t *offsets, int64_t n,
                            int64_t *ids_out);
/* offsets_out: n + 1 entries (host memory); chars_out may be NULL to query chars_needed (GWO_ERR_CAPACITY when
 * chars_cap is too small).  An id the handle never issued: GWO_ERR_INVALID_ARGUMENT. */
gwo_status gwo_key_strings(gwo_handle *h, const int64_t *ids, int64_t n, int64_t *offsets_out, uint16_t *chars_out,
                           int64_t chars_cap, int64_t *chars_needed);

/* Pipelined submission (off by default; caller-owned device columns, no side output: the log layout, the table
 * layout's combine path for tumbling windows with allowedLateness 0 on one GPU, and session windows with
 * allowedLateness 0 -- other batches are resolved inside gwo_submit as usual).  gwo_submit queues the batch's
 * kernels (log: K1; combine: the gather and its speculative merge; sessions: sort and merge) and returns after
 * completing the PREVIOUS batch (its classification checks and pass 2, or its readback; sessions: the batch's
 * readback is read by the next gwo_submit once that batch's slot pass is queued, or by the next call that needs it;
 * a watermark's sweep queues behind the pending batch without reading it), so the host's wait and planning overlap
 * running kernels.  Observable results are unchanged: gwo_sync, gwo_late_dropped, gwo_state_size, the checkpoint
 * calls and the side-output calls complete the pending batch first (and gwo_advance_watermark, except on sessions,
 * where the sweep's own rows do not depend on it).
 * What moves is error reporting: a batch's GWO_ERR_NO_TIMESTAMP / GWO_ERR_KEY_GROUP is returned by the
 * next call on the handle (the batch is still rejected before any window state changes, and the handle
 * stays failed).  Device columns stay borrowed until that next call returns.
 * Readiness when pipelined: the combine path's gather may run on a second stream of the handle, beside the
 * previous batch's merge (GWO_CB_OVERLAP=1; off by default), so a pipelined batch's device columns must be complete
 * before the call or named with gwo_wait_stream (which orders both of the handle's streams); producing them on the
 * handle's stream itself is not enough there. */
gwo_status gwo_set_pipelined_submit(gwo_handle *h, int32_t enabled);

/* Per-kernel HIP-event timing, for bench.py's roofline (off by default). */
typedef enum {
    GWO_KERNEL_SCAN = 0,          /* batch pre-pass: window range, lateness, key-group checks */
    GWO_KERNEL_INSERT = 1,        /* insert into the per-window HBM hash tables */
    GWO_KERNEL_FIRE = 2,          /* watermark fire: compact, emit, reset */
    GWO_KERNEL_PARTITION = 3,     /* multi-GPU: destination partition */
    GWO_KERNEL_EXCHANGE = 4,      /* multi-GPU: RCCL all-to-all */
    GWO_KERNEL_SLIDE = 5,         /* sliding: pane fold/expire */
    GWO_KERNEL_SESSION = 6,       /* sessions: per-key merge */
    GWO_KERNEL_COUNT_ = 7
} gwo_kernel_id;
gwo_status gwo_set_profiling(gwo_handle *h, int32_t enabled);
/* Times only the kernels whose bit (1 << gwo_kernel_id) is set (each timed launch adds two event markers to
 * the stream; 0 turns profiling off). */
gwo_status gwo_set_profiling_mask(gwo_handle *h, uint32_t mask);
gwo_status gwo_kernel_stats(gwo_handle *h, int32_t kernel, int64_t *launches, double *total_ms,
                            int64_t *items);
gwo_status gwo_reset_stats(gwo_handle *h);

/* Bit-exact KeyGroupRangeAssignment over a key column (host or device pointers; outputs may be NULL). */
gwo_status gwo_assign_key_groups(const int64_t *keys, int64_t n, int32_t key_kind, int32_t max_parallelism,
                                 int32_t parallelism, int32_t *key_group_out, int32_t *operator_out,
                                 int32_t device);
/* KeyGroupRangeAssignment for java.lang.String keys (the key selector of a String-keyed stream,
 * KeyGroupRangeAssignment.java:60-73 over String.hashCode): key i is the UTF-16 code units
 * chars[offsets[i] .. offsets[i + 1]) hashed as h = 31 * h + c (wrapping int32, JDK String.hashCode), then
 * murmur -> key group -> operator index.  Any output may be NULL; hash_out receives the hashCodes.
 * Host or device pointers. */
gwo_status gwo_assign_key_groups_utf16(const uint16_t *chars, const int64_t *offsets, int64_t n,
                                       int32_t max_parallelism, int32_t parallelism, int32_t *hash_out,
                                       int32_t *key_group_out, int32_t *operator_out, int32_t device);
/* TimeWindow.getWindowStartWithOffset over a timestamp column (Java '%' semantics). */
gwo_status gwo_window_starts(const int64_t *ts, int64_t n, int64_t offset, int64_t size, int64_t *start_out,
                             int32_t device);

/* ---- multi-GPU keyBy shuffle over RCCL (one process per GPU) ---------------------------------- */
#define GWO_COMM_ID_BYTES 128
gwo_status gwo_comm_unique_id(uint8_t id[GWO_COMM_ID_BYTES]);
/* Collective: every rank calls it with the same id. The handle's key-group range must be
 * computeKeyGroupRangeForOperatorIndex(max_parallelism, nranks, rank). Afterwards gwo_submit and
 * gwo_advance_watermark are collective: gwo_submit routes records to their owner GPU
 * (partition + ncclSend/ncclRecv all-to-all); the watermark becomes the min over ranks. */
gwo_status gwo_comm_init(gwo_handle *h, const uint8_t id[GWO_COMM_ID_BYTES], int32_t nranks, int32_t rank);
/* Watermark agreement without a host wait: each gwo_advance_watermark queues its all-reduce (min over ranks) and applies
 * the min the previous call queued -- every rank the same values, one call later than the default synchronous
 * agreement (a valid StatusWatermarkValve history: one channel's watermark arriving one step later).  The end of input
 * always agrees synchronously.  Off by default (outputs then match a single operator fed the same watermarks). */
gwo_status gwo_comm_set_async_watermark(gwo_handle *h, int32_t enabled);
/* Host round trips of the routed exchange (log layout): routed batches, waits for a batch's exchanged counts (a routed
 * batch's record exchange is posted at the next routed batch, when its counts have arrived: only a flush -- a fire
 * its records may fall into, a snapshot, gwo_sync -- waits), and watermark agreements waited for (every synchronous
 * one; asynchronous: the previous call's all-reduce not yet published).  Waits that happen while the device is still
 * running the newest routed batches' K1 are flow control -- the host ran ahead of the device by more than the 3
 * send/receive slots hold -- and are counted apart by gwo_comm_backpressure, not here. */
gwo_status gwo_comm_stats(gwo_handle *h, int64_t *routed_batches, int64_t *count_waits, int64_t *wm_waits);
/* The same counters, the flow-control waits counted apart, and the host time spent waiting (ns). */
typedef struct {
    int64_t routed_batches, count_waits, wm_waits;
    int64_t flow_count_waits, flow_wm_waits;   /* the awaited result was still queued behind unfinished device work */
    int64_t count_wait_ns, wm_wait_ns;         /* time in count_waits / wm_waits */
    int64_t flow_wait_ns;                      /* time in the flow-control waits */
} gwo_comm_waits;
gwo_status gwo_comm_wait_stats(gwo_handle *h, gwo_comm_waits *out);

/* Batch form of KeyGroupStreamPartitioner.selectChannel (KeyGroupStreamPartitioner.java:51-58): groups n
 * records by destination computeOperatorIndexForKeyGroup(assignToKeyGroup(key)) into per-destination runs
 * of 24-byte {key, ts, value} records -- the route step of the multi-GPU exchange, for hosts with their own
 * transport.  out holds `parallelism` regions of `cap` records (region p at out + 3 * p * cap int64 words);
 * counts[p] = records routed to p (a count above cap: region p overflowed and only cap were written).
 * Order within a region is unspecified.  Host or device pointers; value may be NULL (sent as 0). */
gwo_status gwo_partition_by_operator(const int64_t *key, const int64_t *ts, const int64_t *value, int64_t n,
                                     int32_t key_kind, int32_t max_parallelism, int32_t parallelism, int64_t *out,
                                     int64_t cap, int64_t *counts, int32_t device);

/* ---- synthetic sources (device-resident benchmark/parity inputs; splitmix64) ---- */
typedef struct {
    uint64_t seed;
    int64_t first_index;          /* global record index of row 0 */
    int64_t total_records;        /* N of the whole stream (time spacing = span_ms / N) */
    int64_t num_keys;
    int64_t span_ms;              /* event-time span of the whole stream */
    int64_t disorder_ms;          /* ts = t0 + i*span/N + U[0, disorder) */
    int64_t t0;
    int64_t value_range;          /* value = U[0, value_range) */
    int32_t value_dtype;
    int32_t key_mode;             /* 0: uniform keys; 1: YSB ad_id -> campaign (ad % num_keys) */
} gwo_gen_spec;
gwo_status gwo_generate(const gwo_gen_spec *spec, int64_t n, int64_t *key, int64_t *ts, void *value,
                        void *stream, int32_t device);

#ifdef __cplusplus
}
#endif
#endif /* GWO_H */
