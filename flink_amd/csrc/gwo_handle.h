// gwo_handle.h -- the host-side state of one GPU window operator subtask.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>

#include <map>
#include <string>
#include <vector>

#include "../../include/gwo.h"
#include "gwo_internal.h"
#include "gwo_hash.h"

#define GWO_TRY(expr)                        \
    do {                                     \
        gwo_status s__ = (expr);             \
        if (s__ != GWO_OK) return s__;       \
    } while (0)

struct LogThr;   // gwo_log.h

struct LogRoute;       // gwo_log.h

namespace gwo {

// Checkpoint rows being restored, in host memory (gwo_snapshot.cpp).
struct RestoreRows {
    int64_t n = 0;
    int nw = 0;
    std::vector<int64_t> key, start, end, words;   // words: nw per row, row-major
    std::vector<int32_t> timer;                    // empty: derive fire timers from the restored watermark
    std::vector<char> mine;                        // row's key group lies in this subtask's KeyGroupRange
};

// Restored sliding-window entries read back for an export (gwo_slide.cpp slide_restored_rows).
struct WindowRows {
    std::vector<int64_t> key, words;               // words: plan.nwords per row
    std::vector<long long> j;                      // window index (start = j * slide + floorMod(offset, slide))
    std::vector<char> pending;                     // fire timer pending (else fired, waiting for its cleanup)
};

const char *status_str(gwo_status s);
bool is_device_ptr(const void *p);   // NULL counts as device (nothing to stage)

// Copies to and from caller memory (gwo_xfer.cpp): pageable host memory goes through the library's pinned bounce
// buffer, never through HIP's pageable copy path; pinned host and device memory are copied directly.
enum MemKind { MEM_DEVICE, MEM_PINNED, MEM_PAGEABLE };
MemKind mem_kind(const void *p);   // NULL counts as device
hipError_t copy_out(void *dst, const void *dev_src, size_t bytes, hipStream_t s);   // complete on return
hipError_t copy_in(void *dev_dst, const void *src, size_t bytes, hipStream_t s);   // pageable src reusable on return
hipError_t fetch_host(void *host_dst, const void *src, size_t bytes, hipStream_t s);   // src device or host
int64_t combine_h(int op, int64_t a, int64_t b);   // one accumulator word of a plan op folded on the host (gwo_heapstate.cpp)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

struct Table {
    int64_t *base = nullptr;       // cap entries + side slot
    int64_t *side = nullptr;
    uint64_t cap = 0;
    int counter = -1;              // slot in d_counters
    uint64_t occ = 0;              // occupancy as of the last read_occupancy()
    bool fired = false;            // emitted at maxTs (allowedLateness > 0 keeps it until cleanup)
    bool dirty = false;
};

struct KStat {
    int64_t launches = 0;
    double ms = 0;
    int64_t items = 0;
};

struct PendingEvent {
    int kernel;
    hipEvent_t a, b;
    int64_t items;
};

struct SessionState;   // gwo_session.cpp
struct SlideState;     // gwo_slide.cpp
struct Comm;           // gwo_comm.cpp
struct LogState;       // gwo_log.cpp
struct LogWindow;
struct LogJob;
struct StrDict;        // gwo_strings.cpp
struct SlogState;      // gwo_slog.cpp
struct RestoredWindow; // gwo_slide.h

struct Handle {
    static constexpr double kMaxLoad = 0.7;   // grow above this load factor
    static constexpr double kInitLoad = 0.45; // target load after (re)allocation
    static constexpr uint64_t kMinCap = 1024;

    gwo_config cfg{};
    hipStream_t stream = nullptr;
    bool own_stream = false;
    AccPlan plan{};
    ResultPlan rplan{};
    WindowGeom geom{};
    bool needs_value = true;
    int64_t wm = (int64_t)0x8000000000000000LL;  // Long.MIN_VALUE, InternalTimerServiceImpl.currentWatermark
    // this subtask's input channel watermark (StatusWatermarkValve.InputChannelStatus.watermark): the largest
    // watermark the caller has passed; the operator watermark is the min of it over ranks
    int64_t in_wm = (int64_t)0x8000000000000000LL;

    std::map<long long, Table> tables;         // window / pane index -> table
    // tumbling windows restored with entries already emitted (kept for allowedLateness) at a watermark below their
    // maxTimestamp (a restored timer service starts at Long.MIN_VALUE): a key with new records in the window before
    // the watermark passes maxTimestamp re-registers its fire timer (WindowOperator.java:393-410) and fires with both
    // (fire_tumbling); the others stay emitted
    std::map<long long, Table> rdone;
    std::vector<Table> aux_tables;             // engine-private tables (sliding ring totals)
    std::multimap<uint64_t, int64_t *> pool;   // clean tables by capacity

    // device scratch
    BatchStats *d_stats = nullptr;
    unsigned long long *d_scan_sh = nullptr;   // scan_kernel statistics shards (SCAN_SHARD_WORDS)
    BatchStats *h_stats = nullptr;             // pinned
    BatchStats *h_stats_init = nullptr;        // pinned
    unsigned long long *d_counters = nullptr;
    unsigned long long *h_counters = nullptr;  // pinned
    std::vector<char> counter_used;
    DevBuf dir_buf, stage_key, stage_ts, stage_val;
    DevBuf refire_buf;                         // per-element re-fire scratch (refire_rows)
    std::vector<TableDesc> h_dir;
    long long hist_hint = 0;

    // output
    OutCols out{};
    unsigned long long *d_out_count = nullptr;
    unsigned long long *d_scratch_count = nullptr;
    uint64_t out_rows = 0;
    bool out_count_dirty = false;              // gwo_discard_output: reset d_out_count before the next fire
    uint64_t rows_gone = 0;                    // rows drained or discarded so far (gwo_rows_emitted)
    // asynchronous fire (log layout): the fire runs on fire_stream, overlapping the next batches; its
    // rows become visible when it completes (finish_fire at the next output access or sync point)
    hipStream_t fire_stream = nullptr;
    hipEvent_t ev_main = nullptr, ev_fire = nullptr;
    bool fire_pending = false;
    bool async_fire = false;                   // GWO_ASYNC_FIRE=1: return before the fire completes
    bool discard_after_fire = false;
    // table-layout tumbling fire without a host round trip: the row counter is copied to h_out_cnt behind the
    // fire kernels and out_rows holds an upper bound (the emitted tables' capacities) until settle_out() reads it
    bool out_stale = false, discard_stale = false;
    unsigned long long *h_out_cnt = nullptr;   // pinned
    hipEvent_t ev_out = nullptr;
    hipEvent_t ev_input = nullptr;             // gwo_wait_stream: the producer stream's work so far
    unsigned long long zero_u64 = 0;
    unsigned long long *h_scalar = nullptr;    // pinned scalar staging
    int64_t *h_ident_side = nullptr;           // pinned [0, identity words...] side-slot image

    // late data
    uint64_t late_dropped = 0;
    DevBuf side_key, side_ts, side_val;
    unsigned long long *d_side_count = nullptr;
    long long side_cap = 0;
    unsigned long long side_rows = 0, side_rows_committed = 0;
    bool side_enabled() const { return cfg.side_output != 0; }

    // pre-aggregation policy
    int use_preagg = 1;
    int use_combine = 1;                       // GWO_COMBINE=0: the two-pass scan + insert path only
    int cb_cus = 0;
    uint64_t recent_cap = 0;                           // capacity of the last retired window/pane table
    int cb_max_wg = 0;                                 // gather workgroups at most (GWO_CB_WG; default 4 per CU)
    DevBuf cb_dump_key, cb_dump_acc, cb_ovf, cb_blk, cb_ctr, cb_dir, cb_arr;   // combine path scratch (insert_combined)
    unsigned long long *cb_rb = nullptr, *cb_rb_dev = nullptr;        // host-mapped readback blocks (2 slots)
    unsigned long long cb_seq = 0;
    hipEvent_t cb_ev = nullptr;
    std::vector<TableDesc> cb_dir_host;                                // what cb_dir holds
    long long cb_dir_base = 0;
    int use_combine_spec = 1;                                          // GWO_COMBINE_SPEC=0: no speculative merge
    DevBuf cb_spec_dir;                                                // the speculative merge's directory
    // overlapped pipelining (GWO_CB_OVERLAP=1; off by default: measured slower, profiles/r06_experiments.txt): a
    // pipelined batch's gather runs on cb_side beside the previous batch's merge, which stays on the handle's
    // stream -- so everything later on the handle's stream is ordered behind every merge with no join.  cb_side
    // waits for the handle's stream when a chain starts or this call queued work there (a new table), and for the
    // merge that last read the dump slot it writes.
    bool cb_overlap = false;
    hipStream_t cb_side = nullptr;
    hipEvent_t cb_ev_main = nullptr, cb_ev_gather = nullptr, cb_ev_merge[2] = {nullptr, nullptr};
    bool cb_merge_rec[2] = {false, false};
    DevBuf cb_go;                                                      // [2] per-slot verdicts, [2..9] per-slot incs
    DevBuf cb_dbg;                                                     // GWO_CB_TRACE phase times
    std::vector<TableDesc> cb_spec_host;
    long long cb_spec_base = 0;
    // speculative two-pass insert (insert_speculative): the scan's verdict gates the insert queued behind it
    int use_scan_spec = 1;                                             // GWO_SCAN_SPEC=0: off
    DevBuf sp_dir, sp_go;                                              // directory: tables of hint, hint + 1
    std::vector<TableDesc> sp_dir_host;
    long long sp_dir_base = 0;
    unsigned long long *sp_rb = nullptr, *sp_rb_dev = nullptr;        // host-mapped readback block
    unsigned long long sp_seq = 0;
    hipEvent_t sp_ev = nullptr;
    int cfg_preagg = -1;                       // GWO_PREAGG env override: 0 / 1
    uint64_t batches = 0;
    uint64_t preagg_probe_every = 32, preagg_probe_at = 32;   // adapt_preagg's re-probe schedule (backs off)
    bool preagg_probing = false;

    // errors
    std::string err;
    bool poisoned = false;
    gwo_status poison_status = GWO_OK;

    // profiling
    bool profiling = false;
    // GWO_HOST_PROF=1: mean host time between numbered points of the submit / watermark paths (diagnostics, printed
    // to stderr when the handle is destroyed).  Point p records the time since the previous point; the points that
    // start a call's chain (hp_start) record nothing.
    bool hprof = false;
    long long hp_last = 0, hp_sum[32] = {}, hp_cnt[32] = {};
    void hp(int p, bool start = false) {
        if (!hprof) return;
        const long long now =
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
        if (!start) {
            hp_sum[p] += now - hp_last;
            hp_cnt[p]++;
        }
        hp_last = now;
    }
    uint32_t prof_mask = ~0u;                  // kernels timed while profiling (bit = gwo_kernel_id)
    bool debug = false;                        // GWO_DEBUG=1: trace batches to stderr
    bool ktrace = false;                       // GWO_KTRACE: per-phase K1 / fire cycle sums at destruction
    std::vector<PendingEvent> pending_events;
    std::vector<hipEvent_t> event_pool;        // recycled profiling events
    KStat kstats[GWO_KERNEL_COUNT_];

    SessionState *sess = nullptr;
    SlideState *slide = nullptr;
    Comm *comm = nullptr;
    LogState *logst = nullptr;                 // non-null: log-structured tumbling state
    StrDict *dict = nullptr;                   // String keys: the key dictionary (gwo_strings.cpp)
    SlogState *slog = nullptr;                 // non-null (with logst): sliding windows over logged panes
    size_t log_chunk_min = 0;                  // sliding log: every pane chunk has this size (pool reuse)

    ~Handle();
    gwo_status init(const gwo_config &c);
    gwo_status submit(const int64_t *key, const int64_t *ts, const void *val, int64_t n);
    gwo_status submit_local(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n);
    gwo_status advance_watermark(int64_t wm);
    gwo_status drain(const gwo_out *cols, int64_t cap, int64_t *n_out);
    gwo_status drain_side(const gwo_side_out *cols, int64_t cap, int64_t *n_out);
    gwo_status state_size(int64_t *entries);
    // checkpoint / restore (gwo_snapshot.cpp)
    gwo_status snapshot_quiesce();
    gwo_status snapshot_rows(int64_t *n_rows);
    gwo_status snapshot(const gwo_state_rows *rows, int64_t cap, int64_t *n_out);
    gwo_status restore(const gwo_state_rows *rows, int32_t n_words, int64_t n, int64_t new_wm);
    gwo_status table_restore_rows(const RestoreRows &R, int64_t new_wm);
    // the heap state backend's per-key-group savepoint layout (gwo_heapstate.cpp)
    gwo_status export_heap_state(const gwo_heap_state_ids *ids, uint8_t *buf, int64_t cap, int64_t *len,
                                 int64_t *kg_offsets, int64_t *wm_out);
    gwo_status import_heap_state(const gwo_heap_state_ids *ids, const uint8_t *buf, int64_t len, int64_t new_wm);
    std::vector<uint8_t> heap_img;   // gwo_export_heap_state_begin's image (host memory), until _end
    bool heap_img_open = false;

    // String keys (gwo_strings.cpp)
    gwo_status intern_utf16(const uint16_t *chars, const int64_t *offsets, int64_t n, const int64_t **ids);
    gwo_status key_strings(const int64_t *ids, int64_t n, int64_t *offsets_out, uint16_t *chars_out,
                           int64_t chars_cap, int64_t *chars_needed);
    void dict_free();

    gwo_status fail(gwo_status s, const char *fmt, ...);
    gwo_status poison(gwo_status s, const char *what);
    gwo_status dalloc(void **p, size_t bytes);
    gwo_status hipcheck(hipError_t e, const char *what);
    gwo_status spin_event(hipEvent_t ev, const char *what);
    gwo_status spin_seq(const unsigned long long *word, unsigned long long seq, const char *what,
                        hipStream_t producer = nullptr);   // producer: the stream that publishes the word (default: stream)
    bool known_device(const void *p, size_t bytes);
    std::vector<std::pair<uintptr_t, uintptr_t>> dev_ranges;   // device allocations seen by this stage_inputs call
    gwo_status ensure_buf(DevBuf &b, size_t bytes);
    int take_counter();
    // occupancy counter c: GWO_OCC_WORDS device words (sharded, see gwo_device.h occ_add)
    unsigned long long *ctr(int c) const { return d_counters + (size_t)c * GWO_OCC_WORDS; }
    uint64_t ctr_host(int c) const {
        uint64_t s = 0;
        for (int i = 0; i < GWO_OCC_SHARDS; ++i) s += h_counters[(size_t)c * GWO_OCC_WORDS + i * GWO_OCC_SHARD_STRIDE];
        return s;
    }
    gwo_status ctr_zero(int c) {
        return hipcheck(hipMemsetAsync(ctr(c), 0, GWO_OCC_WORDS * 8, stream), "counter reset");
    }
    gwo_status ctr_read(int c, uint64_t *v);   // D2H + sync
    gwo_status alloc_table(uint64_t cap, Table &t);
    void release_table(Table &t);
    void trim_pool();
    TableDesc desc(const Table &t) const;
    gwo_status ensure_table(long long u, uint64_t incoming);
    gwo_status read_occupancy();
    gwo_status launch_ok(const char *what);
    gwo_status reset_side(const Table &t);
    gwo_status ensure_output(uint64_t extra);
    gwo_status stage_inputs(const int64_t *key, const int64_t *ts, const void *val, int64_t n, const int64_t **dk,
                            const int64_t **dt, const int64_t **dv);
    int64_t unit_start(long long u) const;
    WindowGeom geom_now() const;
    gwo_status insert_windowed(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n,
                               const WindowGeom *at = nullptr);
    gwo_status insert_combined(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, bool *done);
    // Pipelined submission of the combine path (gwo_set_pipelined_submit, tumbling, caller-owned device columns):
    // gwo_submit queues the batch's gather and speculative merge and returns after reading the PREVIOUS batch's
    // readback, so the host's turnaround overlaps the GPU's work.  The gather chains its verdict on the previous
    // one (CombineArgs::chain): a batch the host must take over keeps its successor's merge off, and both are redone
    // in order.
    struct CbPend {
        bool active = false;
        const int64_t *k = nullptr, *t = nullptr, *v = nullptr;
        int64_t n = 0;
        int slot = 0;
        unsigned long long seq = 0;
        long long hint = 0;   // units hint, hint + 1: the speculative merge's tables
        int64_t wm = 0;       // the watermark the batch was classified at
        bool side = false;    // its gather ran on cb_side
    } cb_pend;
    bool pipe_submit = false;   // gwo_set_pipelined_submit
    bool cb_redo = false;       // redoing a batch the pipelined verdict turned down: no pipelining
    bool combine_pipe_ok(const int64_t *k, const int64_t *t, const int64_t *v) const;
    gwo_status combine_resolve_pending(bool *go);
    gwo_status combine_flush();   // resolve the pending pipelined batch (no-op without one)
    gwo_status flush_pending();   // every pipelined batch (combine path, sessions) resolved
    gwo_status sess_publish_err();
    gwo_status sess_collect_err(bool lists_batch = false);
    gwo_status sess_apply_err();
    gwo_status sess_resolve();
    gwo_status insert_speculative(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, bool *done);
    gwo_status refire_rows(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const WindowGeom &g,
                           long long dir_base, int dir_len, uint64_t mmax);
    void adapt_preagg(uint64_t accepted, uint64_t partials);
    void init_stats(long long hist_base);
    gwo_status grow_side(long long need);
    gwo_status fire_tumbling(int64_t new_wm);
    gwo_status settle_out();
    int64_t cleanup_time_host(int64_t max_ts) const;
    OutCols out_cols() {
        OutCols o = out;
        o.count = d_out_count;
        return o;
    }

    // sliding (gwo_slide.cpp)
    int64_t win_start(__int128 j) const;
    long long win_first_pane(__int128 j) const;
    long long win_last_pane(__int128 j) const;
    __int128 first_window_of_pane(long long u) const;
    RingDesc ring_desc();
    gwo_status ensure_ring(uint64_t incoming);
    gwo_status slide_prepare_insert(long long base, int len, const unsigned long long *hist);
    gwo_status ring_rebuild();
    gwo_status release_panes_before(long long first);
    gwo_status slide_init();
    void slide_free();
    gwo_status fire_sliding(int64_t new_wm);
    gwo_status slide_restore_anchor();
    __int128 first_uncleaned_window(int64_t at_wm) const;
    __int128 first_unfired_window(int64_t at_wm) const;
    gwo_status slide_refire_rows(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const WindowGeom &g,
                                 uint64_t records);
    // sliding windows restored from a per-window savepoint (gwo_import_heap_state; gwo_slide.cpp)
    gwo_status slide_restore_windows(const RestoreRows &R, int64_t new_wm);
    gwo_status rwin_fold(RestoredWindow &r, Table &dst, int sign, int live_word, unsigned long long *live);
    void rwin_release_before(long long j);
    bool slide_has_restored() const;
    gwo_status slide_restored_rows(WindowRows &out);
    gwo_status restore_impl(const gwo_state_rows *rows, int32_t n_words, int64_t n, int64_t new_wm, bool per_window);
    // sessions (gwo_session.cpp)
    gwo_status sess_alloc(uint64_t cap, Table &t, int64_t **due);
    gwo_status sess_rebuild_due();
    gwo_status sess_join_sweep();
    int sess_fire_poll();   // a session sweep's completion: 1 published, 0 running, -1 test ev_fire instead
    gwo_status sess_read_err();
    gwo_status sess_ensure(uint64_t incoming);
    gwo_status sess_ensure_pool(uint64_t n);
    gwo_status read_occupancy_one(Table &t);
    gwo_status session_init();
    void session_free();
    gwo_status insert_session(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n);
    gwo_status fire_session(int64_t new_wm);
    gwo_status session_state_size(int64_t *entries);
    gwo_status session_snapshot_collect(const SnapCols &c);
    gwo_status session_restore_rows(const RestoreRows &R, int64_t new_wm);
    uint64_t session_live() const;
    // log-structured tumbling state (gwo_log.cpp)
    gwo_status log_init();
    gwo_status log_reserve();
    void log_free();
    gwo_status log_carve(LogWindow &W, size_t bytes, char **out);
    void log_release(LogWindow &W);
    int log_choose_lp(uint64_t batch_records) const;
    gwo_status log_split_exact(long long base, int nunits, uint64_t cap, const uint64_t *counts, int tmpx);
    gwo_status log_split_dev(const LogJob &J, const unsigned long long *rbp);
    gwo_status log_resolve_split();
    bool log_split_mode() const;          // pass 2 on its own stream (GWO_SPLIT_STREAM, log_p2_begin)
    hipStream_t log_p2_begin(int slot);
    void log_p2_end(int slot);
    // ts32: `t` points at int32 timestamps - tbase (records received in the 20-B wire format)
    gwo_status insert_log(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, int64_t stride = 1,
                          const LogRoute *route = nullptr, bool ts32 = false, int64_t tbase = 0,
                          const WindowGeom *geom_at = nullptr);
    gwo_status log_k1(LogJob &J, bool first_pass);
    LogThr log_thresholds(const LogJob &J) const;
    void log_uncarve(const LogJob &J, int w, uint64_t keep);
    gwo_status log_commit_spec(LogJob &J, const unsigned long long *rbp);
    gwo_status log_resolve_k1(LogJob J);
    gwo_status log_resolve_batch(LogJob &J, bool &refire);
    gwo_status log_fold_raw(const std::vector<long long> &units, const SnapCols &c);
    gwo_status log_migrate(long long u);
    gwo_status log_wait_readback(int slot, unsigned long long seq);
    gwo_status log_flush();                    // resolve the pipelined batch (no-op without one)
    bool log_pending_may_fire(int64_t new_wm) const;
    bool log_may_fire_since(int64_t batch_wm, int64_t new_wm) const;   // a window of records accepted at batch_wm fires by new_wm
    gwo_status set_pipelined(bool on);
    gwo_status fire_log(int64_t new_wm);
    gwo_status log_state_size(int64_t *entries);
    gwo_status log_snapshot_collect(const SnapCols &c);
    gwo_status log_restore_rows(const RestoreRows &R, int64_t new_wm);
    size_t log_window_count() const;
    int64_t log_usize() const;                 // the log's unit: the tumbling window, or the sliding pane
    int64_t log_lateness() const;              // cleanup distance past a unit's end: allowedLateness, or size - slide
    WindowGeom log_geom_now() const;           // K1's geometry (sliding panes: tumbling windows of `slide`)
    // sliding windows over logged panes (gwo_slog.cpp)
    gwo_status slog_init();
    int slog_lp() const;
    void slog_free();
    gwo_status slog_reserve(int64_t n);
    gwo_status slog_anchor();
    gwo_status slog_late_pass(const LogJob &J0);
    void slog_release_before(long long first_pane);
    gwo_status fire_slog(int64_t new_wm);
    gwo_status slog_step(int64_t start, int64_t end, uint64_t bound, size_t s0, size_t s1, bool emit, bool fresh,
                         bool *redo);
    gwo_status slog_rwin_add(long long j, const std::vector<int64_t> &key, const std::vector<int64_t> &words,
                             const std::vector<int64_t> &rows);
    void slog_rwin_release_before(long long j);
    size_t slog_rwin_count() const;
    gwo_status slog_rwin_rows(WindowRows &out);
    // comm (gwo_comm.cpp)
    void comm_free();
    gwo_status comm_exchange(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const int64_t **aos,
                             int64_t *rn, const int64_t **local, int64_t *ln);
    gwo_status comm_unpack(const int64_t *aos, int64_t n, const int64_t **rk, const int64_t **rt, const int64_t **rv);
    gwo_status comm_min_watermark(int64_t wm, int64_t *out);
    gwo_status comm_wait_received();
    // keyBy routing fused into the log layout's K1 (gwo_comm.cpp): arguments of the batch's routed K1 (*on false:
    // nothing to route -- one rank), the exchange after it, and the records received
    gwo_status comm_route_args(int64_t n, LogRoute *rt, bool *on);
    // K1 in route-only mode (rt.mode 3) over a batch's columns: the exact-capacity re-route after a region overflow
    gwo_status log_route_only(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const LogRoute &rt);
    gwo_status comm_mark_routed();
    gwo_status comm_after_route(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n);
    // K1's readback of a routed batch: re-route with exact capacities when a destination region overflowed
    gwo_status comm_check_route(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, uint64_t maxn,
                                uint64_t maxw);
    gwo_status comm_post();   // posts the record exchange of the oldest routed batch not posted yet
    gwo_status comm_post_older(bool wait, bool may_insert);   // posts the exchanges before the newest routed batch's
    // deferred receives of the routed log path: inserted two routed batches later or at log_flush
    bool comm_defers() const;
    gwo_status comm_insert_received(size_t keep);
    gwo_status comm_flush_received();
    bool comm_pending_wm(int64_t *wm) const;   // the oldest watermark a not yet inserted routed batch is classified at

    void prof_begin(int k, hipStream_t s = nullptr);
    void prof_end(int k, int64_t items, hipStream_t s = nullptr);
    gwo_status finish_fire();                  // wait for a pending fire (log layout, sessions) and publish its rows
    gwo_status session_finish_fire();
    gwo_status poll_fire();                    // non-blocking: finish_fire if the fire has completed
    gwo_status prof_collect();
};

}  // namespace gwo
