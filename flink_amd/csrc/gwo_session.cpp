// gwo_session.cpp -- host side of EventTimeSessionWindows (kernels: gwo_session.hip, gwo_sort.hip).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>

#include <cstring>

#include "gwo_handle.h"

namespace gwo {


void launch_sess_slot(const int64_t *key, const int64_t *ts, int64_t n, const TableDesc &t, uint64_t cap, int stride,
                      const SessGeom &g, uint32_t *rec_slot, SessErr *err, const SessLists *ls, hipStream_t s);
void launch_sess_process(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const uint32_t *sslot,
                         const uint32_t *sidx, const TableDesc &t, uint64_t cap, int stride, const AccPlan &p,
                         const ResultPlan &rp, const SessGeom &g, OutCols o, SessErr *err, int64_t *sk, int64_t *st,
                         int64_t *sv, unsigned long long *sc, long long scap, const SessLists *ls, hipStream_t s);
void launch_sess_long(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const uint32_t *rec_slot,
                      const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const ResultPlan &rp,
                      const SessGeom &g, OutCols o, SessErr *err, int64_t *sk, int64_t *st, int64_t *sv,
                      unsigned long long *sc, long long scap, const SessLists &ls, unsigned long long *rb,
                      unsigned long long seq, unsigned long long *reset_rows, hipStream_t s);
void launch_sess_fire(const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const ResultPlan &rp,
                      const SessGeom &g, OutCols o, SessErr *err, unsigned long long *arr, unsigned long long *shards,
                      unsigned long long *rb, unsigned long long seq, hipStream_t s);
void launch_sess_compact(const TableDesc &src, uint64_t cap, const TableDesc &dst, int stride, hipStream_t s);
void launch_sess_pool_compact(const TableDesc &t, uint64_t cap, int stride, int sw, const int64_t *old_pool,
                              const SessGeom &g, hipStream_t s);
void launch_sess_due(const TableDesc &t, uint64_t cap, int stride, int sw, const SessGeom &g, hipStream_t s);

struct SessionState {
    // in-flight sessions held inline per key entry (GWO_SESSION_SLOTS); a key with more spills into the pool.  C5 at
    // 8 / 4 / 2 slots: 0.0548-0.0559 / 0.0527-0.0531 / 0.0517-0.0524 ms/step (profiles/r06_experiments.txt) -- a
    // batch loads and writes back every inline slot of a touched key, and C5's keys hold 1-2 sessions at a time
    int smax = 2;
    int stride = 0;
    Table T;
    int64_t *due = nullptr;         // [T.cap + 1] due watermark per slot (SessGeom::due)
    uint64_t occ_pending = 0;       // entries claimed since T.occ was read, at most (one per record)
    uint64_t live = 0;              // in-flight sessions
    // the batches' statistics block accumulates (no per-batch reset): each read-back's change since the last is
    // the batch's (sess_read_err)
    SessErr *d_err = nullptr;
    SessErr *h_err = nullptr;       // pinned
    SessErr err_prev{};             // d_err as of the last read-back
    SessErr e{};                    // the last read-back's change (bad_kg_key: the value itself)
    SessErr *d_err_fire = nullptr;  // the watermark sweep's own block: its readback completes lazily (finish_fire)
    SessErr *h_err_fire = nullptr;  // d_err_fire as of the sweep's readback
    unsigned long long *rbf = nullptr, *rbf_dev = nullptr;   // host-mapped: the sweep's last workgroup publishes it
    unsigned long long rbf_seq = 0;
    bool reset_behind_fire = false; // a batch reset the row counter behind the pending sweep (its rows discarded)
    SessErr fire_prev{};
    int sort_digits = 8;            // radix digit bits of the slot sort (GWO_SESS_DIGITS: 8 or 10)
    DevBuf rec_slot, k1, v1, k2, v2, hist;
    // records grouped by slot in buckets (SessLists) instead of the radix sort; GWO_SESS_LISTS=0/1 fixes the choice,
    // otherwise the host switches to the sort while batches overflow many buckets (each such key costs a scan of the
    // batch's slots in sess_long_kernel) and back once they stop
    bool lists = true, lists_auto = true;
    DevBuf bkt;                     // [(cap + 1) * SESS_BKT] bucket words (counts zero between batches)
    uint32_t *ctl = nullptr;        // SessLists::ctl
    unsigned long long *arr = nullptr;   // sess_fire_kernel's arrival counters (ARR_WORDS)
    unsigned long long *shards = nullptr;   // SessLists::shards (zero between kernels)
    // spill pool of keys with more in-flight sessions than an entry holds (gwo_internal.h SessGeom)
    int64_t *pool = nullptr;
    uint64_t pool_cap = 0;          // session records
    unsigned long long *d_pool_top = nullptr;
    uint64_t pool_top = 0;          // as of the last read-back
    // host-mapped readback of the statistics block (publish_words_kernel): the batch's read-back is a spin
    unsigned long long *rb = nullptr, *rb_dev = nullptr;
    unsigned long long rb_seq = 0;
    // pipelined submission (gwo_set_pipelined_submit, allowedLateness 0, no side output): the batch's readback is
    // published but not read yet -- read at the watermark right after its sweep is queued, or at any other call
    bool rb_pending = false;
    uint64_t pend_n = 0;
    bool pend_lists = false;        // the pending batch went through the lists path (its release word, fire_session)
    uint64_t n_after_pend = 0;      // records of the batch being submitted behind the pending one (sess_collect_err)
    // the watermark sweep on the handle's fire_stream (pipelined submission, allowedLateness 0, no side output;
    // GWO_SESS_SIDE_SWEEP=1 only: measured slower, profiles/r06_experiments.txt): the next batch's slot pass -- it
    // claims entries and fills buckets, neither of which the sweep reads or writes (a slot's due watermark is SESS_NONE until its key has
    // sessions) -- overlaps it, and the stream joins the sweep (ev_fire) before anything that reads or writes
    // sessions, entries' contents or the pool (sess_join_sweep)
    bool side_sweep = false;
    bool wm_resolve = false;        // GWO_SESS_WM_RESOLVE=1: the watermark reads a pipelined batch's readback
    bool fire_event = false;        // the last sweep recorded ev_fire (side sweep, or GWO_SESS_FIRE_EVENT=1)
    bool fire_event_always = false;
    bool early_slot = true;         // GWO_SESS_EARLY_SLOT=0: a batch reads the previous readback before its slot pass
    bool sweep_on_side = false;     // a sweep queued on fire_stream that the handle's stream has not joined yet
    hipStream_t sweep_stream = nullptr;   // the stream of the last sweep (its readback spin polls it)
};

static constexpr unsigned long long kSessLongMax = 32;   // sess_long_kernel runs 32 workgroups
static constexpr double kSafeLoad = 0.9;   // sess_ensure: the load a slot pass may reach on a bound (one batch)

gwo_status Handle::sess_alloc(uint64_t cap, Table &t, int64_t **due) {
    SessionState &S = *sess;
    void *p = nullptr;
    GWO_TRY(dalloc(&p, ((size_t)cap + 1) * S.stride * 8 + ((size_t)cap + 1) * 8));
    t.base = (int64_t *)p;
    *due = t.base + (cap + 1) * S.stride;   // no sessions anywhere yet
    GWO_TRY(hipcheck(hipMemsetAsync(*due, 0x7f, ((size_t)cap + 1) * 8, stream), "due"));
    t.cap = cap;
    t.side = t.base + cap * S.stride;
    AccPlan fp{};
    fp.stride = S.stride;   // word 0 = EMPTY, every other word 0 (no sessions)
    launch_fill(t.base, cap + 1, fp, stream);
    GWO_TRY(launch_ok("fill"));
    GWO_TRY(hipcheck(hipMemsetAsync(t.side, 0, 8, stream), "side"));
    t.counter = take_counter();
    if (t.counter < 0) return fail(GWO_ERR_OUT_OF_MEMORY, "counter slots exhausted");
    t.occ = 0;
    return ctr_zero(t.counter);
}

gwo_status Handle::session_init() {
    sess = new SessionState();
    SessionState &S = *sess;
    if (const char *e = getenv("GWO_SESSION_SLOTS")) S.smax = std::max(1, std::min(16, atoi(e)));
    if (const char *e = getenv("GWO_SESS_DIGITS")) S.sort_digits = atoi(e) == 10 ? 10 : 8;
    if (const char *e = getenv("GWO_SESS_SIDE_SWEEP")) S.side_sweep = atoi(e) != 0;
    if (const char *e = getenv("GWO_SESS_WM_RESOLVE")) S.wm_resolve = atoi(e) != 0;
    if (const char *e = getenv("GWO_SESS_EARLY_SLOT")) S.early_slot = atoi(e) != 0;
    if (const char *e = getenv("GWO_SESS_FIRE_EVENT")) S.fire_event_always = atoi(e) != 0;
    if (const char *e = getenv("GWO_SESS_LISTS")) {
        S.lists = atoi(e) != 0;
        S.lists_auto = false;
    }
    GWO_TRY(dalloc((void **)&S.ctl, 16));
    GWO_TRY(hipcheck(hipMemsetAsync(S.ctl, 0, 16, stream), "session lists"));
    GWO_TRY(dalloc((void **)&S.arr, ARR_WORDS * 8));
    GWO_TRY(hipcheck(hipMemsetAsync(S.arr, 0, ARR_WORDS * 8, stream), "fire arrivals"));
    GWO_TRY(dalloc((void **)&S.shards, SESS_SHARDS * SESS_SHARD_STRIDE * 8));
    GWO_TRY(hipcheck(hipMemsetAsync(S.shards, 0, SESS_SHARDS * SESS_SHARD_STRIDE * 8, stream), "session shards"));
    S.stride = (2 + S.smax * (3 + plan.nwords) + 1) & ~1;
    // the pool's bump counter sits right behind the batch's SessErr block: one copy reads both back
    GWO_TRY(dalloc((void **)&S.d_err, sizeof(SessErr) + 8));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&S.h_err, sizeof(SessErr) + 8, hipHostMallocDefault), "pinned"));
    GWO_TRY(dalloc((void **)&S.d_err_fire, sizeof(SessErr)));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&S.h_err_fire, sizeof(SessErr), hipHostMallocDefault), "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&S.rbf, sizeof(SessErr) + 8, hipHostMallocCoherent | hipHostMallocMapped),
                     "fire readback"));
    memset(S.rbf, 0, sizeof(SessErr) + 8);
    GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&S.rbf_dev, S.rbf, 0), "fire readback"));
    GWO_TRY(hipcheck(hipEventCreateWithFlags(&ev_fire, hipEventDisableTiming), "event"));
    if (!fire_stream) GWO_TRY(hipcheck(hipStreamCreateWithFlags(&fire_stream, hipStreamNonBlocking), "fire stream"));
    if (!ev_main) GWO_TRY(hipcheck(hipEventCreateWithFlags(&ev_main, hipEventDisableTiming), "event"));
    // [SessErr words, pool top, sequence word, input-release word, table occupancy (the last two: sess_long_kernel)]
    GWO_TRY(hipcheck(hipHostMalloc((void **)&S.rb, sizeof(SessErr) + 32, hipHostMallocCoherent | hipHostMallocMapped),
                     "session readback"));
    memset(S.rb, 0, sizeof(SessErr) + 32);
    GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&S.rb_dev, S.rb, 0), "session readback"));
    S.d_pool_top = (unsigned long long *)((char *)S.d_err + sizeof(SessErr));
    GWO_TRY(hipcheck(hipMemsetAsync(S.d_err, 0, sizeof(SessErr) + 8, stream), "err"));
    GWO_TRY(hipcheck(hipMemsetAsync(S.d_err_fire, 0, sizeof(SessErr), stream), "fire err"));
    uint64_t cap = kMinCap;
    if (cfg.expected_keys > 0)
        while ((double)cfg.expected_keys > kInitLoad * (double)cap) cap <<= 1;
    return sess_alloc(cap, S.T, &S.due);
}

void Handle::session_free() {
    if (!sess) return;
    SessionState &S = *sess;
    if (S.T.base) (void)hipFree(S.T.base);
    if (S.d_err) (void)hipFree(S.d_err);
    if (S.h_err) (void)hipHostFree(S.h_err);
    if (S.rb) (void)hipHostFree(S.rb);
    if (S.rbf) (void)hipHostFree(S.rbf);
    if (S.d_err_fire) (void)hipFree(S.d_err_fire);
    if (S.h_err_fire) (void)hipHostFree(S.h_err_fire);
    if (S.pool) (void)hipFree(S.pool);
    if (S.ctl) (void)hipFree(S.ctl);
    if (S.arr) (void)hipFree(S.arr);
    if (S.shards) (void)hipFree(S.shards);
    S.bkt.release();
    S.rec_slot.release();
    S.k1.release();
    S.v1.release();
    S.k2.release();
    S.v2.release();
    S.hist.release();
    delete sess;
    sess = nullptr;
}

static SessGeom sess_geom(const Handle &h, int smax) {
    SessGeom g{};
    g.pool = h.sess->pool;
    g.pool_top = h.sess->d_pool_top;
    g.pool_cap = h.sess->pool_cap;
    g.due = h.sess->due;
    g.gap = h.cfg.gap;
    g.lateness = h.cfg.allowed_lateness;
    g.wm = h.wm;
    g.smax = smax;
    g.key_kind = h.cfg.key_kind;
    g.max_par = h.cfg.max_parallelism;
    g.kg_lo = h.cfg.key_group_start;
    g.kg_hi = h.cfg.key_group_end;
    g.side_enabled = h.cfg.side_output;
    return g;
}

gwo_status Handle::sess_publish_err() {
    SessionState &S = *sess;
    // the statistics and, right behind them, the pool's bump counter: published into host-mapped memory by a
    // one-wave kernel behind the batch's kernels, spun on (no copy, no stream synchronisation)
    constexpr int NWD = (int)(sizeof(SessErr) / 8) + 1;
    launch_publish_words((const unsigned long long *)S.d_err, NWD, S.rb_dev, ++S.rb_seq, stream);
    return launch_ok("session readback");
}

gwo_status Handle::sess_read_err() {
    GWO_TRY(sess_publish_err());
    return sess_collect_err();
}

gwo_status Handle::sess_collect_err(bool lists_batch) {
    SessionState &S = *sess;
    constexpr int NWD = (int)(sizeof(SessErr) / 8) + 1;
    GWO_TRY(spin_seq(S.rb + NWD, S.rb_seq, "session readback"));
    if (lists_batch) {   // the lists path's readback carries the table's exact occupancy after the batch
        S.T.occ = S.rb[NWD + 2];
        S.occ_pending = S.n_after_pend;   // records submitted behind the batch (a pipelined next batch)
    }
    memcpy(S.h_err, S.rb, sizeof(SessErr) + 8);
    S.pool_top = *(const unsigned long long *)((const char *)S.h_err + sizeof(SessErr));
    constexpr int W = (int)(sizeof(SessErr) / 8);
    const unsigned long long *now = (const unsigned long long *)S.h_err, *was = (const unsigned long long *)&S.err_prev;
    unsigned long long *d = (unsigned long long *)&S.e;
    for (int i = 0; i < W; ++i) d[i] = now[i] - was[i];
    S.e.bad_kg_key = S.h_err->bad_kg_key;
    S.err_prev = *S.h_err;
    return GWO_OK;
}

// A batch of n records can grow the spilled session lists by at most 4 x (live + n) session records (each key's
// arrays double, so one batch's allocations for a key stay within 4x its final count): the pool keeps that
// much room, compacting the spilled lists into a fresh pool (2 x their count each) when it runs short.
gwo_status Handle::sess_ensure_pool(uint64_t n) {
    SessionState &S = *sess;
    const uint64_t need = 4 * (S.live + n);
    if (S.pool_cap - S.pool_top >= need) return GWO_OK;
    GWO_TRY(sess_join_sweep());   // the sweep reads and writes the spilled lists
    const uint64_t ncap = std::max<uint64_t>(6 * (S.live + n), 1 << 16);
    const int sw = 3 + plan.nwords;
    int64_t *np = nullptr;
    GWO_TRY(dalloc((void **)&np, ncap * sw * 8));
    int64_t *old = S.pool;
    S.pool = np;
    S.pool_cap = ncap;
    GWO_TRY(hipcheck(hipMemsetAsync(S.d_pool_top, 0, 8, stream), "pool top"));
    if (old) {
        launch_sess_pool_compact(desc(S.T), S.T.cap, S.stride, sw, old, sess_geom(*this, S.smax), stream);
        GWO_TRY(launch_ok("session pool compaction"));
    }
    GWO_TRY(hipcheck(hipMemcpyAsync((char *)S.h_err + sizeof(SessErr), S.d_pool_top, 8, hipMemcpyDeviceToHost, stream),
                     "pool top"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "pool compaction"));
    S.pool_top = *(const unsigned long long *)((const char *)S.h_err + sizeof(SessErr));
    if (old) (void)hipFree(old);
    return GWO_OK;
}

// The handle's stream waits (on the device) for a sweep queued on fire_stream: before any launch that reads or writes
// sessions, entry contents, due watermarks or the pool.
gwo_status Handle::sess_join_sweep() {
    SessionState &S = *sess;
    if (!S.sweep_on_side) return GWO_OK;
    S.sweep_on_side = false;
    return hipcheck(hipStreamWaitEvent(stream, ev_fire, 0), "sweep join");
}

// Grow the per-key table (dropping keys without sessions) so `incoming` new keys fit.
gwo_status Handle::sess_ensure(uint64_t incoming) {
    SessionState &S = *sess;
    // upper bound without a device read: the last exact occupancy plus one claim per record since
    if ((double)(S.T.occ + S.occ_pending + incoming) <= kMaxLoad * (double)S.T.cap) {
        S.occ_pending += incoming;
        return GWO_OK;
    }
    // A pipelined batch is unread (its readback brings the exact occupancy, without a stream synchronisation): if the
    // table is within the growth threshold but for that batch's claims, the slot pass goes ahead on a safety bound
    // (every record a new key: the probes still find room below kSafeLoad) and the readback decides any growth at
    // the next batch.  C5 read the counter back (a stream synchronisation behind the sweep) every ~4 batches.
    const uint64_t but_pending = S.occ_pending > S.pend_n ? S.occ_pending - S.pend_n : 0;
    if (S.rb_pending && S.pend_lists && (double)(S.T.occ + but_pending + incoming) <= kMaxLoad * (double)S.T.cap &&
        (double)(S.T.occ + S.occ_pending + incoming) <= kSafeLoad * (double)S.T.cap) {
        S.occ_pending += incoming;
        return GWO_OK;
    }
    GWO_TRY(read_occupancy_one(S.T));
    S.occ_pending = incoming;
    if ((double)(S.T.occ + incoming) <= kMaxLoad * (double)S.T.cap) return GWO_OK;
    GWO_TRY(sess_resolve());      // (the live-session count below: exact, not one pipelined batch behind)
    GWO_TRY(sess_join_sweep());   // the compaction reads every entry
    uint64_t need = std::min<uint64_t>(S.T.occ, S.live) + incoming;
    uint64_t cap = kMinCap;
    while ((double)need > kInitLoad * (double)cap) cap <<= 1;
    Table nt;
    int64_t *ndue = nullptr;
    GWO_TRY(sess_alloc(cap, nt, &ndue));
    launch_sess_compact(desc(S.T), S.T.cap, desc(nt), S.stride, stream);
    GWO_TRY(launch_ok("compact"));
    GWO_TRY(hipcheck(hipMemcpyAsync(nt.side, S.T.side, (size_t)S.stride * 8, hipMemcpyDeviceToDevice, stream), "side"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "compact sync"));
    (void)hipFree(S.T.base);
    counter_used[S.T.counter] = 0;
    S.T = nt;
    S.due = ndue;
    GWO_TRY(sess_rebuild_due());
    return read_occupancy_one(S.T);
}

// Every slot's due watermark recomputed from the entries (after entries were written outside the hot path).
gwo_status Handle::sess_rebuild_due() {
    SessionState &S = *sess;
    GWO_TRY(sess_join_sweep());
    launch_sess_due(desc(S.T), S.T.cap, S.stride, 3 + plan.nwords, sess_geom(*this, S.smax), stream);
    return launch_ok("session due");
}

gwo_status Handle::read_occupancy_one(Table &t) {
    return ctr_read(t.counter, &t.occ);
}

gwo_status Handle::insert_session(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n) {
    SessionState &S = *sess;
    hp(0);
    // The last watermark's sweep is left running: the batch's kernels queue right behind it (no idle gap while the
    // host waits for it), and its rows and live-session change are applied at the next output access or watermark
    // (sizing below only needs upper bounds, which the unretired sessions give).  With allowedLateness > 0 the batch
    // emits re-fire rows behind the sweep's, so the sweep's rows are published first.
    if (cfg.allowed_lateness > 0) GWO_TRY(finish_fire());
    // A pipelined batch's readback (the previous batch: live-session count, pool top, errors) is read after this
    // batch's slot pass is queued (early): the slot pass only claims entries (sized by the occupancy bound, which
    // needs no readback) and fills buckets, so it covers the host's wait and the rest of its planning -- read before
    // it, the next batch's launches trailed the watermark's sweep by ~5.5 us of idle GPU per C5 step.  A batch that
    // failed still fails the handle before this batch's sessions change (its slot pass only claimed entries).
    const bool early = S.rb_pending && S.early_slot;
    if (!early) GWO_TRY(sess_resolve());
    if (n > 0xffffffffll) return fail(GWO_ERR_INVALID_ARGUMENT, "session batches are limited to 2^32 records");
    GWO_TRY(sess_ensure((uint64_t)n));
    if (!early) GWO_TRY(sess_ensure_pool((uint64_t)n));
    if (cfg.allowed_lateness > 0) GWO_TRY(ensure_output((uint64_t)n));   // re-fires: at most one row per record
    GWO_TRY(ensure_buf(S.rec_slot, n * 4));
    GWO_TRY(ensure_buf(S.k1, n * 4));
    const bool lists = S.lists;   // (this batch's grouping: a readback read below may switch the next batch's)
    int64_t hist_words = 0;
    if (lists) {
        const size_t was = S.bkt.bytes;
        GWO_TRY(ensure_buf(S.bkt, ((size_t)S.T.cap + 1) * SESS_BKT * 4));
        if (S.bkt.bytes != was)   // a fresh bucket array: every count zero
            GWO_TRY(hipcheck(hipMemsetAsync(S.bkt.ptr, 0, S.bkt.bytes, stream), "session buckets"));
    } else {
        GWO_TRY(ensure_buf(S.v1, n * 4));
        GWO_TRY(ensure_buf(S.k2, n * 4));
        GWO_TRY(ensure_buf(S.v2, n * 4));
        int64_t nblocks = (n + 4095) / 4096;
        hist_words = (int64_t)1024 * std::max<int64_t>(nblocks, 64);   // room for the small-sort tiles
        GWO_TRY(ensure_buf(S.hist, (size_t)hist_words * 4 + 16));
    }
    if (side_enabled() && side_cap - (long long)side_rows_committed < n)
        GWO_TRY(grow_side((long long)side_rows_committed + n));
    SessGeom g = sess_geom(*this, S.smax);
    // lists: the overflowing slots in k1 (radix: the sort's buffers)
    const SessLists ls{(uint32_t *)S.bkt.ptr, (uint32_t *)S.k1.ptr, S.ctl, S.shards};
    OutCols o = out_cols();
    int64_t *sk = (int64_t *)side_key.ptr, *sts = (int64_t *)side_ts.ptr, *sv = (int64_t *)side_val.ptr;
    const long long scap = side_enabled() ? side_cap : 0;
    hp(1);
    prof_begin(GWO_KERNEL_SESSION);
    launch_sess_slot(k, t, n, desc(S.T), S.T.cap, S.stride, g, (uint32_t *)S.rec_slot.ptr, S.d_err, lists ? &ls : nullptr,
                     stream);
    GWO_TRY(launch_ok("sess slot"));
    hp(2);
    if (early) {
        S.n_after_pend = (uint64_t)n;   // (counted in occ_pending by sess_ensure above)
        const gwo_status st = sess_resolve();
        S.n_after_pend = 0;
        GWO_TRY(st);
        GWO_TRY(sess_ensure_pool((uint64_t)n));
    }
    hp(3);
    GWO_TRY(sess_join_sweep());   // the slot pass overlapped the sweep; the rest of the batch follows it
    if (lists) {
        launch_sess_process(k, t, v, n, (const uint32_t *)S.rec_slot.ptr, nullptr, desc(S.T), S.T.cap, S.stride, plan, rplan, g, o, S.d_err, sk,
                            sts, sv, d_side_count, scap, &ls, stream);
        GWO_TRY(launch_ok("sess process"));
        // the batch's statistics are published by the last kernel's last workgroup (no publish launch), which also
        // resets the output's row counter after a discard: without allowedLateness a batch emits no rows, so the
        // counter is free until the next sweep (whose memset this saves).  A sweep still running when the rows
        // were discarded is ahead of it in the stream: its rows go too (session_finish_fire).
        unsigned long long *reset_rows = nullptr;
        if (out_count_dirty && cfg.allowed_lateness == 0 && (!fire_pending || discard_after_fire)) {
            reset_rows = d_out_count;
            out_count_dirty = false;
            S.reset_behind_fire = fire_pending;
        }
        launch_sess_long(k, t, v, n, (const uint32_t *)S.rec_slot.ptr, desc(S.T), S.T.cap, S.stride, plan, rplan, g, o,
                         S.d_err, sk, sts, sv, d_side_count, scap, ls, S.rb_dev, ++S.rb_seq, reset_rows, stream);
        GWO_TRY(launch_ok("sess long"));
        hp(4);
        prof_end(GWO_KERNEL_SESSION, n);
    } else {
        int bits = 1;   // slots are 0..cap (cap: the side slot)
        while (bits < 32 && (S.T.cap >> bits) > 0) bits++;
        int which = radix_sort_pairs((const uint32_t *)S.rec_slot.ptr, nullptr, n, bits, (uint32_t *)S.k1.ptr,
                                     (uint32_t *)S.v1.ptr, (uint32_t *)S.k2.ptr, (uint32_t *)S.v2.ptr,
                                     (uint32_t *)S.hist.ptr, stream, S.sort_digits, hist_words);
        GWO_TRY(launch_ok("radix sort"));
        const uint32_t *ss = which ? (const uint32_t *)S.k2.ptr : (const uint32_t *)S.k1.ptr;
        const uint32_t *si = which ? (const uint32_t *)S.v2.ptr : (const uint32_t *)S.v1.ptr;
        launch_sess_process(k, t, v, n, ss, si, desc(S.T), S.T.cap, S.stride, plan, rplan, g, o, S.d_err, sk, sts, sv,
                            d_side_count, scap, nullptr, stream);
        GWO_TRY(launch_ok("sess process"));
        prof_end(GWO_KERNEL_SESSION, n);
        GWO_TRY(sess_publish_err());
    }
    if (pipe_submit && cfg.allowed_lateness == 0 && !side_enabled()) {   // read by the next call (sess_resolve)
        S.rb_pending = true;
        S.pend_n = (uint64_t)n;
        S.pend_lists = lists;
        return GWO_OK;
    }
    GWO_TRY(sess_collect_err(lists));
    return sess_apply_err();
}

// Reads and applies a pipelined batch's readback (no-op without one).
gwo_status Handle::sess_resolve() {
    if (!sess || !sess->rb_pending) return GWO_OK;
    sess->rb_pending = false;
    GWO_TRY(sess_collect_err(sess->pend_lists));
    return sess_apply_err();
}

gwo_status Handle::sess_apply_err() {
    SessionState &S = *sess;
    const SessErr &e = S.e;
    if (e.bad_ts)
        return poison(GWO_ERR_NO_TIMESTAMP, "Record has Long.MIN_VALUE timestamp (= no timestamp marker).");
    if (e.bad_kg)
        return poison(GWO_ERR_KEY_GROUP, ("Key group of key " + std::to_string(e.bad_kg_key) +
                                          " is not in KeyGroupRange{startKeyGroup=" + std::to_string(cfg.key_group_start) +
                                          ", endKeyGroup=" + std::to_string(cfg.key_group_end) + "}.").c_str());
    if (e.merge_late)
        return poison(GWO_ERR_MERGE_LATE, "The end timestamp of an event-time window cannot become earlier than the "
                                          "current watermark by merging.");
    if (e.pool_full) return poison(GWO_ERR_HIP, "session spill pool exhausted despite its reservation");
    // bucket overflows: a few keys per batch are cheap (a workgroup each scans the batch's slots), many are not
    if (S.lists_auto) {
        if (S.lists && e.long_slots > kSessLongMax) S.lists = false;
        else if (!S.lists && e.long_slots <= kSessLongMax / 4) S.lists = true;
    }
    S.live += e.live_delta;
    out_rows += e.emitted;
    if (side_enabled()) {
        GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_side_count, 8, hipMemcpyDeviceToHost, stream), "side"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side sync"));
        if ((long long)*h_scalar > side_cap)
            return poison(GWO_ERR_CAPACITY, "side output overflow");
        side_rows = side_rows_committed = *h_scalar;
    } else {
        late_dropped += e.late;
    }
    return GWO_OK;
}

// The watermark sweep is queued with its statistics copy behind it and not waited for: its rows and live-session
// change are applied by finish_fire, at the next batch or output access (by then it has usually completed).
gwo_status Handle::fire_session(int64_t new_wm) {
    SessionState &S = *sess;
    hp(8, true);
    GWO_TRY(finish_fire());
    hp(9);
    // a pipelined batch still unread adds at most one live session per record: the sweep is sized for that and
    // queued right behind the batch, then the batch's readback is read
    const uint64_t live_bound = S.live + (S.rb_pending ? S.pend_n : 0);
    if (live_bound == 0) return sess_resolve();
    GWO_TRY(ensure_output(live_bound));
    SessGeom g = sess_geom(*this, S.smax);
    g.wm = new_wm;
    S.reset_behind_fire = false;
    const bool side = S.side_sweep && S.lists && pipe_submit && cfg.allowed_lateness == 0 && !side_enabled();
    hipStream_t fs = stream;
    if (side) {   // behind everything queued so far (the batch's kernels, the output reservation)
        GWO_TRY(hipcheck(hipEventRecord(ev_main, stream), "event"));
        GWO_TRY(hipcheck(hipStreamWaitEvent(fire_stream, ev_main, 0), "event wait"));
        fs = fire_stream;
    }
    prof_begin(GWO_KERNEL_FIRE, fs);
    launch_sess_fire(desc(S.T), S.T.cap, S.stride, plan, rplan, g, out_cols(), S.d_err_fire, S.arr, S.shards,
                     S.rbf_dev, ++S.rbf_seq, fs);
    GWO_TRY(launch_ok("sess fire"));
    prof_end(GWO_KERNEL_FIRE, (int64_t)S.T.cap, fs);
    hp(10);
    // the side sweep's join (and poll_fire's completion test) is an event; otherwise the sweep's readback sequence
    // word is the test: an event recorded behind every sweep held the next batch's first kernel ~5.5 us behind the
    // sweep's end (C5; GWO_SESS_FIRE_EVENT=1 restores it, profiles/r06_experiments.txt)
    S.fire_event = side || S.fire_event_always;
    if (S.fire_event) GWO_TRY(hipcheck(hipEventRecord(ev_fire, fs), "event"));
    S.sweep_on_side = side;
    S.sweep_stream = fs;
    fire_pending = true;
    // A pipelined batch's readback is left to the next call that needs it (the next batch's sizing, gwo_sync, the
    // statistics and checkpoint calls): read here, it held the host until the batch's last kernel ended, and the
    // next batch's launches then trailed the sweep by ~5.5 us of idle GPU per C5 step (GWO_SESS_WM_RESOLVE=1
    // restores the read; profiles/r06_experiments.txt).
    if (S.wm_resolve || !S.rb_pending) return sess_resolve();
    // the batch's device columns are released before this call returns (gwo.h: borrowed until the next call): the
    // lists path's long kernel publishes a release word as it starts (no long slot: nothing reads them any more),
    // the sort path's readback is its release
    constexpr int NWD = (int)(sizeof(SessErr) / 8) + 1;
    const gwo_status st = spin_seq(S.rb + (S.pend_lists ? NWD + 1 : NWD), S.rb_seq, "session input release");
    hp(11);
    return st;
}

int Handle::sess_fire_poll() {
    SessionState &S = *sess;
    if (S.fire_event) return -1;
    constexpr int NW = (int)(sizeof(SessErr) / 8);
    return *(volatile const unsigned long long *)(S.rbf + NW) == S.rbf_seq ? 1 : 0;
}

gwo_status Handle::session_finish_fire() {
    SessionState &S = *sess;
    fire_pending = false;
    constexpr int NW = (int)(sizeof(SessErr) / 8);
    GWO_TRY(spin_seq(S.rbf + NW, S.rbf_seq, "session fire readback", S.sweep_stream));
    GWO_TRY(sess_join_sweep());   // (complete: the join only keeps the stream's order explicit)
    memcpy(S.h_err_fire, S.rbf, sizeof(SessErr));
    const unsigned long long emitted = S.h_err_fire->emitted - S.fire_prev.emitted;
    S.live += S.h_err_fire->live_delta - S.fire_prev.live_delta;
    S.fire_prev = *S.h_err_fire;
    if (discard_after_fire) {   // gwo_discard_output was called while the sweep ran: its rows go too
        discard_after_fire = false;
        rows_gone += emitted;
        out_count_dirty = !S.reset_behind_fire;
    } else {
        out_rows += emitted;
    }
    return GWO_OK;
}

gwo_status Handle::session_state_size(int64_t *entries) {
    GWO_TRY(sess_resolve());
    GWO_TRY(finish_fire());
    *entries = (int64_t)sess->live;
    return GWO_OK;
}

// ---- checkpoint / restore (gwo_snapshot.cpp orchestrates; kernels in gwo_snapshot.hip) ----------------------
void launch_snap_session(const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const int64_t *pool,
                         const SnapCols &c, hipStream_t s);
void launch_sess_restore_wide(const int64_t *key, const int64_t *off, const int64_t *lcap, const int64_t *count,
                              int64_t m, const TableDesc &t, int stride, hipStream_t s);
void launch_sess_restore(const int64_t *key, const int64_t *start, const int64_t *end, const int32_t *timer,
                         const int64_t *words, int64_t n, const TableDesc &t, uint64_t cap, int stride,
                         const AccPlan &p, const SessGeom &g, SessErr *err, hipStream_t s);

gwo_status Handle::session_snapshot_collect(const SnapCols &c) {
    launch_snap_session(desc(sess->T), sess->T.cap, sess->stride, plan, sess->pool, c, stream);
    return launch_ok("session snapshot");
}

uint64_t Handle::session_live() const { return sess->live; }

// Rows of this subtask's key groups become in-flight sessions of their keys, each with its fire-timer flag
// (a pending timer at maxTimestamp, EventTimeTrigger.java:37-45; without flags: pending iff maxTs > watermark).
gwo_status Handle::session_restore_rows(const RestoreRows &R, int64_t new_wm) {
    SessionState &S = *sess;
    std::unordered_map<int64_t, int64_t> per_key;
    uint64_t mine = 0;
    for (int64_t i = 0; i < R.n; ++i) {
        if (!R.mine[i]) continue;
        if (R.end[i] <= R.start[i]) return fail(GWO_ERR_INVALID_ARGUMENT, "restore: empty session window");
        per_key[R.key[i]]++;
        mine++;
    }
    wm = in_wm = new_wm;
    if (mine == 0) return GWO_OK;
    GWO_TRY(sess_ensure(per_key.size()));
    const int sw = 3 + plan.nwords;
    // keys with more sessions than an entry holds: lists built here, uploaded into the spill pool
    std::unordered_map<int64_t, int64_t> wide_at;   // key -> index in the wide lists
    std::vector<int64_t> wk, woff, wcap, wcnt;
    uint64_t wide_records = 0;
    for (auto &kv : per_key)
        if (kv.second > S.smax) {
            wide_at[kv.first] = (int64_t)wk.size();
            wk.push_back(kv.first);
            woff.push_back((int64_t)wide_records);
            wcap.push_back(2 * kv.second);
            wcnt.push_back(0);
            wide_records += 2 * kv.second;
        }
    std::vector<int64_t> pool_img(wide_records * sw, 0);
    std::vector<int64_t> nk, nst, nen, nw;
    std::vector<int32_t> ntm;
    for (int64_t i = 0; i < R.n; ++i) {
        if (!R.mine[i]) continue;
        const bool timer = R.timer.empty() ? (int64_t)((uint64_t)R.end[i] - 1) > new_wm : R.timer[i] != 0;
        auto it = wide_at.find(R.key[i]);
        if (it == wide_at.end()) {
            nk.push_back(R.key[i]);
            nst.push_back(R.start[i]);
            nen.push_back(R.end[i]);
            ntm.push_back(timer ? 1 : 0);
            for (int w = 0; w < R.nw; ++w) nw.push_back(R.words[(size_t)i * R.nw + w]);
            continue;
        }
        const int64_t j = it->second;
        int64_t *X = pool_img.data() + (size_t)(woff[j] + wcnt[j]++) * sw;
        X[0] = R.start[i];
        X[1] = R.end[i];
        X[2] = timer ? 1 : 0;
        for (int w = 0; w < R.nw; ++w) X[3 + w] = R.words[(size_t)i * R.nw + w];
    }
    GWO_TRY(sess_ensure_pool(mine + wide_records));   // a fresh handle: the pool starts empty
    if (!wk.empty()) {
        if (S.pool_top + wide_records > S.pool_cap) return poison(GWO_ERR_HIP, "restore: spill pool too small");
        for (auto &o : woff) o += (int64_t)S.pool_top;
        GWO_TRY(hipcheck(hipMemcpy(S.pool + S.pool_top * sw, pool_img.data(), pool_img.size() * 8, hipMemcpyHostToDevice),
                         "restore pool"));
        const unsigned long long top = S.pool_top + wide_records;
        GWO_TRY(hipcheck(hipMemcpy(S.d_pool_top, &top, 8, hipMemcpyHostToDevice), "restore pool top"));
        S.pool_top = top;
        DevBuf a, b, c, d;
        for (DevBuf *x : {&a, &b, &c, &d}) GWO_TRY(ensure_buf(*x, wk.size() * 8));
        GWO_TRY(hipcheck(hipMemcpy(a.ptr, wk.data(), wk.size() * 8, hipMemcpyHostToDevice), "restore"));
        GWO_TRY(hipcheck(hipMemcpy(b.ptr, woff.data(), wk.size() * 8, hipMemcpyHostToDevice), "restore"));
        GWO_TRY(hipcheck(hipMemcpy(c.ptr, wcap.data(), wk.size() * 8, hipMemcpyHostToDevice), "restore"));
        GWO_TRY(hipcheck(hipMemcpy(d.ptr, wcnt.data(), wk.size() * 8, hipMemcpyHostToDevice), "restore"));
        launch_sess_restore_wide((const int64_t *)a.ptr, (const int64_t *)b.ptr, (const int64_t *)c.ptr,
                                 (const int64_t *)d.ptr, (int64_t)wk.size(), desc(S.T), S.stride, stream);
        GWO_TRY(launch_ok("session restore"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "session restore"));
        for (DevBuf *x : {&a, &b, &c, &d}) x->release();
        S.live += mine - nk.size();
    }
    const int64_t m = (int64_t)nk.size();
    if (m == 0) return sess_rebuild_due();
    DevBuf k, st, en, tm, w;
    GWO_TRY(ensure_buf(k, (size_t)m * 8));
    GWO_TRY(ensure_buf(st, (size_t)m * 8));
    GWO_TRY(ensure_buf(en, (size_t)m * 8));
    GWO_TRY(ensure_buf(tm, (size_t)m * 4));
    GWO_TRY(ensure_buf(w, (size_t)m * R.nw * 8));
    GWO_TRY(hipcheck(hipMemcpyAsync(k.ptr, nk.data(), (size_t)m * 8, hipMemcpyHostToDevice, stream), "restore"));
    GWO_TRY(hipcheck(hipMemcpyAsync(st.ptr, nst.data(), (size_t)m * 8, hipMemcpyHostToDevice, stream), "restore"));
    GWO_TRY(hipcheck(hipMemcpyAsync(en.ptr, nen.data(), (size_t)m * 8, hipMemcpyHostToDevice, stream), "restore"));
    GWO_TRY(hipcheck(hipMemcpyAsync(tm.ptr, ntm.data(), (size_t)m * 4, hipMemcpyHostToDevice, stream), "restore"));
    GWO_TRY(hipcheck(hipMemcpyAsync(w.ptr, nw.data(), (size_t)m * R.nw * 8, hipMemcpyHostToDevice, stream), "restore"));
    launch_sess_restore((const int64_t *)k.ptr, (const int64_t *)st.ptr, (const int64_t *)en.ptr,
                        (const int32_t *)tm.ptr, (const int64_t *)w.ptr, m, desc(S.T), S.T.cap, S.stride, plan,
                        sess_geom(*this, S.smax), S.d_err, stream);
    GWO_TRY(launch_ok("session restore"));
    GWO_TRY(sess_read_err());
    for (DevBuf *x : {&k, &st, &en, &tm, &w}) x->release();
    if (S.e.capacity) return poison(GWO_ERR_HIP, "restore: an entry overflowed its inline sessions");
    S.live += S.e.live_delta;
    return sess_rebuild_due();
}

}  // namespace gwo
