// gwo_slog.cpp -- host side of sliding windows over logged panes (kernel: gwo_slog.hip).
//
// SlidingEventTimeWindows (SlidingEventTimeWindows.java:68-82) with every aggregate word an int64 sum and
// allowedLateness 0, at high key cardinality.  A record is logged once, into its pane (a tumbling window
// of `slide`), by the log layout's K1 + pass 2 (gwo_log.cpp), classified against the pane's windows:
//   * the pane's last window already fired (cleanupTime of that window <= watermark): late, dropped or
//     side output -- WindowOperator.java:386-427 skips every window of the record;
//   * the pane's first window already fired (the pane is in the running total R): the record still
//     belongs to the pane's unfired windows; a second K1 pass over the batch (the "late pass") logs those
//     records into their panes and queues the new segments to be added to R at the next window step;
//   * otherwise it waits in its pane until the pane enters a window.
// The window step of window J (one kernel, gwo_slog.hip): R' = R + entering pane - leaving pane, and every
// key of R' with a positive count emits J's row (WindowOperator.onEventTime / emitWindowContents,
// WindowOperator.java:430-473, 546-550; EventTimeTrigger.onEventTime FIRE at maxTimestamp).  A pane's
// memory is released when it leaves the window.  R is rebuilt from the panes of J (no leaving pane)
// when it became empty, after a restore, and at the first fire.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "gwo_handle.h"
#include "gwo_log.h"
#include "gwo_log_state.h"
#include "gwo_slide.h"
#include "gwo_slog.h"

namespace gwo {

struct SlogState {
    int lp = 0;                    // partition bits of R and of new pane segments
    int cap_log2 = 11;             // LDS table slots of the window step
    bool split_next = false;       // the next window step writes R' at lp + 1
    DevBuf ring[2];                // R (in) and R' (out) alternate
    DevBuf bkt[2];                 // their bucket bytes ([2^lp][nb])
    DevBuf slot[2];                // their entries' table slots ([2^lp][rcap] uint16: the window step places by them)
    uint32_t *cnt[2] = {nullptr, nullptr};   // [2^LOG_MAX_LP] entries per partition
    uint64_t rcap[2] = {0, 0};
    int rlp[2] = {0, 0};
    int cur = 0;                   // ring[cur] holds R
    uint64_t live = 0;             // keys in R (the last fired window)
    uint64_t maxp = 0;             // largest partition of R
    bool rebuild = true;           // R is not the last fired window's total: rebuild from the panes of J
    std::vector<std::pair<long long, size_t>> pending;   // (pane, segment) added at the next window step
    uint64_t pending_records = 0;
    unsigned long long *d_stat = nullptr, *h_stat = nullptr;
    unsigned long long *rb = nullptr, *rb_dev = nullptr, rb_seq = 0;   // host-mapped: the step's folded statistics
    DevBuf segdesc;
    std::vector<SlogSeg> h_segs;
    int groups = 0;                // CUs
    bool reserved = false;
    // windows restored from a per-window savepoint (gwo_import_heap_state): window index -> its entries as a
    // partial-accumulator segment (key + raw words), added to R at the window's step and subtracted at the next
    std::map<long long, LogWindow> rwins;
};

static uint64_t slog_capacity(double mean) { return (uint64_t)std::ceil(mean + 6.0 * std::sqrt(mean) + 16.0); }

int Handle::slog_lp() const { return slog->lp; }

int64_t Handle::log_usize() const { return slog ? cfg.slide : cfg.size; }
int64_t Handle::log_lateness() const { return slog ? cfg.size - cfg.slide : cfg.allowed_lateness; }

// K1's geometry for the log: sliding panes are tumbling windows of `slide` at the assigner's offset (the
// pane start is getWindowStartWithOffset(ts, offset, slide), SlidingEventTimeWindows.java:72), and a pane is
// late when its last window is (cleanup distance size - slide past the pane's end, allowedLateness 0).
WindowGeom Handle::log_geom_now() const {
    WindowGeom g = geom_now();
    if (slog) {
        g.size = cfg.slide;
        g.inv_size = 1.0 / (double)cfg.slide;
        g.offset = cfg.offset;
        g.lateness = cfg.size - cfg.slide;
    }
    return g;
}

gwo_status Handle::slog_init() {
    slog = new SlogState();
    SlogState &G = *slog;
    // a table of <= 32 KiB (1024 slots for avg's two words; the sweep's slots per thread: 2..8) so about five
    // workgroups share a CU and overlap their partitions' HBM round trips
    const int c = slog_table_log2(plan.nwords);   // (the kernel instance for nwords is built for this size)
    G.cap_log2 = c;
    // R partitions: ~0.6 of the LDS table per partition at the caller's distinct-key hint (or the first batch)
    const double per = 0.6 * (double)(1 << c);
    G.lp = LOG_MIN_LP;
    if (cfg.expected_keys > 0)
        while (G.lp < LOG_MAX_LP && (double)cfg.expected_keys / (double)(1u << G.lp) > per) G.lp++;
    for (int i = 0; i < 2; ++i) {
        GWO_TRY(dalloc((void **)&G.cnt[i], ((size_t)1 << LOG_MAX_LP) * 4));
        GWO_TRY(hipcheck(hipMemsetAsync(G.cnt[i], 0, ((size_t)1 << LOG_MAX_LP) * 4, stream), "ring counts"));
        G.rlp[i] = G.lp;
    }
    GWO_TRY(dalloc((void **)&G.d_stat, SLOG_SHARDS * SLOG_STAT_STRIDE * 8));
    GWO_TRY(hipcheck(hipMemsetAsync(G.d_stat, 0, SLOG_SHARDS * SLOG_STAT_STRIDE * 8, stream), "ring stats"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&G.h_stat, SLOG_SHARDS * SLOG_STAT_STRIDE * 8, hipHostMallocDefault),
                     "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&G.rb, (SLS_WORDS + 1) * 8, hipHostMallocCoherent | hipHostMallocMapped),
                     "slog readback"));
    memset(G.rb, 0, (SLS_WORDS + 1) * 8);
    GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&G.rb_dev, G.rb, 0), "slog readback"));
    GWO_TRY(ensure_buf(G.segdesc, SLOG_MAX_SEGS * sizeof(SlogSeg)));
    int cus = 0;
    GWO_TRY(hipcheck(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg.device), "CU count"));
    G.groups = std::max(cus, 1);   // CUs (the launcher multiplies by the kernel's occupancy)
    if (cfg.expected_keys > 0) {   // R and R' for the hinted key count, so the steady state allocates nothing
        const uint64_t P = 1ull << G.lp;
        const uint64_t rcap = slog_capacity(1.25 * (double)cfg.expected_keys / (double)P);
        for (int i = 0; i < 2; ++i) {
            GWO_TRY(ensure_buf(G.ring[i], P * rcap * (1 + plan.nwords) * 8));
            G.rcap[i] = rcap;
        }
        GWO_TRY(ensure_output((uint64_t)cfg.expected_keys + (uint64_t)cfg.expected_keys / 4 + 4096));
    }
    const size_t nb = ((size_t)1 << G.cap_log2) / 8;
    for (int i = 0; i < 2; ++i) GWO_TRY(ensure_buf(G.bkt[i], ((size_t)1 << G.lp) * nb));
    // the window step's code object: one partition, no entries, no segments (HIP loads a kernel on its first launch)
    SlogArgs a{};
    a.in = SlogRing{nullptr, G.cnt[0], (uint8_t *)G.bkt[0].ptr, 0, 0, 0};
    a.out = SlogRing{nullptr, G.cnt[1], (uint8_t *)G.bkt[1].ptr, 0, 0, 0};
    a.p = plan;
    a.rp = rplan;
    a.count_word = slide->count_word;
    a.cap_log2 = G.cap_log2;
    a.stat = G.d_stat;
    a.o.count = d_scratch_count;
    launch_slog_fire(a, 1, stream);
    GWO_TRY(launch_ok("slog warm-up"));
    return hipcheck(hipMemsetAsync(G.d_stat, 0, SLOG_SHARDS * SLOG_STAT_STRIDE * 8, stream), "ring stats");
}

void Handle::slog_free() {
    if (!slog) return;
    SlogState &G = *slog;
    for (auto &kv : G.rwins) log_release(kv.second);
    for (int i = 0; i < 2; ++i) {
        G.ring[i].release();
        G.bkt[i].release();
        G.slot[i].release();
        if (G.cnt[i]) (void)hipFree(G.cnt[i]);
    }
    G.segdesc.release();
    if (G.d_stat) (void)hipFree(G.d_stat);
    if (G.h_stat) (void)hipHostFree(G.h_stat);
    if (G.rb) (void)hipHostFree(G.rb);
    delete slog;
    slog = nullptr;
}

// The pane chunk pool, sized from the first batch: every pane of a window plus a few in flight, each
// chunk holding a pane's segments (speculative carves included), touched now so no step allocates.
gwo_status Handle::slog_reserve(int64_t n) {
    SlogState &G = *slog;
    if (G.reserved) return GWO_OK;
    G.reserved = true;
    const double P = (double)(1u << G.lp);
    const double seg = (double)n + 6.0 * std::sqrt(P * (double)n) + 5.0 * P + 64.0;
    size_t chunk = (size_t)1 << 20;
    while ((double)chunk < 2.2 * seg * (needs_value ? 16.0 : 8.0) + 16.0 * P) chunk <<= 1;
    log_chunk_min = chunk;
    size_t free_b = 0, total_b = 0;
    GWO_TRY(hipcheck(hipMemGetInfo(&free_b, &total_b), "memory info"));
    const size_t panes = (size_t)(cfg.size / cfg.slide) + 8;
    const size_t want = std::min(panes * chunk, free_b / 4);
    for (size_t got = 0; got + chunk <= want; got += chunk) {
        void *p = nullptr;
        GWO_TRY(dalloc(&p, chunk));
        GWO_TRY(hipcheck(hipMemsetAsync(p, 0, chunk, stream), "pane pool"));
        logst->free_chunks.emplace(chunk, (char *)p);
    }
    return GWO_OK;
}

// After a restore: windows ending at or before the watermark fired before the checkpoint; R is rebuilt
// from the restored panes at the next window step.
gwo_status Handle::slog_anchor() {
    SlideState &S = *slide;
    S.J = first_unfired_window(wm);
    S.j_set = true;
    slog->rebuild = true;
    slog->pending.clear();
    slog->pending_records = 0;
    return GWO_OK;
}

// Restored window j's pending entries (rows of key / words, words already carrying a positive count word) as a
// partial segment partitioned like R (top lp bits of digit_hash; lp never shrinks, so it is never finer than R's).
gwo_status Handle::slog_rwin_add(long long j, const std::vector<int64_t> &key, const std::vector<int64_t> &words,
                                 const std::vector<int64_t> &rows) {
    SlogState &G = *slog;
    const int NW = plan.nwords, RW = 1 + NW;
    LogWindow &W = G.rwins[j];
    W.lp = G.lp;
    const uint32_t F = 1u << W.lp;
    std::vector<uint32_t> cnt(F, 0), off(F, 0);
    for (int64_t i : rows) cnt[digit_hash(key[i]) >> (32 - W.lp)]++;
    uint32_t run = 0;
    for (uint32_t p = 0; p < F; ++p) {
        off[p] = run;
        run += cnt[p];
    }
    std::vector<uint32_t> fill(off);
    std::vector<int64_t> rec((size_t)rows.size() * RW);
    for (int64_t i : rows) {
        int64_t *r = rec.data() + (size_t)fill[digit_hash(key[i]) >> (32 - W.lp)]++ * RW;
        r[0] = key[i];
        for (int w = 0; w < NW; ++w) r[1 + w] = words[(size_t)i * NW + w];
    }
    char *p_rec = nullptr, *p_off = nullptr, *p_cnt = nullptr;
    GWO_TRY(log_carve(W, rec.size() * 8, &p_rec));
    GWO_TRY(log_carve(W, (size_t)F * 4, &p_off));
    GWO_TRY(log_carve(W, (size_t)F * 4, &p_cnt));
    GWO_TRY(hipcheck(hipMemcpy(p_rec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice), "restore records"));
    GWO_TRY(hipcheck(hipMemcpy(p_off, off.data(), (size_t)F * 4, hipMemcpyHostToDevice), "restore offsets"));
    GWO_TRY(hipcheck(hipMemcpy(p_cnt, cnt.data(), (size_t)F * 4, hipMemcpyHostToDevice), "restore counts"));
    W.partial = LogSegDesc{(int64_t *)p_rec, (uint32_t *)p_off, (uint32_t *)p_cnt, W.lp, (uint32_t)rows.size()};
    W.partial_rows = rows.size();
    return GWO_OK;
}

void Handle::slog_rwin_release_before(long long j) {
    SlogState &G = *slog;
    for (auto it = G.rwins.begin(); it != G.rwins.end() && it->first < j;) {
        log_release(it->second);
        it = G.rwins.erase(it);
    }
}

size_t Handle::slog_rwin_count() const {
    size_t n = 0;
    for (auto &kv : slog->rwins) n += kv.second.partial_rows;
    return n;
}

gwo_status Handle::slog_rwin_rows(WindowRows &out) {
    const int NW = plan.nwords, RW = 1 + NW;
    std::vector<int64_t> rec;
    for (auto &kv : slog->rwins) {
        const LogWindow &W = kv.second;
        rec.resize((size_t)W.partial_rows * RW);
        if (rec.empty()) continue;
        GWO_TRY(hipcheck(hipMemcpy(rec.data(), W.partial.rec, rec.size() * 8, hipMemcpyDeviceToHost), "restored window"));
        for (uint64_t r = 0; r < W.partial_rows; ++r) {
            out.key.push_back(rec[r * RW]);
            out.j.push_back(kv.first);
            out.pending.push_back(1);
            out.words.insert(out.words.end(), rec.begin() + r * RW + 1, rec.begin() + (r + 1) * RW);
        }
    }
    return GWO_OK;
}

// The late pass (see the file comment): K1 over the batch again, accepting only the records whose pane is
// already in R; their new segments are added to R at the next window step (and leave with their pane).
gwo_status Handle::slog_late_pass(const LogJob &J0) {
    LogState &L = *logst;
    SlogState &G = *slog;
    std::map<long long, std::pair<size_t, uint64_t>> before;
    for (auto &kv : L.wins) before[kv.first] = {kv.second.segs.size(), kv.second.records};
    LogJob J = J0;
    J.only_refire = true;
    J.spec = false;
    if (J.rt.mode != 0) J.rt.mode = 2;   // other GPUs' records were routed by the first K1
    J.nunits = LOG_NU;
    J.slot = L.free_slot();
    const long long hint = hist_hint, span = L.span_hint;
    GWO_TRY(log_k1(J, false));
    bool refire = false;
    gwo_status s = log_resolve_batch(J, refire);
    hist_hint = hint;   // the next batch's window-range guess stays the stream's, not the late panes'
    L.span_hint = span;
    GWO_TRY(s);
    GWO_TRY(log_resolve_split());
    for (auto &kv : L.wins) {
        auto it = before.find(kv.first);
        const size_t s0 = it == before.end() ? 0 : it->second.first;
        const uint64_t r0 = it == before.end() ? 0 : it->second.second;
        for (size_t i = s0; i < kv.second.segs.size(); ++i) G.pending.push_back({kv.first, i});
        G.pending_records += kv.second.records - r0;
    }
    return GWO_OK;
}

void Handle::slog_release_before(long long first_pane) {
    LogState &L = *logst;
    for (auto it = L.wins.begin(); it != L.wins.end() && it->first < first_pane;) {
        log_release(it->second);
        it = L.wins.erase(it);
    }
}

// One launch of a window step over segments h_segs[s0, s1): R' = R + those segments (rows only when `emit`).
// redo: set when the step ran speculatively behind a pass 2 that overflowed (its rows are rewound; the caller
// redoes the split exactly and the step).
gwo_status Handle::slog_step(int64_t start, int64_t end, uint64_t bound, size_t s0, size_t s1, bool emit, bool fresh,
                             bool *redo) {
    SlideState &S = *slide;
    SlogState &G = *slog;
    LogState &L = *logst;
    *redo = false;
    const int NW = plan.nwords, RW = 1 + NW;
        // R' geometry: the partitions split when the largest one nears the LDS table
        const int in = G.cur, outb = 1 - G.cur;
        const int lp_in = fresh ? G.lp : G.rlp[in];
        const int lp_out = (G.split_next && lp_in < LOG_MAX_LP) ? lp_in + 1 : lp_in;
        const uint64_t Pout = 1ull << lp_out;
        uint64_t rcap = slog_capacity((double)bound / (double)Pout);
        if (G.ring[outb].bytes < Pout * rcap * RW * 8)
            GWO_TRY(ensure_buf(G.ring[outb], (size_t)((double)(Pout * rcap * RW * 8) * 1.5)));
        rcap = G.ring[outb].bytes / (Pout * RW * 8);   // use all of it
        GWO_TRY(ensure_buf(G.bkt[outb], (size_t)Pout * (((size_t)1 << G.cap_log2) / 8)));
        GWO_TRY(ensure_buf(G.slot[outb], (size_t)Pout * rcap * 2));
        if (emit) GWO_TRY(ensure_output(bound));
        if (fresh)   // R is empty: every partition of the input reads zero entries
            GWO_TRY(hipcheck(hipMemsetAsync(G.cnt[in], 0, ((size_t)1 << lp_in) * 4, stream), "ring reset"));
        SlogArgs a{};
        a.in = SlogRing{(int64_t *)G.ring[in].ptr, G.cnt[in], (uint8_t *)G.bkt[in].ptr, G.rcap[in], lp_in, 0,
                        (uint16_t *)G.slot[in].ptr};
        a.out = SlogRing{(int64_t *)G.ring[outb].ptr, G.cnt[outb], (uint8_t *)G.bkt[outb].ptr, rcap, lp_out, 0,
                         (uint16_t *)G.slot[outb].ptr};
        a.segs = nullptr;
        a.nseg = (int)(s1 - s0);
        for (size_t i = s0; i < s1; ++i) a.seg[i - s0] = G.h_segs[i];
        a.emit = emit ? 1 : 0;
        a.has_val = needs_value ? 1 : 0;
        a.count_word = S.count_word;
        a.cap_log2 = G.cap_log2;
        a.start = start;
        a.end = end;
        a.p = plan;
        a.rp = rplan;
        a.stat = G.d_stat;
        static int trace = getenv("GWO_SLOG_TRACE") ? atoi(getenv("GWO_SLOG_TRACE")) : 0;
        static unsigned long long *d_dbg = nullptr;
        if (trace && !d_dbg) {
            (void)hipMalloc((void **)&d_dbg, (SLOG_DBG_PHASES + 2 * SLOG_DBG_BLOCKS) * 8);
            (void)hipMemset(d_dbg, 0, (SLOG_DBG_PHASES + 2 * SLOG_DBG_BLOCKS) * 8);
        }
        a.dbg = trace ? d_dbg : nullptr;
        static int mode = getenv("GWO_SLOG_MODE") ? atoi(getenv("GWO_SLOG_MODE")) : 0;
        a.mode = mode;
#if GWO_SLOG_CHECK
        static unsigned long long *h_viol = nullptr, *d_viol = nullptr;
        if (!h_viol) {
            GWO_TRY(hipcheck(hipHostMalloc((void **)&h_viol, 8 * 8, hipHostMallocCoherent | hipHostMallocMapped), "check"));
            memset(h_viol, 0, 8 * 8);
            GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&d_viol, h_viol, 0), "check"));
        }
        a.chk.viol = d_viol;
#endif
        const uint64_t rows0 = out_rows;
        for (int attempt = 0;; ++attempt) {
            a.o = out_cols();
#if GWO_SLOG_CHECK
            a.chk.in_rec = G.ring[in].bytes / 8;
            a.chk.in_slot = G.slot[in].bytes / 2;
            a.chk.out_rec = G.ring[outb].bytes / 8;
            a.chk.out_slot = G.slot[outb].bytes / 2;
#endif
            // (the statistics shards are zero: reset at creation and by every step's publish)
            prof_begin(GWO_KERNEL_FIRE);
            launch_slog_fire(a, G.groups, stream);
            GWO_TRY(launch_ok("slog window step"));
            prof_end(GWO_KERNEL_FIRE, (int64_t)bound);
            launch_slog_stat_publish(G.d_stat, G.rb_dev, ++G.rb_seq, stream);
            GWO_TRY(launch_ok("slog statistics"));
            GWO_TRY(spin_seq(G.rb + SLS_WORDS, G.rb_seq, "slog window step"));
            uint64_t st[SLS_WORDS] = {};
            for (int w = 0; w < SLS_WORDS; ++w) st[w] = G.rb[w];
#if GWO_SLOG_CHECK
            if (h_viol[0]) {
                fprintf(stderr, "[slog-check] window %lld attempt %d: %llu violations; first: what=%llu partition=%llu "
                                "index=%llu bound=%llu width=%llu lp %llu->%llu (in rcap %llu, out rcap %llu, segs %d, fresh %d)\n",
                        (long long)start, attempt, h_viol[0], h_viol[1], h_viol[2], h_viol[3], h_viol[4], h_viol[5],
                        h_viol[6], h_viol[7], (unsigned long long)a.in.rcap, (unsigned long long)a.out.rcap, a.nseg,
                        (int)fresh);
                memset(h_viol, 0, 8 * 8);
            }
#endif
            if (L.pend.active) {   // queued behind a pass 2 not checked yet (fire_slog): it completed before this step
                if (L.h_split_flag[L.pend.tmpx] != 0) {   // it overflowed: this step read an incomplete segment
                    *h_scalar = rows0;
                    GWO_TRY(hipcheck(hipMemcpyAsync(d_out_count, h_scalar, 8, hipMemcpyHostToDevice, stream),
                                     "row rewind"));
                    *redo = true;
                    return GWO_OK;
                }
                L.pend.active = false;   // (log_resolve_split's no-overflow outcome)
            }
            if (st[SLS_NEG] && !mode) return poison(GWO_ERR_HIP, "sliding log: a key's window count became negative");
            if (st[SLS_LDS]) return poison(GWO_ERR_CAPACITY, "sliding log: a partition overflowed its LDS table");
            if (st[SLS_ROVF]) {   // a partition of R' outgrew its region: larger regions, same step again
                if (attempt >= 4) return poison(GWO_ERR_CAPACITY, "sliding log: running-total partition overflow");
                rcap = std::max<uint64_t>(rcap * 2, st[SLS_MAXP] + st[SLS_MAXP] / 4 + 64);
                GWO_TRY(ensure_buf(G.ring[outb], Pout * rcap * RW * 8));
                GWO_TRY(ensure_buf(G.slot[outb], (size_t)Pout * rcap * 2));
                a.out.rec = (int64_t *)G.ring[outb].ptr;
                a.out.slot = (uint16_t *)G.slot[outb].ptr;
                a.out.rcap = rcap;
                *h_scalar = rows0;
                GWO_TRY(hipcheck(hipMemcpyAsync(d_out_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "row rewind"));
                continue;
            }
            if (debug)
                fprintf(stderr, "[gwo] slog window %lld: segs=%zu live=%llu maxp=%llu slow=%llu lp %d->%d\n",
                        (long long)start, G.h_segs.size(), (unsigned long long)st[SLS_LIVE],
                        (unsigned long long)st[SLS_MAXP], (unsigned long long)st[SLS_SLOW], lp_in, lp_out);
            G.live = st[SLS_LIVE];
            G.maxp = st[SLS_MAXP];
            if (trace && (S.J % 16) == 0) {   // phase times of workgroup 0 (device wall clock, 100 MHz)
                static std::vector<unsigned long long> hv(SLOG_DBG_PHASES + 2 * SLOG_DBG_BLOCKS);
                (void)hipMemcpy(hv.data(), d_dbg, hv.size() * 8, hipMemcpyDeviceToHost);
                const unsigned long long *h = hv.data();
                {   // workgroup start/end spread (ticks of 10 ns from the first start)
                    std::vector<long long> st, en;
                    for (int b = 0; b < SLOG_DBG_BLOCKS; ++b)
                        if (h[SLOG_DBG_PHASES + 2 * b] && h[SLOG_DBG_PHASES + 2 * b + 1]) {
                            st.push_back((long long)h[SLOG_DBG_PHASES + 2 * b]);
                            en.push_back((long long)h[SLOG_DBG_PHASES + 2 * b + 1]);
                        }
                    if (!st.empty()) {
                        const long long t0 = *std::min_element(st.begin(), st.end());
                        for (auto &x : st) x -= t0;
                        for (auto &x : en) x -= t0;
                        std::sort(st.begin(), st.end());
                        std::sort(en.begin(), en.end());
                        const size_t n = st.size();
                        fprintf(stderr, "[slog] window %lld workgroups %zu start p50/p90/max %lld/%lld/%lld end min/p10/p50/p90/max "
                                        "%lld/%lld/%lld/%lld/%lld\n", (long long)start, n, st[n / 2], st[n * 9 / 10], st[n - 1],
                                en[0], en[n / 10], en[n / 2], en[n * 9 / 10], en[n - 1]);
                    }
                    (void)hipMemset(d_dbg, 0, hv.size() * 8);
                }
                fprintf(stderr, "[slog] window %lld slow=%llu maxp=%llu:", (long long)start, (unsigned long long)st[SLS_SLOW],
                        (unsigned long long)st[SLS_MAXP]);
                // per partition: ranges, placement, fold (to the barrier after it), sweep loop 1, pass A, pass B, tail
                for (int q = 0; q < 16; ++q) {
                    const unsigned long long *x = h + q * 8;
                    fprintf(stderr, " [%lld %lld %lld %lld %lld %lld %lld]", (long long)(x[1] - x[0]), (long long)(x[2] - x[1]),
                            (long long)(x[3] - x[2]), (long long)(x[6] - x[3]), (long long)(x[7] - x[6]),
                            (long long)(x[4] - x[7]), (long long)(x[5] - x[4]));
                }
                fprintf(stderr, "\n");
            }
            break;
        }
        if (emit) out_rows = rows0 + G.live;
        if ((long long)out_rows > out.cap)   // never hand out rows past the output columns (a drain would read them)
            return poison(GWO_ERR_HIP, ("sliding log: " + std::to_string(out_rows) + " rows exceed the output capacity " +
                                        std::to_string(out.cap) + " (window step bound " + std::to_string(bound) + ")")
                                           .c_str());
        G.cur = outb;
        G.rcap[outb] = rcap;
        G.rlp[outb] = lp_out;
        G.lp = lp_out;   // new panes are logged at R's partitioning
        G.split_next = (double)G.maxp > 0.75 * (double)(1 << G.cap_log2);
    return GWO_OK;
}

// Window steps for every window whose maxTimestamp the watermark passed (EventTimeTrigger.onEventTime FIRE,
// InternalTimerServiceImpl.advanceWatermark fires timers in timestamp order: window J before J + 1).
gwo_status Handle::fire_slog(int64_t new_wm) {
    SlideState &S = *slide;
    SlogState &G = *slog;
    LogState &L = *logst;
    GWO_TRY(log_flush());
    // a pass 2 still unchecked is not waited for: the first window step is queued right behind it and checks its
    // overflow flag with the step's own readback (an overflow -- rare -- rewinds the step's rows, redoes the split
    // exactly and then the step); r03 waited here for pass 2, ~30 us of idle GPU per C3 step
    const __int128 j_new = first_unfired_window(new_wm);
    if (!S.j_set) {
        S.J = j_new;
        if (!L.wins.empty()) S.J = std::min(first_window_of_pane(L.wins.begin()->first), j_new);
        S.j_set = true;
        G.rebuild = true;
    }
    while (S.J < j_new) {
        long long lo = win_first_pane(S.J), hi = win_last_pane(S.J);
        G.h_segs.clear();
        uint64_t plus_records = 0;
        std::vector<long long> leaving;
        auto add_pane = [&](LogWindow &W, int sign) {
            for (auto &d : W.segs) G.h_segs.push_back(SlogSeg{d.rec, d.off, d.cnt, d.lp, sign, 0, d.nrec});
            if (W.partial.rec)
                G.h_segs.push_back(SlogSeg{W.partial.rec, W.partial.off, W.partial.cnt, W.partial.lp, sign, 1, W.partial.nrec});
            if (sign > 0) plus_records += W.records + W.partial_rows;
        };
        auto add_restored = [&](__int128 j, int sign) {   // a restored window's entries: in R for its own step only
            auto r = G.rwins.find((long long)j);
            if (r != G.rwins.end() && r->second.partial.rec) add_pane(r->second, sign);
        };
        if (G.rebuild) {
            // R holds nothing of window J - 1: skip to the first window holding a pane with records (or restored
            // entries) and sum its panes
            slog_release_before(lo);
            slog_rwin_release_before((long long)S.J);
            auto it = L.wins.begin();
            while (it != L.wins.end() && it->second.segs.empty() && !it->second.partial.rec) {
                log_release(it->second);   // offsets carved for a K1 range that got no records
                it = L.wins.erase(it);
            }
            if (it == L.wins.end() && G.rwins.empty()) {
                S.J = j_new;
                break;
            }
            __int128 ja = it == L.wins.end() ? j_new : std::max(S.J, first_window_of_pane(it->first));
            if (!G.rwins.empty()) ja = std::min(ja, (__int128)G.rwins.begin()->first);
            if (ja >= j_new) break;
            S.J = ja;
            lo = win_first_pane(S.J);
            hi = win_last_pane(S.J);
            slog_release_before(lo);
            for (auto jt = L.wins.lower_bound(lo); jt != L.wins.end() && jt->first <= hi; ++jt) add_pane(jt->second, +1);
            add_restored(S.J, +1);
            G.live = 0;
        } else {
            const long long plo = win_first_pane(S.J - 1), phi = win_last_pane(S.J - 1);
            for (auto jt = L.wins.upper_bound(phi); jt != L.wins.end() && jt->first <= hi; ++jt) add_pane(jt->second, +1);
            for (auto &pe : G.pending) {
                auto jt = L.wins.find(pe.first);
                if (jt == L.wins.end() || pe.second >= jt->second.segs.size()) continue;
                const LogSegDesc &d = jt->second.segs[pe.second];
                G.h_segs.push_back(SlogSeg{d.rec, d.off, d.cnt, d.lp, +1, 0, d.nrec});
            }
            plus_records += G.pending_records;
            for (auto jt = L.wins.lower_bound(plo); jt != L.wins.end() && jt->first < lo; ++jt) {
                add_pane(jt->second, -1);
                leaving.push_back(jt->first);
            }
            add_restored(S.J, +1);
            add_restored(S.J - 1, -1);
        }
        const auto pending_was = G.pending;
        const uint64_t pending_records_was = G.pending_records;
        G.pending.clear();
        G.pending_records = 0;
        // more segments than one step takes (a rebuild over a whole window, many small batches per pane): chunks
        // of SLOG_MAX_SEGS, entering segments first, so a key's count only falls towards its final value; only the
        // last chunk emits rows
        std::stable_sort(G.h_segs.begin(), G.h_segs.end(), [](const SlogSeg &x, const SlogSeg &y) { return x.sign > y.sign; });
        const int64_t start = win_start(S.J);
        const int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
        const uint64_t bound = G.live + plus_records;
        if (G.live == 0 && G.h_segs.empty()) {   // nothing in R and nothing enters: the window is empty
            for (long long u : leaving) {
                log_release(L.wins[u]);
                L.wins.erase(u);
            }
            G.rebuild = true;
            S.J += 1;
            continue;
        }
        const size_t nchunks = std::max<size_t>(1, (G.h_segs.size() + SLOG_MAX_SEGS - 1) / SLOG_MAX_SEGS);
        bool redo = false;
        for (size_t ch = 0; ch < nchunks && !redo; ++ch) {
            const bool last = ch + 1 == nchunks;
            const size_t s0 = ch * SLOG_MAX_SEGS, s1 = std::min(G.h_segs.size(), s0 + SLOG_MAX_SEGS);
            GWO_TRY(slog_step(start, end, bound, s0, s1, last, ch == 0 && G.rebuild, &redo));
        }
        if (redo) {   // (only the first chunk can be speculative: R is untouched, the window is built again)
            if (debug) fprintf(stderr, "[gwo] slog: the pass 2 ahead of window %lld overflowed: step redone\n", (long long)start);
            G.pending = pending_was;
            G.pending_records = pending_records_was;
            GWO_TRY(log_resolve_split());
            continue;
        }
        G.rebuild = G.live == 0;
        for (long long u : leaving) {
            log_release(L.wins[u]);
            L.wins.erase(u);
        }
        slog_rwin_release_before((long long)S.J);   // R holds window J's restored entries until the next step
        S.J += 1;
    }
    return GWO_OK;
}

}  // namespace gwo
