// gwo_log.cpp -- host side of the log-structured tumbling-window state (kernels: gwo_log.hip).
//
// Bookkeeping only: which windows are open, the device memory of their segments, the partition
// count of each window, bucket/partition capacities, and the per-batch partition/split/fire launch
// sequence.  The reference's equivalents are the window-contents state table and the timer queue
// of WindowOperator (WindowOperator.java:218-273 open(), :430-473 onEventTime,
// InternalTimerServiceImpl.java:268-278).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <vector>

#include "gwo_handle.h"
#include "gwo_log.h"
#include "gwo_log_state.h"

namespace gwo {

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static constexpr size_t kRbBytes = (size_t)LOG_RB_WORDS * 8;
static constexpr size_t kPlanBytes = (LOG_NU * LOG_ND + 1) * sizeof(LogBucket);

// Capacity of a fixed-size group that receives Binomial(n, 1/k) records: mean + 6 sigma + slack.
static uint64_t group_capacity(double mean) {
    return (uint64_t)std::ceil(mean + 6.0 * std::sqrt(mean) + 4.0);
}

gwo_status Handle::log_init() {
    logst = new LogState();
    LogState &L = *logst;
    GWO_TRY(dalloc((void **)&L.d_cursor, (LOG_CURSOR_WORDS + LOG_K1_TRASH_WORDS) * 8));
    GWO_TRY(hipcheck(hipMemsetAsync(L.d_cursor, 0, (LOG_CURSOR_WORDS + LOG_K1_TRASH_WORDS) * 8, stream), "cursor"));
    GWO_TRY(dalloc((void **)&L.d_bk, kPlanBytes * LOG_SLOTS));
    GWO_TRY(dalloc((void **)&L.d_plan, kPlanBytes));
    GWO_TRY(dalloc((void **)&L.d_overflow, 16));
    GWO_TRY(dalloc((void **)&L.d_slow, (LOG_SLOW_CAP + 1) * 4));   // the fire's slow-path partition list + count
    GWO_TRY(hipcheck(hipMemsetAsync(L.d_overflow, 0, 16, stream), "overflow"));
    GWO_TRY(dalloc((void **)&L.d_go, LOG_SLOTS * sizeof(unsigned)));
    GWO_TRY(dalloc((void **)&L.d_t0, 8));
    if (hipDeviceGetAttribute(&L.clock_khz, hipDeviceAttributeWallClockRate, cfg.device) != hipSuccess) L.clock_khz = 0;
    GWO_TRY(dalloc((void **)&L.d_done, LOG_DONE_WORDS * 8));
    GWO_TRY(hipcheck(hipMemsetAsync(L.d_done, 0, LOG_DONE_WORDS * 8, stream), "done"));
    {
        std::vector<unsigned long long> sh((size_t)LOG_SHARDS * LOG_CUR_STRIDE, 0ull);
        for (int q = 0; q < LOG_SHARDS; ++q) {
            sh[(size_t)q * LOG_CUR_STRIDE + K1S_MIN] = 0x7fffffffffffffffull;
            sh[(size_t)q * LOG_CUR_STRIDE + K1S_MAX] = 0x8000000000000000ull;
            sh[(size_t)q * LOG_CUR_STRIDE + K1S_NEXT] = 0x7fffffffffffffffull;
        }
        GWO_TRY(dalloc((void **)&L.d_k1sh, sh.size() * 8));
        GWO_TRY(hipcheck(hipMemcpy(L.d_k1sh, sh.data(), sh.size() * 8, hipMemcpyHostToDevice), "K1 shards"));
    }
    // written by kernels, read by the host after an event: coherent, mapped
    GWO_TRY(hipcheck(hipHostMalloc((void **)&L.h_rb, kRbBytes * LOG_SLOTS, hipHostMallocCoherent | hipHostMallocMapped),
                     "pinned"));
    GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&L.d_rbh, L.h_rb, 0), "mapped readback"));
    for (int i = 0; i < LOG_SLOTS; ++i)
        GWO_TRY(hipcheck(hipEventCreateWithFlags(&L.ev_rb[i], hipEventDisableTiming), "event"));
    GWO_TRY(hipcheck(hipEventCreateWithFlags(&L.ev_split, hipEventDisableTiming), "event"));
    if (const char *e = getenv("GWO_SPLIT_STREAM")) L.split_mode = atoi(e) != 0;
    if (L.split_mode) {
        GWO_TRY(hipcheck(hipStreamCreateWithFlags(&L.split_stream, hipStreamNonBlocking), "pass-2 stream"));
        for (int i = 0; i < LOG_SLOTS; ++i) {
            GWO_TRY(hipcheck(hipEventCreateWithFlags(&L.ev_k1done[i], hipEventDisableTiming), "event"));
            GWO_TRY(hipcheck(hipEventCreateWithFlags(&L.ev_p2[i], hipEventDisableTiming), "event"));
        }
    }
    GWO_TRY(hipcheck(hipHostMalloc((void **)&L.h_buckets, kPlanBytes, hipHostMallocDefault), "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&L.h_split_flag, 16, hipHostMallocCoherent | hipHostMallocMapped),
                     "pinned"));
    GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&L.d_split_flag, L.h_split_flag, 0), "mapped flag"));
    GWO_TRY(ensure_buf(L.firedesc, 4096 * sizeof(LogSegDesc)));   // no reallocation inside a fire
    GWO_TRY(hipcheck(hipHostMalloc((void **)&L.h_fire_out, 32, hipHostMallocDefault), "pinned"));
    GWO_TRY(hipcheck(hipStreamCreateWithFlags(&fire_stream, hipStreamNonBlocking), "fire stream"));
    GWO_TRY(hipcheck(hipEventCreateWithFlags(&ev_main, hipEventDisableTiming), "event"));
    GWO_TRY(hipcheck(hipEventCreateWithFlags(&ev_fire, hipEventDisableTiming), "event"));
    init_stats(0);   // afterwards K1's last workgroup resets the device stats after every launch
    L.cap_log2 = log_fire_cap_log2(plan.nwords);
    warm_log_kernels(plan.nwords, needs_value, stream);
    GWO_TRY(launch_ok("warm-up"));
    {   // pass 2's code object too: a speculative launch whose verdict word is 0 exits at once
        GWO_TRY(hipcheck(hipMemsetAsync(L.d_go, 0, LOG_SLOTS * sizeof(unsigned), stream), "go"));
        GWO_TRY(hipcheck(hipMemsetAsync(L.d_bk, 0, kPlanBytes, stream), "plan"));
        launch_log_split(nullptr, 1, needs_value, L.d_bk, 0, LogSegSet{}, L.d_split_flag, 1, L.d_go, stream);
        GWO_TRY(launch_ok("warm-up"));
    }
    return log_reserve();
}

// With a distinct-keys hint, the steady state's device memory is reserved (and touched) at creation, so no
// batch or fire allocates: the output rows of one window, and a chunk pool for the records of three
// windows in flight (one filling, one fired, the next -- 16-B records, about two records per key, 1.4x for
// the partitions' capacity slack), capped at a quarter of the free device memory.
gwo_status Handle::log_reserve() {
    if (cfg.expected_keys <= 0 || slog) return GWO_OK;   // (the sliding log reserves at its first batch)
    LogState &L = *logst;
    const uint64_t keys = (uint64_t)cfg.expected_keys;
    GWO_TRY(ensure_output(keys + keys / 8 + 4096));
    for (int64_t *c : {out.key, out.start, out.end, out.res[0], out.res[1], out.res[2], out.res[3]})
        if (c) GWO_TRY(hipcheck(hipMemsetAsync(c, 0, (size_t)out.cap * 8, stream), "output reserve"));
    size_t free_b = 0, total_b = 0;
    GWO_TRY(hipcheck(hipMemGetInfo(&free_b, &total_b), "memory info"));
    const double per_window = (double)keys * 2.0 * (needs_value ? 16.0 : 8.0) * 1.4;
    for (int i = 0; i < 8; ++i) {   // a new window's first carves (its partition offsets/counters) take 1-MB chunks
        void *p = nullptr;
        GWO_TRY(dalloc(&p, (size_t)1 << 20));
        GWO_TRY(hipcheck(hipMemsetAsync(p, 0, (size_t)1 << 20, stream), "pool reserve"));
        L.free_chunks.emplace((size_t)1 << 20, (char *)p);
    }
    const size_t chunk = (size_t)1 << 30;
    size_t want = (size_t)std::min(3.0 * per_window, (double)free_b / 4.0);
    for (size_t got = 0; got + chunk <= want; got += chunk) {
        void *p = nullptr;
        GWO_TRY(dalloc(&p, chunk));
        GWO_TRY(hipcheck(hipMemsetAsync(p, 0, chunk, stream), "pool reserve"));
        L.free_chunks.emplace(chunk, (char *)p);
    }
    return GWO_OK;
}

void Handle::log_free() {
    if (!logst) return;
    LogState &L = *logst;
    for (auto &kv : L.wins)
        for (auto &c : kv.second.chunks) (void)hipFree(c.base);
    for (auto &kv : L.free_chunks) (void)hipFree(kv.second);
    for (int i = 0; i < LOG_SLOTS; ++i) {
        L.tmp[i].release();
        if (L.ev_rb[i]) (void)hipEventDestroy(L.ev_rb[i]);
    }
    if (L.ev_split) (void)hipEventDestroy(L.ev_split);
    if (L.split_stream) {
        (void)hipStreamSynchronize(L.split_stream);
        (void)hipStreamDestroy(L.split_stream);
    }
    for (int i = 0; i < LOG_SLOTS; ++i) {
        if (L.ev_k1done[i]) (void)hipEventDestroy(L.ev_k1done[i]);
        if (L.ev_p2[i]) (void)hipEventDestroy(L.ev_p2[i]);
    }
    L.firedesc.release();
    if (L.h_split_flag) (void)hipHostFree(L.h_split_flag);
    if (L.h_fire_out) (void)hipHostFree(L.h_fire_out);
    if (L.d_cursor) (void)hipFree(L.d_cursor);
    if (L.d_bk) (void)hipFree(L.d_bk);
    if (L.d_plan) (void)hipFree(L.d_plan);
    if (L.d_overflow) (void)hipFree(L.d_overflow);
    if (L.d_slow) (void)hipFree(L.d_slow);
    if (L.d_go) (void)hipFree(L.d_go);
    if (L.d_done) (void)hipFree(L.d_done);
    if (L.d_t0) (void)hipFree(L.d_t0);
    if (L.d_k1sh) (void)hipFree(L.d_k1sh);
    if (L.h_rb) (void)hipHostFree(L.h_rb);
    if (L.h_buckets) (void)hipHostFree(L.h_buckets);
    delete logst;
    logst = nullptr;
}

// Carves `bytes` (256-B aligned) out of the window's chunks; new chunks come from the pool.
gwo_status Handle::log_carve(LogWindow &W, size_t bytes, char **out) {
    bytes = align256(bytes);
    if (W.chunks.empty() || W.chunks.back().size - W.chunks.back().used < bytes) {
        size_t want = 1 << 20;
        while (want < bytes * 4 && want < ((size_t)1 << 30)) want <<= 1;
        want = std::max(want, bytes);
        if (log_chunk_min && bytes <= log_chunk_min) want = log_chunk_min;   // sliding log: one pane size
        LogChunk c;
        auto it = logst->free_chunks.lower_bound(want);
        if (it != logst->free_chunks.end() && it->first <= want * 2) {
            c.base = it->second;
            c.size = it->first;
            logst->free_chunks.erase(it);
        } else {
            void *p = nullptr;
            gwo_status s = dalloc(&p, want);
            if (s != GWO_OK) {
                GWO_TRY(hipcheck(hipStreamSynchronize(stream), "pool trim"));
                for (auto &kv : logst->free_chunks) (void)hipFree(kv.second);
                logst->free_chunks.clear();
                GWO_TRY(dalloc(&p, want));
            }
            c.base = (char *)p;
            c.size = want;
        }
        W.chunks.push_back(c);
    }
    LogChunk &c = W.chunks.back();
    *out = c.base + c.used;
    c.used += bytes;
    return GWO_OK;
}

void Handle::log_release(LogWindow &W) {
    for (auto &c : W.chunks) logst->free_chunks.emplace(c.size, c.base);
    W.chunks.clear();
    W.segs.clear();
    W.partial = LogSegDesc{};
    W.partial_rows = 0;
}

// Partitions of a new window: about 3/4 of the fire kernel's fast-path capacity (FIRE_RCAP records)
// per partition, from the last fired window's record count, else the caller's distinct-key hint
// (records >= keys; x2 covers the usual duplication) or this batch's size.  An underestimate only
// sends partitions to the fire's slow path.
int Handle::log_choose_lp(uint64_t batch_records) const {
    if (slog) return slog_lp();   // sliding log: panes are partitioned like the running total
    const LogState &L = *logst;
    uint64_t est = L.last_window_records;
    if (est == 0) est = std::max<uint64_t>((uint64_t)std::max<int64_t>(cfg.expected_keys, 0) * 2, batch_records * 8);
    const uint64_t per = (uint64_t)FIRE_RCAP * LOG_PART_FILL / 8;
    int lp = LOG_MIN_LP;
    while (lp < LOG_MAX_LP && ((uint64_t)1 << lp) * per < est) lp++;
    return lp;
}

// Pass 2 planned on the host, synchronous: the exact re-run after a deferred pass 2 overflowed (skewed
// keys).  Fresh segments for windows [base, base + nunits) of batch buffer `tmpx` (bucket counts in
// `counts`); re-runs with each bucket's partitions sized to its measured largest one until nothing
// overflows.
gwo_status Handle::log_split_exact(long long base, int nunits, uint64_t cap, const uint64_t *counts, int tmpx) {
    LogState &L = *logst;
    const int W = needs_value ? 2 : 1;
    const int nb = nunits * LOG_ND;
    std::vector<LogWindow *> wins(nunits, nullptr);
    std::vector<uint64_t> wcount(nunits, 0);
    for (int b = 0; b < nb; ++b) wcount[b >> LOG_DB] += counts[b];
    std::vector<uint32_t> pcap_exact(nb, 0);   // after an overflow: the measured partition maximum
    LogSegSet set{};
    // the device plan of this batch buffer holds each bucket's region-group offsets (xoff)
    GWO_TRY(hipcheck(hipMemcpyAsync(L.h_buckets, L.bk(tmpx), (nb + 1) * sizeof(LogBucket), hipMemcpyDeviceToHost,
                                    stream), "plan"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "plan"));
    while (true) {
        uint32_t chunks = 0;
        for (int w = 0; w < nunits; ++w) {
            LogSegDesc d{};
            const int c0 = w * LOG_ND;
            if (wcount[w]) {
                LogWindow &Wn = L.wins[base + w];   // exists: created when K1 was launched over it
                wins[w] = &Wn;
                const int lp = Wn.lp, F = 1 << (lp - LOG_DB);
                uint64_t seg = 0;
                for (int dgt = 0; dgt < LOG_ND; ++dgt) {
                    const uint64_t n_b = counts[c0 + dgt];
                    LogBucket &B = L.h_buckets[c0 + dgt];
                    B.n = (uint32_t)n_b;
                    B.pcap = n_b ? std::max<uint32_t>((uint32_t)group_capacity((double)n_b / F), pcap_exact[c0 + dgt])
                                 : 0u;
                    B.seg_base = (uint32_t)seg;
                    B.chunk0 = chunks;
                    seg += (uint64_t)F * B.pcap;
                    chunks += (uint32_t)((n_b + LOG_TILE - 1) / LOG_TILE);
                }
                if (seg >= (1ull << 32)) return poison(GWO_ERR_CAPACITY, "log layout: batch segment exceeds 2^32 records");
                char *p = nullptr;
                GWO_TRY(log_carve(Wn, seg * W * 8, &p));
                d.rec = (int64_t *)p;
                GWO_TRY(log_carve(Wn, ((size_t)1 << lp) * 4, &p));
                d.off = (uint32_t *)p;
                GWO_TRY(log_carve(Wn, ((size_t)1 << lp) * 4, &p));
                d.cnt = (uint32_t *)p;
                d.lp = lp;
                d.nrec = (uint32_t)seg;
                GWO_TRY(hipcheck(hipMemsetAsync(d.cnt, 0, ((size_t)1 << lp) * 4, stream), "segment counts"));
            } else {
                for (int dgt = 0; dgt < LOG_ND; ++dgt) {
                    LogBucket &B = L.h_buckets[c0 + dgt];
                    B = LogBucket{};
                    B.chunk0 = chunks;
                }
            }
            set.s[w] = d;
        }
        L.h_buckets[nb] = LogBucket{};
        L.h_buckets[nb].chunk0 = chunks;
        L.h_split_flag[tmpx] = 0;
        GWO_TRY(hipcheck(hipMemcpyAsync(L.d_plan, L.h_buckets, (nb + 1) * sizeof(LogBucket), hipMemcpyHostToDevice, stream),
                         "split plan"));
        launch_log_split((const int64_t *)L.tmp[tmpx].ptr, cap, needs_value, L.d_plan, nb, set, L.d_split_flag + tmpx,
                         chunks, nullptr, stream);
        GWO_TRY(launch_ok("log split"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "log split"));
        if (L.h_split_flag[tmpx] == 0) break;
        // the cursors hold the exact counts: redo with each bucket's partitions sized to its largest one
        // (the segments carved above stay unused until the window is released)
        for (int w = 0; w < nunits; ++w) {
            if (!wins[w]) continue;
            const int F = 1 << (set.s[w].lp - LOG_DB);
            std::vector<uint32_t> cnt((size_t)LOG_ND * F);
            GWO_TRY(hipcheck(hipMemcpy(cnt.data(), set.s[w].cnt, cnt.size() * 4, hipMemcpyDeviceToHost), "counts"));
            for (int dgt = 0; dgt < LOG_ND; ++dgt)
                for (int f = 0; f < F; ++f)
                    pcap_exact[w * LOG_ND + dgt] = std::max(pcap_exact[w * LOG_ND + dgt], cnt[(size_t)dgt * F + f]);
        }
    }
    for (int w = 0; w < nunits; ++w) {
        if (!wins[w]) continue;
        wins[w]->segs.push_back(set.s[w]);
        wins[w]->records += wcount[w];
    }
    return GWO_OK;
}

// The stream a pass 2 of batch buffer `slot` runs on: the handle's, or (split mode; not with the sliding log, the
// multi-GPU exchange or pipelined submission, whose steps and inserts queue behind pass 2 on the handle's stream) the
// pass-2 stream behind an event marking everything queued on the handle's stream so far -- its K1.
bool Handle::log_split_mode() const {
    const LogState &L = *logst;
    return L.split_mode && !slog && !comm && !L.pipeline;
}
hipStream_t Handle::log_p2_begin(int slot) {
    LogState &L = *logst;
    if (!log_split_mode()) return stream;
    (void)hipEventRecord(L.ev_k1done[slot], stream);
    (void)hipStreamWaitEvent(L.split_stream, L.ev_k1done[slot], 0);
    return L.split_stream;
}
void Handle::log_p2_end(int slot) {
    LogState &L = *logst;
    if (log_split_mode()) (void)hipEventRecord(L.ev_p2[slot], L.split_stream);
}

// Commits a speculative pass 2 that runs the device plan (rb[LOG_RB_GO]): each window's segment records
// are trimmed to the plan's size and the segments join their windows; the partition-overflow flag is checked
// at the next sync point as for every pass 2 (log_resolve_split).
gwo_status Handle::log_commit_spec(LogJob &J, const unsigned long long *rbp) {
    LogState &L = *logst;
    uint64_t wcount[LOG_NU] = {};
    for (int b = 0; b < J.nunits * LOG_ND; ++b) wcount[b >> LOG_DB] += rbp[b];
    for (int w = 0; w < J.nunits; ++w) log_uncarve(J, w, wcount[w] ? rbp[LOG_RB_SEG + w] : 0);
    L.pend.after_seq = J.seq;   // any later readback implies this pass 2 completed (stream order; not in split mode)
    L.pend.has_event = false;
    L.pend.active = true;
    L.pend.tmpx = J.slot;
    L.pend.nunits = J.nunits;
    L.pend.base = J.base;
    L.pend.cap = J.cap;
    L.pend.counts.assign(rbp, rbp + J.nunits * LOG_ND);
    for (int w = 0; w < J.nunits; ++w) {
        if (!wcount[w]) continue;
        LogWindow &Wn = L.wins[J.base + w];
        J.desc[w].nrec = (uint32_t)std::min<uint64_t>(rbp[LOG_RB_SEG + w], J.seg_cap[w]);   // the device plan's size
        Wn.segs.push_back(J.desc[w]);
        Wn.records += wcount[w];
    }
    return GWO_OK;
}

// Pass 2 of job J from the device plan log_collect_kernel left in bk(J.slot): carve each window's segment
// records (sizes from the readback), launch, and return; the overflow flag is checked by
// log_resolve_split at the next sync point.
gwo_status Handle::log_split_dev(const LogJob &J, const unsigned long long *rbp) {
    LogState &L = *logst;
    const int W = needs_value ? 2 : 1;
    LogSegSet set{};
    uint64_t wcount[LOG_NU] = {}, total = 0;
    for (int b = 0; b < J.nunits * LOG_ND; ++b) wcount[b >> LOG_DB] += rbp[b];
    for (int w = 0; w < J.nunits; ++w) {
        set.s[w] = J.desc[w];
        if (!wcount[w]) continue;
        const uint64_t seg = rbp[LOG_RB_SEG + w];
        if (seg >= (1ull << 32)) return poison(GWO_ERR_CAPACITY, "log layout: batch segment exceeds 2^32 records");
        char *p = nullptr;
        GWO_TRY(log_carve(L.wins[J.base + w], seg * W * 8, &p));
        set.s[w].rec = (int64_t *)p;
        set.s[w].nrec = (uint32_t)seg;
        total += wcount[w];
    }
    L.h_split_flag[J.slot] = 0;
    hipStream_t ps = log_p2_begin(J.slot);
    prof_begin(GWO_KERNEL_PARTITION, ps);
    launch_log_split((const int64_t *)L.tmp[J.slot].ptr, J.cap, needs_value, L.bk(J.slot), J.nunits * LOG_ND, set,
                     L.d_split_flag + J.slot, (uint32_t)rbp[LOG_RB_CHUNKS], nullptr, ps);
    GWO_TRY(launch_ok("log split"));
    prof_end(GWO_KERNEL_PARTITION, (int64_t)total, ps);
    log_p2_end(J.slot);
    // completion is implied by the next K1's readback (stream order); only a pipelined K1, queued before
    // this pass 2, needs an event (a marker between the kernels costs several microseconds)
    L.pend.after_seq = L.seq;
    L.pend.has_event = L.pipeline;
    if (L.pipeline) GWO_TRY(hipcheck(hipEventRecord(L.ev_split, stream), "event"));
    L.pend.active = true;
    L.pend.tmpx = J.slot;
    L.pend.nunits = J.nunits;
    L.pend.base = J.base;
    L.pend.cap = J.cap;
    L.pend.counts.assign(rbp, rbp + J.nunits * LOG_ND);
    for (int w = 0; w < J.nunits; ++w) {
        if (!wcount[w]) continue;
        LogWindow &Wn = L.wins[J.base + w];
        Wn.segs.push_back(set.s[w]);
        Wn.records += wcount[w];
    }
    return GWO_OK;
}

// Checks the deferred pass 2: on overflow, its segments come out of their windows and pass 2 re-runs
// synchronously on the same batch buffer (which no later K1 touched).
gwo_status Handle::log_resolve_split() {
    LogState &L = *logst;
    if (!L.pend.active) return GWO_OK;
    if (log_split_mode()) {   // on its own stream: only its event says it completed
        GWO_TRY(spin_event(L.ev_p2[L.pend.tmpx], "pass 2"));
    } else if (L.seen_seq <= L.pend.after_seq) {   // the event, not the stream: a pipelined K1 may be queued behind it
        if (L.pend.has_event) GWO_TRY(spin_event(L.ev_split, "pass 2"));
        else GWO_TRY(hipcheck(hipStreamSynchronize(stream), "pass 2"));
    }
    L.pend.active = false;
    if (L.h_split_flag[L.pend.tmpx] == 0) return GWO_OK;
    for (int w = 0; w < L.pend.nunits; ++w) {
        uint64_t c = 0;
        for (int d = 0; d < LOG_ND; ++d) c += L.pend.counts[(size_t)w * LOG_ND + d];
        if (!c) continue;
        LogWindow &Wn = L.wins[L.pend.base + w];
        Wn.segs.pop_back();   // the deferred split's segment is the window's last one
        Wn.records -= c;
    }
    std::vector<uint64_t> counts = L.pend.counts;
    return log_split_exact(L.pend.base, L.pend.nunits, L.pend.cap, counts.data(), L.pend.tmpx);
}

// Upper bound of the segment records one window receives from a batch of n records: the device plan
// gives each of its LOG_ND coarse buckets F * pcap records (F = 2^lp / LOG_ND partitions each), pcap =
// ceil(n_b/F + 6 sqrt(n_b/F) + 4), so the window's segment is at most
//   n + 6 sqrt(F) * sum_b sqrt(n_b) + 5 * 2^lp <= n + 6 sqrt(2^lp n) + 5 * 2^lp   (Cauchy-Schwarz over the buckets).
static uint64_t seg_upper_bound(uint64_t n, int lp) {
    const double P = (double)(1u << lp);
    return (uint64_t)std::ceil((double)n + 6.0 * std::sqrt(P * (double)n) + 5.0 * P) + 64;
}

// Window bounds of K1's launch range [base, base + nunits) and each window's class at the batch's watermark
// (WindowOperator.java:386-427: isWindowLate via cleanupTime, EventTimeTrigger.onElement FIRE for maxTs <= wm),
// so K1 classifies a record inside the range by comparing its timestamp with the bounds.  Off when a bound
// leaves the int64 range or lies where getWindowStartWithOffset is not monotone (ts < offset - size).
LogThr Handle::log_thresholds(const LogJob &J) const {
    LogThr t{};
    for (int j = 0; j <= LOG_NU; ++j) t.bound[j] = (int64_t)0x7fffffffffffffffLL;
    t.full_range = cfg.key_group_start == 0 && cfg.key_group_end == cfg.max_parallelism - 1;
    const __int128 size = log_usize(), s0 = (__int128)J.base * size + (__int128)geom.unit_off_mod;
    const __int128 lo = (__int128)(int64_t)0x8000000000000000LL, hi = (__int128)(int64_t)0x7fffffffffffffffLL;
    if (s0 <= lo || s0 + (__int128)J.nunits * size > hi || s0 < (__int128)geom.offset - size) return t;
    for (int j = 0; j <= J.nunits; ++j) t.bound[j] = (int64_t)(s0 + (__int128)j * size);
    for (int j = 0; j < J.nunits; ++j) {
        const int64_t max_ts = (int64_t)(s0 + (__int128)(j + 1) * size - 1);
        const int64_t c_late = (int64_t)((uint64_t)max_ts + (uint64_t)log_lateness());
        const int64_t cleanup = c_late >= max_ts ? c_late : (int64_t)0x7fffffffffffffffLL;
        uint32_t c = cleanup <= J.g.wm ? 1u : (max_ts <= J.g.wm ? 2u : 0u);
        if (J.only_refire) c = c == 2u ? 0u : 1u;   // the late pass takes class-2 units inline, the rest out of line
        t.cls |= c << (2 * j);
    }
    t.only_refire = J.only_refire ? 1 : 0;
    t.ok = 1;
    return t;
}

// K1 of job J (one window range of a batch) into batch buffer J.slot; its last workgroup writes the readback
// block (bucket counts, statistics, device plan of pass 2); ev_rb[J.slot] marks the readback's completion.
// J.spec: each window's segment records are carved now with an upper bound and pass 2 is queued right
// behind K1 with an upper bound of workgroups; it runs the device plan unless K1's verdict says the batch
// needs the host (log_resolve_k1 then un-carves and re-plans), so no host round trip sits between them.
gwo_status Handle::log_k1(LogJob &J, bool first_pass) {
    LogState &L = *logst;
    const int W = needs_value ? 2 : 1;
    CollectArgs ca{};
    ca.nunits = J.nunits;
    ca.cap = J.cap;
    ca.bk = L.bk(J.slot);
    ca.go = L.d_go + J.slot;
    ca.rb = L.rb_dev(J.slot);
    ca.done = L.d_done;
    ca.shard = L.d_k1sh;
    ca.seq = J.seq = ++L.seq;
    ca.spec = J.spec ? 1 : 0;
    for (int w = 0; w < J.nunits; ++w) {
        auto it = L.wins.find(J.base + w);
        if (it == L.wins.end()) {
            LogWindow Wn;
            Wn.lp = log_choose_lp((uint64_t)J.n);
            it = L.wins.emplace(J.base + w, std::move(Wn)).first;
        }
        const int lp = it->second.lp;
        char *p = nullptr;
        LogSegDesc d{};
        GWO_TRY(log_carve(it->second, ((size_t)1 << lp) * 4, &p));
        d.off = (uint32_t *)p;
        GWO_TRY(log_carve(it->second, ((size_t)1 << lp) * 4, &p));
        d.cnt = (uint32_t *)p;
        d.lp = lp;
        if (J.spec) {
            J.seg_cap[w] = seg_upper_bound((uint64_t)J.n, lp);
            GWO_TRY(log_carve(it->second, J.seg_cap[w] * W * 8, &p));
            d.rec = (int64_t *)p;
            J.carve_at[w] = p;
            J.carve_end[w] = it->second.chunks.back().base + it->second.chunks.back().used;
            ca.seg_cap[w] = J.seg_cap[w];
        }
        J.desc[w] = d;
        ca.lp[w] = lp;
        ca.cnt[w] = d.cnt;
    }
    DevBuf &tmp = L.tmp[J.slot];
    if (tmp.bytes < (size_t)J.nunits * LOG_ND * LOG_XG * J.cap * W * 8) {
        GWO_TRY(log_resolve_split());   // ensure_buf may free: nothing may still read it
        // sized for LOG_NU windows, so a batch spanning more windows than the last one does not reallocate
        GWO_TRY(ensure_buf(tmp, (size_t)std::max(J.nunits, LOG_NU) * LOG_ND * LOG_XG * J.cap * W * 8));
    }
    const bool side = first_pass && side_enabled();
    LogThr thr = log_thresholds(J);
    thr.ts32 = J.ts32 ? 1 : 0;
    thr.tbase = J.tbase;
    // profiling: K1 times itself on the device wall clock (workgroup 0's start, the tail's end; read back with the
    // plan) -- no stream markers around it
    J.timed = profiling && ((prof_mask >> GWO_KERNEL_INSERT) & 1u) && L.clock_khz > 0;
    ca.t0 = J.timed ? L.d_t0 : nullptr;
    // sliding window steps run synchronously (no sweep in flight): after a discard the row counter is reset by this
    // K1's tail, ahead of the next step, instead of by a memset right before it
    if (slog && out_count_dirty && !fire_pending && !out_stale) {
        ca.reset_rows = d_out_count;
        out_count_dirty = false;
    }
    launch_log_part(J.k, J.t, J.v, J.n, J.stride, J.g, J.base, J.nunits, needs_value, L.d_cursor, J.cap,
                    (int64_t *)tmp.ptr, d_stats, (int64_t *)side_key.ptr, (int64_t *)side_ts.ptr,
                    (int64_t *)side_val.ptr, d_side_count, side ? side_cap : 0, side, ca, thr, J.rt, stream);
    GWO_TRY(launch_ok("log partition"));
    if (J.rt.mode == 1) {   // routed once: the exchange may start behind this K1; re-runs skip other GPUs' records
        GWO_TRY(comm_mark_routed());
        J.rt.mode = 2;
    }
    // The readback's own sequence word tells the host K1 is done; an event is recorded only behind the side-output
    // count copy (each event marker between K1 and pass 2 costs the stream ~5 us on MI355X, measured in the trace).
    L.rb_event[J.slot] = side;
    if (side) {
        GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_side_count, 8, hipMemcpyDeviceToHost, stream), "side count"));
        GWO_TRY(hipcheck(hipEventRecord(L.ev_rb[J.slot], stream), "event"));
    }
    if (J.spec) {
        LogSegSet set{};
        for (int w = 0; w < J.nunits; ++w) set.s[w] = J.desc[w];
        // chunks = sum over buckets of ceil(n_b / TILE) <= ceil(n / TILE) + buckets
        const uint64_t grid = ((uint64_t)J.n + LOG_TILE - 1) / LOG_TILE + (uint64_t)J.nunits * LOG_ND;
        L.h_split_flag[J.slot] = 0;
        hipStream_t ps = log_p2_begin(J.slot);
        prof_begin(GWO_KERNEL_PARTITION, ps);
        launch_log_split((const int64_t *)tmp.ptr, J.cap, needs_value, L.bk(J.slot), J.nunits * LOG_ND, set,
                         L.d_split_flag + J.slot, (uint32_t)grid, L.d_go + J.slot, ps);
        GWO_TRY(launch_ok("log split"));
        prof_end(GWO_KERNEL_PARTITION, J.n, ps);
        log_p2_end(J.slot);
    }
    return GWO_OK;
}

// Gives back the speculative segment carve of window w of job J (the device did not run the plan, or the
// window got no records), or trims it to `keep` records -- only while it is still the last carve of its
// chunk; otherwise the tail simply stays unused until the window is released.
void Handle::log_uncarve(const LogJob &J, int w, uint64_t keep) {
    auto it = logst->wins.find(J.base + w);
    if (it == logst->wins.end() || it->second.chunks.empty() || !J.carve_at[w]) return;
    LogChunk &c = it->second.chunks.back();
    if (c.base + c.used != J.carve_end[w]) return;
    const size_t bytes = keep ? ((keep * (needs_value ? 2 : 1) * 8 + 255) & ~(size_t)255) : 0;
    c.used = (size_t)(J.carve_at[w] - c.base) + bytes;
}

// Waits for K1's readback by spinning on its sequence word in pinned host memory (the collect kernel
// writes it last), which wakes the host as soon as the data lands instead of through the runtime's
// completion wait; the stream (or the slot's event, when one was recorded) is polled now and then so a failed
// launch cannot spin forever.
gwo_status Handle::log_wait_readback(int slot, unsigned long long seq) {
    LogState &L = *logst;
    volatile unsigned long long *w = L.rb(slot) + LOG_RB_SEQ;
    if (!L.rb_event[slot]) {   // the stream is queried only after a while (spin_seq: a query is a stream marker)
        GWO_TRY(spin_seq((const unsigned long long *)w, seq, "log partition"));
    } else {
        for (unsigned it = 1;; ++it) {
            if (*w == seq) break;
            if ((it & 1023) == 0) {
                hipError_t e = hipEventQuery(L.ev_rb[slot]);
                if (e != hipSuccess && e != hipErrorNotReady) return hipcheck(e, "log partition");
                if (e == hipSuccess && *w != seq)   // completed, yet the word never arrived: fail loudly
                    return poison(GWO_ERR_HIP, "log partition: readback sequence word not visible after completion");
            }
            __builtin_ia32_pause();
        }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    L.seen_seq = std::max(L.seen_seq, seq);
    return GWO_OK;
}

// Completes a batch whose first K1 is queued: waits for its readback, rejects the batch on a
// classification error (before any window state changes), re-runs K1 when the window range guess or a
// region capacity was wrong, and launches pass 2 (deferred) for each window range.
gwo_status Handle::log_resolve_k1(LogJob J) {
    const LogJob J0 = J;
    bool refire = false;
    GWO_TRY(log_resolve_batch(J, refire));
    if (!refire) return GWO_OK;
    if (slog) return slog_late_pass(J0);
    // allowedLateness > 0: records of fired, not yet cleaned windows re-fire them (EventTimeTrigger.onElement
    // FIRE, WindowOperator.java:393-406).  Those windows live in hash tables (log_migrate); a table pass over
    // the batch takes the re-fire records only -- the log took the accepted ones, K1 counted the late ones.
    WindowGeom g = J0.g;
    g.refire_ok = 1;
    g.refire_only = 1;
    const long long hint = hist_hint;   // the log's window-range guess, not the fired windows'
    const gwo_status s = insert_windowed(J0.k, J0.t, J0.v, J0.n, &g);
    hist_hint = hint;
    return s;
}

gwo_status Handle::log_resolve_batch(LogJob &J, bool &refire) {
    LogState &L = *logst;
    BatchStats &hs = *h_stats;
    bool first_pass = true;
    long long lo = 0, hi = -1;
    while (true) {
        GWO_TRY(log_wait_readback(J.slot, J.seq));
        if (J.timed) {   // the launch's own device timestamps
            const unsigned long long *rb = L.rb(J.slot);
            KStat &ks = kstats[GWO_KERNEL_INSERT];
            ks.launches++;
            ks.ms += (double)(rb[LOG_RB_T1] - rb[LOG_RB_T0]) / (double)L.clock_khz;
            ks.items += J.n;
            J.timed = false;
        }
        // the side-output row count follows the collect kernel by a copy: wait for that too
        if (first_pass && side_enabled() && !J.only_refire) GWO_TRY(spin_event(L.ev_rb[J.slot], "side count"));
        const unsigned long long *rbp = L.rb(J.slot);
        memcpy(h_stats, rbp + LOG_RB_STATS, sizeof(BatchStats));
        GWO_TRY(log_resolve_split());   // the previous pass 2 (also frees its plan staging for reuse)
        if (first_pass) {
            if (hs.bad_ts) return poison(GWO_ERR_NO_TIMESTAMP,
                                         "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time "
                                         "characteristic set to 'ProcessingTime', or did you forget to call "
                                         "'DataStream.assignTimestampsAndWatermarks(...)'?");
            if (hs.bad_range) return poison(GWO_ERR_UNSUPPORTED, "sliding windows: timestamp < offset - slide (Java '%' "
                                                                 "quirk range) is outside the pane restatement");
            if (hs.refire) {
                if (J.stride != 1 && !slog)
                    return poison(GWO_ERR_UNSUPPORTED, "allowedLateness > 0 re-fire on records received by the "
                                                       "multi-GPU exchange: use the table layout");
                refire = true;
            }
            if (hs.bad_kg) return poison(GWO_ERR_KEY_GROUP, ("Key group of key " + std::to_string(hs.bad_kg_key) +
                                                             " is not in KeyGroupRange{startKeyGroup=" +
                                                             std::to_string(cfg.key_group_start) + ", endKeyGroup=" +
                                                             std::to_string(cfg.key_group_end) + "}.").c_str());
            if (side_enabled() && !J.only_refire) {
                side_rows = *h_scalar;
                if ((long long)side_rows > side_cap) {
                    side_rows = side_rows_committed;
                    GWO_TRY(grow_side((long long)hs.late + (long long)side_rows_committed));
                    *h_scalar = side_rows;
                    GWO_TRY(hipcheck(hipMemcpyAsync(d_side_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "side reset"));
                    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side reset sync"));
                    GWO_TRY(log_k1(J, true));
                    continue;
                }
                side_rows_committed = side_rows;
            } else {
                late_dropped += hs.late;
            }
            // routed K1: a destination region that overflowed is re-routed now (the columns are still the caller's)
            if (J.rt.mode == 2 && comm)
                GWO_TRY(comm_check_route(J.k, J.t, J.v, J.n, rbp[LOG_RB_RMAX], rbp[LOG_RB_RWMAX]));
            if (hs.accepted == 0) {
                if (J.spec)
                    for (int w = 0; w < J.nunits; ++w) log_uncarve(J, w, 0);
                return GWO_OK;
            }
            lo = hs.min_idx;
            hi = hs.max_idx;
            first_pass = false;
            if (J.spec) {
                if (rbp[LOG_RB_GO] && J.base <= lo && lo < J.base + J.nunits) {
                    // the speculative pass 2 is running the device plan: commit its segments
                    GWO_TRY(log_commit_spec(J, rbp));
                    const long long chunk_hi = J.base + J.nunits - 1, nx = (long long)rbp[LOG_RB_NEXT];
                    if (chunk_hi >= hi || nx > hi) break;
                    J.spec = false;
                    J.base = std::max(chunk_hi + 1, nx);   // the next window holding records (not every empty one between)
                    J.nunits = (int)std::min<long long>(LOG_NU, hi - J.base + 1);
                    J.slot = L.free_slot();
                    GWO_TRY(log_k1(J, false));
                    continue;
                }
                // it exited: give its carves back and plan on the host from this readback
                for (int w = 0; w < J.nunits; ++w) log_uncarve(J, w, 0);
                J.spec = false;
            }
            if (J.base > lo || J.base + J.nunits <= lo) {   // wrong window range guess: redo from the first window
                J.base = lo;
                J.nunits = (int)std::min<long long>(LOG_NU, hi - lo + 1);
                GWO_TRY(log_k1(J, false));
                continue;
            }
        }
        const uint64_t maxc = rbp[LOG_RB_MAXREG];
        if (maxc > J.cap) {   // a region overflowed its capacity (skewed keys): redo this range exactly
            J.cap = maxc;
            GWO_TRY(log_k1(J, false));
            continue;
        }
        GWO_TRY(log_split_dev(J, rbp));
        const long long chunk_hi = J.base + J.nunits - 1, nx = (long long)rbp[LOG_RB_NEXT];
        if (chunk_hi >= hi || nx > hi) break;
        J.base = std::max(chunk_hi + 1, nx);   // the next window holding records (not every empty one between)
        J.nunits = (int)std::min<long long>(LOG_NU, hi - J.base + 1);
        J.slot = L.free_slot();
        GWO_TRY(log_k1(J, false));
    }
    hist_hint = lo;
    static const int span_margin = getenv("GWO_LOG_SPAN_MARGIN") ? atoi(getenv("GWO_LOG_SPAN_MARGIN")) : 1;
    L.span_hint = hi - lo + 1 + span_margin;
    return GWO_OK;
}

// Route-only K1 (rt.mode 3): every other GPU's record of the batch goes to the send regions again (exact
// capacities after an overflow); this GPU's records -- partitioned by the batch's first K1 -- are skipped, and the
// tail moves only the route counts (no plan, no readback: the first K1's are in use).
gwo_status Handle::log_route_only(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const LogRoute &rt) {
    LogState &L = *logst;
    if (n == 0) return GWO_OK;
    CollectArgs ca{};
    ca.done = L.d_done;
    ca.shard = L.d_k1sh;
    LogThr thr{};
    for (int j = 0; j <= LOG_NU; ++j) thr.bound[j] = (int64_t)0x7fffffffffffffffLL;
    thr.full_range = 1;
    const DevBuf &tmp = L.tmp[0];
    launch_log_part(k, t, v, n, 1, log_geom_now(), 0, 1, needs_value, L.d_cursor, 0, (int64_t *)tmp.ptr, d_stats,
                    nullptr, nullptr, nullptr, d_side_count, 0, 0, ca, thr, rt, stream);
    return launch_ok("route-only partition");
}

// Resolves the pipelined batch, if any (every call that observes state or fires windows comes here first).
gwo_status Handle::log_flush() {
    if (logst && logst->job.active) {
        LogJob J = logst->job;
        logst->job.active = false;
        GWO_TRY(log_resolve_k1(J));
    }
    return comm_flush_received();   // records received by the multi-GPU exchange and not yet inserted
}

gwo_status Handle::insert_log(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, int64_t stride,
                              const LogRoute *route, bool ts32, int64_t tbase, const WindowGeom *geom_at) {
    LogState &L = *logst;
    LogJob J;
    if (route) J.rt = *route;
    J.ts32 = ts32;
    J.tbase = tbase;
    J.k = k;
    J.t = t;
    J.v = v;
    J.n = n;
    J.stride = stride;
    J.g = geom_at ? *geom_at : log_geom_now();
    if (slog) GWO_TRY(slog_reserve(n));
    J.base = hist_hint;
    J.nunits = (int)std::min<long long>(LOG_NU, std::max<long long>(1, L.span_hint));
    J.cap = group_capacity((double)n / ((double)LOG_ND * LOG_XG));
    // speculative pass 2 (no host round trip between K1 and pass 2) unless late records go to the side output
    // (K1's first pass appends them; a re-run must not repeat that)
    J.spec = !side_enabled();
    // Pipelined: this batch's K1 is queued before the previous batch is resolved, so the host's wait,
    // checks and pass-2 planning overlap a running K1.  Only for caller-owned device columns (borrowed
    // until the next call returns, gwo.h) -- staged host input and received exchange buffers are reused
    // by the next batch -- and without a side output (K1 appends to it on the first pass).
    // With allowedLateness > 0 a batch resolves before the next watermark: its re-fire records must reach the
    // fired windows' tables before a watermark cleans them up.
    const bool pipe = L.pipeline && !slog && cfg.allowed_lateness == 0 && stride == 1 && !side_enabled() && !comm && !dict &&
                      (const void *)k != stage_key.ptr &&
                      (const void *)t != stage_ts.ptr && (!v || (const void *)v != stage_val.ptr);
    if (L.job.active && !pipe) GWO_TRY(log_flush());
    J.slot = L.free_slot();
    GWO_TRY(log_k1(J, true));
    // multi-GPU: the exchange of the routed records is queued now, so it overlaps this batch's own records' work
    if (route) GWO_TRY(comm_after_route(k, t, v, n));
    if (!pipe) return log_resolve_k1(J);
    LogJob prev = L.job;
    L.job = J;
    L.job.active = true;
    if (!prev.active) return GWO_OK;
    gwo_status s = log_resolve_k1(prev);
    // a window range guess taken before the previous batch resolved is refreshed for the next launch
    return s;
}

// A pipelined batch may hold records of a window this watermark fires: any accepted record has
// end - 1 > (watermark at its K1), so that needs a window end in (that watermark, new_wm].
bool Handle::log_pending_may_fire(int64_t new_wm) const {
    const LogState &L = *logst;
    int64_t rwm;
    if (comm_pending_wm(&rwm) && log_may_fire_since(rwm, new_wm)) return true;   // deferred received records
    if (!L.job.active) return false;
    return log_may_fire_since(L.job.g.wm, new_wm);
}

bool Handle::log_may_fire_since(int64_t batch_wm, int64_t new_wm) const {
    const __int128 w0 = (__int128)batch_wm + 1;
    const __int128 size = cfg.size, off = geom.unit_off_mod;
    __int128 q = (w0 - off) / size;
    if ((w0 - off) % size < 0) q -= 1;                  // floor division
    const __int128 end_m1 = q * size + off + size - 1;  // max timestamp of the window holding w0
    return end_m1 <= (__int128)new_wm;
}

// Launches the fold of every window whose end the watermark passed (EventTimeTrigger.onEventTime FIRE,
// WindowOperator.java:430-473) on fire_stream, one workgroup per CU so that the next batches' kernels
// run beside it, and returns.  finish_fire publishes the rows and releases the windows' memory.
gwo_status Handle::fire_log(int64_t new_wm) {
    LogState &L = *logst;
    GWO_TRY(poll_fire());
    auto due = [&](std::vector<long long> &out) {   // windows this watermark fires, not already firing
        out.clear();
        for (auto &kv : L.wins) {
            if ((int64_t)((uint64_t)unit_start(kv.first) + (uint64_t)cfg.size - 1) > new_wm) continue;
            if (fire_pending &&
                std::find(L.fire_units.begin(), L.fire_units.end(), kv.first) != L.fire_units.end())
                continue;
            out.push_back(kv.first);
        }
    };
    if (log_pending_may_fire(new_wm)) GWO_TRY(log_flush());
    std::vector<long long> fire;
    due(fire);
    if (cfg.allowed_lateness == 0 && (!tables.empty() || !rdone.empty()))
        GWO_TRY(fire_tumbling(new_wm));   // restored fired windows
    if (cfg.allowed_lateness > 0) {
        // a fired window stays until its cleanup time and takes late records: it moves to a hash table,
        // which the table path fires, re-fires and cleans up (fire_tumbling, refire_rows)
        if (!fire.empty()) {
            GWO_TRY(finish_fire());
            GWO_TRY(log_resolve_split());
            due(fire);
            for (long long u : fire) GWO_TRY(log_migrate(u));
        }
        return fire_tumbling(new_wm);
    }
    if (fire.empty()) return GWO_OK;
    GWO_TRY(finish_fire());         // the previous fire's rows and memory first
    GWO_TRY(log_resolve_split());   // the fired windows' last segments must be complete
    due(fire);
    for (auto it = fire.begin(); it != fire.end();) {   // a window with no segment has nothing to emit
        if (L.wins[*it].segs.empty() && !L.wins[*it].partial.rec) {
            log_release(L.wins[*it]);   // offsets/counters carved for a K1 range that got no records
            L.wins.erase(*it);
            it = fire.erase(it);
        } else {
            ++it;
        }
    }
    if (fire.empty()) return GWO_OK;
    for (long long u : fire)
        if (L.wins[u].segs.size() > LOG_MAX_SEGS)
            return poison(GWO_ERR_CAPACITY, "log layout: a window collected more than 512 batches; use the table layout "
                                            "for windows that span that many watermark intervals");
    // Output rows: one per distinct key.  Reserve for the expected count (last window's keys, or the
    // caller's hint) rather than the record count; if the fire emits more, finish_fire re-runs it into
    // a bigger buffer (the fire only reads the segments, so a re-run is exact).
    uint64_t bound = 0, expect = 0;
    const uint64_t per_window = std::max<uint64_t>(L.last_window_keys, (uint64_t)std::max<int64_t>(cfg.expected_keys, 0));
    for (long long u : fire) {
        const uint64_t r = L.wins[u].records + L.wins[u].partial_rows;
        bound += r;
        expect += std::min<uint64_t>(r, per_window + per_window / 8 + 4096);
    }
    GWO_TRY(ensure_output(expect));
    size_t ndesc = 0;
    for (long long u : fire) ndesc += L.wins[u].segs.size();
    L.h_fire.clear();
    for (long long u : fire)
        for (auto &d : L.wins[u].segs) L.h_fire.push_back(d);
    GWO_TRY(ensure_buf(L.firedesc, ndesc * sizeof(LogSegDesc)));
    GWO_TRY(hipcheck(hipMemcpyAsync(L.firedesc.ptr, L.h_fire.data(), ndesc * sizeof(LogSegDesc), hipMemcpyHostToDevice,
                                    stream), "fire desc"));
    if (L.max_groups == 0) {
        int cus = 0;
        GWO_TRY(hipcheck(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg.device), "CU count"));
        L.max_groups = std::max(cus, 1);
    }
    L.fire_rows0 = out_rows;
    L.fire_bound = bound;
    L.fire_units = fire;
    // synchronous fire: on the handle's stream (no cross-stream event); asynchronous: on fire_stream
    hipStream_t fs = async_fire ? fire_stream : stream;
    if (async_fire) {
        GWO_TRY(hipcheck(hipEventRecord(ev_main, stream), "event"));   // segments, descriptors, row counter
        GWO_TRY(hipcheck(hipStreamWaitEvent(fire_stream, ev_main, 0), "event wait"));
    }
    OutCols o = out_cols();
    size_t at = 0;
    for (long long u : fire) {
        LogWindow &W = L.wins[u];
        int64_t start = unit_start(u);
        int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
        prof_begin(GWO_KERNEL_FIRE, fs);
        launch_log_fire((const LogSegDesc *)L.firedesc.ptr + at, (int)W.segs.size(), W.lp, needs_value, plan, rplan,
                        start, end, o, L.d_overflow, L.max_groups, async_fire ? 1 : 2, W.partial.rec ? 1 : 0, W.partial,
                        L.d_slow, L.d_slow + LOG_SLOW_CAP, fs);
        GWO_TRY(launch_ok("log fire"));
        prof_end(GWO_KERNEL_FIRE, (int64_t)W.records, fs);
        at += W.segs.size();
    }
    GWO_TRY(hipcheck(hipMemcpyAsync(L.h_fire_out, d_out_count, 8, hipMemcpyDeviceToHost, fs), "out count"));
    GWO_TRY(hipcheck(hipMemcpyAsync(L.h_fire_out + 1, L.d_overflow, 16, hipMemcpyDeviceToHost, fs), "overflow"));
    GWO_TRY(hipcheck(hipEventRecord(ev_fire, fs), "event"));
    fire_pending = true;
    // Measured on MI355X (C4): letting the fire overlap the next batches is slower -- beside a 1-per-CU
    // fire the partition kernel loses its occupancy (0.36 vs 0.26 ms) and the fire takes 4.9 vs 2.9 ms;
    // at 2 per CU the next batch simply queues behind it.  So the fire completes here; the stream and
    // event machinery stays for callers that interleave other work (GWO_ASYNC_FIRE=1).
    if (!async_fire) return finish_fire();
    return GWO_OK;
}

gwo_status Handle::finish_fire() {
    GWO_TRY(settle_out());
    if (!fire_pending) return GWO_OK;
    if (sess) return session_finish_fire();
    LogState &L = *logst;
    fire_pending = false;
    GWO_TRY(spin_event(ev_fire, "fire"));
    if (L.h_fire_out[1]) return poison(GWO_ERR_CAPACITY, "log fire: a partition overflowed its LDS table");
    uint64_t count = L.h_fire_out[0];
    if ((long long)count > out.cap) {
        // more rows than reserved: rewind the row counter, grow to the exact need, fire again (synchronous)
        const uint64_t need = count - L.fire_rows0;
        *h_scalar = L.fire_rows0;
        GWO_TRY(hipcheck(hipMemcpyAsync(d_out_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "out rewind"));
        GWO_TRY(ensure_output(std::min(need, L.fire_bound)));
        OutCols o = out_cols();
        size_t at = 0;
        for (long long u : L.fire_units) {
            LogWindow &W = L.wins[u];
            int64_t start = unit_start(u);
            int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
            launch_log_fire((const LogSegDesc *)L.firedesc.ptr + at, (int)W.segs.size(), W.lp, needs_value, plan,
                            rplan, start, end, o, L.d_overflow, L.max_groups, 2, W.partial.rec ? 1 : 0, W.partial,
                            L.d_slow, L.d_slow + LOG_SLOW_CAP, stream);
            GWO_TRY(launch_ok("log fire"));
            at += W.segs.size();
        }
        GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_out_count, 8, hipMemcpyDeviceToHost, stream), "out count"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "log fire"));
        count = *h_scalar;
    }
    const uint64_t emitted = count - L.fire_rows0;
    if (debug)
        fprintf(stderr, "[gwo] fire %zu window(s): rows=%llu slow_partitions=%llu lp=%d records=%llu\n",
                L.fire_units.size(), (unsigned long long)emitted, (unsigned long long)L.h_fire_out[2],
                L.wins[L.fire_units[0]].lp, (unsigned long long)L.wins[L.fire_units[0]].records);
    if (discard_after_fire) {   // gwo_discard_output was called while the fire ran
        discard_after_fire = false;
        rows_gone += emitted;
        out_rows = 0;
        out_count_dirty = true;
    } else {
        out_rows = count;
    }
    L.last_window_keys = emitted / L.fire_units.size();
    L.last_window_records = 0;
    for (long long u : L.fire_units) L.last_window_records = std::max<uint64_t>(L.last_window_records, L.wins[u].records);
    for (long long u : L.fire_units) {
        log_release(L.wins[u]);   // allowedLateness 0: the window's cleanup time is its fire
        L.wins.erase(u);
    }
    L.fire_units.clear();
    return GWO_OK;
}

gwo_status Handle::set_pipelined(bool on) {
    if (!on) GWO_TRY(flush_pending());
    pipe_submit = on;             // the combine path (tumbling tables; combine_pipe_ok) and sessions
    if (!logst) return GWO_OK;    // other layouts resolve every batch inside gwo_submit
    if (!on) GWO_TRY(log_flush());
    logst->pipeline = on;
    return GWO_OK;
}

gwo_status Handle::log_state_size(int64_t *entries) {
    GWO_TRY(log_flush());
    uint64_t s = 0;
    for (auto &kv : logst->wins) s += kv.second.records + kv.second.partial_rows;
    if (!tables.empty() || !rdone.empty()) {   // fired windows kept for allowedLateness
        GWO_TRY(read_occupancy());
        for (auto &kv : tables) s += kv.second.occ;
        for (auto &kv : rdone) s += kv.second.occ;
    }
    *entries = (int64_t)s;
    return GWO_OK;
}

}  // namespace gwo

// ---- checkpoint / restore of the log layout (gwo_snapshot.cpp orchestrates) ---------------------------------
namespace gwo {

size_t Handle::log_window_count() const { return logst->wins.size(); }

// Folds windows without releasing them -- the fire kernel, LDS hash-table path only, with a result plan that
// emits the raw accumulator words -- into rows (key, window, words) of `c`.
gwo_status Handle::log_fold_raw(const std::vector<long long> &units, const SnapCols &c) {
    LogState &L = *logst;
    ResultPlan raw{};
    raw.naggs = plan.nwords;
    for (int w = 0; w < plan.nwords; ++w) {
        raw.kind[w] = GWO_AGG_COUNT;   // a COUNT result is its accumulator word as it is
        raw.word[w] = w;
    }
    OutCols o{};
    o.key = c.key;
    o.start = c.start;
    o.end = c.end;
    for (int w = 0; w < plan.nwords; ++w) o.res[w] = c.w[w];
    o.count = c.count;
    o.cap = c.cap;
    if (L.max_groups == 0) {
        int cus = 0;
        GWO_TRY(hipcheck(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg.device), "CU count"));
        L.max_groups = std::max(cus, 1);
    }
    L.h_fire.clear();
    for (long long u : units)
        for (auto &d : L.wins[u].segs) L.h_fire.push_back(d);
    if (!L.h_fire.empty()) {
        GWO_TRY(ensure_buf(L.firedesc, L.h_fire.size() * sizeof(LogSegDesc)));
        GWO_TRY(hipcheck(hipMemcpyAsync(L.firedesc.ptr, L.h_fire.data(), L.h_fire.size() * sizeof(LogSegDesc),
                                        hipMemcpyHostToDevice, stream), "fold desc"));
    }
    GWO_TRY(hipcheck(hipMemsetAsync(L.d_overflow, 0, 16, stream), "overflow"));
    size_t at = 0;
    for (long long u : units) {
        LogWindow &W = L.wins[u];
        const int64_t start = unit_start(u);
        const int64_t end = (int64_t)((uint64_t)start + (uint64_t)log_usize());   // sliding: the pane
        launch_log_fire((const LogSegDesc *)L.firedesc.ptr + at, (int)W.segs.size(), W.lp, needs_value, plan, raw, start,
                        end, o, L.d_overflow, L.max_groups, 2, 1, W.partial, L.d_slow, L.d_slow + LOG_SLOW_CAP, stream);
        GWO_TRY(launch_ok("log fold"));
        at += W.segs.size();
    }
    GWO_TRY(hipcheck(hipMemcpyAsync(L.h_fire_out + 1, L.d_overflow, 16, hipMemcpyDeviceToHost, stream), "overflow"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "log fold"));
    if (L.h_fire_out[1]) return poison(GWO_ERR_CAPACITY, "log fold: a partition overflowed its LDS table");
    return GWO_OK;
}

// Checkpoint rows of every collecting window (fire timers pending: a log window leaves the log at its fire).
gwo_status Handle::log_snapshot_collect(const SnapCols &c) {
    std::vector<long long> units;
    for (auto &kv : logst->wins) units.push_back(kv.first);
    return log_fold_raw(units, c);
}

// allowedLateness > 0: window u, due to fire, leaves the log for a hash table (its state, one entry per key),
// where the table path emits it, re-fires it for late records and clears it at its cleanup time.
gwo_status Handle::log_migrate(long long u) {
    LogState &L = *logst;
    LogWindow &W = L.wins[u];
    const uint64_t bound = W.records + W.partial_rows;
    if (bound > 0 && (!W.segs.empty() || W.partial.rec)) {
        const int NW = plan.nwords;
        DevBuf b[3 + GWO_MAX_WORDS];
        for (int i = 0; i < 3 + NW; ++i) GWO_TRY(ensure_buf(b[i], (size_t)bound * 8));
        SnapCols c{};
        c.key = (int64_t *)b[0].ptr;
        c.start = (int64_t *)b[1].ptr;
        c.end = (int64_t *)b[2].ptr;
        for (int w = 0; w < NW; ++w) c.w[w] = (int64_t *)b[3 + w].ptr;
        c.count = d_scratch_count;
        c.cap = (long long)bound;
        GWO_TRY(hipcheck(hipMemsetAsync(d_scratch_count, 0, 8, stream), "migrate count"));
        GWO_TRY(log_fold_raw({u}, c));
        GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_scratch_count, 8, hipMemcpyDeviceToHost, stream), "migrate count"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "migrate count"));
        const int64_t n = (int64_t)*h_scalar;
        if (n > (int64_t)bound) return poison(GWO_ERR_HIP, "log migrate: more keys than records");
        if (n > 0) {
            GWO_TRY(ensure_table(u, (uint64_t)n));
            launch_table_load(c, n, desc(tables[u]), plan, stream);
            GWO_TRY(launch_ok("log migrate"));
            tables[u].dirty = true;
        }
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "log migrate"));
        for (auto &x : b) x.release();
    }
    log_release(L.wins[u]);
    L.wins.erase(u);
    return read_occupancy();
}

// Restored rows of a window become that window's partial-accumulator segment: records of (key, raw words)
// grouped by partition (top lp bits of digit_hash, as every later batch's segments), folded into the window's
// rows at its fire.
// Rows of windows that already fired (timer flag 0: kept for allowedLateness) go to hash tables, as
// log_migrate leaves them.
gwo_status Handle::log_restore_rows(const RestoreRows &R, int64_t new_wm) {
    LogState &L = *logst;
    std::map<long long, std::vector<int64_t>> rows_of;
    std::map<long long, int> kinds;   // bit 0: rows with a pending fire timer, bit 1: rows already emitted
    std::vector<int64_t> fired;
    for (int64_t i = 0; i < R.n; ++i) {
        if (!R.mine[i]) continue;
        const __int128 a = (__int128)R.start[i] - (__int128)geom.unit_off_mod;
        __int128 q = a / geom.unit;
        if (a % geom.unit != 0 && a < 0) q -= 1;
        const long long u = (long long)q;
        if (unit_start(u) != R.start[i])
            return fail(GWO_ERR_INVALID_ARGUMENT, "restore: %lld is not a window start", (long long)R.start[i]);
        if (!R.timer.empty() && R.timer[i] == 0) {
            fired.push_back(i);
            kinds[u] |= 2;
        } else {
            rows_of[u].push_back(i);
            kinds[u] |= 1;
        }
    }
    for (auto &kv : kinds)   // emitted rows beside pending ones: only above the watermark (table_restore_rows: rdone)
        if (kv.second == 3 && (int64_t)((uint64_t)unit_start(kv.first) + (uint64_t)cfg.size - 1) <= new_wm)
            return fail(GWO_ERR_UNSUPPORTED, "restore: window %lld has rows already emitted and rows still pending "
                                             "at a watermark past its end", (long long)unit_start(kv.first));
    if (!fired.empty()) {
        RestoreRows T;
        T.n = (int64_t)fired.size();
        T.nw = R.nw;
        for (int64_t i : fired) {
            T.key.push_back(R.key[i]);
            T.start.push_back(R.start[i]);
            T.end.push_back(R.end[i]);
            T.timer.push_back(0);
            T.words.insert(T.words.end(), R.words.begin() + (size_t)i * R.nw, R.words.begin() + (size_t)(i + 1) * R.nw);
        }
        T.mine.assign(T.n, 1);
        GWO_TRY(table_restore_rows(T, new_wm));
    }
    wm = in_wm = new_wm;
    const int RW = 1 + plan.nwords;
    for (auto &kv : rows_of) {
        const std::vector<int64_t> &ix = kv.second;
        LogWindow &W = L.wins[kv.first];
        W.lp = log_choose_lp((uint64_t)ix.size());
        const uint32_t F = 1u << W.lp;
        std::vector<uint32_t> cnt(F, 0), off(F, 0);
        for (int64_t i : ix) cnt[digit_hash(R.key[i]) >> (32 - W.lp)]++;
        uint32_t run = 0;
        for (uint32_t p = 0; p < F; ++p) {
            off[p] = run;
            run += cnt[p];
        }
        std::vector<uint32_t> fill(off);
        std::vector<int64_t> rec((size_t)ix.size() * RW);
        for (int64_t i : ix) {
            const uint32_t p = digit_hash(R.key[i]) >> (32 - W.lp);
            int64_t *r = rec.data() + (size_t)fill[p]++ * RW;
            r[0] = R.key[i];
            for (int w = 0; w < plan.nwords; ++w) r[1 + w] = R.words[(size_t)i * R.nw + w];
        }
        char *p_rec = nullptr, *p_off = nullptr, *p_cnt = nullptr;
        GWO_TRY(log_carve(W, rec.size() * 8, &p_rec));
        GWO_TRY(log_carve(W, (size_t)F * 4, &p_off));
        GWO_TRY(log_carve(W, (size_t)F * 4, &p_cnt));
        GWO_TRY(hipcheck(hipMemcpy(p_rec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice), "restore records"));
        GWO_TRY(hipcheck(hipMemcpy(p_off, off.data(), (size_t)F * 4, hipMemcpyHostToDevice), "restore offsets"));
        GWO_TRY(hipcheck(hipMemcpy(p_cnt, cnt.data(), (size_t)F * 4, hipMemcpyHostToDevice), "restore counts"));
        W.partial = LogSegDesc{(int64_t *)p_rec, (uint32_t *)p_off, (uint32_t *)p_cnt, W.lp, (uint32_t)ix.size()};
        W.partial_rows = ix.size();
    }
    return slog ? slog_anchor() : GWO_OK;
}

}  // namespace gwo
