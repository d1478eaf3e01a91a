// gwo_log.cpp -- host side of the log-structured tumbling-window state (kernels: gwo_log.hip).
//
// Bookkeeping only: which windows are open, the device memory of their segments, the partition
// count of each window, and the per-batch scan/scatter/fire launch sequence.  The reference's
// equivalents are the window-contents state table and the timer queue of WindowOperator
// (WindowOperator.java:218-273 open(), :430-473 onEventTime, InternalTimerServiceImpl.java:268-278).
#include <algorithm>
#include <cstring>
#include <map>
#include <vector>

#include "gwo_handle.h"
#include "gwo_log.h"

namespace gwo {

struct LogChunk {
    char *base = nullptr;
    size_t size = 0;
    size_t used = 0;
};

struct LogWindow {
    int lp = 0;
    std::vector<LogSegDesc> segs;
    std::vector<LogChunk> chunks;
    uint64_t records = 0;
};

struct LogState {
    std::map<long long, LogWindow> wins;
    std::multimap<size_t, char *> free_chunks;
    DevBuf tkey, tval, cbase, segdesc, firedesc;
    unsigned *d_chist = nullptr;
    unsigned *h_chist = nullptr;                 // pinned [LOG_UNITS * 256]
    unsigned long long *h_cbase = nullptr;       // pinned [LOG_UNITS * 256 + 1]
    LogSegDesc *h_desc = nullptr;                // pinned [LOG_UNITS]
    std::vector<LogSegDesc> h_fire;
    unsigned long long *d_overflow = nullptr;
    uint64_t last_window_records = 0;
    int cap_log2 = 0;
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

gwo_status Handle::log_init() {
    logst = new LogState();
    LogState &L = *logst;
    GWO_TRY(dalloc((void **)&L.d_chist, LOG_UNITS * 256 * sizeof(unsigned)));
    GWO_TRY(dalloc((void **)&L.d_overflow, 8));
    GWO_TRY(hipcheck(hipMemsetAsync(L.d_overflow, 0, 8, stream), "overflow"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&L.h_chist, LOG_UNITS * 256 * sizeof(unsigned), hipHostMallocDefault), "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&L.h_cbase, (LOG_UNITS * 256 + 1) * 8, hipHostMallocDefault), "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&L.h_desc, LOG_UNITS * sizeof(LogSegDesc), hipHostMallocDefault), "pinned"));
    GWO_TRY(ensure_buf(L.cbase, (LOG_UNITS * 256 + 1) * 8 * 2));
    GWO_TRY(ensure_buf(L.segdesc, LOG_UNITS * sizeof(LogSegDesc)));
    L.cap_log2 = log_fire_cap_log2(plan.nwords);
    return GWO_OK;
}

void Handle::log_free() {
    if (!logst) return;
    LogState &L = *logst;
    for (auto &kv : L.wins)
        for (auto &c : kv.second.chunks) (void)hipFree(c.base);
    for (auto &kv : L.free_chunks) (void)hipFree(kv.second);
    L.tkey.release();
    L.tval.release();
    L.cbase.release();
    L.segdesc.release();
    L.firedesc.release();
    if (L.d_chist) (void)hipFree(L.d_chist);
    if (L.d_overflow) (void)hipFree(L.d_overflow);
    if (L.h_chist) (void)hipHostFree(L.h_chist);
    if (L.h_cbase) (void)hipHostFree(L.h_cbase);
    if (L.h_desc) (void)hipHostFree(L.h_desc);
    delete logst;
    logst = nullptr;
}

// Carves `bytes` (256-B aligned) out of the window's chunks; new chunks come from the pool.
gwo_status Handle::log_carve(LogWindow &W, size_t bytes, char **out) {
    bytes = align256(bytes);
    if (W.chunks.empty() || W.chunks.back().size - W.chunks.back().used < bytes) {
        size_t want = 1 << 20;
        while (want < bytes * 4 && want < ((size_t)512 << 20)) want <<= 1;
        want = std::max(want, bytes);
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
}

// Partitions of a new window: about 5/8 of the fire kernel's LDS table per partition, sized from
// the previous window's record count, the caller's key hint and what this batch already brings.
int Handle::log_choose_lp(uint64_t batch_records) const {
    const LogState &L = *logst;
    uint64_t est = std::max<uint64_t>(L.last_window_records, (uint64_t)std::max<int64_t>(cfg.expected_keys, 0) * 2);
    est = std::max<uint64_t>(est, batch_records * 8);
    uint64_t per = ((uint64_t)1 << L.cap_log2) * 5 / 8;
    int lp = 0;
    while (lp < LOG_MAX_LP && ((uint64_t)1 << lp) * per < est) lp++;
    return lp;
}

gwo_status Handle::insert_log(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n) {
    LogState &L = *logst;
    WindowGeom g = geom_now();
    BatchStats &hs = *h_stats;
    long long base = hist_hint;
    bool first_pass = true;
    long long lo = 0, hi = -1;
    const int64_t *val = needs_value ? v : nullptr;
    while (true) {
        init_stats(base);
        GWO_TRY(hipcheck(hipMemsetAsync(L.d_chist, 0, LOG_UNITS * 256 * sizeof(unsigned), stream), "chist"));
        prof_begin(GWO_KERNEL_SCAN);
        launch_log_scan(k, t, v, n, g, base, d_stats, L.d_chist, (int64_t *)side_key.ptr, (int64_t *)side_ts.ptr,
                        (int64_t *)side_val.ptr, d_side_count, first_pass && side_enabled() ? side_cap : 0,
                        first_pass && side_enabled(), stream);
        GWO_TRY(launch_ok("log scan"));
        prof_end(GWO_KERNEL_SCAN, n);
        GWO_TRY(hipcheck(hipMemcpyAsync(h_stats, d_stats, sizeof(BatchStats), hipMemcpyDeviceToHost, stream), "stats"));
        GWO_TRY(hipcheck(hipMemcpyAsync(L.h_chist, L.d_chist, LOG_UNITS * 256 * sizeof(unsigned), hipMemcpyDeviceToHost,
                                        stream), "chist"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "log scan sync"));
        if (first_pass) {
            if (hs.bad_ts) return poison(GWO_ERR_NO_TIMESTAMP,
                                         "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time "
                                         "characteristic set to 'ProcessingTime', or did you forget to call "
                                         "'DataStream.assignTimestampsAndWatermarks(...)'?");
            if (hs.refire) return poison(GWO_ERR_UNSUPPORTED,
                                         "allowedLateness > 0: a record re-fires an already emitted window "
                                         "(EventTimeTrigger.onElement FIRE) -- not supported by the GPU operator");
            if (hs.bad_kg) return poison(GWO_ERR_KEY_GROUP, ("Key group of key " + std::to_string(hs.bad_kg_key) +
                                                             " is not in KeyGroupRange{startKeyGroup=" +
                                                             std::to_string(cfg.key_group_start) + ", endKeyGroup=" +
                                                             std::to_string(cfg.key_group_end) + "}.").c_str());
            if (side_enabled()) {
                GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_side_count, 8, hipMemcpyDeviceToHost, stream), "side count"));
                GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side count sync"));
                side_rows = *h_scalar;
                if ((long long)side_rows > side_cap) {
                    side_rows = side_rows_committed;
                    GWO_TRY(grow_side((long long)hs.late + (long long)side_rows_committed));
                    *h_scalar = side_rows;
                    GWO_TRY(hipcheck(hipMemcpyAsync(d_side_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "side reset"));
                    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side reset sync"));
                    continue;
                }
                side_rows_committed = side_rows;
            } else {
                late_dropped += hs.late;
            }
            if (hs.accepted == 0) return GWO_OK;
            lo = hs.min_idx;
            hi = hs.max_idx;
            first_pass = false;
            if (base > lo || base + LOG_UNITS <= lo) {
                base = lo;
                continue;
            }
        }
        const long long chunk_hi = std::min<long long>(hi, base + LOG_UNITS - 1);
        const int nunits = (int)(chunk_hi - base + 1);
        const int nb = nunits * 256;
        // coarse bucket bases (exclusive scan) and per-window record counts
        uint64_t run = 0;
        std::vector<uint64_t> wcount(nunits, 0);
        for (int b = 0; b < nb; ++b) {
            L.h_cbase[b] = run;
            run += L.h_chist[b];
            wcount[b >> 8] += L.h_chist[b];
        }
        L.h_cbase[nb] = run;
        const uint64_t total = run;
        if (total > 0) {
            GWO_TRY(ensure_buf(L.tkey, total * 8));
            if (val) GWO_TRY(ensure_buf(L.tval, total * 8));
            // cursors (consumed by pass 1) and a pristine copy of the bases (read by pass 2)
            unsigned long long *d_cursor = (unsigned long long *)L.cbase.ptr;
            unsigned long long *d_cb = d_cursor + (LOG_UNITS * 256 + 1);
            GWO_TRY(hipcheck(hipMemcpyAsync(d_cursor, L.h_cbase, (nb + 1) * 8, hipMemcpyHostToDevice, stream), "cursor"));
            GWO_TRY(hipcheck(hipMemcpyAsync(d_cb, L.h_cbase, (nb + 1) * 8, hipMemcpyHostToDevice, stream), "cbase"));
            for (int w = 0; w < nunits; ++w) {
                LogSegDesc d{};
                if (wcount[w]) {
                    long long u = base + w;
                    auto it = L.wins.find(u);
                    if (it == L.wins.end()) {
                        LogWindow W;
                        W.lp = log_choose_lp(wcount[w]);
                        it = L.wins.emplace(u, std::move(W)).first;
                    }
                    LogWindow &W = it->second;
                    d.lp = W.lp;
                    char *p = nullptr;
                    GWO_TRY(log_carve(W, wcount[w] * 8, &p));
                    d.key = (int64_t *)p;
                    if (val) {
                        GWO_TRY(log_carve(W, wcount[w] * 8, &p));
                        d.val = (int64_t *)p;
                    }
                    GWO_TRY(log_carve(W, (((size_t)1 << W.lp) + 1) * 4, &p));
                    d.off = (uint32_t *)p;
                    W.segs.push_back(d);
                    W.records += wcount[w];
                }
                L.h_desc[w] = d;
            }
            GWO_TRY(hipcheck(hipMemcpyAsync(L.segdesc.ptr, L.h_desc, nunits * sizeof(LogSegDesc), hipMemcpyHostToDevice,
                                            stream), "segdesc"));
            prof_begin(GWO_KERNEL_INSERT);
            launch_log_pass1(k, t, val, n, g, base, nunits, d_cursor, (int64_t *)L.tkey.ptr,
                             val ? (int64_t *)L.tval.ptr : nullptr, stream);
            GWO_TRY(launch_ok("log pass1"));
            prof_end(GWO_KERNEL_INSERT, n);
            prof_begin(GWO_KERNEL_PARTITION);
            launch_log_pass2((const int64_t *)L.tkey.ptr, val ? (const int64_t *)L.tval.ptr : nullptr, d_cb, nunits,
                             (const LogSegDesc *)L.segdesc.ptr, stream);
            GWO_TRY(launch_ok("log pass2"));
            prof_end(GWO_KERNEL_PARTITION, (int64_t)total);
            // the pinned staging above is reused by the next chunk/batch
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "log insert"));
        }
        if (chunk_hi >= hi) break;
        base = chunk_hi + 1;
    }
    hist_hint = lo;
    return GWO_OK;
}

gwo_status Handle::fire_log(int64_t new_wm) {
    LogState &L = *logst;
    std::vector<long long> fire;
    for (auto &kv : L.wins) {
        if (kv.second.segs.size() > LOG_MAX_SEGS)
            return poison(GWO_ERR_CAPACITY, "log layout: a window collected more than 512 batches; use the table layout "
                                            "for windows that span that many watermark intervals");
        int64_t start = unit_start(kv.first);
        int64_t max_ts = (int64_t)((uint64_t)start + (uint64_t)cfg.size - 1);
        if (max_ts <= new_wm) fire.push_back(kv.first);   // EventTimeTrigger.onEventTime FIRE
    }
    if (fire.empty()) return GWO_OK;
    uint64_t bound = 0;
    for (long long u : fire) bound += L.wins[u].records;
    GWO_TRY(ensure_output(bound));
    OutCols o = out_cols();
    // one descriptor array per fired window, uploaded together
    size_t ndesc = 0;
    for (long long u : fire) ndesc += L.wins[u].segs.size();
    L.h_fire.clear();
    for (long long u : fire)
        for (auto &d : L.wins[u].segs) L.h_fire.push_back(d);
    GWO_TRY(ensure_buf(L.firedesc, ndesc * sizeof(LogSegDesc)));
    GWO_TRY(hipcheck(hipMemcpyAsync(L.firedesc.ptr, L.h_fire.data(), ndesc * sizeof(LogSegDesc), hipMemcpyHostToDevice,
                                    stream), "fire desc"));
    size_t at = 0;
    for (long long u : fire) {
        LogWindow &W = L.wins[u];
        int64_t start = unit_start(u);
        int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
        prof_begin(GWO_KERNEL_FIRE);
        launch_log_fire((const LogSegDesc *)L.firedesc.ptr + at, (int)W.segs.size(), W.lp, plan, rplan, start, end, o,
                        L.d_overflow, stream);
        GWO_TRY(launch_ok("log fire"));
        prof_end(GWO_KERNEL_FIRE, (int64_t)W.records);
        at += W.segs.size();
    }
    GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_out_count, 8, hipMemcpyDeviceToHost, stream), "out count"));
    GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar + 1, L.d_overflow, 8, hipMemcpyDeviceToHost, stream), "overflow"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "log fire"));
    out_rows = h_scalar[0];
    if (h_scalar[1]) return poison(GWO_ERR_CAPACITY, "log fire: a partition overflowed its LDS table");
    for (long long u : fire) {
        LogWindow &W = L.wins[u];
        L.last_window_records = std::max<uint64_t>(W.records, L.last_window_records / 2);
        log_release(W);
        // allowedLateness > 0: any later record of this window is a re-fire and is rejected at
        // scan time, so nothing of the window is kept until its cleanup time
        L.wins.erase(u);
    }
    return GWO_OK;
}

gwo_status Handle::log_state_size(int64_t *entries) {
    uint64_t s = 0;
    for (auto &kv : logst->wins) s += kv.second.records;
    *entries = (int64_t)s;
    return GWO_OK;
}

}  // namespace gwo
