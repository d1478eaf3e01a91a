// gwo_snapshot.cpp -- checkpoint / restore of the keyed window state for every layout (kernels:
// gwo_snapshot.hip; layout-specific collection and restore in gwo_log.cpp / gwo_session.cpp).
//
// Reference: the heap backend writes, per key group, the window-contents entries (namespace, key, state)
// (CopyOnWriteStateMapSnapshot.java:127-129, HeapSnapshotStrategy.java:97-222) and the window-timers of
// the timer service (InternalTimeServiceManager.java:160-198); restore reads only the key groups of the
// subtask's KeyGroupRange (HeapRestoreOperation), which is how a job is rescaled.  A row here is
// (key, TimeWindow{start, end}, raw accumulator words, fire-timer pending), rows ordered by key group.
#include <algorithm>
#include <cstring>
#include <map>
#include <vector>

#include "gwo_handle.h"

namespace gwo {

void launch_snap_table(const TableDesc &t, uint64_t cap, const AccPlan &p, int64_t start, int64_t end, int32_t timer,
                       const SnapCols &c, hipStream_t s);
void launch_snap_gather(const SnapCols &c, const uint32_t *perm, const uint32_t *kg_sorted, int64_t n, int nw,
                        int64_t *key, int64_t *start, int64_t *end, int64_t *words, int32_t *kg, int32_t *timer,
                        hipStream_t s);
void launch_snap_fill_i32(int32_t *p, int64_t n, int32_t v, hipStream_t s);

namespace {
struct Scratch {
    DevBuf b[5 + GWO_MAX_WORDS];
    ~Scratch() {
        for (auto &x : b) x.release();
    }
};
}  // namespace

// Completes everything queued (a pipelined batch, a deferred pass 2, a running fire): a checkpoint is taken
// between records (prepareSnapshotPreBarrier flushes the operator's batch first, AbstractStreamOperator.java:303).
gwo_status Handle::snapshot_quiesce() {
    GWO_TRY(flush_pending());
    if (logst) {
        GWO_TRY(log_flush());
        GWO_TRY(log_resolve_split());
    }
    GWO_TRY(finish_fire());
    return hipcheck(hipStreamSynchronize(stream), "snapshot sync");
}

// Upper bound of the rows a snapshot writes (exact for tables and sessions; the log layout's unfolded records).
gwo_status Handle::snapshot_rows(int64_t *n_rows) {
    GWO_TRY(snapshot_quiesce());
    if (sess) return session_state_size(n_rows);
    if (logst) return log_state_size(n_rows);
    GWO_TRY(read_occupancy());
    int64_t r = 0;
    for (auto &kv : tables) r += (int64_t)kv.second.occ;
    for (auto &kv : rdone) r += (int64_t)kv.second.occ;
    *n_rows = r;
    return GWO_OK;
}

gwo_status Handle::snapshot(const gwo_state_rows *rows, int64_t cap, int64_t *n_out) {
    int64_t bound = 0;
    GWO_TRY(snapshot_rows(&bound));
    const int NW = plan.nwords;
    const size_t m = (size_t)std::max<int64_t>(bound, 1);
    Scratch S;
    for (int i = 0; i < 3; ++i) GWO_TRY(ensure_buf(S.b[i], m * 8));
    GWO_TRY(ensure_buf(S.b[3], m * 4));
    for (int w = 0; w < NW; ++w) GWO_TRY(ensure_buf(S.b[5 + w], m * 8));
    SnapCols c{};
    c.key = (int64_t *)S.b[0].ptr;
    c.start = (int64_t *)S.b[1].ptr;
    c.end = (int64_t *)S.b[2].ptr;
    c.timer = (int32_t *)S.b[3].ptr;
    for (int w = 0; w < NW; ++w) c.w[w] = (int64_t *)S.b[5 + w].ptr;
    c.count = d_scratch_count;
    c.cap = (long long)m;
    GWO_TRY(hipcheck(hipMemsetAsync(d_scratch_count, 0, 8, stream), "snapshot count"));
    if (sess) {
        GWO_TRY(session_snapshot_collect(c));
    } else {
        if (logst) {   // collecting windows: fire timers pending; then any fired windows kept in tables
            GWO_TRY(log_snapshot_collect(c));
            GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_scratch_count, 8, hipMemcpyDeviceToHost, stream), "snapshot count"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "snapshot count"));
            const int64_t n_log = std::min<int64_t>((int64_t)*h_scalar, (int64_t)m);
            if (n_log > 0) launch_snap_fill_i32(c.timer, n_log, 1, stream);
        }
        for (auto &kv : tables) {
            const int64_t start = unit_start(kv.first);
            const int64_t span = slide ? geom.unit : cfg.size;   // sliding rows carry their pane
            const int32_t timer = (cfg.assigner == GWO_ASSIGNER_TUMBLING && kv.second.fired) ? 0 : 1;
            launch_snap_table(desc(kv.second), kv.second.cap, plan, start, (int64_t)((uint64_t)start + (uint64_t)span),
                              timer, c, stream);
        }
        for (auto &kv : rdone) {   // emitted entries (a key with new records also has a pending row from `tables`)
            const int64_t start = unit_start(kv.first);
            launch_snap_table(desc(kv.second), kv.second.cap, plan, start, (int64_t)((uint64_t)start + (uint64_t)cfg.size),
                              0, c, stream);
        }
        GWO_TRY(launch_ok("snapshot"));
    }
    GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_scratch_count, 8, hipMemcpyDeviceToHost, stream), "snapshot count"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "snapshot count"));
    int64_t n = (int64_t)*h_scalar;
    *n_out = n;
    if (n > (int64_t)m) return poison(GWO_ERR_HIP, "snapshot: more rows than the state holds");
    if (n > cap) return fail(GWO_ERR_CAPACITY, "snapshot: %lld rows, buffer holds %lld", (long long)n, (long long)cap);
    if (n == 0) return GWO_OK;
    // key groups, then a stable radix sort by key group (KeyGroupRangeAssignment.java:60-73)
    DevBuf kg, k1, v1, k2, v2, hist, ok, os, oe, ow, okg, ot;
    GWO_TRY(ensure_buf(kg, (size_t)n * 4));
    launch_key_groups(c.key, n, cfg.key_kind, cfg.max_parallelism, 1, (int32_t *)kg.ptr, nullptr, stream);
    GWO_TRY(launch_ok("snapshot key groups"));
    for (DevBuf *d : {&k1, &v1, &k2, &v2}) GWO_TRY(ensure_buf(*d, (size_t)n * 4));
    GWO_TRY(ensure_buf(hist, (size_t)256 * ((n + 4095) / 4096) * 4 + 16));
    const int bits = cfg.max_parallelism <= 256 ? 8 : 16;
    const int which = radix_sort_pairs((const uint32_t *)kg.ptr, nullptr, n, bits, (uint32_t *)k1.ptr,
                                       (uint32_t *)v1.ptr, (uint32_t *)k2.ptr, (uint32_t *)v2.ptr,
                                       (uint32_t *)hist.ptr, stream);
    GWO_TRY(launch_ok("snapshot sort"));
    const uint32_t *skg = (const uint32_t *)(which ? k2.ptr : k1.ptr);
    const uint32_t *perm = (const uint32_t *)(which ? v2.ptr : v1.ptr);
    for (DevBuf *d : {&ok, &os, &oe}) GWO_TRY(ensure_buf(*d, (size_t)n * 8));
    GWO_TRY(ensure_buf(ow, (size_t)n * NW * 8));
    GWO_TRY(ensure_buf(okg, (size_t)n * 4));
    GWO_TRY(ensure_buf(ot, (size_t)n * 4));
    launch_snap_gather(c, perm, skg, n, NW, (int64_t *)ok.ptr, (int64_t *)os.ptr, (int64_t *)oe.ptr, (int64_t *)ow.ptr,
                       (int32_t *)okg.ptr, (int32_t *)ot.ptr, stream);
    GWO_TRY(launch_ok("snapshot gather"));
    if (!rdone.empty() && !sess) {
        // a tumbling window restored with emitted entries (rdone) holds a key twice once the key got new records: a
        // pending row (tables) and an emitted one (rdone).  The heap backend keeps one entry per (key, window)
        // (CopyOnWriteStateMapSnapshot.java:127-129) whose fire timer is pending -- the rows are merged here as
        // gwo_export_heap_state merges them (rare path: host copies, the device buffers are rewritten)
        std::vector<int64_t> hk(n), hs(n), he(n), hw((size_t)n * NW);
        std::vector<int32_t> hg(n), ht(n);
        GWO_TRY(hipcheck(copy_out(hk.data(), ok.ptr, (size_t)n * 8, stream), "dedup"));
        GWO_TRY(hipcheck(copy_out(hs.data(), os.ptr, (size_t)n * 8, stream), "dedup"));
        GWO_TRY(hipcheck(copy_out(he.data(), oe.ptr, (size_t)n * 8, stream), "dedup"));
        GWO_TRY(hipcheck(copy_out(hw.data(), ow.ptr, (size_t)n * NW * 8, stream), "dedup"));
        GWO_TRY(hipcheck(copy_out(hg.data(), okg.ptr, (size_t)n * 4, stream), "dedup"));
        GWO_TRY(hipcheck(copy_out(ht.data(), ot.ptr, (size_t)n * 4, stream), "dedup"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "dedup"));
        std::map<std::pair<int64_t, int64_t>, int64_t> at;
        int64_t m2 = 0;
        for (int64_t i = 0; i < n; ++i) {
            auto it = at.find({hk[i], hs[i]});
            if (it != at.end()) {   // same key group as the row it joins: the key-group order stays
                const int64_t j = it->second;
                for (int w = 0; w < NW; ++w)
                    hw[(size_t)j * NW + w] = combine_h(plan.op[w], hw[(size_t)j * NW + w], hw[(size_t)i * NW + w]);
                ht[j] = ht[j] || ht[i];
                continue;
            }
            at[{hk[i], hs[i]}] = m2;
            hk[m2] = hk[i];
            hs[m2] = hs[i];
            he[m2] = he[i];
            hg[m2] = hg[i];
            ht[m2] = ht[i];
            for (int w = 0; w < NW; ++w) hw[(size_t)m2 * NW + w] = hw[(size_t)i * NW + w];
            m2++;
        }
        if (m2 < n) {
            n = m2;
            *n_out = n;
            GWO_TRY(hipcheck(copy_in(ok.ptr, hk.data(), (size_t)n * 8, stream), "dedup"));
            GWO_TRY(hipcheck(copy_in(os.ptr, hs.data(), (size_t)n * 8, stream), "dedup"));
            GWO_TRY(hipcheck(copy_in(oe.ptr, he.data(), (size_t)n * 8, stream), "dedup"));
            GWO_TRY(hipcheck(copy_in(ow.ptr, hw.data(), (size_t)n * NW * 8, stream), "dedup"));
            GWO_TRY(hipcheck(copy_in(okg.ptr, hg.data(), (size_t)n * 4, stream), "dedup"));
            GWO_TRY(hipcheck(copy_in(ot.ptr, ht.data(), (size_t)n * 4, stream), "dedup"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "dedup"));
        }
    }
    struct {
        void *dst;
        DevBuf *src;
        size_t bytes;
    } cp[] = {{rows->key, &ok, (size_t)n * 8},         {rows->window_start, &os, (size_t)n * 8},
              {rows->window_end, &oe, (size_t)n * 8},  {rows->words, &ow, (size_t)n * NW * 8},
              {rows->key_group, &okg, (size_t)n * 4},  {rows->timer, &ot, (size_t)n * 4}};
    gwo_status st = GWO_OK;
    for (auto &x : cp)
        if (x.dst && st == GWO_OK)
            st = hipcheck(copy_out(x.dst, x.src->ptr, x.bytes, stream), "snapshot copy");
    if (st == GWO_OK) st = hipcheck(hipStreamSynchronize(stream), "snapshot sync");
    for (DevBuf *d : {&kg, &k1, &v1, &k2, &v2, &hist, &ok, &os, &oe, &ow, &okg, &ot}) d->release();
    return st;
}

// ---- restore -----------------------------------------------------------------------------------------------
// Host copies of the rows (checkpoints are read from storage into host memory; device rows work too).
gwo_status Handle::restore(const gwo_state_rows *rows, int32_t n_words, int64_t n, int64_t new_wm) {
    return restore_impl(rows, n_words, n, new_wm, false);
}

// per_window: sliding rows are windows (a per-window savepoint, gwo_import_heap_state), not panes.
gwo_status Handle::restore_impl(const gwo_state_rows *rows, int32_t n_words, int64_t n, int64_t new_wm,
                                bool per_window) {
    if (n_words != plan.nwords)
        return fail(GWO_ERR_INVALID_ARGUMENT, "restore: rows carry %d accumulator words, this operator's aggregates use %d",
                    n_words, plan.nwords);
    const bool fresh = wm == (int64_t)0x8000000000000000LL && tables.empty() && rdone.empty() &&
                       (!sess || session_live() == 0) &&
                       (!logst || log_window_count() == 0) && !slide_has_restored();
    if (!fresh) return fail(GWO_ERR_STATE, "restore: the handle already holds state");
    RestoreRows R;
    R.n = n;
    R.nw = n_words;
    if (n > 0) {
        R.key.resize(n);
        R.start.resize(n);
        R.end.resize(n);
        R.words.resize((size_t)n * n_words);
        struct {
            void *dst;
            const void *src;
            size_t bytes;
        } cp[] = {{R.key.data(), rows->key, (size_t)n * 8},
                  {R.start.data(), rows->window_start, (size_t)n * 8},
                  {R.end.data(), rows->window_end, (size_t)n * 8},
                  {R.words.data(), rows->words, (size_t)n * n_words * 8}};
        for (auto &x : cp) GWO_TRY(hipcheck(fetch_host(x.dst, x.src, x.bytes, stream), "restore rows"));
        if (rows->timer) {
            R.timer.resize(n);
            GWO_TRY(hipcheck(fetch_host(R.timer.data(), rows->timer, (size_t)n * 4, stream), "restore timers"));
        }
    }
    // only this subtask's key groups (a rescaled job restores the union of the old subtasks' rows)
    R.mine.assign(n, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int32_t kg = key_group(R.key[i], cfg.key_kind, cfg.max_parallelism);
        R.mine[i] = kg >= cfg.key_group_start && kg <= cfg.key_group_end;
    }
    if (sess) return session_restore_rows(R, new_wm);
    if (slide && per_window) return slide_restore_windows(R, new_wm);
    if (logst) return log_restore_rows(R, new_wm);
    return table_restore_rows(R, new_wm);
}

// Table layout (tumbling, sliding panes): rows grouped into per-window (per-pane) hash tables; every check
// happens before the handle changes (rows must be window (pane) starts).  A tumbling row's timer flag says whether its
// fire timer is pending or the window already emitted it (kept for allowedLateness):
//   * pending rows -> the window's table, which fires at maxTimestamp;
//   * emitted rows of a window the restore watermark passed -> the window's table, marked fired (re-fires, cleanup);
//   * emitted rows of a window whose maxTimestamp lies above the restore watermark (a restored WindowOperator's timer
//     service starts at Long.MIN_VALUE; or subtasks checkpointed at different watermarks, rescaled into one) -> rdone:
//     such an entry stays emitted unless its key gets new records before the watermark passes maxTimestamp, which
//     re-registers that (key, window) timer (WindowOperator.java:393-410), so the key fires with both (fire_tumbling);
//     so do emitted rows of a window that also has pending rows (subtasks checkpointed at different watermarks).
gwo_status Handle::table_restore_rows(const RestoreRows &R, int64_t new_wm) {
    std::map<long long, uint64_t> per_unit, per_done;
    std::map<long long, int> timers;   // bit 0: a row with a pending timer, bit 1: a row already emitted
    std::vector<char> to_done(R.n, 0);
    std::vector<long long> unit_of(R.n, 0);
    const bool tumbling = cfg.assigner == GWO_ASSIGNER_TUMBLING;
    for (int64_t i = 0; i < R.n; ++i) {
        if (!R.mine[i]) continue;
        const __int128 a = (__int128)R.start[i] - (__int128)geom.unit_off_mod;
        __int128 q = a / geom.unit;
        if (a % geom.unit != 0 && a < 0) q -= 1;   // floor (unit > 0)
        const long long u = (long long)q;
        if (unit_start(u) != R.start[i])
            return fail(GWO_ERR_INVALID_ARGUMENT, "restore: %lld is not a window start", (long long)R.start[i]);
        if (!R.timer.empty()) timers[u] |= R.timer[i] ? 1 : 2;
        unit_of[i] = u;
    }
    for (int64_t i = 0; i < R.n; ++i) {
        if (!R.mine[i]) continue;
        const long long u = unit_of[i];
        const int64_t max_ts = (int64_t)((uint64_t)R.start[i] + (uint64_t)cfg.size - 1);
        if (tumbling && !R.timer.empty() && R.timer[i] == 0 && (max_ts > new_wm || timers[u] == 3)) {
            if (logst && cfg.allowed_lateness == 0)   // (a window fires and clears at once: no such state exists)
                return fail(GWO_ERR_UNSUPPORTED, "restore: window %lld holds entries already emitted (above the "
                                                 "restore watermark or beside pending ones) with allowedLateness 0",
                            (long long)unit_start(u));
            to_done[i] = 1;
            per_done[u]++;
        } else {
            per_unit[u]++;
        }
    }
    long long lo = 0, hi = -1;
    for (auto *m : {&per_unit, &per_done})
        if (!m->empty()) {
            lo = hi < lo ? m->begin()->first : std::min(lo, m->begin()->first);
            hi = std::max(hi, m->rbegin()->first);
        }
    if (hi >= lo && hi - lo >= (1LL << 20)) return fail(GWO_ERR_UNSUPPORTED, "restore: windows span more than 2^20 units");
    wm = in_wm = new_wm;   // validated: from here on the handle holds the restored state
    if (hi < lo) return slide ? slide_restore_anchor() : GWO_OK;
    for (auto &kv : per_unit) {
        GWO_TRY(ensure_table(kv.first, kv.second));   // marks windows whose end the watermark passed as fired
        auto t = timers.find(kv.first);
        if (tumbling && t != timers.end()) tables[kv.first].fired = t->second == 2;
    }
    for (auto &kv : per_done) {
        Table t;
        uint64_t cap = kMinCap;
        while ((double)kv.second > kInitLoad * (double)cap) cap <<= 1;
        GWO_TRY(alloc_table(cap, t));
        t.fired = true;
        rdone.emplace(kv.first, t);
    }
    const int dir_len = (int)(hi - lo + 1);
    DevBuf bk, bs, bw;
    gwo_status st = GWO_OK;
    for (int pass = 0; pass < 2 && st == GWO_OK; ++pass) {   // pending / fired rows, then rows for rdone
        std::map<long long, Table> &dst = pass ? rdone : tables;
        std::vector<int64_t> k, s, w;
        for (int64_t i = 0; i < R.n; ++i)
            if (R.mine[i] && to_done[i] == pass) {
                k.push_back(R.key[i]);
                s.push_back(R.start[i]);
                w.insert(w.end(), R.words.begin() + (size_t)i * R.nw, R.words.begin() + (size_t)(i + 1) * R.nw);
            }
        if (k.empty()) continue;
        h_dir.assign(dir_len, TableDesc{});
        for (auto &kv : dst) h_dir[kv.first - lo] = desc(kv.second);
        GWO_TRY(ensure_buf(dir_buf, dir_len * sizeof(TableDesc)));
        GWO_TRY(hipcheck(hipMemcpyAsync(dir_buf.ptr, h_dir.data(), dir_len * sizeof(TableDesc), hipMemcpyHostToDevice,
                                        stream), "restore dir"));
        GWO_TRY(ensure_buf(bk, k.size() * 8));
        GWO_TRY(ensure_buf(bs, s.size() * 8));
        GWO_TRY(ensure_buf(bw, w.size() * 8));
        GWO_TRY(hipcheck(copy_in(bk.ptr, k.data(), k.size() * 8, stream), "restore keys"));
        GWO_TRY(hipcheck(copy_in(bs.ptr, s.data(), s.size() * 8, stream), "restore starts"));
        GWO_TRY(hipcheck(copy_in(bw.ptr, w.data(), w.size() * 8, stream), "restore words"));
        launch_restore((const int64_t *)bk.ptr, (const int64_t *)bs.ptr, (const int64_t *)bw.ptr, (int64_t)k.size(), plan,
                       geom_now(), (const TableDesc *)dir_buf.ptr, lo, dir_len, stream);
        st = launch_ok("restore");
        if (st == GWO_OK) st = hipcheck(hipStreamSynchronize(stream), "restore sync");   // (host columns are reused)
    }
    bk.release();
    bs.release();
    bw.release();
    for (auto &kv : tables) kv.second.dirty = true;
    if (st == GWO_OK) st = read_occupancy();
    for (auto it = tables.begin(); it != tables.end();) {   // a table left empty goes back to the pool
        if (it->second.occ == 0) {
            release_table(it->second);
            it = tables.erase(it);
        } else {
            ++it;
        }
    }
    if (st == GWO_OK && slide) st = slide_restore_anchor();
    return st;
}

}  // namespace gwo
