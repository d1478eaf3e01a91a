// gwo_slide.cpp -- SlidingEventTimeWindows on panes.
//
// The reference assigns every record to ceil(size/slide) windows (SlidingEventTimeWindows.java:
// 68-82) and keeps one state entry + timer per (key, window).  Here a record updates exactly one
// pane (a tumbling window of gcd(size, slide), the pane design of the Blink SQL runtime:
// flink-table/flink-table-runtime-blink/.../window/assigners/SlidingWindowAssigner.java:66-95).
// With allowedLateness = 0 a pane's contents only reach windows that have not fired yet, which is
// exactly the reference's per-window accept set (WindowOperator.java:388-390), so outputs match.
//
// Fire strategies:
//  * ring (every accumulator word is a wrap-around int64 sum: COUNT, SUM/AVG over int64): the
//    running total T of the next window J to fire is kept in HBM; records in J's panes update T
//    as they arrive; firing J emits T's live entries, then T -= leaving panes, T += entering panes.
//    Int64 addition is a group, so subtraction is exact (bit-identical to summing the window).
//  * recompute (MIN/MAX, float64 sums): firing J folds J's panes into a scratch table and emits it.
#include <algorithm>

#include "gwo_handle.h"
#include "gwo_slide.h"

namespace gwo {

#define GWO_LONG_MIN_H ((int64_t)0x8000000000000000LL)
#define GWO_LONG_MAX_H ((int64_t)0x7fffffffffffffffLL)

static int64_t fmod64(int64_t a, int64_t b) {
    int64_t r = a % b;
    return r < 0 ? r + b : r;
}
static __int128 fdiv128(__int128 a, __int128 b) {
    __int128 q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

gwo_status Handle::slide_init() {
    slide = new SlideState();
    SlideState &S = *slide;
    S.om = fmod64(cfg.offset, cfg.slide);
    bool all_add = true;
    for (int w = 0; w < plan.nwords; ++w) all_add &= plan.op[w] == ACC_ADD_I64;
    S.ring = all_add && getenv("GWO_SLIDE_RECOMPUTE") == nullptr;
    if (S.ring) {
        // presence of a key in the window: an existing record count word (COUNT, AVG) serves, else a hidden one
        for (int w = 0; w < plan.nwords && S.count_word < 0; ++w)
            if (plan.op[w] == ACC_ADD_I64 && plan.src[w] == SRC_ONE) S.count_word = w;
        if (S.count_word < 0) {
            if (plan.nwords >= GWO_MAX_WORDS) return fail(GWO_ERR_UNSUPPORTED, "too many accumulator words");
            S.count_word = plan.nwords;
            plan.op[plan.nwords] = ACC_ADD_I64;
            plan.src[plan.nwords] = SRC_ONE;
            plan.ident[plan.nwords] = 0;
            plan.nwords++;
            plan.stride = ((1 + plan.nwords) + 1) & ~1;
        }
        GWO_TRY(dalloc((void **)&S.d_live, 8));
        GWO_TRY(hipcheck(hipMemsetAsync(S.d_live, 0, 8, stream), "live"));
        Table t;
        GWO_TRY(alloc_table(std::max<uint64_t>(kMinCap, 1 << 16), t));
        aux_tables.push_back(t);
        S.t_idx = (int)aux_tables.size() - 1;
    }
    return GWO_OK;
}

void Handle::slide_free() {
    if (!slide) return;
    if (slide->d_live) (void)hipFree(slide->d_live);
    delete slide;
    slide = nullptr;
}

// pane index of a pane-aligned time x
static inline long long pane_of(int64_t x, int64_t unit) { return (long long)fdiv128(x, unit); }

int64_t Handle::win_start(__int128 j) const { return (int64_t)(j * cfg.slide + slide->om); }
long long Handle::win_first_pane(__int128 j) const { return pane_of(win_start(j), geom.unit); }
long long Handle::win_last_pane(__int128 j) const {
    return (long long)(fdiv128((__int128)win_start(j) + cfg.size, geom.unit) - 1);
}
// first window containing pane u: smallest j with start_j + size > pane_start(u)
__int128 Handle::first_window_of_pane(long long u) const {
    __int128 ps = (__int128)u * geom.unit + geom.unit_off_mod;
    return fdiv128(ps - cfg.size - slide->om, cfg.slide) + 1;
}

RingDesc Handle::ring_desc() {
    RingDesc r{};
    r.lo = 1;
    r.hi = 0;
    if (slide && slide->ring && slide->j_set) {
        Table &T = aux_tables[slide->t_idx];
        r.t = desc(T);
        r.lo = win_first_pane(slide->J);
        r.hi = win_last_pane(slide->J);
        r.live = slide->d_live;
        r.count_word = slide->count_word;
    }
    return r;
}

// Grow (or compact away dead entries of) the ring table so `incoming` more entries fit.
gwo_status Handle::ensure_ring(uint64_t incoming) {
    SlideState &S = *slide;
    Table &T = aux_tables[S.t_idx];
    GWO_TRY(read_occupancy());
    if ((double)(T.occ + incoming) <= kMaxLoad * (double)T.cap) return GWO_OK;
    GWO_TRY(hipcheck(hipMemcpyAsync(&S.h_live, S.d_live, 8, hipMemcpyDeviceToHost, stream), "live"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "live sync"));
    uint64_t need = S.h_live + incoming;
    uint64_t ncap = kMinCap;
    while ((double)need > kInitLoad * (double)ncap) ncap <<= 1;
    Table nt;
    GWO_TRY(alloc_table(ncap, nt));
    launch_rehash_live(desc(T), T.cap, desc(nt), plan, S.count_word, stream);
    GWO_TRY(hipcheck(hipMemcpyAsync(nt.side, T.side, (size_t)plan.stride * 8, hipMemcpyDeviceToDevice, stream), "side"));
    GWO_TRY(reset_side(T));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "ring rehash"));
    release_table(T);
    aux_tables[S.t_idx] = nt;
    return read_occupancy();
}

gwo_status Handle::slide_prepare_insert(long long base, int len, const unsigned long long *hist) {
    if (!slide || !slide->ring || !slide->j_set) return GWO_OK;
    long long lo = win_first_pane(slide->J), hi = win_last_pane(slide->J);
    uint64_t incoming = 0;
    for (int d = 0; d < len; ++d)
        if (base + d >= lo && base + d <= hi) incoming += hist[d];
    return incoming ? ensure_ring(incoming) : GWO_OK;
}

// T := sum of the existing panes of window J (after a jump).
gwo_status Handle::ring_rebuild() {
    SlideState &S = *slide;
    Table &T0 = aux_tables[S.t_idx];
    launch_fill(T0.base, T0.cap, plan, stream);
    GWO_TRY(launch_ok("fill"));
    GWO_TRY(reset_side(T0));
    GWO_TRY(ctr_zero(T0.counter));
    GWO_TRY(hipcheck(hipMemsetAsync(S.d_live, 0, 8, stream), "live reset"));
    T0.occ = 0;
    GWO_TRY(read_occupancy());
    long long lo = win_first_pane(S.J), hi = win_last_pane(S.J);
    for (auto it = tables.lower_bound(lo); it != tables.end() && it->first <= hi; ++it) {
        GWO_TRY(ensure_ring(it->second.occ));
        Table &T = aux_tables[S.t_idx];
        launch_fold(desc(it->second), it->second.cap, desc(T), plan, +1, S.count_word, S.d_live, stream);
        T.occ += it->second.occ;   // upper bound until the next read
    }
    return GWO_OK;
}

// After gwo_restore: every window that ends at or before the restored watermark fired before the
// checkpoint, so the next window to fire is the first one open at it; the ring total is rebuilt from
// the restored panes.
gwo_status Handle::slide_restore_anchor() {
    SlideState &S = *slide;
    __int128 j = fdiv128((__int128)wm - cfg.size + 1 - S.om, cfg.slide) + 1;
    const __int128 j_lo = fdiv128((__int128)GWO_LONG_MIN_H + 2 * (__int128)cfg.size + cfg.slide, cfg.slide);
    const __int128 j_hi = fdiv128((__int128)GWO_LONG_MAX_H - 2 * (__int128)cfg.size - cfg.slide, cfg.slide);
    S.J = std::max(j_lo, std::min(j_hi, j));
    S.j_set = true;
    if (S.ring) GWO_TRY(ring_rebuild());
    return GWO_OK;
}

// Window indices are kept where start_j + size cannot overflow a long.
static __int128 clamp_window(__int128 j, int64_t size, int64_t slide) {
    const __int128 j_lo = fdiv128((__int128)GWO_LONG_MIN_H + 2 * (__int128)size + slide, slide);
    const __int128 j_hi = fdiv128((__int128)GWO_LONG_MAX_H - 2 * (__int128)size - slide, slide);
    return std::max(j_lo, std::min(j_hi, j));
}

// first window not fired at watermark w: start_j + size - 1 > w
__int128 Handle::first_unfired_window(int64_t w) const {
    return clamp_window(fdiv128((__int128)w - cfg.size + 1 - slide->om, cfg.slide) + 1, cfg.size, cfg.slide);
}

// first window not cleaned up at watermark w: start_j + size - 1 + allowedLateness > w (WindowOperator.java:
// 639-646 saturates the cleanup time at Long.MAX_VALUE; keeping such windows' panes a little longer is harmless)
__int128 Handle::first_uncleaned_window(int64_t w) const {
    const __int128 j =
        fdiv128((__int128)w - cfg.size + 1 - (__int128)cfg.allowed_lateness - slide->om, cfg.slide) + 1;
    return std::min(first_unfired_window(w), clamp_window(j, cfg.size, cfg.slide));
}

gwo_status Handle::fire_sliding(int64_t new_wm) {
    SlideState &S = *slide;
    const __int128 j_new = first_unfired_window(new_wm);
    // panes stay while a window holding them is not cleaned up: with allowedLateness > 0 fired windows
    // still take (and re-fire for) late records until their cleanup time
    const long long keep_from = win_first_pane(first_uncleaned_window(new_wm));
    if (!S.j_set) {
        // anchor: windows before j_new have fired (were empty); the first window with data may be earlier
        S.J = j_new;
        if (!tables.empty()) S.J = std::min(first_window_of_pane(tables.begin()->first), j_new);
        S.j_set = true;
        if (S.ring) GWO_TRY(ring_rebuild());
    }
    OutCols o = out_cols();
    while (S.J < j_new) {
        // ---- skip windows that hold no data (restored entries with a pending fire timer count as data) ----
        long long lo = win_first_pane(S.J), hi = win_last_pane(S.J);
        auto rw = S.rwin.find((long long)S.J);
        const bool rpend = rw != S.rwin.end() && rw->second.n_pend > 0;
        bool empty;
        if (S.ring) {
            GWO_TRY(hipcheck(hipMemcpyAsync(&S.h_live, S.d_live, 8, hipMemcpyDeviceToHost, stream), "live"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "live sync"));
            empty = S.h_live == 0;
        } else {
            auto it = tables.lower_bound(lo);
            empty = it == tables.end() || it->first > hi;
        }
        if (empty && !rpend) {
            __int128 target = j_new;
            auto it = tables.lower_bound(lo);
            if (it != tables.end()) target = std::min(j_new, std::max(S.J + 1, first_window_of_pane(it->first)));
            for (auto nx = S.rwin.upper_bound((long long)S.J); nx != S.rwin.end(); ++nx)
                if (nx->second.n_pend) {
                    target = std::min(target, (__int128)nx->first);
                    break;
                }
            // panes before the target window are in no unfired (or uncleaned) window any more
            GWO_TRY(release_panes_before(std::min(win_first_pane(target), keep_from)));
            S.J = target;
            if (S.ring) GWO_TRY(ring_rebuild());
            continue;
        }
        const int64_t start = win_start(S.J);
        const int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
        // ---- emit window J ----
        if (S.ring) {
            if (rw != S.rwin.end()) {   // restored entries join J's rows: T += them for the emission, -= after it
                GWO_TRY(ensure_ring(rw->second.n_pend));
                GWO_TRY(rwin_fold(rw->second, aux_tables[S.t_idx], +1, S.count_word, S.d_live));
                GWO_TRY(hipcheck(hipMemcpyAsync(&S.h_live, S.d_live, 8, hipMemcpyDeviceToHost, stream), "live"));
                GWO_TRY(hipcheck(hipStreamSynchronize(stream), "live sync"));
            }
            Table &T = aux_tables[S.t_idx];
            GWO_TRY(ensure_output(S.h_live));
            o = out_cols();
            prof_begin(GWO_KERNEL_FIRE);
            launch_fire(desc(T), T.cap, plan, rplan, start, end, o, 0, S.count_word, stream);
            prof_end(GWO_KERNEL_FIRE, (int64_t)T.cap);
            out_rows += S.h_live;
            if (rw != S.rwin.end()) GWO_TRY(rwin_fold(rw->second, T, -1, S.count_word, S.d_live));
        } else {
            uint64_t total = rw != S.rwin.end() ? rw->second.n_pend : 0;
            GWO_TRY(read_occupancy());
            for (auto it = tables.lower_bound(lo); it != tables.end() && it->first <= hi; ++it) total += it->second.occ;
            Table W;
            uint64_t cap = kMinCap;
            while ((double)total > kInitLoad * (double)cap) cap <<= 1;
            GWO_TRY(alloc_table(cap, W));
            prof_begin(GWO_KERNEL_SLIDE);
            for (auto it = tables.lower_bound(lo); it != tables.end() && it->first <= hi; ++it)
                launch_fold(desc(it->second), it->second.cap, desc(W), plan, +1, -1, nullptr, stream);
            if (rw != S.rwin.end()) GWO_TRY(rwin_fold(rw->second, W, +1, -1, nullptr));   // after the panes
            prof_end(GWO_KERNEL_SLIDE, (int64_t)total);
            uint64_t rows = 0;
            GWO_TRY(ctr_read(W.counter, &rows));
            GWO_TRY(ensure_output(rows));
            o = out_cols();
            prof_begin(GWO_KERNEL_FIRE);
            launch_fire(desc(W), W.cap, plan, rplan, start, end, o, 1, -1, stream);
            prof_end(GWO_KERNEL_FIRE, (int64_t)W.cap);
            out_rows += rows;
            release_table(W);
        }
        // ---- advance J -> J+1: T -= leaving panes, T += entering panes ----
        const long long nlo = win_first_pane(S.J + 1), nhi = win_last_pane(S.J + 1);
        if (S.ring) {
            GWO_TRY(read_occupancy());
            prof_begin(GWO_KERNEL_SLIDE);
            for (auto it = tables.lower_bound(lo); it != tables.end() && it->first < nlo; ++it)
                launch_fold(desc(it->second), it->second.cap, desc(aux_tables[S.t_idx]), plan, -1, S.count_word,
                            S.d_live, stream);
            prof_end(GWO_KERNEL_SLIDE, 0);
            uint64_t entering = 0;
            for (auto it = tables.upper_bound(hi); it != tables.end() && it->first <= nhi; ++it) entering += it->second.occ;
            if (entering) GWO_TRY(ensure_ring(entering));
            prof_begin(GWO_KERNEL_SLIDE);
            for (auto it = tables.upper_bound(hi); it != tables.end() && it->first <= nhi; ++it)
                launch_fold(desc(it->second), it->second.cap, desc(aux_tables[S.t_idx]), plan, +1, S.count_word,
                            S.d_live, stream);
            prof_end(GWO_KERNEL_SLIDE, 0);
        }
        GWO_TRY(release_panes_before(std::min(nlo, keep_from)));
        S.J += 1;
    }
    // windows whose cleanup time this watermark passed (no fire needed) free their panes too
    rwin_release_before((long long)std::min(S.J, first_uncleaned_window(new_wm)));
    return release_panes_before(std::min(win_first_pane(S.J), keep_from));
}

// ---- sliding windows restored from a per-window savepoint (gwo_import_heap_state) ------------------------------
// Restored entries of window j: pend (fire timer pending) inserted into the window's rows, done (already fired,
// waiting for the cleanup) only into keys the window holds from new records; sign -1 takes them out again.
gwo_status Handle::rwin_fold(RestoredWindow &r, Table &dst, int sign, int live_word, unsigned long long *live) {
    if (r.pend.base) launch_fold(desc(r.pend), r.pend.cap, desc(dst), plan, sign, live_word, live, stream, 0);
    if (r.done.base) launch_fold(desc(r.done), r.done.cap, desc(dst), plan, sign, live_word, live, stream, 1);
    GWO_TRY(launch_ok("restored window fold"));
    if (sign > 0) dst.occ += r.n_pend;   // an upper bound until the next read
    return GWO_OK;
}

void Handle::rwin_release_before(long long j) {
    if (!slide) return;
    for (auto it = slide->rwin.begin(); it != slide->rwin.end() && it->first < j;) {
        for (Table *t : {&it->second.pend, &it->second.done})
            if (t->base) {   // back to the pool clean: a no-output sweep resets every entry
                OutCols none = out_cols();
                none.cap = 0;
                (void)hipMemsetAsync(d_scratch_count, 0, 8, stream);
                none.count = d_scratch_count;
                launch_fire(desc(*t), t->cap, plan, rplan, 0, 0, none, 1, -1, stream);
                release_table(*t);
            }
        it = slide->rwin.erase(it);
    }
    if (slog) slog_rwin_release_before(j);
}

bool Handle::slide_has_restored() const {
    return slide && (!slide->rwin.empty() || (slog && slog_rwin_count() > 0));
}

// Rows (key, window start, raw words, fire timer pending) of a per-window savepoint: validated, then kept per
// window (RestoredWindow / the sliding log's partial segments).  New records after the restore go to panes as
// always; a window's rows combine both when it fires.
gwo_status Handle::slide_restore_windows(const RestoreRows &R, int64_t new_wm) {
    SlideState &S = *slide;
    const int NW = plan.nwords;
    std::map<long long, std::vector<int64_t>> pend, done;   // window -> row indices
    for (int64_t i = 0; i < R.n; ++i) {
        if (!R.mine[i]) continue;
        const __int128 a = (__int128)R.start[i] - S.om;
        const __int128 j = fdiv128(a, cfg.slide);
        if (win_start(j) != R.start[i] || (int64_t)((uint64_t)R.start[i] + (uint64_t)cfg.size) != R.end[i])
            return fail(GWO_ERR_INVALID_ARGUMENT, "import: [%lld, %lld) is not a window of this sliding assigner",
                        (long long)R.start[i], (long long)R.end[i]);
        const int64_t max_ts = (int64_t)((uint64_t)R.end[i] - 1);
        const bool pending = R.timer.empty() ? max_ts > new_wm : R.timer[i] != 0;
        if (pending && max_ts <= new_wm)
            return fail(GWO_ERR_UNSUPPORTED, "import: window [%lld, %lld) has a pending fire timer at or below the "
                                             "restore watermark %lld (restore at the checkpoint's watermark or "
                                             "Long.MIN_VALUE)", (long long)R.start[i], (long long)R.end[i],
                        (long long)new_wm);
        if (!pending && cleanup_time_host(max_ts) <= new_wm) continue;   // its state is gone at this watermark
        if (!pending && slog)
            return fail(GWO_ERR_UNSUPPORTED, "import: window [%lld, %lld) already fired; the sliding log keeps no "
                                             "fired windows (allowedLateness 0)", (long long)R.start[i],
                        (long long)R.end[i]);
        (pending ? pend : done)[(long long)j].push_back(i);
    }
    // the count word marks a key present in a window (ring strategies): a restored entry holds >= 1 record
    std::vector<int64_t> words(R.words);
    if (S.count_word >= 0) {
        bool hidden = true;   // slide_init's own count word (no COUNT / AVG aggregate supplies one)
        for (int a = 0; a < rplan.naggs; ++a) {
            if (rplan.kind[a] == GWO_AGG_COUNT && rplan.word[a] == S.count_word) hidden = false;
            if (rplan.kind[a] == GWO_AGG_AVG && rplan.word[a] + 1 == S.count_word) hidden = false;
        }
        for (auto *m : {&pend, &done})
            for (auto &kv : *m)
                for (int64_t i : kv.second) {
                    int64_t &c = words[(size_t)i * NW + S.count_word];
                    if (hidden) c = 1;
                    else if (c <= 0)
                        return fail(GWO_ERR_INVALID_ARGUMENT, "import: a window accumulator of key %lld counts %lld "
                                                              "records", (long long)R.key[i], (long long)c);
                }
    }
    // validated: from here on the handle holds the restored state
    wm = in_wm = new_wm;
    if (slog) {
        GWO_TRY(slog_anchor());
        for (auto &kv : pend) GWO_TRY(slog_rwin_add(kv.first, R.key, words, kv.second));
        return GWO_OK;
    }
    GWO_TRY(slide_restore_anchor());
    std::vector<int64_t> hk, hw;
    DevBuf dk, dw;
    for (int kind = 0; kind < 2; ++kind)
        for (auto &kv : kind ? done : pend) {
            const std::vector<int64_t> &ix = kv.second;
            hk.clear();
            hw.clear();
            for (int64_t i : ix) {
                hk.push_back(R.key[i]);
                hw.insert(hw.end(), words.begin() + (size_t)i * NW, words.begin() + (size_t)(i + 1) * NW);
            }
            RestoredWindow &rw = S.rwin[kv.first];
            Table &t = kind ? rw.done : rw.pend;
            uint64_t cap = kMinCap;
            while ((double)ix.size() > kInitLoad * (double)cap) cap <<= 1;
            GWO_TRY(alloc_table(cap, t));
            (kind ? rw.n_done : rw.n_pend) = ix.size();
            GWO_TRY(ensure_buf(dk, hk.size() * 8));
            GWO_TRY(ensure_buf(dw, hw.size() * 8));
            GWO_TRY(hipcheck(hipMemcpyAsync(dk.ptr, hk.data(), hk.size() * 8, hipMemcpyHostToDevice, stream), "rows"));
            GWO_TRY(hipcheck(hipMemcpyAsync(dw.ptr, hw.data(), hw.size() * 8, hipMemcpyHostToDevice, stream), "rows"));
            launch_rows_insert((const int64_t *)dk.ptr, (const int64_t *)dw.ptr, (int64_t)ix.size(), desc(t), plan,
                               stream);
            GWO_TRY(launch_ok("restore window"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "restore window"));   // (dk, dw are reused)
        }
    dk.release();
    dw.release();
    return GWO_OK;
}

// The restored entries still held (table layout and sliding log): key, window index, raw words, fire timer pending.
gwo_status Handle::slide_restored_rows(WindowRows &out) {
    if (!slide) return GWO_OK;
    if (slog) return slog_rwin_rows(out);
    const int NW = plan.nwords;
    std::vector<int64_t> img;
    for (auto &kv : slide->rwin)
        for (int kind = 0; kind < 2; ++kind) {
            const Table &t = kind ? kv.second.done : kv.second.pend;
            if (!t.base) continue;
            img.resize((size_t)(t.cap + 1) * plan.stride);
            GWO_TRY(hipcheck(hipMemcpy(img.data(), t.base, img.size() * 8, hipMemcpyDeviceToHost), "restored window"));
            for (uint64_t e = 0; e <= t.cap; ++e) {
                const int64_t *x = img.data() + e * plan.stride;
                const bool side = e == t.cap;
                if (side ? x[0] == 0 : x[0] == (int64_t)0x8000000000000000LL) continue;
                out.key.push_back(side ? (int64_t)0x8000000000000000LL : x[0]);
                out.j.push_back(kv.first);
                out.pending.push_back(kind == 0);
                out.words.insert(out.words.end(), x + 1, x + 1 + NW);
            }
        }
    return GWO_OK;
}

// Reset and return to the pool every pane table with index < first.
gwo_status Handle::release_panes_before(long long first) {
    for (auto it = tables.begin(); it != tables.end() && it->first < first;) {
        Table &t = it->second;
        OutCols none = out_cols();
        none.cap = 0;
        GWO_TRY(hipcheck(hipMemsetAsync(d_scratch_count, 0, 8, stream), "z"));
        none.count = d_scratch_count;
        launch_fire(desc(t), t.cap, plan, rplan, 0, 0, none, 1, -1, stream);
        recent_cap = t.cap;
        release_table(t);
        it = tables.erase(it);
    }
    return GWO_OK;
}

// Per-element re-fire on sliding windows (allowedLateness > 0).  The reference adds a record to each of its
// windows that is not late (WindowOperator.java:386-427) and EventTimeTrigger.onElement FIREs the ones whose
// maxTimestamp the watermark passed (EventTimeTrigger.java:37-45): one row per (record, fired-but-not-cleaned
// window) with that window's contents including the record.  Every record of the batch that reaches such a
// window re-fires it, so pair q's row is
//     window state before the batch  (+)  the batch's values for that (key, window) up to q, arrival order,
// where the state before the batch is the combine of the window's panes for the key.  The pairs are written in
// arrival order, sorted stably by (key, window) and scanned (refire_emit_kernel); then the batch's insert adds
// the records to their panes.
gwo_status Handle::slide_refire_rows(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n,
                                     const WindowGeom &g, uint64_t records) {
    SlideState &S = *slide;
    const __int128 j_fire = first_unfired_window(g.wm), j_clean = first_uncleaned_window(g.wm);
    if (j_fire <= j_clean) return poison(GWO_ERR_HIP, "sliding re-fire records but no fired, uncleaned window");
    if (j_fire - j_clean >= ((__int128)1 << 24))
        return fail(GWO_ERR_UNSUPPORTED, "allowedLateness re-fire: more than 2^24 fired, uncleaned windows");
    const uint32_t nj = (uint32_t)(j_fire - j_clean);
    const uint64_t per = std::min<uint64_t>((uint64_t)((cfg.size + cfg.slide - 1) / cfg.slide), nj);
    const uint64_t mmax = std::max<uint64_t>(records * per, 1);
    uint64_t kcap = 64;
    while (kcap < 2 * records) kcap <<= 1;
    const unsigned __int128 groups = (unsigned __int128)(kcap + 1) * nj;
    if (groups >= ((unsigned __int128)1 << 32))
        return poison(GWO_ERR_CAPACITY, "allowedLateness re-fire: (re-fire keys x fired windows) exceeds 2^32");
    int bits = 8;
    while (bits < 32 && ((unsigned __int128)1 << bits) < groups) bits += 8;
    const long long pane_base = win_first_pane(j_clean), pane_hi = win_last_pane(j_fire - 1);
    const long long pane_len = pane_hi - pane_base + 1;
    if (pane_len <= 0 || pane_len > (1LL << 24))
        return fail(GWO_ERR_UNSUPPORTED, "allowedLateness re-fire: fired windows span more than 2^24 panes");
    std::vector<TableDesc> pdir((size_t)pane_len, TableDesc{});
    for (auto it = tables.lower_bound(pane_base); it != tables.end() && it->first <= pane_hi; ++it)
        pdir[(size_t)(it->first - pane_base)] = desc(it->second);
    // restored windows' entries (pending, fired) of the fired, uncleaned windows [j_clean, j_fire)
    std::vector<TableDesc> wdir;
    for (auto it = S.rwin.lower_bound((long long)j_clean); it != S.rwin.end() && it->first < (long long)j_fire; ++it) {
        if (wdir.empty()) wdir.assign((size_t)nj * 2, TableDesc{});
        const size_t d = (size_t)(it->first - (long long)j_clean);
        if (it->second.pend.base) wdir[2 * d] = desc(it->second.pend);
        if (it->second.done.base) wdir[2 * d + 1] = desc(it->second.done);
    }
    const uint64_t rs_blocks = (mmax + 4095) / 4096;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    // carve: blk[256] u32 | pdir | wdir | r_idx[m] | r_u[m] | before[m][MAX_WORDS] | r_slot, k1, v1, k2, v2 [m] u32 |
    //        hist | keytab[kcap] u64
    const size_t o_blk = 0, o_pdir = 1024, o_wdir = up(o_pdir + (size_t)pane_len * sizeof(TableDesc));
    const size_t o_idx = up(o_wdir + wdir.size() * sizeof(TableDesc));
    const size_t o_u = o_idx + mmax * 8, o_before = o_u + mmax * 8, o_slot = o_before + mmax * GWO_MAX_WORDS * 8;
    const size_t o_k1 = o_slot + mmax * 4, o_v1 = o_k1 + mmax * 4, o_k2 = o_v1 + mmax * 4, o_v2 = o_k2 + mmax * 4;
    const size_t o_hist = up(o_v2 + mmax * 4), o_keys = up(o_hist + 256 * 4 * rs_blocks), total = o_keys + kcap * 8;
    GWO_TRY(ensure_buf(refire_buf, total));
    char *b = (char *)refire_buf.ptr;
    GWO_TRY(hipcheck(hipMemcpyAsync(b + o_pdir, pdir.data(), (size_t)pane_len * sizeof(TableDesc),
                                    hipMemcpyHostToDevice, stream), "refire panes"));
    if (!wdir.empty())
        GWO_TRY(hipcheck(hipMemcpyAsync(b + o_wdir, wdir.data(), wdir.size() * sizeof(TableDesc), hipMemcpyHostToDevice,
                                        stream), "refire windows"));
    GWO_TRY(hipcheck(hipMemsetAsync(b + o_keys, 0, kcap * 8, stream), "refire keys"));
    launch_refire_collect(t, n, g, 0, 0, (uint32_t *)(b + o_blk), (int64_t *)(b + o_idx), (long long *)(b + o_u),
                          stream);
    GWO_TRY(launch_ok("refire collect"));
    std::vector<uint32_t> blk(256);
    GWO_TRY(hipcheck(hipMemcpyAsync(blk.data(), b + o_blk, 256 * 4, hipMemcpyDeviceToHost, stream), "refire count"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "refire count"));
    uint64_t m = 0;
    for (uint32_t c : blk) m += c;
    if (m == 0 || m > mmax) return poison(GWO_ERR_HIP, "allowedLateness re-fire: pair count disagrees with the scan");
    launch_slide_refire_slots(k, (const int64_t *)(b + o_idx), (const long long *)(b + o_u), (int64_t)m, plan, g,
                              (unsigned long long *)(b + o_keys), kcap - 1, (long long)j_clean, nj,
                              (const TableDesc *)(b + o_pdir), pane_base, pane_len,
                              wdir.empty() ? nullptr : (const TableDesc *)(b + o_wdir), (uint32_t *)(b + o_slot),
                              (int64_t *)(b + o_before), stream);
    GWO_TRY(launch_ok("refire slots"));
    const int which = radix_sort_pairs((const uint32_t *)(b + o_slot), nullptr, (int64_t)m, bits,
                                       (uint32_t *)(b + o_k1), (uint32_t *)(b + o_v1), (uint32_t *)(b + o_k2),
                                       (uint32_t *)(b + o_v2), (uint32_t *)(b + o_hist), stream);
    GWO_TRY(launch_ok("refire sort"));
    GWO_TRY(ensure_output(m));
    const uint32_t *sk = (const uint32_t *)(b + (which ? o_k2 : o_k1));
    const uint32_t *sp = (const uint32_t *)(b + (which ? o_v2 : o_v1));
    launch_refire_emit(k, v, (const int64_t *)(b + o_idx), (const long long *)(b + o_u), (int64_t)m, sk, sp,
                       (const int64_t *)(b + o_before), plan, rplan, cfg.slide, S.om, cfg.size, out_cols(), stream);
    GWO_TRY(launch_ok("refire emit"));
    out_rows += m;
    return GWO_OK;
}

}  // namespace gwo
