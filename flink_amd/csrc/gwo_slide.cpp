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

namespace gwo {

struct SlideState {
    bool ring = false;
    int count_word = -1;          // hidden per-entry count (ring): presence of a key in window J
    int t_idx = -1;               // aux_tables index of T
    bool j_set = false;
    __int128 J = 0;               // next window to fire
    unsigned long long *d_live = nullptr;
    unsigned long long h_live = 0;
    int64_t om = 0;               // floorMod(offset, slide): window j starts at j*slide + om
};

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
    if (cfg.allowed_lateness != 0)
        return fail(GWO_ERR_UNSUPPORTED, "sliding windows with allowedLateness > 0 are not in the GPU subset");
    slide = new SlideState();
    SlideState &S = *slide;
    S.om = fmod64(cfg.offset, cfg.slide);
    bool all_add = true;
    for (int w = 0; w < plan.nwords; ++w) all_add &= plan.op[w] == ACC_ADD_I64;
    S.ring = all_add && getenv("GWO_SLIDE_RECOMPUTE") == nullptr;
    if (S.ring) {
        if (plan.nwords >= GWO_MAX_WORDS) return fail(GWO_ERR_UNSUPPORTED, "too many accumulator words");
        S.count_word = plan.nwords;
        plan.op[plan.nwords] = ACC_ADD_I64;
        plan.src[plan.nwords] = SRC_ONE;
        plan.ident[plan.nwords] = 0;
        plan.nwords++;
        plan.stride = ((1 + plan.nwords) + 1) & ~1;
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

gwo_status Handle::fire_sliding(int64_t new_wm) {
    SlideState &S = *slide;
    // first window that is not fired at new_wm: start_j + size - 1 > wm
    __int128 j_new = fdiv128((__int128)new_wm - cfg.size + 1 - S.om, cfg.slide) + 1;
    // keep window starts representable: start_j + size must not overflow a long
    const __int128 j_lo = fdiv128((__int128)GWO_LONG_MIN_H + 2 * (__int128)cfg.size + cfg.slide, cfg.slide);
    const __int128 j_hi = fdiv128((__int128)GWO_LONG_MAX_H - 2 * (__int128)cfg.size - cfg.slide, cfg.slide);
    j_new = std::max(j_lo, std::min(j_hi, j_new));
    if (!S.j_set) {
        // anchor: windows before j_new have fired (were empty); the first window with data may be earlier
        S.J = j_new;
        if (!tables.empty()) S.J = std::min(first_window_of_pane(tables.begin()->first), j_new);
        S.j_set = true;
        if (S.ring) GWO_TRY(ring_rebuild());
    }
    OutCols o = out_cols();
    while (S.J < j_new) {
        // ---- skip windows that hold no data ----
        long long lo = win_first_pane(S.J), hi = win_last_pane(S.J);
        bool empty;
        if (S.ring) {
            GWO_TRY(hipcheck(hipMemcpyAsync(&S.h_live, S.d_live, 8, hipMemcpyDeviceToHost, stream), "live"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "live sync"));
            empty = S.h_live == 0;
        } else {
            auto it = tables.lower_bound(lo);
            empty = it == tables.end() || it->first > hi;
        }
        if (empty) {
            __int128 target = j_new;
            auto it = tables.lower_bound(lo);
            if (it != tables.end()) target = std::min(j_new, std::max(S.J + 1, first_window_of_pane(it->first)));
            // panes before the target window are in no unfired window any more
            GWO_TRY(release_panes_before(win_first_pane(target)));
            S.J = target;
            if (S.ring) GWO_TRY(ring_rebuild());
            continue;
        }
        const int64_t start = win_start(S.J);
        const int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
        // ---- emit window J ----
        if (S.ring) {
            Table &T = aux_tables[S.t_idx];
            GWO_TRY(ensure_output(S.h_live));
            o = out_cols();
            prof_begin(GWO_KERNEL_FIRE);
            launch_fire(desc(T), T.cap, plan, rplan, start, end, o, 0, S.count_word, stream);
            prof_end(GWO_KERNEL_FIRE, (int64_t)T.cap);
            out_rows += S.h_live;
        } else {
            uint64_t total = 0;
            GWO_TRY(read_occupancy());
            for (auto it = tables.lower_bound(lo); it != tables.end() && it->first <= hi; ++it) total += it->second.occ;
            Table W;
            uint64_t cap = kMinCap;
            while ((double)total > kInitLoad * (double)cap) cap <<= 1;
            GWO_TRY(alloc_table(cap, W));
            prof_begin(GWO_KERNEL_SLIDE);
            for (auto it = tables.lower_bound(lo); it != tables.end() && it->first <= hi; ++it)
                launch_fold(desc(it->second), it->second.cap, desc(W), plan, +1, -1, nullptr, stream);
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
        GWO_TRY(release_panes_before(nlo));
        S.J += 1;
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
        release_table(t);
        it = tables.erase(it);
    }
    return GWO_OK;
}

}  // namespace gwo
