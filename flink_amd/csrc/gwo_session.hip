// gwo_session.hip -- EventTimeSessionWindows on gfx950.
//
// Reference: WindowOperator.processElement's merging branch (WindowOperator.java:303-383),
// MergingWindowSet.addWindow (MergingWindowSet.java:156-225), TimeWindow.mergeWindows/intersects
// (TimeWindow.java:120-129, 217-262), EventTimeTrigger.onElement/onMerge (EventTimeTrigger.java:37-81)
// and onEventTime/clearAllState (WindowOperator.java:430-473, 528-540).
//
// State: one HBM hash-table entry per key holding that key's in-flight sessions inline:
//   word 0 key | word 1 number of sessions | smax x [start, end, flags, acc words...]
// (flags bit 0 = an event-time timer at maxTimestamp is pending).  In-flight sessions of a key are
// pairwise non-intersecting (every addWindow merges all intersecting windows), so merging a new
// window touches a contiguous run of them.
//
// A batch is processed key-parallel but arrival-ordered within a key: records are grouped by
// their key's table slot with a stable radix sort (gwo_sort.hip) and one lane walks each key's
// records in order.  That keeps the reference's order-dependent cases exact (an on-time record
// arriving after a late one can bridge sessions; allowedLateness > 0 re-fires).
#include "gwo_device.h"

namespace gwo {

__device__ __forceinline__ int64_t *entry_ptr(const TableDesc &t, uint32_t slot, int stride, uint64_t cap) {
    return slot < cap ? t.base + (uint64_t)slot * stride : t.side;
}

// pass 1: slot of every record's key (claims entries for new keys)
__global__ __launch_bounds__(256) void sess_slot_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                        int64_t n, TableDesc t, uint64_t cap, int stride, SessGeom g,
                                                        uint32_t *__restrict__ rec_slot, SessErr *err) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        int64_t k = key[i];
        if (ts[i] == GWO_LONG_MIN) atomicAdd(&err->bad_ts, 1ull);
        int32_t kg = key_group(k, g.key_kind, g.max_par);
        if (kg < g.kg_lo || kg > g.kg_hi) {
            atomicAdd(&err->bad_kg, 1ull);
            err->bad_kg_key = k;
        }
        bool claimed;
        int64_t *a = find_or_insert(t, stride, k, claimed);
        count_claims(t.occ, claimed);
        rec_slot[i] = k == GWO_EMPTY_KEY ? (uint32_t)cap : (uint32_t)((a - 1 - t.base) / stride);
    }
}

__device__ __forceinline__ void emit_row(const OutCols &o, const AccPlan &p, const ResultPlan &rp, int64_t key,
                                         int64_t start, int64_t end, const int64_t *acc) {
    unsigned long long pos = atomicAdd(o.count, 1ull);
    if ((long long)pos >= o.cap) return;
    o.key[pos] = key;
    o.start[pos] = start;
    o.end[pos] = end;
    for (int a = 0; a < rp.naggs; ++a) {
        int w = rp.word[a];
        int64_t r;
        switch (rp.kind[a]) {
            case 2:
            case 3: r = rp.value_is_f64 ? f64_from_order_key(acc[w]) : acc[w]; break;
            case 4: {
                double s = rp.value_is_f64 ? __longlong_as_double(acc[w]) : (double)acc[w];
                r = __double_as_longlong(s / (double)acc[w + 1]);
                break;
            }
            default: r = acc[w]; break;
        }
        o.res[a][pos] = r;
    }
}

#define SESS_MAXS 16
#define SESS_MAXW (3 + GWO_MAX_WORDS)

// pass 2: one lane per key, records in arrival order
__global__ __launch_bounds__(64) void sess_process_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                          const int64_t *__restrict__ val, int64_t n,
                                                          const uint32_t *__restrict__ sorted_slot,
                                                          const uint32_t *__restrict__ sorted_idx, TableDesc t,
                                                          uint64_t cap, int stride, AccPlan p, ResultPlan rp, SessGeom g,
                                                          OutCols o, SessErr *err, int64_t *side_key, int64_t *side_ts,
                                                          int64_t *side_val, unsigned long long *side_count,
                                                          long long side_cap) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int sw = 3 + p.nwords;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += step) {
        uint32_t slot = sorted_slot[q];
        if (q > 0 && sorted_slot[q - 1] == slot) continue;  // not the head of this key's run
        int64_t *e = entry_ptr(t, slot, stride, cap);
        int ns = (int)e[1];
        int64_t S[SESS_MAXS][SESS_MAXW];  // start, end, flags, acc...
        for (int s = 0; s < ns; ++s)
            for (int w = 0; w < sw; ++w) S[s][w] = e[2 + s * sw + w];
        long long created = 0;
        bool dirty = false;
        for (int64_t r = q; r < n && sorted_slot[r] == slot; ++r) {
            const uint32_t i = sorted_idx[r];
            const int64_t k = key[i], tsi = ts[i];
            const int64_t v = val ? val[i] : 0;
            if (tsi == GWO_LONG_MIN) continue;  // the whole batch is rejected by the host
            const int64_t ws = tsi, we = jadd(tsi, g.gap);
            // in-flight sessions intersecting [ws, we) (TimeWindow.intersects is inclusive)
            int64_t ms = ws, me = we;
            int nm = 0, first = -1;
            for (int s = 0; s < ns; ++s) {
                if (S[s][0] <= we && S[s][1] >= ws) {
                    if (first < 0) first = s;
                    nm++;
                    ms = S[s][0] < ms ? S[s][0] : ms;
                    me = S[s][1] > me ? S[s][1] : me;
                }
            }
            int actual;
            bool fresh = false;
            if (nm == 0) {
                if (ns >= g.smax) {
                    atomicAdd(&err->capacity, 1ull);
                    continue;
                }
                actual = ns++;
                S[actual][0] = ws;
                S[actual][1] = we;
                S[actual][2] = 0;
                for (int w = 0; w < p.nwords; ++w) S[actual][3 + w] = p.ident[w];
                fresh = true;
                created++;
            } else if (nm == 1 && S[first][0] == ms && S[first][1] == me) {
                actual = first;  // new window inside an existing session: no merge callback
            } else {
                int64_t rmax = jsub(me, 1);
                if (jadd(rmax, g.lateness) <= g.wm) {  // WindowOperator.java:318-323
                    atomicAdd(&err->merge_late, 1ull);
                    continue;
                }
                // mergeNamespaces: fold every merged session into the first
                int64_t acc[GWO_MAX_WORDS];
                for (int w = 0; w < p.nwords; ++w) acc[w] = p.ident[w];
                int keep = 0;
                for (int s = 0; s < ns; ++s) {
                    bool m = S[s][0] <= we && S[s][1] >= ws;
                    if (m) {
                        for (int w = 0; w < p.nwords; ++w) acc[w] = combine(p.op[w], acc[w], S[s][3 + w]);
                    } else {
                        if (keep != s)
                            for (int w = 0; w < sw; ++w) S[keep][w] = S[s][w];
                        keep++;
                    }
                }
                created -= nm - 1;
                ns = keep + 1;
                actual = keep;
                S[actual][0] = ms;
                S[actual][1] = me;
                S[actual][2] = rmax > g.wm ? 1 : 0;  // EventTimeTrigger.onMerge: timer iff maxTs > watermark
                for (int w = 0; w < p.nwords; ++w) S[actual][3 + w] = acc[w];
            }
            dirty = true;
            const int64_t amax = jsub(S[actual][1], 1);
            if (cleanup_time(amax, g.lateness) <= g.wm) {  // isWindowLate -> retireWindow
                if (fresh) {
                    ns--;
                    created--;
                }
                if (jadd(tsi, g.lateness) <= g.wm) {       // isElementLate
                    atomicAdd(&err->late, 1ull);
                    if (g.side_enabled) {
                        unsigned long long pos = atomicAdd(side_count, 1ull);
                        if ((long long)pos < side_cap) {
                            side_key[pos] = k;
                            side_ts[pos] = tsi;
                            side_val[pos] = v;
                        }
                    }
                }
                continue;
            }
            for (int w = 0; w < p.nwords; ++w) S[actual][3 + w] = combine(p.op[w], S[actual][3 + w], lift_word(p, w, v));
            if (amax <= g.wm) {
                emit_row(o, p, rp, k, S[actual][0], S[actual][1], &S[actual][3]);  // onElement FIRE
                atomicAdd(&err->emitted, 1ull);
            } else {
                S[actual][2] = 1;                                                 // registerEventTimeTimer
            }
        }
        if (dirty) {
            e[1] = ns;
            for (int s = 0; s < ns; ++s)
                for (int w = 0; w < sw; ++w) e[2 + s * sw + w] = S[s][w];
            if (created) atomicAdd(&err->live_delta, (unsigned long long)created);
        }
    }
}

// watermark: fire pending timers <= wm, clear sessions whose cleanup time <= wm
__global__ __launch_bounds__(256) void sess_fire_kernel(TableDesc t, uint64_t cap, int stride, AccPlan p, ResultPlan rp,
                                                        SessGeom g, OutCols o, SessErr *err) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const int sw = 3 + p.nwords;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= cap; i += step) {
        int64_t *e;
        int64_t k;
        if (i < cap) {
            e = t.base + i * (uint64_t)stride;
            k = e[0];
            if (k == GWO_EMPTY_KEY) continue;
        } else {
            e = t.side;
            if (e[0] == 0) continue;
            k = GWO_EMPTY_KEY;
        }
        int ns = (int)e[1];
        if (ns == 0) continue;
        int keep = 0;
        long long removed = 0;
        for (int s = 0; s < ns; ++s) {
            int64_t *S = e + 2 + s * sw;
            int64_t mx = jsub(S[1], 1);
            bool changed = false;
            if ((S[2] & 1) && mx <= g.wm) {
                emit_row(o, p, rp, k, S[0], S[1], S + 3);
                atomicAdd(&err->emitted, 1ull);
                S[2] &= ~1ll;
                changed = true;
            }
            (void)changed;
            if (cleanup_time(mx, g.lateness) <= g.wm) {
                removed++;
                continue;
            }
            if (keep != s)
                for (int w = 0; w < sw; ++w) e[2 + keep * sw + w] = S[w];
            keep++;
        }
        if (keep != ns) e[1] = keep;
        if (removed) atomicAdd(&err->live_delta, (unsigned long long)(-removed));
    }
}

// compaction: copy keys that still hold sessions into a fresh table
__global__ __launch_bounds__(256) void sess_compact_kernel(TableDesc src, uint64_t cap, TableDesc dst, int stride) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += step) {
        int64_t *e = src.base + i * (uint64_t)stride;
        int64_t k = e[0];
        if (k == GWO_EMPTY_KEY || e[1] == 0) continue;
        bool claimed;
        int64_t *a = find_or_insert(dst, stride, k, claimed) - 1;
        count_claims(dst.occ, claimed);
        for (int w = 1; w < stride; ++w) a[w] = e[w];
    }
}

// ---- launchers -------------------------------------------------------------------------------------
static inline int sgrid(int64_t n, int threads, int cap) {
    int64_t g = (n + threads - 1) / threads;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

void launch_sess_slot(const int64_t *key, const int64_t *ts, int64_t n, const TableDesc &t, uint64_t cap, int stride,
                      const SessGeom &g, uint32_t *rec_slot, SessErr *err, hipStream_t s) {
    hipLaunchKernelGGL(sess_slot_kernel, dim3(sgrid(n, 256, 8192)), dim3(256), 0, s, key, ts, n, t, cap, stride, g,
                       rec_slot, err);
}

void launch_sess_process(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const uint32_t *sslot,
                         const uint32_t *sidx, const TableDesc &t, uint64_t cap, int stride, const AccPlan &p,
                         const ResultPlan &rp, const SessGeom &g, OutCols o, SessErr *err, int64_t *sk, int64_t *st,
                         int64_t *sv, unsigned long long *sc, long long scap, hipStream_t s) {
    hipLaunchKernelGGL(sess_process_kernel, dim3(sgrid(n, 64, 65536)), dim3(64), 0, s, key, ts, val, n, sslot, sidx,
                       t, cap, stride, p, rp, g, o, err, sk, st, sv, sc, scap);
}

void launch_sess_fire(const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const ResultPlan &rp,
                      const SessGeom &g, OutCols o, SessErr *err, hipStream_t s) {
    hipLaunchKernelGGL(sess_fire_kernel, dim3(sgrid((int64_t)cap + 1, 256, 8192)), dim3(256), 0, s, t, cap, stride,
                       p, rp, g, o, err);
}

void launch_sess_compact(const TableDesc &src, uint64_t cap, const TableDesc &dst, int stride, hipStream_t s) {
    hipLaunchKernelGGL(sess_compact_kernel, dim3(sgrid((int64_t)cap, 256, 8192)), dim3(256), 0, s, src, cap, dst,
                       stride);
}

}  // namespace gwo
