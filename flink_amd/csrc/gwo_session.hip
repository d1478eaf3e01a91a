// gwo_session.hip -- EventTimeSessionWindows on gfx950.
//
// Reference: WindowOperator.processElement's merging branch (WindowOperator.java:303-383),
// MergingWindowSet.addWindow (MergingWindowSet.java:156-225), TimeWindow.mergeWindows/intersects
// (TimeWindow.java:120-129, 217-262), EventTimeTrigger.onElement/onMerge (EventTimeTrigger.java:37-81)
// and onEventTime/clearAllState (WindowOperator.java:430-473, 528-540).
//
// State: one HBM hash-table entry per key holding that key's in-flight sessions inline:
//   word 0 key | word 1 number of sessions | smax x [start, end, flags, acc words...]
// (flags bit 0 = an event-time timer at maxTimestamp is pending).  A key with more in-flight sessions
// than its entry holds spills them into a pool array (word 1 = -1, words 2..4 = pool record, capacity,
// count; SessGeom): MergingWindowSet (MergingWindowSet.java:156-225) bounds nothing per key, nor does
// this.  In-flight sessions of a key are pairwise non-intersecting (every addWindow merges all
// intersecting windows).
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

// One output row at a reserved position (rows past the output capacity are counted, not written).
__device__ __forceinline__ void emit_row_at(const OutCols &o, const AccPlan &p, const ResultPlan &rp,
                                            unsigned long long pos, int64_t key, int64_t start, int64_t end,
                                            const int64_t *acc) {
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

__device__ __forceinline__ void emit_row(const OutCols &o, const AccPlan &p, const ResultPlan &rp, int64_t key,
                                         int64_t start, int64_t end, const int64_t *acc) {
    emit_row_at(o, p, rp, atomicAdd(o.count, 1ull), key, start, end, acc);
}

#define SESS_MAXS 16
#define SESS_MAXW (3 + GWO_MAX_WORDS)

// The earliest watermark at which an entry's sessions need the fire sweep: a pending event-time timer fires at
// maxTimestamp = end - 1 (EventTimeTrigger.onEventTime), a session retires at cleanupTime(maxTimestamp)
// (WindowOperator.java:528-540).  The sweep only visits slots whose value the watermark reached.
__device__ __forceinline__ int64_t sess_due(const int64_t *S, int ns, int sw, int64_t lateness) {
    int64_t d = SESS_NONE;
    for (int s = 0; s < ns; ++s) {
        const int64_t mx = jsub(S[s * sw + 1], 1);
        const int64_t t = (S[s * sw + 2] & 1) ? mx : cleanup_time(mx, lateness);
        d = t < d ? t : d;
    }
    return d;
}

// Moves a key's session list into a fresh pool array of at least `want` sessions (doubling); returns the
// array or nullptr when the pool is exhausted (the host sizes the pool so that cannot happen).
__device__ __forceinline__ int64_t *sess_grow(const SessGeom &g, const int64_t *S, int ns, int sw, int want,
                                              int64_t &off, int &scap) {
    const unsigned long long o = atomicAdd(g.pool_top, (unsigned long long)want);
    if (o + (unsigned long long)want > g.pool_cap) return nullptr;
    int64_t *dst = g.pool + o * (unsigned long long)sw;
    for (int i = 0; i < ns * sw; ++i) dst[i] = S[i];
    off = (int64_t)o;
    scap = want;
    return dst;
}

// pass 2: one lane per key, records in arrival order
__global__ __launch_bounds__(64) void sess_process_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                          const int64_t *__restrict__ val, int64_t n,
                                                          const uint32_t *__restrict__ sorted_slot,
                                                          const uint32_t *__restrict__ sorted_idx, TableDesc t,
                                                          uint64_t cap, int stride, AccPlan p, ResultPlan rp, SessGeom g,
                                                          OutCols o, SessErr *err, int64_t *side_key, int64_t *side_ts,
                                                          int64_t *side_val, unsigned long long *side_count,
                                                          long long side_cap) {
    extern __shared__ int64_t s_L[];   // [64][smax * sw]: each lane's copy of its key's inline sessions
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int sw = 3 + p.nwords;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += step) {
        uint32_t slot = sorted_slot[q];
        if (q > 0 && sorted_slot[q - 1] == slot) continue;  // not the head of this key's run
        int64_t *e = entry_ptr(t, slot, stride, cap);
        // the key's session list: the inline sessions copied into L (written back at the end), or its pool array
        // in this lane's LDS slice (a private array indexed at run time would live in scratch memory)
        int64_t *L = s_L + (size_t)threadIdx.x * g.smax * sw;
        int64_t *S = L;
        int ns, scap = g.smax;
        int64_t off = 0;
        bool spilled = e[1] < 0;
        if (spilled) {
            off = e[2];
            scap = (int)e[3];
            ns = (int)e[4];
            S = g.pool + (uint64_t)off * sw;
        } else {
            ns = (int)e[1];
            for (int i = 0; i < ns * sw; ++i) L[i] = e[2 + i];
        }
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
                const int64_t *X = S + s * sw;
                if (X[0] <= we && X[1] >= ws) {
                    if (first < 0) first = s;
                    nm++;
                    ms = X[0] < ms ? X[0] : ms;
                    me = X[1] > me ? X[1] : me;
                }
            }
            int actual;
            bool fresh = false;
            if (nm == 0) {
                if (ns >= scap) {   // the list is full: spill (or grow) into a pool array twice its size
                    int64_t *nS = sess_grow(g, S, ns, sw, 2 * scap, off, scap);
                    if (!nS) {
                        atomicAdd(&err->pool_full, 1ull);
                        continue;
                    }
                    S = nS;
                    spilled = true;
                }
                actual = ns++;
                int64_t *X = S + actual * sw;
                X[0] = ws;
                X[1] = we;
                X[2] = 0;
                for (int w = 0; w < p.nwords; ++w) X[3 + w] = p.ident[w];
                fresh = true;
                created++;
            } else if (nm == 1 && S[first * sw] == ms && S[first * sw + 1] == me) {
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
                    const int64_t *X = S + s * sw;
                    bool m = X[0] <= we && X[1] >= ws;
                    if (m) {
                        for (int w = 0; w < p.nwords; ++w) acc[w] = combine(p.op[w], acc[w], X[3 + w]);
                    } else {
                        if (keep != s)
                            for (int w = 0; w < sw; ++w) S[keep * sw + w] = X[w];
                        keep++;
                    }
                }
                created -= nm - 1;
                ns = keep + 1;
                actual = keep;
                int64_t *X = S + actual * sw;
                X[0] = ms;
                X[1] = me;
                X[2] = rmax > g.wm ? 1 : 0;  // EventTimeTrigger.onMerge: timer iff maxTs > watermark
                for (int w = 0; w < p.nwords; ++w) X[3 + w] = acc[w];
            }
            dirty = true;
            int64_t *A = S + actual * sw;
            const int64_t amax = jsub(A[1], 1);
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
            for (int w = 0; w < p.nwords; ++w) A[3 + w] = combine(p.op[w], A[3 + w], lift_word(p, w, v));
            if (amax <= g.wm) {
                emit_row(o, p, rp, k, A[0], A[1], A + 3);  // onElement FIRE
                atomicAdd(&err->emitted, 1ull);
            } else {
                A[2] = 1;                                  // registerEventTimeTimer
            }
        }
        if (dirty) {
            if (spilled) {
                e[1] = -1;
                e[2] = off;
                e[3] = scap;
                e[4] = ns;
            } else {
                e[1] = ns;
                for (int i = 0; i < ns * sw; ++i) e[2 + i] = L[i];
            }
            g.due[slot < cap ? slot : cap] = sess_due(S, ns, sw, g.lateness);
            if (created) atomicAdd(&err->live_delta, (unsigned long long)created);
        }
    }
}

// watermark: fire pending timers <= wm, clear sessions whose cleanup time <= wm
// Persistent workgroups (about one per CU) sweep the slots in rounds of SF_SPT slots per thread; a round counts
// its rows first and reserves them with ONE returning atomic per workgroup (block_reserve), then emits.  A
// reservation per wave or per row serialised on the shared row counter: ~180 us per watermark at C5's ~5K
// fired sessions, for a kernel that does a few microseconds of work.  Statistics: one add per workgroup.
#define SF_SPT 8
__device__ __forceinline__ int64_t *sess_slot_entry(const TableDesc &t, uint64_t cap, int stride, uint64_t i,
                                                    int64_t &k) {
    if (i < cap) {
        int64_t *e = t.base + i * (uint64_t)stride;
        k = e[0];
        return k == GWO_EMPTY_KEY ? nullptr : e;
    }
    k = GWO_EMPTY_KEY;
    return t.side[0] == 0 ? nullptr : t.side;
}

__global__ __launch_bounds__(256) void sess_fire_kernel(TableDesc t, uint64_t cap, int stride, AccPlan p, ResultPlan rp,
                                                        SessGeom g, OutCols o, SessErr *err) {
    const int sw = 3 + p.nwords;
    const uint64_t span = (uint64_t)gridDim.x * 256;   // slots one pass of the grid covers
    unsigned long long emitted = 0;
    long long removed_all = 0;
    // rounds are workgroup-uniform (block_reserve synchronises the workgroup)
    for (uint64_t r0 = 0; r0 <= cap; r0 += span * SF_SPT) {
        unsigned due_m = 0, nrow = 0;
        // the round's due words load together (most slots are not due: one round trip for all of them)
        bool due[SF_SPT];
#pragma unroll
        for (int j = 0; j < SF_SPT; ++j) {
            const uint64_t i = r0 + (uint64_t)j * span + (uint64_t)blockIdx.x * 256 + threadIdx.x;
            const int64_t dv = g.due[i <= cap ? i : cap];   // unconditional (clamped): no branch between the loads
            due[j] = i <= cap && dv <= g.wm;
        }
#pragma unroll
        for (int j = 0; j < SF_SPT; ++j) {
            const uint64_t i = r0 + (uint64_t)j * span + (uint64_t)blockIdx.x * 256 + threadIdx.x;
            if (!due[j]) continue;   // a slot whose due watermark is ahead: nothing to do
            int64_t k;
            const int64_t *e = sess_slot_entry(t, cap, stride, i, k);
            if (!e) continue;
            const bool spilled = e[1] < 0;
            const int ns = spilled ? (int)e[4] : (int)e[1];
            const int64_t *base = spilled ? g.pool + (uint64_t)e[2] * sw : e + 2;
            for (int s = 0; s < ns; ++s)   // rows: pending timers at maxTs <= wm (EventTimeTrigger.onEventTime)
                nrow += (base[s * sw + 2] & 1) && jsub(base[s * sw + 1], 1) <= g.wm;
            if (ns) due_m |= 1u << j;
        }
        unsigned long long pos = block_reserve(nrow, o.count);
        emitted += nrow;
#pragma unroll
        for (int j = 0; j < SF_SPT; ++j) {
            if (!((due_m >> j) & 1u)) continue;
            const uint64_t i = r0 + (uint64_t)j * span + (uint64_t)blockIdx.x * 256 + threadIdx.x;
            int64_t k;
            int64_t *e = sess_slot_entry(t, cap, stride, i, k);
            const bool spilled = e[1] < 0;
            const int ns = spilled ? (int)e[4] : (int)e[1];
            int64_t *base = spilled ? g.pool + (uint64_t)e[2] * sw : e + 2;
            int keep = 0;
            for (int s = 0; s < ns; ++s) {
                int64_t *S = base + s * sw;
                const int64_t mx = jsub(S[1], 1);
                if ((S[2] & 1) && mx <= g.wm) {
                    emit_row_at(o, p, rp, pos++, k, S[0], S[1], S + 3);
                    S[2] &= ~1ll;
                }
                if (cleanup_time(mx, g.lateness) <= g.wm) {
                    removed_all++;
                    continue;
                }
                if (keep != s)
                    for (int w = 0; w < sw; ++w) base[keep * sw + w] = S[w];
                keep++;
            }
            if (keep != ns) {
                if (!spilled) e[1] = keep;
                else if (keep == 0) e[1] = 0;   // every spilled session retired: the key is inline (and empty) again
                else e[4] = keep;
            }
            g.due[i] = sess_due(base, keep, sw, g.lateness);
        }
    }
    // workgroup totals: one add each
    __shared__ unsigned long long s_e[4];
    __shared__ long long s_r[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
        emitted += __shfl_xor(emitted, o2);
        removed_all += __shfl_xor(removed_all, o2);
    }
    if (lane == 0) {
        s_e[wid] = emitted;
        s_r[wid] = removed_all;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long e = s_e[0] + s_e[1] + s_e[2] + s_e[3];
        const long long r = s_r[0] + s_r[1] + s_r[2] + s_r[3];
        if (e) atomicAdd(&err->emitted, e);
        if (r) atomicAdd(&err->live_delta, (unsigned long long)(-r));
    }
}

// Every slot's due watermark from its entry (after a compaction or a restore wrote entries directly).
__global__ __launch_bounds__(256) void sess_due_kernel(TableDesc t, uint64_t cap, int stride, int sw, SessGeom g) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= cap; i += step) {
        const int64_t *e = i < cap ? t.base + i * (uint64_t)stride : t.side;
        int64_t d = SESS_NONE;
        if (i < cap ? e[0] != GWO_EMPTY_KEY : e[0] != 0) {
            const bool spilled = e[1] < 0;
            const int ns = spilled ? (int)e[4] : (int)e[1];
            d = sess_due(spilled ? g.pool + (uint64_t)e[2] * sw : e + 2, ns, sw, g.lateness);
        }
        g.due[i] = d;
    }
}

// compaction: copy keys that still hold sessions into a fresh table
__global__ __launch_bounds__(256) void sess_compact_kernel(TableDesc src, uint64_t cap, TableDesc dst, int stride) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += step) {
        int64_t *e = src.base + i * (uint64_t)stride;
        int64_t k = e[0];
        if (k == GWO_EMPTY_KEY || e[1] == 0) continue;   // (e[1] < 0: spilled, kept with its pool reference)
        bool claimed;
        int64_t *a = find_or_insert(dst, stride, k, claimed) - 1;
        count_claims(dst.occ, claimed);
        for (int w = 1; w < stride; ++w) a[w] = e[w];
    }
}

// pool compaction: every spilled list moves to a fresh pool (capacity 2 x its count, at least 2 x smax)
__global__ __launch_bounds__(256) void sess_pool_compact_kernel(TableDesc t, uint64_t cap, int stride, int sw,
                                                                const int64_t *__restrict__ old_pool, SessGeom g) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= cap; i += step) {
        int64_t *e = i < cap ? t.base + i * (uint64_t)stride : t.side;
        if (i < cap ? e[0] == GWO_EMPTY_KEY : e[0] == 0) continue;
        if (e[1] >= 0) continue;
        const int ns = (int)e[4];
        const int want = 2 * ns > 2 * g.smax ? 2 * ns : 2 * g.smax;
        const unsigned long long o = atomicAdd(g.pool_top, (unsigned long long)want);
        const int64_t *src = old_pool + (uint64_t)e[2] * sw;
        int64_t *dst = g.pool + o * (uint64_t)sw;
        for (int k = 0; k < ns * sw; ++k) dst[k] = src[k];
        e[2] = (int64_t)o;
        e[3] = want;
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
    const size_t lds = (size_t)64 * g.smax * (3 + p.nwords) * 8;
    hipLaunchKernelGGL(sess_process_kernel, dim3(sgrid(n, 64, 65536)), dim3(64), lds, s, key, ts, val, n, sslot, sidx,
                       t, cap, stride, p, rp, g, o, err, sk, st, sv, sc, scap);
}

void launch_sess_fire(const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const ResultPlan &rp,
                      const SessGeom &g, OutCols o, SessErr *err, hipStream_t s) {
    // about one workgroup per CU (MI355X: 256), fewer for small tables
    hipLaunchKernelGGL(sess_fire_kernel, dim3(sgrid((int64_t)cap + 1, 256 * SF_SPT, 256)), dim3(256), 0, s, t, cap,
                       stride, p, rp, g, o, err);
}

void launch_sess_pool_compact(const TableDesc &t, uint64_t cap, int stride, int sw, const int64_t *old_pool,
                              const SessGeom &g, hipStream_t s) {
    hipLaunchKernelGGL(sess_pool_compact_kernel, dim3(sgrid((int64_t)cap + 1, 256, 8192)), dim3(256), 0, s, t, cap,
                       stride, sw, old_pool, g);
}

void launch_sess_due(const TableDesc &t, uint64_t cap, int stride, int sw, const SessGeom &g, hipStream_t s) {
    hipLaunchKernelGGL(sess_due_kernel, dim3(sgrid((int64_t)cap + 1, 256, 4096)), dim3(256), 0, s, t, cap, stride, sw,
                       g);
}

void launch_sess_compact(const TableDesc &src, uint64_t cap, const TableDesc &dst, int stride, hipStream_t s) {
    hipLaunchKernelGGL(sess_compact_kernel, dim3(sgrid((int64_t)cap, 256, 8192)), dim3(256), 0, s, src, cap, dst,
                       stride);
}

}  // namespace gwo
