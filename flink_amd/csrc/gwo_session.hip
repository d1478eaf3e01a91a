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
// their key's table slot -- in per-slot buckets filled by the slot pass (SessLists; three launches per
// batch), or, when the host sees many keys overflow their buckets, with a stable radix sort
// (gwo_sort.hip) -- and one lane walks each key's records in order.  That keeps the reference's
// order-dependent cases exact (an on-time record arriving after a late one can bridge sessions;
// allowedLateness > 0 re-fires).
#include "gwo_device.h"

namespace gwo {

__device__ __forceinline__ int64_t *entry_ptr(const TableDesc &t, uint32_t slot, int stride, uint64_t cap) {
    return slot < cap ? t.base + (uint64_t)slot * stride : t.side;
}

// pass 1: slot of every record's key (claims entries for new keys); with lists (SessLists) also the record's place in
// its slot's bucket, and the slot's first record of the batch marked as the one whose lane applies the bucket
// (SESS_OWNER in rec_slot)
template <bool LISTS>
__global__ __launch_bounds__(256) void sess_slot_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                        int64_t n, TableDesc t, uint64_t cap, int stride, SessGeom g,
                                                        uint32_t *__restrict__ rec_slot, SessErr *err, SessLists ls) {
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
        const uint32_t slot = k == GWO_EMPTY_KEY ? (uint32_t)cap : (uint32_t)((a - 1 - t.base) / stride);
        if (LISTS) {
            uint32_t *bk = ls.bkt + (uint64_t)slot * SESS_BKT;
            const uint32_t r = atomicAdd(bk, 1u);
            if (r < SESS_BKT_N) bk[1 + r] = (uint32_t)i;
            rec_slot[i] = slot | (r == 0 ? SESS_OWNER : 0u);
        } else {
            rec_slot[i] = slot;
        }
    }
}

// One output row at a reserved position (rows past the output capacity are counted, not written).
__device__ __forceinline__ void emit_row_at(const OutCols &o, const AccPlan &p, const ResultPlan &rp,
                                            unsigned long long pos, int64_t key, int64_t start, int64_t end,
                                            const int64_t *acc, int ast = 1) {
    if ((long long)pos >= o.cap) return;
    o.key[pos] = key;
    o.start[pos] = start;
    o.end[pos] = end;
    for (int a = 0; a < rp.naggs; ++a) {
        int w = rp.word[a];
        int64_t r;
        switch (rp.kind[a]) {
            case 2:
            case 3: r = rp.value_is_f64 ? f64_from_order_key(acc[w * ast]) : acc[w * ast]; break;
            case 4: {
                double s = rp.value_is_f64 ? __longlong_as_double(acc[w * ast]) : (double)acc[w * ast];
                r = __double_as_longlong(s / (double)acc[(w + 1) * ast]);
                break;
            }
            default: r = acc[w * ast]; break;
        }
        o.res[a][pos] = r;
    }
}

#define SESS_MAXS 16
#define SESS_MAXW (3 + GWO_MAX_WORDS)

// The earliest watermark at which an entry's sessions need the fire sweep: a pending event-time timer fires at
// maxTimestamp = end - 1 (EventTimeTrigger.onEventTime), a session retires at cleanupTime(maxTimestamp)
// (WindowOperator.java:528-540).  The sweep only visits slots whose value the watermark reached.
__device__ __forceinline__ int64_t sess_due(const int64_t *S, int ns, int sw, int64_t lateness, int sst = 1) {
    int64_t d = SESS_NONE;
    for (int s = 0; s < ns; ++s) {
        const int64_t mx = jsub(S[(s * sw + 1) * sst], 1);
        const int64_t t = (S[(s * sw + 2) * sst] & 1) ? mx : cleanup_time(mx, lateness);
        d = t < d ? t : d;
    }
    return d;
}

// Moves a key's session list (element stride sst) into a fresh pool array of at least `want` sessions (doubling);
// returns the array or nullptr when the pool is exhausted (the host sizes the pool so that cannot happen).
__device__ __forceinline__ int64_t *sess_grow(const SessGeom &g, const int64_t *S, int sst, int ns, int sw, int want,
                                              int64_t &off, int &scap) {
    const unsigned long long o = atomicAdd(g.pool_top, (unsigned long long)want);
    if (o + (unsigned long long)want > g.pool_cap) return nullptr;
    int64_t *dst = g.pool + o * (unsigned long long)sw;
    for (int i = 0; i < ns * sw; ++i) dst[i] = S[i * sst];
    off = (int64_t)o;
    scap = want;
    return dst;
}

// One key's session list while a batch's records are applied to it (sess_key_*): the inline sessions copied into
// LDS (written back at the end), or its pool array.  Word i of the list is S[i * sst]: a lane's LDS copy is
// interleaved with its wave's other lanes (sst = 64: word i of lane l at L0[i * 64 + l]), so the lanes of a wave
// touch consecutive words -- a slice per lane (a 256-B stride) put every lane's access on the same LDS bank.  A
// private array indexed at run time would live in scratch memory.
struct SessKey {
    int64_t *e;
    int64_t *L;      // the LDS copy (word i at L[i * lst])
    int64_t *S;      // the list being edited: L, or the key's pool array
    int64_t off;
    int ns, scap;
    int lst, sst;    // element strides of L and of S
    bool spilled, dirty;
    long long created;
};

__device__ __forceinline__ void sess_key_begin(SessKey &K, int64_t *e, int64_t *L, int lst, const SessGeom &g, int sw) {
    K.e = e;
    K.L = L;
    K.lst = lst;
    K.S = L;
    K.sst = lst;
    K.scap = g.smax;
    K.off = 0;
    K.spilled = e[1] < 0;
    K.dirty = false;
    K.created = 0;
    if (K.spilled) {
        K.off = e[2];
        K.scap = (int)e[3];
        K.ns = (int)e[4];
        K.S = g.pool + (uint64_t)K.off * sw;
        K.sst = 1;
    } else {
        K.ns = (int)e[1];
        for (int i = 0; i < K.ns * sw; ++i) L[i * lst] = e[2 + i];
    }
}

// The same with every inline word loaded at once (smax sessions, used or not: one round trip instead of a chain of
// dependent loads), the entry's key and session count in the same round trip.
__device__ __forceinline__ void sess_key_begin_bulk(SessKey &K, int64_t *e, int64_t *L, int lst, const SessGeom &g,
                                                    int sw) {
    const int nwd = g.smax * sw;
    const int64_t e1 = e[1], e2 = e[2], e3 = e[3], e4 = e[4];
    for (int i0 = 0; i0 < nwd; i0 += 16) {   // e + 2 is 16-B aligned (even stride); words past nwd stay in the entry
        longlong2 w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            w[j] = i0 + 2 * j < nwd ? ((const longlong2 *)(e + 2 + i0))[j] : make_longlong2(0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (i0 + 2 * j < nwd) L[(i0 + 2 * j) * lst] = w[j].x;
            if (i0 + 2 * j + 1 < nwd) L[(i0 + 2 * j + 1) * lst] = w[j].y;
        }
    }
    K.e = e;
    K.L = L;
    K.lst = lst;
    K.S = L;
    K.sst = lst;
    K.scap = g.smax;
    K.off = 0;
    K.spilled = e1 < 0;
    K.dirty = false;
    K.created = 0;
    K.ns = (int)e1;
    if (K.spilled) {
        K.off = e2;
        K.scap = (int)e3;
        K.ns = (int)e4;
        K.S = g.pool + (uint64_t)K.off * sw;
        K.sst = 1;
    }
}

// Record (k, tsi, v) applied to its key's sessions: WindowOperator.processElement's merging branch.
// NWT: the plan's accumulator words at compile time (1-4; 0: p.nwords at run time) -- the word loops unroll.
template <int NWT = 0>
__device__ __forceinline__ void sess_key_record(SessKey &K, int64_t k, int64_t tsi, int64_t v, const AccPlan &p,
                                                const ResultPlan &rp, const SessGeom &g, const OutCols &o,
                                                SessErr *err, int64_t *side_key, int64_t *side_ts, int64_t *side_val,
                                                unsigned long long *side_count, long long side_cap, int sw) {
    if (tsi == GWO_LONG_MIN) return;  // the whole batch is rejected by the host
    const int NWP = NWT > 0 ? NWT : p.nwords;
    if (NWT > 0) sw = 3 + NWT;
    const int64_t ws = tsi, we = jadd(tsi, g.gap);
    int64_t *S = K.S;
    int sst = K.sst;
    int ssw = sw * sst;   // one session's step
    int ns = K.ns;
    // in-flight sessions intersecting [ws, we) (TimeWindow.intersects is inclusive)
    int64_t ms = ws, me = we, f0 = 0, f1 = 0;   // (f0, f1): the first intersecting session
    int nm = 0, first = -1;
    for (int s = 0; s < ns; ++s) {
        const int64_t x0 = S[s * ssw], x1 = S[s * ssw + sst];
        if (x0 <= we && x1 >= ws) {
            if (first < 0) {
                first = s;
                f0 = x0;
                f1 = x1;
            }
            nm++;
            ms = x0 < ms ? x0 : ms;
            me = x1 > me ? x1 : me;
        }
    }
    int actual;
    bool fresh = false;
    if (nm == 0) {
        if (ns >= K.scap) {   // the list is full: spill (or grow) into a pool array twice its size
            int64_t *nS = sess_grow(g, S, sst, ns, sw, 2 * K.scap, K.off, K.scap);
            if (!nS) {
                atomicAdd(&err->pool_full, 1ull);
                return;
            }
            S = K.S = nS;
            sst = K.sst = 1;
            ssw = sw;
            K.spilled = true;
        }
        actual = ns++;
        int64_t *X = S + actual * sw * sst;
        X[0] = ws;
        X[sst] = we;
        X[2 * sst] = 0;
        for (int w = 0; w < NWP; ++w) X[(3 + w) * sst] = p.ident[w];
        fresh = true;
        K.created++;
    } else if (nm == 1 && f0 == ms && f1 == me) {
        actual = first;  // new window inside an existing session: no merge callback
    } else {
        int64_t rmax = jsub(me, 1);
        if (jadd(rmax, g.lateness) <= g.wm) {  // WindowOperator.java:318-323
            atomicAdd(&err->merge_late, 1ull);
            return;
        }
        // mergeNamespaces: fold every merged session into the first
        int64_t acc[GWO_MAX_WORDS];
        for (int w = 0; w < NWP; ++w) acc[w] = p.ident[w];
        int keep = 0;
        for (int s = 0; s < ns; ++s) {
            const int64_t *X = S + s * ssw;
            bool m = X[0] <= we && X[sst] >= ws;
            if (m) {
                for (int w = 0; w < NWP; ++w) acc[w] = combine(p.op[w], acc[w], X[(3 + w) * sst]);
            } else {
                if (keep != s)
                    for (int w = 0; w < sw; ++w) S[keep * ssw + w * sst] = X[w * sst];
                keep++;
            }
        }
        K.created -= nm - 1;
        ns = keep + 1;
        actual = keep;
        int64_t *X = S + actual * ssw;
        X[0] = ms;
        X[sst] = me;
        X[2 * sst] = rmax > g.wm ? 1 : 0;  // EventTimeTrigger.onMerge: timer iff maxTs > watermark
        for (int w = 0; w < NWP; ++w) X[(3 + w) * sst] = acc[w];
    }
    K.dirty = true;
    K.ns = ns;
    int64_t *A = S + actual * ssw;
    const int64_t amax = jsub(me, 1);   // the session's end: [ws, we) new, the one it lies in, or the merged one
    if (cleanup_time(amax, g.lateness) <= g.wm) {  // isWindowLate -> retireWindow
        if (fresh) {
            K.ns--;
            K.created--;
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
        return;
    }
    for (int w = 0; w < NWP; ++w) A[(3 + w) * sst] = combine(p.op[w], A[(3 + w) * sst], lift_word(p, w, v));
    if (amax <= g.wm) {
        emit_row_at(o, p, rp, atomicAdd(o.count, 1ull), k, A[0], A[sst], A + 3 * sst, sst);  // onElement FIRE
        atomicAdd(&err->emitted, 1ull);
    } else {
        A[2 * sst] = 1;                            // registerEventTimeTimer
    }
}

// Writes the key's sessions back; returns the change in its number of sessions (summed per wave by the caller:
// one device-scope add per key on one address serialised ~10K adds per batch).
__device__ __forceinline__ long long sess_key_end(SessKey &K, uint32_t slot, uint64_t cap, const SessGeom &g, int sw) {
    if (!K.dirty) return 0;
    int64_t *e = K.e;
    if (K.spilled) {
        e[1] = -1;
        e[2] = K.off;
        e[3] = K.scap;
        e[4] = K.ns;
    } else {
        e[1] = K.ns;
        for (int i = 0; i < K.ns * sw; ++i) e[2 + i] = K.L[i * K.lst];
    }
    g.due[slot < cap ? slot : cap] = sess_due(K.S, K.ns, sw, g.lateness, K.sst);
    return K.created;
}

#define SESS_REC_ARGS p, rp, g, o, err, side_key, side_ts, side_val, side_count, side_cap, sw
#define SESS_REC(i) key[i], ts[i], val ? val[i] : 0

// pass 2: one lane per key, records in arrival order.  LISTS: the lane of each slot's first record (the owner flag
// in rec_slot) loads the bucket, the entry and every bucketed record's timestamp and value at once, then applies the
// records smallest index first (a bucket holds at most SESS_BKT_N records: a slot with more is queued for
// sess_long_kernel); otherwise the slot-sorted records (stable radix sort, gwo_sort.hip), a lane per run head.
#ifndef SESS_PROC_WAVES
#define SESS_PROC_WAVES 1   // waves per process workgroup (each wave its own LDS columns)
#endif
template <bool LISTS, int NWT = 0>
__global__ __launch_bounds__(64 * SESS_PROC_WAVES) void sess_process_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                          const int64_t *__restrict__ val, int64_t n,
                                                          const uint32_t *__restrict__ sorted_slot,
                                                          const uint32_t *__restrict__ sorted_idx, TableDesc t,
                                                          uint64_t cap, int stride, AccPlan p, ResultPlan rp, SessGeom g,
                                                          OutCols o, SessErr *err, int64_t *side_key, int64_t *side_ts,
                                                          int64_t *side_val, unsigned long long *side_count,
                                                          long long side_cap, SessLists ls) {
    extern __shared__ int64_t s_L[];   // [smax * sw][64]: the lanes' copies of their keys' inline sessions, interleaved
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int sw = 3 + (NWT > 0 ? NWT : p.nwords);
    // this wave's LDS columns: [smax * sw + 2 * SESS_BKT_N][64] words per wave
    int64_t *L = s_L + (size_t)(threadIdx.x >> 6) * ((size_t)g.smax * sw + (LISTS ? 2 * SESS_BKT_N : 0)) * 64 +
                 (threadIdx.x & 63);
    unsigned long long nlong = 0;
    long long created = 0;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += step) {
        SessKey K;
        if (LISTS) {
            const uint32_t xs = sorted_slot[q];   // rec_slot: the lane of a slot's first record applies its bucket
            if (!(xs & SESS_OWNER)) continue;
            const uint32_t slot = xs & ~SESS_OWNER;
            uint32_t *bk = ls.bkt + (uint64_t)slot * SESS_BKT;
            const uint4 b0 = ((const uint4 *)bk)[0], b1 = ((const uint4 *)bk)[1];
            const uint4 b2 = ((const uint4 *)bk)[2], b3 = ((const uint4 *)bk)[3];
            int64_t *e = entry_ptr(t, slot, stride, cap);
            sess_key_begin_bulk(K, e, L, 64, g, sw);   // in flight with the bucket
            const uint32_t c = b0.x;
            bk[0] = 0;   // the bucket is empty again for the next batch
            if (c > SESS_BKT_N) {
                ls.longs[atomicAdd(&ls.ctl[1], 1u)] = slot;
                nlong++;
                continue;
            }
            // the bucket's indices sorted (arrival order) by a bitonic network over 16 registers, then every record's
            // timestamp and value gathered in that order into this lane's LDS column (one round trip; the record loop
            // reads them by position -- a selection per record over 15 registers with its payload measured 9 us of
            // the kernel's 24)
            uint32_t r[16] = {b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w, b3.x, b3.y, b3.z, b3.w,
                              0xffffffffu};
#pragma unroll
            for (int x = 0; x < SESS_BKT_N; ++x) r[x] = x < (int)c ? r[x] : 0xffffffffu;
            // the network and the gathers sized to the largest bucket among the wave's owner lanes (wave-uniform:
            // C5's buckets hold 1-3 records mostly, and a 16-wide network and 30 gathers per lane were most of the
            // lane's instructions)
            const int P = __ballot(c > 8u) ? 16 : __ballot(c > 4u) ? 8 : __ballot(c > 2u) ? 4 : __ballot(c > 1u) ? 2 : 1;
            auto bitonic = [&](auto NP) {
                constexpr int N_ = decltype(NP)::value;
#pragma unroll
                for (int kk = 2; kk <= N_; kk <<= 1)
#pragma unroll
                    for (int jj = kk >> 1; jj > 0; jj >>= 1)
#pragma unroll
                        for (int x = 0; x < N_; ++x) {
                            const int y = x ^ jj;
                            if (y > x) {
                                const uint32_t lo = min(r[x], r[y]), hi = max(r[x], r[y]);
                                r[x] = (x & kk) == 0 ? lo : hi;
                                r[y] = (x & kk) == 0 ? hi : lo;
                            }
                        }
            };
            if (P == 16) bitonic(std::integral_constant<int, 16>{});
            else if (P == 8) bitonic(std::integral_constant<int, 8>{});
            else if (P == 4) bitonic(std::integral_constant<int, 4>{});
            else if (P == 2) bitonic(std::integral_constant<int, 2>{});
            int64_t *R = L + (size_t)g.smax * sw * 64;   // [2 * SESS_BKT_N][64]: (ts, value) of the sorted records
            int64_t rt[SESS_BKT_N], rv[SESS_BKT_N];   // every load issued before the first is used
#pragma unroll
            for (int x = 0; x < SESS_BKT_N; ++x) {
                if (x >= P) break;   // (wave-uniform)
                const uint32_t i = x < (int)c ? r[x] : r[0];
                rt[x] = ts[i];
                rv[x] = val ? val[i] : 0;
            }
#pragma unroll
            for (int x = 0; x < SESS_BKT_N; ++x) {
                if (x < (int)c) {
                    R[(2 * x) * 64] = rt[x];
                    R[(2 * x + 1) * 64] = rv[x];
                }
            }
            const int64_t k = slot < cap ? e[0] : GWO_EMPTY_KEY;   // the side slot holds the empty-key marker's key
            for (uint32_t j = 0; j < c; ++j) sess_key_record<NWT>(K, k, R[(2 * j) * 64], R[(2 * j + 1) * 64], SESS_REC_ARGS);
#ifdef GWO_SP_NOEND
            created += K.created + K.ns;
#else
            created += sess_key_end(K, slot, cap, g, sw);
#endif
        } else {
            const uint32_t slot = sorted_slot[q];
            if (q > 0 && sorted_slot[q - 1] == slot) continue;  // not the head of this key's run
            sess_key_begin(K, entry_ptr(t, slot, stride, cap), L, 64, g, sw);
            int64_t r = q;
            for (; r < n && sorted_slot[r] == slot; ++r) {
                const uint32_t i = sorted_idx[r];
                sess_key_record(K, SESS_REC(i), SESS_REC_ARGS);
            }
            nlong += r - q > SESS_BKT_N;   // what the lists would have sent to sess_long_kernel (the host's choice)
            created += sess_key_end(K, slot, cap, g, sw);
        }
    }
    wave_atomic_add(LISTS ? &ls.shards[(blockIdx.x % SESS_SHARDS) * SESS_SHARD_STRIDE] : &err->live_delta,
                    (unsigned long long)created);
    wave_atomic_add(&err->long_slots, nlong);
}

// Folds (reads and resets) shard words wa (threads 0-63) and wb (threads 64-127) of every shard in one round of
// exchanges (256-thread workgroups; both totals returned to all threads).
__device__ __forceinline__ void sess_fold_shards2(unsigned long long *shards, int wa, int wb, unsigned long long &ra,
                                                  unsigned long long &rb) {
    __shared__ unsigned long long s_fold2[2];
    if (threadIdx.x < 128) {
        const int h = threadIdx.x >> 6, q = threadIdx.x & 63;
        unsigned long long v = q < SESS_SHARDS ? atomicExch(&shards[q * SESS_SHARD_STRIDE + (h ? wb : wa)], 0ull) : 0ull;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (q == 0) s_fold2[h] = v;
    }
    __syncthreads();
    ra = s_fold2[0];
    rb = s_fold2[1];
    __syncthreads();
}

// pass 3 (lists only): the slots whose records overflowed their buckets, a workgroup each: the records' slots are
// scanned in index order, a chunk at a time, and thread 0 applies the chunk's matches in order.  The batch's last
// kernel: its last workgroup publishes the statistics block (and the pool's bump counter behind it) into the
// host-mapped readback, sequence word last, and resets the list counters.
#define SL_PER 8
#define SL_CHUNK (256 * SL_PER)
__global__ __launch_bounds__(256) void sess_long_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                        const int64_t *__restrict__ val, int64_t n,
                                                        const uint32_t *__restrict__ rec_slot, TableDesc t,
                                                        uint64_t cap, int stride, AccPlan p, ResultPlan rp, SessGeom g,
                                                        OutCols o, SessErr *err, int64_t *side_key, int64_t *side_ts,
                                                        int64_t *side_val, unsigned long long *side_count,
                                                        long long side_cap, SessLists ls, unsigned long long *rb,
                                                        unsigned long long seq, unsigned long long *reset_rows) {
    extern __shared__ int64_t s_L[];       // thread 0's copy of the key's inline sessions
    __shared__ uint32_t s_idx[SL_CHUNK];   // a chunk's records of the key, in arrival order
    const int sw = 3 + p.nwords;
    const uint32_t nl = ls.ctl[1];
    // no slot overflowed its bucket (C5: every batch): workgroup 0 alone publishes, with no arrival count
    const bool none = nl == 0;
    if (none && blockIdx.x != 0) return;
    constexpr int NWD = (int)(sizeof(SessErr) / 8) + 1;
    // the batch's input columns are no longer read (the slot and process kernels are done, no slot is long): the
    // release word, which a pipelined watermark waits for instead of the whole readback (gwo_session.cpp fire_session)
    if (none && threadIdx.x == 0) rb_put(&rb[NWD + 1], seq);
    for (uint32_t j = blockIdx.x; j < nl; j += gridDim.x) {
        const uint32_t slot = ls.longs[j];
        SessKey K;
        if (threadIdx.x == 0) sess_key_begin(K, entry_ptr(t, slot, stride, cap), s_L, 1, g, sw);
        for (int64_t c0 = 0; c0 < n; c0 += SL_CHUNK) {
            const int64_t i0 = c0 + (int64_t)threadIdx.x * SL_PER;
            uint32_t m = 0;
            if (i0 + SL_PER <= n) {
                const uint4 a = ((const uint4 *)(rec_slot + i0))[0], b = ((const uint4 *)(rec_slot + i0))[1];
                constexpr uint32_t S_ = ~SESS_OWNER;
                m = ((a.x & S_) == slot) | ((a.y & S_) == slot) << 1 | ((a.z & S_) == slot) << 2 |
                    ((a.w & S_) == slot) << 3 | ((b.x & S_) == slot) << 4 | ((b.y & S_) == slot) << 5 |
                    ((b.z & S_) == slot) << 6 | ((b.w & S_) == slot) << 7;
            } else {
                for (int x = 0; x < SL_PER; ++x)
                    m |= (i0 + x < n && (rec_slot[i0 + x] & ~SESS_OWNER) == slot) ? 1u << x : 0u;
            }
            unsigned tot;
            unsigned pos = block_exclusive_scan(__popc(m), &tot);
            for (int x = 0; x < SL_PER; ++x)
                if ((m >> x) & 1u) s_idx[pos++] = (uint32_t)(i0 + x);
            __syncthreads();
            if (threadIdx.x == 0)
                for (unsigned r = 0; r < tot; ++r) {
                    const uint32_t i = s_idx[r];
                    sess_key_record(K, SESS_REC(i), SESS_REC_ARGS);
                }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            const long long c = sess_key_end(K, slot, cap, g, sw);
            if (c) atomicAdd(&err->live_delta, (unsigned long long)c);
        }
    }
    // statistics are device-scope atomics, read back here with read-modify-write atomics (coherent across XCDs)
    // after every workgroup's stores and atomics completed (vmcnt) and its arrival was counted
    __shared__ int s_last;
    if (!none) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) s_last = atomicAdd(&ls.ctl[2], 1u) == gridDim.x - 1;
        __syncthreads();
        if (!s_last) return;
    }
    // one round of device-scope atomics: the process kernel's live-session change folded from its shards (wave 0),
    // the statistics words read (wave 1) and the table's occupancy summed from its counter shards (wave 2: the host
    // sizes the next batches on it without reading the counter back, a stream synchronisation); the fold goes back
    // into the statistics block without a return (rb_publish's wait covers it)
    __shared__ unsigned long long s_live, s_w[NWD];
    const int wv = threadIdx.x >> 6, q = threadIdx.x & 63;
    if (wv == 0) {
        unsigned long long v = q < SESS_SHARDS ? atomicExch(&ls.shards[q * SESS_SHARD_STRIDE], 0ull) : 0ull;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (q == 0) s_live = v;
    } else if (wv == 1) {
        if (q < NWD) s_w[q] = atomicAdd((unsigned long long *)err + q, 0ull);
    } else if (wv == 2) {
        unsigned long long c = q < GWO_OCC_SHARDS
                                   ? __hip_atomic_load(&t.occ[q * GWO_OCC_SHARD_STRIDE], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : 0ull;
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if (q == 0) rb_put(&rb[NWD + 2], c);
    }
    __syncthreads();
    if (threadIdx.x < NWD) {
        const unsigned long long add = threadIdx.x == (int)(offsetof(SessErr, live_delta) / 8) ? s_live : 0ull;
        if (add) atomicAdd((unsigned long long *)err + threadIdx.x, add);
        rb_put(&rb[threadIdx.x], s_w[threadIdx.x] + add);
    }
    if (!none && threadIdx.x == NWD) rb_put(&rb[NWD + 1], seq);   // (every long slot's records applied)
    if (threadIdx.x == 0) {
        ls.ctl[1] = 0;
        ls.ctl[2] = 0;
        if (reset_rows) *reset_rows = 0;   // the output's row counter after a discard (instead of a memset)
    }
    rb_publish(&rb[NWD], seq);
}

// watermark: fire pending timers <= wm, clear sessions whose cleanup time <= wm
// Persistent workgroups (about one per CU) sweep the slots in rounds of SF_SPT slots per thread; a round counts
// its rows first and reserves them with ONE returning atomic per workgroup (block_reserve), then emits.  A
// reservation per wave or per row serialised on the shared row counter: ~180 us per watermark at C5's ~5K
// fired sessions, for a kernel that does a few microseconds of work.  Statistics: one add per workgroup.  A round's
// due slots are compacted into a workgroup list and a thread takes one each (C5: 19.1 -> 14.6 us per watermark);
// more workgroups with fewer slots per thread measured slower (SF_SPT 2 / 1024 workgroups: 33 us, 1 / 2048: 54 us).
#ifndef SF_SPT
#define SF_SPT 8
#endif
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

// One due slot of the sweep: its pending timers at maxTs <= wm emit rows at pos, pos + 1, ... (reserved by the caller;
// pos is advanced past them for the thread's next due slot), its
// sessions past their cleanup time retire (WindowOperator.java:430-473, 528-540), its due watermark is recomputed.
// Returns the number of retired sessions.
__device__ __forceinline__ long long sf_sweep_slot(int64_t *e, uint64_t i, int64_t k, const TableDesc &t, uint64_t cap,
                                                   int sw, const AccPlan &p, const ResultPlan &rp, const SessGeom &g,
                                                   const OutCols &o, unsigned long long &pos) {
    const bool spilled = e[1] < 0;
    const int ns = spilled ? (int)e[4] : (int)e[1];
    int64_t *base = spilled ? g.pool + (uint64_t)e[2] * sw : e + 2;
    long long removed = 0;
    int keep = 0;
    for (int s = 0; s < ns; ++s) {
        int64_t *S = base + s * sw;
        const int64_t mx = jsub(S[1], 1);
        if ((S[2] & 1) && mx <= g.wm) {
            emit_row_at(o, p, rp, pos++, k, S[0], S[1], S + 3);
            S[2] &= ~1ll;
        }
        if (cleanup_time(mx, g.lateness) <= g.wm) {
            removed++;
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
    return removed;
}

__global__ __launch_bounds__(256) void sess_fire_kernel(TableDesc t, uint64_t cap, int stride, AccPlan p, ResultPlan rp,
                                                        SessGeom g, OutCols o, SessErr *err, unsigned long long *arr,
                                                        unsigned long long *shards, unsigned long long *rb,
                                                        unsigned long long seq) {
    const int sw = 3 + p.nwords;
    const uint64_t span = (uint64_t)gridDim.x * 256;   // slots one pass of the grid covers
    unsigned long long emitted = 0;
    long long removed_all = 0;
#ifndef GWO_SF_ROUNDS   // (the r03 sweep, kept for A/B: a thread walks its due slots one after another)
    // the round's due slots compacted into a workgroup list first, then a thread per due slot: its entry header and
    // first session load in one round trip (a thread with several due slots no longer walks them one after another)
    __shared__ uint32_t s_due[256 * SF_SPT];
    for (uint64_t r0 = 0; r0 <= cap; r0 += span * SF_SPT) {
        unsigned m = 0;
#pragma unroll
        for (int j = 0; j < SF_SPT; ++j) {
            const uint64_t i = r0 + (uint64_t)j * span + (uint64_t)blockIdx.x * 256 + threadIdx.x;
            const int64_t dv = g.due[i <= cap ? i : cap];
            m |= (i <= cap && dv <= g.wm) ? 1u << j : 0u;
        }
        unsigned tot;
        unsigned at = block_exclusive_scan(__popc(m), &tot);
#pragma unroll
        for (int j = 0; j < SF_SPT; ++j)
            if ((m >> j) & 1u) s_due[at++] = (uint32_t)((uint64_t)j * span + (uint64_t)blockIdx.x * 256 + threadIdx.x);
        __syncthreads();
        for (unsigned b0 = 0; b0 < tot; b0 += 256) {   // workgroup-uniform
            const uint64_t i = b0 + threadIdx.x < tot ? r0 + s_due[b0 + threadIdx.x] : cap + 1;
            int64_t *e = nullptr;
            int64_t k = GWO_EMPTY_KEY, h1 = 0, h2 = 0, h4 = 0, x1 = 0, x2 = 0;
            if (i <= cap) {
                int64_t *ee = i < cap ? t.base + i * (uint64_t)stride : t.side;
                const int64_t h0 = ee[0];   // header and the first inline session's end and flags: one round trip
                h1 = ee[1];
                h2 = ee[2];
                h4 = ee[4];
                x1 = ee[3];
                x2 = ee[4];
                if (i < cap ? h0 != GWO_EMPTY_KEY : h0 != 0) e = ee;
                k = i < cap ? h0 : GWO_EMPTY_KEY;
            }
            unsigned nrow = 0;
            int ns = 0;
            const int64_t *base = nullptr;
            if (e) {
                const bool spilled = h1 < 0;
                ns = spilled ? (int)h4 : (int)h1;
                base = spilled ? g.pool + (uint64_t)h2 * sw : e + 2;
                for (int s = 0; s < ns; ++s) {   // rows: pending timers at maxTs <= wm (EventTimeTrigger.onEventTime)
                    const int64_t end = (s || spilled) ? base[s * sw + 1] : x1;
                    const int64_t fl = (s || spilled) ? base[s * sw + 2] : x2;
                    nrow += (fl & 1) && jsub(end, 1) <= g.wm;
                }
            }
            unsigned long long pos = block_reserve(nrow, o.count);
            emitted += nrow;
            if (e && ns) removed_all += sf_sweep_slot(e, i, k, t, cap, sw, p, rp, g, o, pos);
        }
        __syncthreads();   // s_due is rewritten by the next round
    }
#else
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
            removed_all += sf_sweep_slot(e, i, k, t, cap, sw, p, rp, g, o, pos);
        }
    }
#endif
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
        unsigned long long *sh = shards + (blockIdx.x % SESS_SHARDS) * SESS_SHARD_STRIDE;
        if (e) atomicAdd(sh + 1, e);
        if (r) atomicAdd(sh + 2, (unsigned long long)(-r));
    }
    // the last workgroup publishes the sweep's statistics into the host-mapped readback, sequence word last (no
    // copy behind the kernel): read with read-modify-write atomics after every workgroup's adds completed
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) s_last = grid_arrive_last(arr);
    __syncthreads();
    if (!s_last) return;
    constexpr int NW = (int)(sizeof(SessErr) / 8);
    unsigned long long em, lv;   // (one round of exchanges for both words: the sweep's last round trips)
    sess_fold_shards2(shards, 1, 2, em, lv);
    if (threadIdx.x < NW) {
        const int w = threadIdx.x;
        const unsigned long long add = w == (int)(offsetof(SessErr, emitted) / 8)      ? em
                                       : w == (int)(offsetof(SessErr, live_delta) / 8) ? lv
                                                                                       : 0ull;
        rb_put(&rb[w], atomicAdd((unsigned long long *)err + w, add) + add);
    }
    rb_publish(&rb[NW], seq);
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
                      const SessGeom &g, uint32_t *rec_slot, SessErr *err, const SessLists *ls, hipStream_t s) {
    if (ls)
        hipLaunchKernelGGL(sess_slot_kernel<true>, dim3(sgrid(n, 256, 8192)), dim3(256), 0, s, key, ts, n, t, cap,
                           stride, g, rec_slot, err, *ls);
    else
        hipLaunchKernelGGL(sess_slot_kernel<false>, dim3(sgrid(n, 256, 8192)), dim3(256), 0, s, key, ts, n, t, cap,
                           stride, g, rec_slot, err, SessLists{});
}

void launch_sess_process(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const uint32_t *sslot,
                         const uint32_t *sidx, const TableDesc &t, uint64_t cap, int stride, const AccPlan &p,
                         const ResultPlan &rp, const SessGeom &g, OutCols o, SessErr *err, int64_t *sk, int64_t *st,
                         int64_t *sv, unsigned long long *sc, long long scap, const SessLists *ls, hipStream_t s) {
    const size_t lds = (size_t)SESS_PROC_WAVES * 64 * (g.smax * (3 + p.nwords) + (ls ? 2 * SESS_BKT_N : 0)) * 8;
    constexpr int PT = 64 * SESS_PROC_WAVES;
#define GWO_SESS_PROC(NWT)                                                                                    \
    hipLaunchKernelGGL((sess_process_kernel<true, NWT>), dim3(sgrid(n, PT, 65536 / SESS_PROC_WAVES)), dim3(PT), lds, s,  \
                       key, ts, val, n, \
                       sslot, sidx, t, cap, stride, p, rp, g, o, err, sk, st, sv, sc, scap, *ls)
    if (ls) {   // (the plan's word count at compile time for 1-4 words)
        switch (p.nwords) {
            case 1: GWO_SESS_PROC(1); break;
            case 2: GWO_SESS_PROC(2); break;
            case 3: GWO_SESS_PROC(3); break;
            case 4: GWO_SESS_PROC(4); break;
            default: GWO_SESS_PROC(0); break;
        }
    } else
        hipLaunchKernelGGL(sess_process_kernel<false>, dim3(sgrid(n, PT, 65536 / SESS_PROC_WAVES)), dim3(PT), lds, s, key, ts, val, n,
                           sslot, sidx, t, cap, stride, p, rp, g, o, err, sk, st, sv, sc, scap, SessLists{});
#undef GWO_SESS_PROC
}

void launch_sess_long(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const uint32_t *rec_slot,
                      const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const ResultPlan &rp,
                      const SessGeom &g, OutCols o, SessErr *err, int64_t *sk, int64_t *st, int64_t *sv,
                      unsigned long long *sc, long long scap, const SessLists &ls, unsigned long long *rb,
                      unsigned long long seq, unsigned long long *reset_rows, hipStream_t s) {
    const size_t lds = (size_t)g.smax * (3 + p.nwords) * 8;
#ifndef SESS_LONG_WG
#define SESS_LONG_WG 32
#endif
    hipLaunchKernelGGL(sess_long_kernel, dim3(SESS_LONG_WG), dim3(256), lds, s, key, ts, val, n, rec_slot, t, cap, stride, p, rp,
                       g, o, err, sk, st, sv, sc, scap, ls, rb, seq, reset_rows);
}

void launch_sess_fire(const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const ResultPlan &rp,
                      const SessGeom &g, OutCols o, SessErr *err, unsigned long long *arr, unsigned long long *shards,
                      unsigned long long *rb, unsigned long long seq, hipStream_t s) {
    // about one workgroup per CU (MI355X: 256), fewer for small tables
#ifndef SF_WG
#define SF_WG 256
#endif
    hipLaunchKernelGGL(sess_fire_kernel, dim3(sgrid((int64_t)cap + 1, 256 * SF_SPT, SF_WG)), dim3(256), 0, s, t, cap,
                       stride, p, rp, g, o, err, arr, shards, rb, seq);
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
