// gwo_kernels.hip -- hand-written gfx950 kernels of the keyed event-time window path.
//
//   scan      per batch: window/pane range of the accepted records, histogram for table sizing,
//             late-record accounting (numLateRecordsDropped / side output), Long.MIN_VALUE check
//   insert    records -> per-window HBM hash tables, keyed (key) within a window's table;
//             optional per-workgroup LDS pre-aggregation of duplicate (key, window) pairs before
//             the device-scope atomics (low-cardinality streams, e.g. YSB's 1K campaigns)
//   fire      watermark-driven onEventTime: sweep a window's table, stream-compact the occupied
//             entries into the output columns (key, start, end, results) and reset them
//   rehash    table growth
//
// All of these are HBM-bandwidth-bound integer/byte work (no MFMA).  See DESIGN.md for the
// algorithmic bytes per unit that bench.py prices each kernel with.
#include "gwo_device.h"

namespace gwo {

enum RecClass : int { REC_ACCEPT = 0, REC_LATE = 1, REC_SKIP = 2, REC_REFIRE = 3, REC_BAD_TS = 4, REC_BAD_SLIDE = 5 };

// Classifies one record against the batch's watermark; returns the unit (window or pane) index.
// Tumbling: WindowOperator.java:386-427 with TumblingEventTimeWindows.java:68-81.
// Sliding:  SlidingEventTimeWindows.java:68-82 restated on panes of gcd(size, slide).
__device__ __forceinline__ int classify(int64_t ts, const WindowGeom &g, long long &unit_idx) {
    if (ts == GWO_LONG_MIN) return REC_BAD_TS;
    int64_t last_start, first_start;
    if (!g.sliding) {
        last_start = window_start_f(ts, g.offset, g.size, g.inv_size);
        first_start = last_start;
    } else {
        // Java's '%' gives a start > ts for ts - offset + slide < 0; the pane restatement covers
        // the well-defined range only and rejects the rest loudly (never a silent difference).
        if (jadd(jsub(ts, g.offset), g.slide) < 0) return REC_BAD_SLIDE;
        last_start = window_start_f(ts, g.offset, g.slide, g.inv_slide);
        // smallest start s = last_start - k*slide with s > ts - size
        int64_t k = fdiv_floor(jsub(last_start, jsub(ts, g.size)) - 1, g.slide, g.inv_slide);
        first_start = jsub(last_start, k * g.slide);
    }
    int64_t last_max_ts = jsub(jadd(last_start, g.size), 1);
    if (cleanup_time(last_max_ts, g.lateness) <= g.wm) {
        // every window of the record is late (isWindowLate); isElementLate decides the count
        return jadd(ts, g.lateness) <= g.wm ? REC_LATE : REC_SKIP;
    }
    int64_t first_max_ts = jsub(jadd(first_start, g.size), 1);
    if (!g.sliding) {
        unit_idx = fdiv_floor(last_start, g.size, g.inv_size);
        // EventTimeTrigger.onElement FIRE: window.maxTs <= watermark (the unit is the window)
        return first_max_ts <= g.wm ? REC_REFIRE : REC_ACCEPT;
    }
    int64_t pane_start =
        jsub(ts, jsub(jsub(ts, g.unit_off), fdiv_floor(jsub(ts, g.unit_off), g.unit, g.inv_unit) * g.unit));
    unit_idx = fdiv_floor(pane_start, g.unit, g.inv_unit);
    // The pane feeds every window of the record: cleaned ones never emit again, unfired ones fire later,
    // and fired-but-not-cleaned ones (only with allowedLateness > 0) re-fire now, one row each.
    if (first_max_ts > g.wm || g.lateness == 0) return REC_ACCEPT;
    int64_t newest_fired = last_start;   // newest window of the record with maxTs <= watermark
    if (last_max_ts > g.wm) {
        const int64_t d = last_max_ts - g.wm;   // in (0, size): no overflow
        newest_fired = jsub(last_start, (fdiv_floor(d - 1, g.slide, g.inv_slide) + 1) * g.slide);
    }
    return cleanup_time(jsub(jadd(newest_fired, g.size), 1), g.lateness) > g.wm ? REC_REFIRE : REC_ACCEPT;
}

// Sliding re-fire record: its fired-but-not-cleaned windows are j in [ja, jb] (window j starts at
// j * slide + floorMod(offset, slide)); call only for records classify() calls REC_REFIRE.
__device__ __forceinline__ void slide_refire_windows(int64_t ts, const WindowGeom &g, long long &ja, long long &jb) {
    const int64_t last_start = window_start_f(ts, g.offset, g.slide, g.inv_slide);
    const int64_t k = fdiv_floor(jsub(last_start, jsub(ts, g.size)) - 1, g.slide, g.inv_slide);
    const int64_t first_start = jsub(last_start, k * g.slide);
    const int64_t om = jsub(g.offset, fdiv_floor(g.offset, g.slide, g.inv_slide) * g.slide);
    const long long j_first = fdiv_floor(jsub(first_start, om), g.slide, g.inv_slide);
    const long long j_last = j_first + k;
    // cleaned: maxTs + lateness <= wm (never saturated here: the record's last window is not cleaned)
    const int64_t first_max_ts = jsub(jadd(first_start, g.size), 1);
    const int64_t first_cleanup = cleanup_time(first_max_ts, g.lateness);
    ja = first_cleanup > g.wm ? j_first : j_first + fdiv_floor(g.wm - first_cleanup, g.slide, g.inv_slide) + 1;
    // fired: maxTs <= wm
    const int64_t last_max_ts = jsub(jadd(last_start, g.size), 1);
    jb = last_max_ts <= g.wm ? j_last : j_last - (fdiv_floor(last_max_ts - g.wm - 1, g.slide, g.inv_slide) + 1);
}

// Records a table pass inserts: accepted ones and (re-fire enabled) re-fire ones; a refire_only pass (the
// log layout's fired windows, gwo_log.cpp) leaves accepted records and late accounting to the log's K1.
__device__ __forceinline__ bool takes(int c, const WindowGeom &g) {
    return (c == REC_ACCEPT && !g.refire_only) || (c == REC_REFIRE && g.refire_ok);
}

// ------------------------------------------------------------------------------------------------
// scan
// ------------------------------------------------------------------------------------------------
// Statistics: every workgroup reduces its counters and histogram in LDS and adds them to shard blockIdx %
// SCAN_SHARDS (same-address device atomics serialise at ~12 ns each on MI355X: per-wave atomics of a 1.6K-
// workgroup scan on one word cost ~80 us); the last workgroup folds the shards into *st (and resets them).
__global__ __launch_bounds__(256) void scan_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                   const int64_t *__restrict__ val, int64_t n, WindowGeom g,
                                                   long long hist_base, BatchStats *st, int64_t *side_key,
                                                   int64_t *side_ts, int64_t *side_val,
                                                   unsigned long long *side_count, long long side_cap,
                                                   int side_enabled, unsigned long long *sh, ScanSpec sp) {
    __shared__ unsigned long long s_hist[GWO_HIST_BINS];
    for (int i = threadIdx.x; i < GWO_HIST_BINS; i += blockDim.x) s_hist[i] = 0;
    __syncthreads();
    long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000LL;
    unsigned long long acc = 0, late = 0, refire = 0, bad_ts = 0, bad_slide = 0, hout = 0, bad_kg = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        long long u = 0;
        int c = classify(ts[i], g, u);
        if (c == REC_REFIRE && g.refire_ok) refire++;   // also inserted: counted with the accepted records
        if (takes(c, g)) {
            if (sp.check_kg) {   // the speculative insert runs only if no key is outside the KeyGroupRange
                const int64_t k = key[i];
                const int32_t kg = key_group(k, g.key_kind, g.max_par);
                if (kg < g.kg_lo || kg > g.kg_hi) {
                    bad_kg++;
                    atomicExch((unsigned long long *)&st->bad_kg_key, (unsigned long long)k);
                }
            }
            acc++;
            mn = u < mn ? u : mn;
            mx = u > mx ? u : mx;
            long long b = u - hist_base;
            if (b >= 0 && b < GWO_HIST_BINS) atomicAdd(&s_hist[b], 1ull);
            else hout++;
        } else if (c == REC_LATE && !g.refire_only) {
            late++;
            if (side_enabled) {
                unsigned long long pos = atomicAdd(side_count, 1ull);
                if ((long long)pos < side_cap) {
                    side_key[pos] = key[i];
                    side_ts[pos] = ts[i];
                    side_val[pos] = val ? val[i] : 0;
                }
            }
        } else if (c == REC_REFIRE) {
            refire++;
        } else if (c == REC_BAD_TS) {
            bad_ts++;
        } else if (c == REC_BAD_SLIDE) {
            bad_slide++;
        }
    }
    // workgroup reduction -> shard blockIdx % SCAN_SHARDS (zero words skipped)
    unsigned long long v[SCAN_CNT] = {(unsigned long long)mn, (unsigned long long)mx, acc, late, refire, bad_ts,
                                      bad_slide, hout, bad_kg};
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const long long a = __shfl_xor((long long)v[0], o), b = __shfl_xor((long long)v[1], o);
        v[0] = a < (long long)v[0] ? (unsigned long long)a : v[0];
        v[1] = b > (long long)v[1] ? (unsigned long long)b : v[1];
#pragma unroll
        for (int f = 2; f < SCAN_CNT; ++f) v[f] += __shfl_xor(v[f], o);
    }
    __shared__ unsigned long long s_red[4][SCAN_CNT];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int f = 0; f < SCAN_CNT; ++f) s_red[wid][f] = v[f];
    __syncthreads();
    unsigned long long *my = sh + (size_t)(blockIdx.x % SCAN_SHARDS) * SCAN_SW;
    const int t = threadIdx.x;
    if (t < SCAN_CNT) {
        unsigned long long r = s_red[0][t];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            const unsigned long long x = s_red[w][t];
            if (t == 0) r = (long long)x < (long long)r ? x : r;
            else if (t == 1) r = (long long)x > (long long)r ? x : r;
            else r += x;
        }
        if (t == 0) {
            if ((long long)r != 0x7fffffffffffffffLL) atomicMin((long long *)&my[0], (long long)r);
        } else if (t == 1) {
            if ((long long)r != (long long)0x8000000000000000LL) atomicMax((long long *)&my[1], (long long)r);
        } else if (r) {
            atomicAdd(&my[t], r);
        }
    } else if (t >= 64 && t < 64 + GWO_HIST_BINS) {
        if (s_hist[t - 64]) atomicAdd(&my[SCAN_CNT + t - 64], s_hist[t - 64]);
    }
    // the last workgroup folds the shards (arrivals counted per shard, the last of a shard counts the shard;
    // every workgroup's atomics have completed before its arrival)
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned long long *done = sh + (size_t)SCAN_SHARDS * SCAN_SW;
    if (t == 0) {
        const unsigned q = blockIdx.x % SCAN_SHARDS;
        const unsigned members = (gridDim.x - q + SCAN_SHARDS - 1) / SCAN_SHARDS;
        const unsigned nsh = gridDim.x < SCAN_SHARDS ? gridDim.x : SCAN_SHARDS;
        bool last = false;
        if (atomicAdd(&done[q * 16], 1ull) == members - 1) last = atomicAdd(&done[SCAN_SHARDS * 16], 1ull) == nsh - 1;
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    __shared__ unsigned long long s_tot[SCAN_CNT + GWO_HIST_BINS];
    __shared__ unsigned long long s_spec[3];   // occupancy of the hint tables, side-output count
#define RBW(f) (int)(offsetof(BatchStats, f) / 8)
    if (t < SCAN_CNT + GWO_HIST_BINS) {
        const unsigned long long init = t == 0 ? 0x7fffffffffffffffull : (t == 1 ? 0x8000000000000000ull : 0ull);
        const unsigned long long r = xchg_fold<SCAN_SHARDS>(&sh[t], SCAN_SW, init, t == 0 ? 1 : (t == 1 ? 2 : 0));
        s_tot[t] = r;
        int w = RBW(hist) + t - SCAN_CNT;
        switch (t) {
            case 0: st->min_idx = (long long)r; w = RBW(min_idx); break;
            case 1: st->max_idx = (long long)r; w = RBW(max_idx); break;
            case 2: st->accepted = r; w = RBW(accepted); break;
            case 3: st->late = r; w = RBW(late); break;
            case 4: st->refire = r; w = RBW(refire); break;
            case 5: st->bad_ts = r; w = RBW(bad_ts); break;
            case 6: st->bad_range = r; w = RBW(bad_range); break;
            case 7: st->hist_out = r; w = RBW(hist_out); break;
            case 8: w = RBW(bad_kg); break;   // (a plain scan: the insert counts key-group violations)
            default: st->hist[t - SCAN_CNT] = r; break;
        }
        if (sp.rb) rb_put(&sp.rb[w], r);
    } else if (t >= 128 && t < 128 + SCAN_SHARDS + 1) {
        atomicExch(&done[(t - 128) * 16], 0ull);   // the next scan counts from zero
    } else if (sp.rb && t >= 192 && t < 195) {
        const int q = t - 192;   // 0-1: occupancy of the hint tables, 2: side-output count
        unsigned long long tot = 0;
        if (q < 2) {
            unsigned long long *o = sp.occ[q];
            if (o)
                for (int s = 0; s < GWO_OCC_SHARDS; ++s) tot += atomicAdd(o + s * GWO_OCC_SHARD_STRIDE, 0ull);
            rb_put(&sp.rb[CB_RB_OCC + q], tot);
        } else {
            tot = side_enabled ? atomicAdd(side_count, 0ull) : 0ull;
            rb_put(&sp.rb[CB_RB_SIDE], tot);
        }
        s_spec[q] = tot;
    }
    if (!sp.rb) return;
    __syncthreads();
    if (t == 0) {   // the speculative insert's verdict (the host's checks and ensure_table's load factor)
        bool go = s_tot[2] > 0 && s_tot[5] == 0 && s_tot[6] == 0 && s_tot[8] == 0 && s_tot[4] == 0 && s_tot[7] == 0 &&
                  (long long)s_tot[0] >= sp.hint && (long long)s_tot[1] <= sp.hint + 1 &&
                  (!side_enabled || (long long)s_spec[2] <= side_cap);
        for (int r = 0; r < 2 && go; ++r) {
            const unsigned long long recs = s_tot[SCAN_CNT + r];
            if (recs) go = sp.occ[r] != nullptr && 10 * (s_spec[r] + recs) <= 7 * sp.cap[r];
        }
        *sp.go = go ? 1u : 0u;
        rb_put(&sp.rb[CB_RB_GO], go ? 1ull : 0ull);
        rb_put(&sp.rb[RBW(bad_kg_key)], s_tot[8] ? atomicAdd((unsigned long long *)&st->bad_kg_key, 0ull) : 0ull);
    }
#undef RBW
    rb_publish(&sp.rb[CB_RB_SEQ], sp.seq);
}

// ------------------------------------------------------------------------------------------------
// insert (direct): one lane per record, device-scope atomics into the window's table
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void apply_record(const TableDesc &t, const AccPlan &p, int64_t k, int64_t vbits) {
    bool claimed;
    int64_t *acc = find_or_insert(t, p.stride, k, claimed);
    count_claims(t.occ, claimed);
    for (int w = 0; w < p.nwords; ++w) atomic_combine(acc + w, p.op[w], lift_word(p, w, vbits));
}

// Ring update with live-entry accounting on the hidden count word; returns the entries it made live (0 or 1)
// for the caller to add up -- one add per wave on r.live, not one per key.
__device__ __forceinline__ unsigned ring_update(const RingDesc &r, const AccPlan &p, int64_t k, const int64_t *words) {
    bool claimed;
    int64_t *acc = find_or_insert(r.t, p.stride, k, claimed);
    count_claims(r.t.occ, claimed);
    unsigned became = 0;
    for (int w = 0; w < p.nwords; ++w) {
        if (w == r.count_word) {
            unsigned long long old = atomicAdd((unsigned long long *)(acc + w), (unsigned long long)words[w]);
            became = old == 0 && words[w] != 0;
        } else {
            atomic_combine(acc + w, p.op[w], words[w]);
        }
    }
    return became;
}

// Wave sum of per-lane counts added to *dst by one lane (every lane of the wave calls it).
__device__ __forceinline__ void wave_add_signed(unsigned long long *dst, long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, (unsigned long long)v);
}

__device__ __forceinline__ void apply_ring(const RingDesc &r, const AccPlan &p, int64_t k, const int64_t *words) {
    if (ring_update(r, p, k, words)) atomicAdd(r.live, 1ull);
}

__device__ __forceinline__ void check_key_group(int64_t k, const WindowGeom &g, BatchStats *st) {
    int32_t kg = key_group(k, g.key_kind, g.max_par);
    if (kg < g.kg_lo || kg > g.kg_hi) {
        atomicAdd(&st->bad_kg, 1ull);
        st->bad_kg_key = k;
    }
}

__global__ __launch_bounds__(256) void insert_direct_kernel(const int64_t *__restrict__ key,
                                                            const int64_t *__restrict__ ts,
                                                            const int64_t *__restrict__ val, int64_t n,
                                                            WindowGeom g, AccPlan p,
                                                            const TableDesc *__restrict__ dir, long long dir_base,
                                                            int dir_len, BatchStats *st, RingDesc ring,
                                                            const uint32_t *go) {
    if (go && *go == 0) return;   // speculative launch the scan's verdict turned down: the host takes over
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    long long became = 0;   // ring entries made live by this lane
    // whole waves iterate together (the bound is rounded up to whole waves) so the live count is wave-reduced
    const int64_t lane = threadIdx.x & 63;
    const int64_t nw = (n + 63) & ~(int64_t)63;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i - lane < nw; i += stride) {
        if (i >= n) continue;
        long long u = 0;
        int64_t t = ts[i];
        const int c = classify(t, g, u);
        if (!takes(c, g)) continue;
        long long d = u - dir_base;
        if (d < 0 || d >= dir_len) continue;
        int64_t k = key[i];
        check_key_group(k, g, st);
        int64_t v = val ? val[i] : 0;
        apply_record(dir[d], p, k, v);
        if (u >= ring.lo && u <= ring.hi) {
            int64_t words[GWO_MAX_WORDS];
            for (int w = 0; w < p.nwords; ++w) words[w] = lift_word(p, w, v);
            became += ring_update(ring, p, k, words);
        }
    }
    if (ring.lo <= ring.hi) wave_add_signed(ring.live, became);
}

// ------------------------------------------------------------------------------------------------
// insert (pre-aggregated): each workgroup folds a tile of records into an LDS hash table keyed
// on (key, unit) first, then flushes one device-scope update per distinct pair.
// Claim protocol: a 64-bit tag = mix(key, unit)|1 is claimed with an LDS CAS; the claimant writes
// the exact (key, unit) and the identity accumulator; after a barrier every lane verifies the
// exact pair (a tag collision falls back to the direct global path, so results never depend on it).
// ------------------------------------------------------------------------------------------------
#define PREAGG_SLOTS 2048   // LDS: 2048 x (8 + 8 + 4 + 8*8) B = 168 KiB worst case -> words cap below
#define PREAGG_WORDS 6      // pre-aggregation is used for <= 6 accumulator words
#define PREAGG_TILE 4096

__device__ __forceinline__ uint64_t pair_tag(int64_t k, long long u) {
    uint64_t h = slot_hash(k ^ (int64_t)((uint64_t)u * 0xD1B54A32D192ED03ull));
    return h | 1ull;
}

__device__ __forceinline__ void lds_combine(int64_t *dst, int op, int64_t x) {
    switch (op) {
        case ACC_ADD_I64: atomicAdd((unsigned long long *)dst, (unsigned long long)x); break;
        case ACC_ADD_F64: atomicAdd((double *)dst, __longlong_as_double(x)); break;
        case ACC_MIN_I64: atomicMin((long long *)dst, (long long)x); break;
        default: atomicMax((long long *)dst, (long long)x); break;
    }
}

__global__ __launch_bounds__(256) void insert_preagg_kernel(const int64_t *__restrict__ key,
                                                            const int64_t *__restrict__ ts,
                                                            const int64_t *__restrict__ val, int64_t n,
                                                            WindowGeom g, AccPlan p,
                                                            const TableDesc *__restrict__ dir, long long dir_base,
                                                            int dir_len, BatchStats *st,
                                                            unsigned long long *partials, RingDesc ring) {
    __shared__ unsigned long long s_tag[PREAGG_SLOTS];
    __shared__ int64_t s_key[PREAGG_SLOTS];
    __shared__ int32_t s_unit[PREAGG_SLOTS];
    __shared__ int64_t s_acc[PREAGG_SLOTS * PREAGG_WORDS];
    const int NW = p.nwords;
    constexpr int PER = PREAGG_TILE / 256;
    unsigned long long flushed = 0;
    for (int64_t tile = (int64_t)blockIdx.x * PREAGG_TILE; tile < n; tile += (int64_t)gridDim.x * PREAGG_TILE) {
        for (int i = threadIdx.x; i < PREAGG_SLOTS; i += 256) s_tag[i] = 0;
        __syncthreads();
        int slot[PER];
        int64_t rk[PER], rv[PER];
        int32_t ru[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            slot[j] = -2;  // -2: not accepted, -1: go direct
            int64_t i = tile + j * 256 + threadIdx.x;
            if (i >= n) continue;
            long long u = 0;
            const int c = classify(ts[i], g, u);
            if (!takes(c, g)) continue;
            long long d = u - dir_base;
            if (d < 0 || d >= dir_len) continue;
            int64_t k = key[i];
            check_key_group(k, g, st);
            rk[j] = k;
            rv[j] = val ? val[i] : 0;
            ru[j] = (int32_t)d;
            uint64_t tag = pair_tag(k, d);
            int s = (int)(tag >> 40) & (PREAGG_SLOTS - 1);
            slot[j] = -1;
            for (int probe = 0; probe < 32; ++probe) {
                unsigned long long prev = atomicCAS(&s_tag[s], 0ull, tag);
                if (prev == 0ull) {
                    s_key[s] = k;
                    s_unit[s] = (int32_t)d;
                    for (int w = 0; w < NW; ++w) s_acc[s * NW + w] = p.ident[w];
                    slot[j] = s;
                    break;
                }
                if (prev == tag) {
                    slot[j] = s;
                    break;
                }
                s = (s + 1) & (PREAGG_SLOTS - 1);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (slot[j] == -2) continue;
            int s = slot[j];
            if (s >= 0 && s_key[s] == rk[j] && s_unit[s] == ru[j]) {
                for (int w = 0; w < NW; ++w) lds_combine(&s_acc[s * NW + w], p.op[w], lift_word(p, w, rv[j]));
            } else {
                apply_record(dir[ru[j]], p, rk[j], rv[j]);
                long long u = dir_base + ru[j];
                if (u >= ring.lo && u <= ring.hi) {
                    int64_t words[GWO_MAX_WORDS];
                    for (int w = 0; w < p.nwords; ++w) words[w] = lift_word(p, w, rv[j]);
                    apply_ring(ring, p, rk[j], words);
                }
            }
        }
        __syncthreads();
        for (int s = threadIdx.x; s < PREAGG_SLOTS; s += 256) {
            if (s_tag[s] == 0ull) continue;
            flushed++;
            bool claimed;
            const TableDesc &ft = dir[s_unit[s]];
            int64_t *a = find_or_insert(ft, p.stride, s_key[s], claimed);
            count_claims(ft.occ, claimed);
            for (int w = 0; w < NW; ++w) atomic_combine(a + w, p.op[w], s_acc[s * NW + w]);
            long long u = dir_base + s_unit[s];
            if (u >= ring.lo && u <= ring.hi) apply_ring(ring, p, s_key[s], &s_acc[s * NW]);
        }
        __syncthreads();
    }
    wave_atomic_add(partials, flushed);
}

// ------------------------------------------------------------------------------------------------
// Combine path (table layout, low-cardinality batches such as YSB's 1K campaigns): the scan and the
// pre-aggregated insert as ONE pass over the records plus a merge, with the host's checks in between.
//   gather  persistent workgroups: every record is classified (the scan's statistics, histogram, side
//           output, key-group check); a wave first folds runs of lanes holding one (unit, key) into one lane
//           (ballot + masked wave reduction: hot keys), then every record is folded into the workgroup's LDS
//           table of units hint and hint + 1
//           (key-indexed, accumulators preset to the identity, so a claim is one CAS of the key word); the
//           table is then dumped densely per workgroup.  Records of other units, of a full table or with
//           the empty-key marker are listed for the merge.  Statistics go to a per-workgroup slot and the
//           last workgroup reduces them into BatchStats: device-scope atomics on one address serialise at
//           ~12 ns each on MI355X (measured), so per-wave counter atomics cost more than the pass itself.
//   merge   after the host accepted the batch (nothing changed before -- the reject-before-any-change rule
//           holds): per dump slot and run of workgroups, entries of one key fold in registers into one
//           find-or-insert + combine; then the listed records one by one.
// ------------------------------------------------------------------------------------------------
#define CB_NU 2
#ifndef CB_THREADS
#define CB_THREADS 1024
#endif
#ifndef CB_PER
#define CB_PER 4
#endif
#define CB_TILE (CB_THREADS * CB_PER)
#ifndef CB_MERGE_RUN
#define CB_MERGE_RUN 8
#endif
#ifndef CB_MERGE_EAGER
#define CB_MERGE_EAGER 1
#endif
#define CB_SHARDS 16      // statistics shards (gather)
#define CB_HOT 8          // lanes of one (unit, key) in a wave that take the wave pre-reduction

// The workgroup's LDS table of one unit (S slots, key-indexed): the slot holding k, claimed if absent; -1 when
// 32 probes found no room (the record is listed for the merge).  Two 32-bit multiplies place a key: the table
// is private to the pass, any spread will do.  (Linear probing keeps a key at the same slot in most workgroups'
// tables, which the merge's runs fold in registers; 4-slot buckets measured no faster here and scattered them.)
__device__ __forceinline__ int lds_slot(int64_t *kb, int S, int sbits, int64_t k) {
    uint32_t sl = ((uint32_t)k * 0x9E3779B1u ^ (uint32_t)((uint64_t)k >> 32) * 0x85EBCA77u) >> (32 - sbits);
    for (int probe = 0; probe < 32; ++probe) {
        int64_t cur = kb[sl];
        if (cur == GWO_EMPTY_KEY) {
            cur = (int64_t)atomicCAS((unsigned long long *)&kb[sl], (unsigned long long)GWO_EMPTY_KEY,
                                     (unsigned long long)k);
            if (cur == GWO_EMPTY_KEY) return (int)sl;
        }
        if (cur == k) return (int)sl;
        sl = (sl + 1) & (uint32_t)(S - 1);
    }
    return -1;
}

// Lane `src` (wave-uniform) of x: a scalar read (v_readlane), no LDS permute.
__device__ __forceinline__ int64_t lane64(int64_t x, int src) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// x folded over the 64 lanes of the wave with the word's monoid (every lane gets the result; lanes that do
// not take part pass the identity).  Float sums are re-associated: within the 1e-6 relative bound.
__device__ __forceinline__ int64_t wave_fold(int op, int64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = combine(op, x, __shfl_xor(x, o));
    return x;
}

enum : int { CS_ACC = 0, CS_LATE, CS_REFIRE, CS_BADTS, CS_BADRANGE, CS_BADKG, CS_HOUT, CS_MIN, CS_MAX, CS_D0, CS_D1,
             CS_HIST = 16, CS_WORDS = CS_HIST + GWO_HIST_BINS };

// NWT: the accumulator words at compile time (1-4; 0: p.nwords at run time) -- loops over words unroll and the plan's
// per-word fields become scalar constants instead of run-time indexed arrays (the kernel was VALU-bound on them)
// The gather's arguments, one struct: read through the kernarg segment pointer (offset 0) where the slow path and the
// tail use them, so that only the per-record fields stay in scalar registers across the tile loop (the ~600 B of
// arguments had spilled from SGPRs into VGPR lanes: a v_readlane per use, most of the kernel's VALU).
struct GatherArgs {
    const int64_t *key, *ts, *val;
    int64_t n;
    WindowGeom g;
    AccPlan p;
    CombineArgs a;
    BatchStats *st;
    int64_t *side_key, *side_ts, *side_val;
    unsigned long long *side_count;
    long long side_cap;
    int side_enabled;
};
typedef __attribute__((address_space(4))) const GatherArgs KGatherArgs;
// The kernarg segment behind an opaque copy of its pointer: loads through it stay where they are written.
__device__ __forceinline__ KGatherArgs *gather_args() {
    KGatherArgs *ka = (KGatherArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    return ka;
}
__device__ __forceinline__ WindowGeom load_geom(__attribute__((address_space(4))) const WindowGeom *s) {
    WindowGeom g;
    g.unit = s->unit;
    g.unit_off = s->unit_off;
    g.unit_off_mod = s->unit_off_mod;
    g.size = s->size;
    g.slide = s->slide;
    g.offset = s->offset;
    g.lateness = s->lateness;
    g.wm = s->wm;
    g.inv_size = s->inv_size;
    g.inv_slide = s->inv_slide;
    g.inv_unit = s->inv_unit;
    g.sliding = s->sliding;
    g.key_kind = s->key_kind;
    g.max_par = s->max_par;
    g.kg_lo = s->kg_lo;
    g.kg_hi = s->kg_hi;
    g.refire_ok = s->refire_ok;
    g.refire_only = s->refire_only;
    return g;
}

template <int NWT>
__global__ __launch_bounds__(CB_THREADS) void gather_kernel(GatherArgs A) {
    const int64_t *__restrict__ key = A.key;
    const int64_t *__restrict__ ts = A.ts;
    const int64_t *__restrict__ val = A.val;
    const int64_t n = A.n;
    const AccPlan &p = A.p;
    const CombineArgs &a = A.a;
    // the per-record fields of the geometry (the rest is read in the slow path)
    const int32_t g_key_kind = A.g.key_kind, g_max_par = A.g.max_par, g_kg_lo = A.g.kg_lo, g_kg_hi = A.g.kg_hi;
    const int32_t g_refire_only = A.g.refire_only;
    unsigned long long *const dbg = A.a.dbg;
    extern __shared__ __attribute__((aligned(16))) int64_t s_dyn[];
    const int S = a.S, NW = NWT > 0 ? NWT : p.nwords, tid = threadIdx.x;
    // trace: per-workgroup slot of 8 words, plain stores (start, then phase ends), reduced on the host
#define CB_STAMP(k)                                                        \
    do {                                                                   \
        if (dbg && tid == 0) dbg[blockIdx.x * 8 + (k)] = wall_clock64(); \
    } while (0)
    CB_STAMP(0);
    int64_t *s_key = s_dyn;                     // [CB_NU * S]
    int64_t *s_acc = s_dyn + CB_NU * S;         // [CB_NU * S * NW]
    int64_t *s_spare = s_acc + CB_NU * S * NW;  // [64]: each lane's spare word for the find-or-claim rounds
    __shared__ unsigned s_hist[GWO_HIST_BINS];
    __shared__ unsigned long long s_red[CB_THREADS / 64][CS_HIST];
    for (int i = tid; i < CB_NU * S; i += CB_THREADS) s_key[i] = GWO_EMPTY_KEY;
    if (tid < 64) s_spare[tid] = GWO_EMPTY_KEY;
    for (int i = tid; i < CB_NU * S; i += CB_THREADS)
        for (int w = 0; w < NW; ++w) s_acc[i * NW + w] = p.ident[w];
    if (tid < GWO_HIST_BINS) s_hist[tid] = 0;
    __syncthreads();
    unsigned acc = 0, late = 0, refire = 0, bad_ts = 0, bad_range = 0, bad_kg = 0, hout = 0;
    long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000LL;
    int run_b = -1;
    unsigned run_n = 0;
    // a tile's loads all in flight before any record is processed; the next tile's are issued once this tile's
    // records are in LDS (workgroups loop over tiles when the launch has fewer workgroups than tiles)
    int64_t tt[CB_PER], kk[CB_PER], vv[CB_PER];
    auto load_tile = [&](int64_t tile) {
#pragma unroll
        for (int j = 0; j < CB_PER; ++j) {
            int64_t i = tile + j * CB_THREADS + tid;
            i = i < n ? i : tile;
            tt[j] = __builtin_nontemporal_load(ts + i);
            kk[j] = __builtin_nontemporal_load(key + i);
            vv[j] = val ? __builtin_nontemporal_load(val + i) : 0;
        }
    };
    const int64_t tstride = (int64_t)gridDim.x * CB_TILE;
    if ((int64_t)blockIdx.x * CB_TILE < n) load_tile((int64_t)blockIdx.x * CB_TILE);
    if (dbg) {   // trace: when the first tile's loads have all arrived
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        CB_STAMP(6);
    }
    for (int64_t tile = (int64_t)blockIdx.x * CB_TILE; tile < n; tile += tstride) {
        unsigned ovm = 0;   // records of this tile left to the merge (bit j: record tile + j * CB_THREADS + tid)
        unsigned candm = 0;   // bit j: record j goes into the LDS table of unit cbu[j]
        int cbu[CB_PER];
        // the common case inline: an accepted record of one of the batch's windows (a few compares); everything
        // else -- late, re-fire, bad timestamps, windows outside the range -- is reloaded and classified in full
        // out of line below (the full classification inside the unrolled loop bloats the code every record runs)
        unsigned slow = 0;
#pragma unroll
        for (int j = 0; j < CB_PER; ++j) {
            const int64_t i = tile + j * CB_THREADS + tid;
            if (i >= n) continue;
            const int64_t tv = tt[j];
            const int jj = (tv >= a.bound[1]) + (tv >= a.bound[2]) + (tv >= a.bound[3]);
            if (!(a.thr_ok && tv >= a.bound[0] && tv < a.bound[4] && ((a.cls >> (2 * jj)) & 3u) == 0 &&
                  !g_refire_only)) {
                slow |= 1u << j;
                continue;
            }
            acc++;
            const int64_t k = kk[j];
            if (!a.full_range) {
                const int32_t kg = key_group(k, g_key_kind, g_max_par);
                if (kg < g_kg_lo || kg > g_kg_hi) {
                    bad_kg++;
                    atomicExch((unsigned long long *)&gather_args()->st->bad_kg_key, (unsigned long long)k);
                }
            }
            const long long u = a.hint + jj;
            mn = u < mn ? u : mn;
            mx = u > mx ? u : mx;
            if (jj != run_b) {   // run-length histogram: a batch's records share few units
                if (run_n) atomicAdd(&s_hist[run_b], run_n);
                run_b = jj;
                run_n = 0;
            }
            run_n++;
            cbu[j] = jj;
            if (jj < CB_NU && k != GWO_EMPTY_KEY) candm |= 1u << j;
            else ovm |= 1u << j;
        }
#pragma unroll 1
        while (slow) {
            const int j = __builtin_ctz(slow);
            slow &= slow - 1;
            const int64_t i = tile + j * CB_THREADS + tid;
            KGatherArgs *ka = gather_args();   // (the rare path reads its arguments here, not from registers)
            const WindowGeom g = load_geom(&ka->g);
            long long u = 0;
            const int64_t tv = ts[i];
            const int c = classify(tv, g, u);
            if (c == REC_BAD_TS) {
                bad_ts++;
            } else if (c == REC_BAD_SLIDE) {
                bad_range++;
            } else if (c == REC_LATE) {
                if (g.refire_only) continue;
                late++;
                if (ka->side_enabled) {
                    const unsigned long long pos = atomicAdd(ka->side_count, 1ull);
                    if ((long long)pos < ka->side_cap) {
                        ka->side_key[pos] = key[i];
                        ka->side_ts[pos] = tv;
                        ka->side_val[pos] = val ? val[i] : 0;
                    }
                }
            } else if (takes(c, g)) {
                acc++;
                refire += c == REC_REFIRE;
                const int64_t k = key[i];
                const int32_t kg = a.full_range ? g.kg_lo : key_group(k, g.key_kind, g.max_par);
                if (kg < g.kg_lo || kg > g.kg_hi) {
                    bad_kg++;
                    atomicExch((unsigned long long *)&ka->st->bad_kg_key, (unsigned long long)k);
                }
                mn = u < mn ? u : mn;
                mx = u > mx ? u : mx;
                const long long b = u - a.hint;
                if (b >= 0 && b < GWO_HIST_BINS) {
                    if ((int)b != run_b) {
                        if (run_n) atomicAdd(&s_hist[run_b], run_n);
                        run_b = (int)b;
                        run_n = 0;
                    }
                    run_n++;
                } else {
                    hout++;
                }
                const bool cand = b >= 0 && b < CB_NU && k != GWO_EMPTY_KEY;
#pragma unroll
                for (int q = 0; q < CB_PER; ++q)   // cbu[j] without a run-time register index
                    if (q == j) cbu[q] = (int)b;
                if (cand) candm |= 1u << j;
                else ovm |= 1u << j;
            }
        }
        CB_STAMP(1);
        // wave pre-reduction of duplicate keys, then the LDS tables (every lane of the wave is here)
        const int lane = tid & 63;
        unsigned rem = 0;   // bit j: record j still goes into an LDS table after the hot-key rounds
#pragma unroll
        for (int j = 0; j < CB_PER; ++j) {
            bool cand = (candm >> j) & 1u;
            const int64_t k = kk[j];
            const int b = cand ? cbu[j] : 0;
            // rounds over the wave's first remaining (unit, key): while it is a hot key (>= CB_HOT lanes), its
            // lanes' words fold into one lane with a masked wave reduction and that lane updates LDS once
            unsigned long long m = __ballot(cand);
            for (int r = 0; r < 8 && m; ++r) {
                const int leader = __ffsll((long long)m) - 1;   // wave-uniform: scalar lane reads
                const int64_t lk = lane64(k, leader);
                const int lb = __builtin_amdgcn_readlane(b, leader);
                const bool mine = cand && k == lk && b == lb;
                const unsigned long long peers = __ballot(mine);
                if (__popcll(peers) < CB_HOT) break;
                int slot = -1;
                if (lane == leader) slot = lds_slot(s_key + lb * S, S, a.sbits, lk);
                slot = __builtin_amdgcn_readlane(slot, leader);
                if (slot >= 0) {
                    int64_t *dst = s_acc + ((size_t)lb * S + slot) * NW;
                    for (int w = 0; w < NW; ++w) {
                        const int64_t x = wave_fold(p.op[w], mine ? lift_word(p, w, vv[j]) : p.ident[w]);
                        if (lane == leader) lds_combine(dst + w, p.op[w], x);
                    }
                    if (mine) cand = false;
                }
                m &= ~peers;
            }
            if (cand) rem |= 1u << j;
        }
        // find-or-claim of every remaining record at once: per probe round ONE compare-and-swap per record, all
        // CB_PER in flight together (a record already placed swaps this lane's spare word, so no swap is
        // conditional: a swap under a branch is waited for at the branch's join -- r03's gather waited for every
        // record's read and swap in turn).  Linear probing from the key's home slot, as lds_slot.
        uint32_t sl[CB_PER];
        int slot[CB_PER];
#pragma unroll
        for (int j = 0; j < CB_PER; ++j) {
            const int64_t k = kk[j];
            sl[j] = ((uint32_t)k * 0x9E3779B1u ^ (uint32_t)((uint64_t)k >> 32) * 0x85EBCA77u) >> (32 - a.sbits);
            slot[j] = -1;
        }
        unsigned pend = rem;
        for (int probe = 0; probe < 32 && pend; ++probe) {
            int64_t prev[CB_PER];
#pragma unroll
            for (int j = 0; j < CB_PER; ++j) {
                const bool pj = (pend >> j) & 1u;
                int64_t *at = pj ? &s_key[cbu[j] * S + (int)sl[j]] : &s_spare[lane];
                prev[j] = (int64_t)atomicCAS((unsigned long long *)at, (unsigned long long)GWO_EMPTY_KEY,
                                             (unsigned long long)(pj ? kk[j] : GWO_EMPTY_KEY));
            }
#pragma unroll
            for (int j = 0; j < CB_PER; ++j) {
                if (!((pend >> j) & 1u)) continue;
                if (prev[j] == GWO_EMPTY_KEY || prev[j] == kk[j]) {
                    slot[j] = (int)sl[j];
                    pend &= ~(1u << j);
                } else {
                    sl[j] = (sl[j] + 1) & (uint32_t)(S - 1);
                }
            }
        }
        ovm |= pend;   // no room within 32 probes: listed for the merge
#pragma unroll
        for (int j = 0; j < CB_PER; ++j) {
            if (!((rem >> j) & 1u) || slot[j] < 0) continue;
            int64_t *dst = s_acc + ((size_t)cbu[j] * S + slot[j]) * NW;
            for (int w = 0; w < NW; ++w) lds_combine(dst + w, p.op[w], lift_word(p, w, vv[j]));   // (no return value)
        }
        if (tile + tstride < n) load_tile(tile + tstride);
        // the tile's listed records: one reservation per workgroup
        unsigned long long at = block_reserve((unsigned)__popc(ovm), a.ovf_count);
        for (int j = 0; j < CB_PER; ++j)
            if ((ovm >> j) & 1u) {
                if (at < a.ovf_cap) a.ovf[at] = (uint32_t)(tile + j * CB_THREADS + tid);
                at++;
            }
    }
    CB_STAMP(2);
    KGatherArgs *const kt = gather_args();   // the tail's arguments, loaded here
    if (run_n) atomicAdd(&s_hist[run_b], run_n);
    // per-workgroup statistics slot
    unsigned long long v[CS_HIST] = {acc, late, refire, bad_ts, bad_range, bad_kg, hout, 0, 0, 0, 0};
    for (int o = 32; o > 0; o >>= 1) {
        for (int f = 0; f < CS_MIN; ++f) v[f] += __shfl_xor(v[f], o);
        const long long x = __shfl_xor(mn, o), y = __shfl_xor(mx, o);
        mn = x < mn ? x : mn;
        mx = y > mx ? y : mx;
    }
    __syncthreads();   // every LDS table update and histogram run is in
    // the occupied slots of the tables of units that took records of this workgroup (a batch usually spans one
    // window: half the tables) -- counted here, dumped after the arrival below, so that the statistics' round
    // trips do not wait for the dump's stores
    unsigned d0 = 0, d1 = 0;
    const unsigned used = (s_hist[0] ? 1u : 0u) | (s_hist[1] ? 2u : 0u);
    for (int i = tid; i < CB_NU * S; i += CB_THREADS) {
        if (!((used >> (i >= S ? 1 : 0)) & 1u)) continue;
        if (s_key[i] != GWO_EMPTY_KEY) (i < S ? d0 : d1)++;
    }
    CB_STAMP(3);
    unsigned long long e0 = d0, e1 = d1;
    for (int o = 32; o > 0; o >>= 1) {
        e0 += __shfl_xor(e0, o);
        e1 += __shfl_xor(e1, o);
    }
    const int lane = tid & 63, wid = tid >> 6;
    if (lane == 0) {
        for (int f = 0; f < CS_HIST; ++f) s_red[wid][f] = 0;
        for (int f = 0; f < CS_MIN; ++f) s_red[wid][f] = v[f];
        s_red[wid][CS_MIN] = (unsigned long long)mn;
        s_red[wid][CS_MAX] = (unsigned long long)mx;
        s_red[wid][CS_D0] = e0;
        s_red[wid][CS_D1] = e1;
    }
    __syncthreads();
    // this workgroup's statistics go into shard blockIdx % CB_SHARDS of the statistics words (device-scope
    // atomics, zero words skipped: ~G / CB_SHARDS operations per address)
    unsigned long long *shard = kt->a.blk + (size_t)(blockIdx.x % CB_SHARDS) * CS_WORDS;
    if (tid < CS_HIST) {
        unsigned long long r = tid == CS_MIN ? 0x7fffffffffffffffull : 0ull;
        for (int w = 0; w < CB_THREADS / 64; ++w) {
            const unsigned long long x = s_red[w][tid];
            if (tid == CS_MIN) r = (long long)x < (long long)r ? x : r;
            else if (tid == CS_MAX) r = (w == 0 || (long long)x > (long long)r) ? x : r;
            else r += x;
        }
        if (tid == CS_MIN) atomicMin((long long *)&shard[tid], (long long)r);
        else if (tid == CS_MAX) atomicMax((long long *)&shard[tid], (long long)r);
        else if (r) atomicAdd(&shard[tid], r);
    } else if (tid < CS_WORDS) {
        if (s_hist[tid - CS_HIST]) atomicAdd(&shard[tid], (unsigned long long)s_hist[tid - CS_HIST]);
    }
    // the last workgroup reduces the shards into BatchStats (and resets them).  Shards are updated and read with
    // device-scope read-modify-write atomics, coherent across XCDs without an L2 write-back; each workgroup's
    // have completed (vmcnt) before its arrival is counted.  No release fence: on gfx950 one writes back the
    // XCD's whole L2, per workgroup costlier than the pass (the dumps reach the merge through the kernel boundary).
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) s_last = grid_arrive_last(kt->a.done);
    __syncthreads();
    CB_STAMP(4);
    // the dump (accumulators only of occupied slots; dump_used tells the merge which tables) reaches the merge
    // through the kernel boundary; the last workgroup's tail below overlaps its stores
    auto dump = [&]() {
        if (tid == 0) kt->a.dump_used[blockIdx.x] = used;
        int64_t *dk = kt->a.dump_key + (size_t)blockIdx.x * CB_NU * S;
        int64_t *da = kt->a.dump_acc + (size_t)blockIdx.x * CB_NU * S * NW;
        for (int i = tid; i < CB_NU * S; i += CB_THREADS) {
            if (!((used >> (i >= S ? 1 : 0)) & 1u)) continue;
            const int64_t k = s_key[i];
            __builtin_nontemporal_store(k, &dk[i]);   // streamed out: no dirty dump lines left for the kernel's end
            if (k == GWO_EMPTY_KEY) continue;
            for (int w = 0; w < NW; ++w) __builtin_nontemporal_store(s_acc[i * NW + w], &da[(size_t)i * NW + w]);
        }
    };
    if (!s_last) {
        dump();
        return;
    }
    __shared__ unsigned long long s_tot[CS_WORDS];
    if (tid < CS_WORDS) {
        const unsigned long long init =
            tid == CS_MIN ? 0x7fffffffffffffffull : (tid == CS_MAX ? 0x8000000000000000ull : 0ull);
        // read and reset for the next batch
        s_tot[tid] = xchg_fold<CB_SHARDS>(&kt->a.blk[tid], CS_WORDS, init, tid == CS_MIN ? 1 : (tid == CS_MAX ? 2 : 0));
    }
    // the readback block: BatchStats image, side-output count, occupancy of the hint tables, sequence word last
    __shared__ unsigned long long s_spec[4];   // listed records, side-output count, occupancy of the hint tables
    __shared__ uint32_t s_goprev;   // the previous batch's verdict (pipelined chain), read in this same round
    if (tid == CB_THREADS - 5) s_goprev = kt->a.chain ? *(volatile const uint32_t *)kt->a.go_prev : 1u;
    if (tid < CS_WORDS && (tid < CS_HIST ? tid <= CS_D1 : true)) {
#define RBW(f) (int)(offsetof(BatchStats, f) / 8)
        // (static: a constant table in global memory; a local array indexed by tid was 20 B of scratch per lane,
        // and a kernel with scratch waits ~6 us at dispatch behind the previous kernel)
        static constexpr int word[CS_HIST] = {RBW(accepted), RBW(late),    RBW(refire),      RBW(bad_ts),
                                       RBW(bad_range), RBW(bad_kg), RBW(hist_out),    RBW(min_idx),
                                       RBW(max_idx),  RBW(distinct), RBW(distinct) + 1, 0};
        const unsigned long long r = s_tot[tid];
        rb_put(&kt->a.rb[tid < CS_HIST ? word[tid] : RBW(hist) + tid - CS_HIST], r);
        if (tid == CS_BADKG)
            rb_put(&kt->a.rb[RBW(bad_kg_key)], r ? atomicAdd((unsigned long long *)&kt->st->bad_kg_key, 0ull) : 0ull);
    } else if (tid >= CB_THREADS - 4) {
        const int q = tid - (CB_THREADS - 4);   // 0: overflow, 1: side count, 2-3: occupancy
        if (q == 0) {
            const unsigned long long ov = atomicExch(kt->a.ovf_count, 0ull);   // read and reset for the next batch
            rb_put(&kt->a.rb[RBW(overflow)], ov);
#undef RBW
            s_spec[0] = ov;
        } else if (q == 1) {
            const unsigned long long sc = kt->a.side_enabled ? atomicAdd(kt->side_count, 0ull) : 0ull;
            rb_put(&kt->a.rb[CB_RB_SIDE], sc);
            s_spec[1] = sc;
        } else {
            unsigned long long *o = kt->a.occ[q - 2];
            unsigned long long tot = 0;
            if (o)
                for (int sh = 0; sh < GWO_OCC_SHARDS; ++sh) tot += atomicAdd(o + sh * GWO_OCC_SHARD_STRIDE, 0ull);
            rb_put(&kt->a.rb[CB_RB_OCC + q - 2], tot);
            s_spec[q] = tot;
        }
    }
    __syncthreads();
    CB_STAMP(5);
    if (tid == 0) {   // the speculative merge's verdict
        bool go = kt->a.go != nullptr && s_goprev != 0u && s_tot[CS_ACC] > 0 && s_tot[CS_BADTS] == 0 && s_tot[CS_BADRANGE] == 0 &&
                  s_tot[CS_BADKG] == 0 && s_tot[CS_REFIRE] == 0 && s_tot[CS_HOUT] == 0 && s_spec[0] == 0 &&
                  (!kt->a.side_enabled || (long long)s_spec[1] <= kt->a.side_cap) &&
                  (long long)s_tot[CS_MIN] >= kt->a.hint && (long long)s_tot[CS_MAX] <= kt->a.hint + 1;
        const unsigned long long *ip = kt->a.inc_prev;
        unsigned long long incs[2];
        for (int r = 0; r < 2; ++r) incs[r] = min(s_tot[CS_HIST + r], s_tot[CS_D0 + r]);
        for (int r = 0; r < 2 && go; ++r) {
            if (!s_tot[CS_HIST + r]) continue;
            // overlapped: the previous batch's merge may still be claiming its keys of this table (at most its
            // distinct keys there); the bound is looser, so the limit is 0.9 -- a table never fills (a full one
            // would leave find_or_insert probing forever)
            unsigned long long extra = 0;
            const long long u = kt->a.hint + r;
            if (ip) extra = (long long)ip[0] == u ? ip[1] : ((long long)ip[0] + 1 == u ? ip[2] : 0ull);
            go = kt->a.occ[r] != nullptr &&
                 10 * (s_spec[2 + r] + incs[r] + extra) <= (ip ? 9ull : 7ull) * kt->a.cap[r];   // the host's kMaxLoad 0.7
        }
        if (kt->a.inc_out) {
            kt->a.inc_out[0] = (unsigned long long)kt->a.hint;
            kt->a.inc_out[1] = incs[0];
            kt->a.inc_out[2] = incs[1];
        }
        if (kt->a.go) *kt->a.go = go ? 1u : 0u;
        rb_put(&kt->a.rb[CB_RB_GO], go ? 1ull : 0ull);
    }
#undef CB_STAMP
    rb_publish(&kt->a.rb[CB_RB_SEQ], kt->a.seq);
    dump();   // the last workgroup's own dump: after the readback, which waits for every store issued before it
}

// merge: threads [0, dump_threads) take (slot, run of CB_MERGE_RUN workgroups) of the dumps; the rest take the
// listed records.  dir covers units [dir_base, dir_base + dir_len) (the host includes hint, hint + 1 whenever
// their dumps hold entries).
__global__ __launch_bounds__(256) void merge_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                    const int64_t *__restrict__ val, WindowGeom g, AccPlan p,
                                                    CombineArgs a, int G, int64_t dump_threads, uint64_t novf,
                                                    const TableDesc *__restrict__ dir, long long dir_base,
                                                    int dir_len, RingDesc ring, const uint32_t *go) {
    if (go && *go == 0) return;   // speculative launch the gather's verdict turned down: the host takes over
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int S = a.S, NW = p.nwords, slots = CB_NU * S;
    if ((int64_t)blockIdx.x * 256 < dump_threads) {   // whole workgroups: count_claims needs the full wave
        const int slot = (int)(t % slots);
        const int w0 = (int)(t / slots) * CB_MERGE_RUN;
        const bool live = t < dump_threads && w0 < G;
        const long long d = a.hint + slot / S - dir_base;
        // keys and table flags load together (a table not dumped holds a stale key: masked by its flag)
        int64_t k[CB_MERGE_RUN];
        uint32_t used[CB_MERGE_RUN];
#pragma unroll
        for (int j = 0; j < CB_MERGE_RUN; ++j) {
            const bool in = live && w0 + j < G;
            k[j] = in ? a.dump_key[(size_t)(w0 + j) * slots + slot] : GWO_EMPTY_KEY;
            used[j] = in ? a.dump_used[w0 + j] : 0u;
        }
#pragma unroll
        for (int j = 0; j < CB_MERGE_RUN; ++j)
            if (!((used[j] >> (slot >= S ? 1 : 0)) & 1u)) k[j] = GWO_EMPTY_KEY;
        int64_t run_k = GWO_EMPTY_KEY;
        int64_t run[GWO_MAX_WORDS];
        auto flush = [&]() {   // entries exist only for units of accepted records: inside the directory
            if (run_k == GWO_EMPTY_KEY || d < 0 || d >= dir_len) return;
            const TableDesc &tb = dir[d];
            bool cl;
            int64_t *e = find_or_insert(tb, p.stride, run_k, cl);
            if (cl) occ_add(tb.occ, 1ull);
            for (int w = 0; w < NW; ++w) atomic_combine(e + w, p.op[w], run[w]);
            const long long u = a.hint + slot / S;
            if (u >= ring.lo && u <= ring.hi) apply_ring(ring, p, run_k, run);
        };
        // the first CB_MW accumulator words of every entry load before any is folded (one round trip, not one
        // per entry); further words, if any, load in the fold.  CB_MERGE_EAGER: issued with the keys, not behind
        // them (an empty slot's words are never written: read and ignored -- inside the dump allocation)
        constexpr int CB_MW = 2;
        int64_t av[CB_MERGE_RUN][CB_MW];
#pragma unroll
        for (int j = 0; j < CB_MERGE_RUN; ++j)
#pragma unroll
            for (int w = 0; w < CB_MW; ++w)
#if CB_MERGE_EAGER
                av[j][w] = live && w0 + j < G && w < NW ? a.dump_acc[((size_t)(w0 + j) * slots + slot) * NW + w] : 0;
#else
                av[j][w] = k[j] != GWO_EMPTY_KEY && w < NW ? a.dump_acc[((size_t)(w0 + j) * slots + slot) * NW + w] : 0;
#endif
#pragma unroll
        for (int j = 0; j < CB_MERGE_RUN; ++j) {
            if (k[j] == GWO_EMPTY_KEY) continue;
            const int64_t *src = a.dump_acc + ((size_t)(w0 + j) * slots + slot) * NW;
            const bool same = k[j] == run_k;
            if (!same) {
                flush();
                run_k = k[j];
            }
            for (int w = 0; w < NW; ++w) {
                const int64_t x = w < CB_MW ? av[j][w < CB_MW ? w : 0] : src[w];
                run[w] = same ? combine(p.op[w], run[w], x) : x;
            }
        }
        flush();
        return;
    }
    // listed records: insert_direct's per-record path
    const int64_t q = t - dump_threads;
    if (q >= (int64_t)novf) return;
    const int64_t i = a.ovf[q];
    long long u = 0;
    const int c = classify(ts[i], g, u);
    if (!takes(c, g)) return;
    const long long d = u - dir_base;
    if (d < 0 || d >= dir_len) return;
    const int64_t k = key[i];
    const int64_t v = val ? val[i] : 0;
    bool cl;
    int64_t *e = find_or_insert(dir[d], p.stride, k, cl);
    if (cl) occ_add(dir[d].occ, 1ull);
    for (int w = 0; w < p.nwords; ++w) atomic_combine(e + w, p.op[w], lift_word(p, w, v));
    if (u >= ring.lo && u <= ring.hi) {
        int64_t words[GWO_MAX_WORDS];
        for (int w = 0; w < p.nwords; ++w) words[w] = lift_word(p, w, v);
        apply_ring(ring, p, k, words);
    }
}

// ------------------------------------------------------------------------------------------------
// fire: EventTimeTrigger.onEventTime FIRE + clearAllState for one window's table
// (WindowOperator.java:430-473, 528-550).  Occupied entries -> output rows via wave ballot
// stream compaction (one device atomic per wave); entries are reset to EMPTY/identity in place
// so the table returns to the pool clean.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void write_results(const AccPlan &p, const ResultPlan &rp, const int64_t *acc,
                                              const OutCols &o, unsigned long long pos) {
    for (int a = 0; a < rp.naggs; ++a) {
        int w = rp.word[a];
        int64_t r;
        switch (rp.kind[a]) {
            case 2:  // MIN
            case 3:  // MAX
                r = rp.value_is_f64 ? f64_from_order_key(acc[w]) : acc[w];
                break;
            case 4: {  // AVG: (double) sum / count
                double s = rp.value_is_f64 ? __longlong_as_double(acc[w]) : (double)acc[w];
                r = __double_as_longlong(s / (double)acc[w + 1]);
                break;
            }
            default: r = acc[w]; break;  // COUNT, SUM (int64 or double bits)
        }
        o.res[a][pos] = r;
    }
}

#ifndef FIRE_FPT
#define FIRE_FPT 8   // slots per thread per chunk: one output reservation per 2048 slots
#endif

__device__ __forceinline__ const int64_t *fire_entry(const TableDesc &t, uint64_t cap, int stride, uint64_t i) {
    return i < cap ? t.base + i * (uint64_t)stride : t.side;   // i == cap: the side slot
}

// Rows of a chunk are ordered (slot round j, thread): the 256 lanes that emit in round j write one contiguous run
// of every output column (coalesced stores); one row reservation per chunk.  (Ordering rows by thread instead --
// each thread's rows adjacent -- makes a store instruction touch up to 64 scattered 8-B words per column.)
__global__ __launch_bounds__(256) void fire_kernel(TableDesc t, uint64_t cap, AccPlan p, ResultPlan rp, int64_t start,
                                                   int64_t end, OutCols o, int reset, int live_word) {
    constexpr uint64_t CH = 256 * FIRE_FPT;
    const int NW = p.nwords;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ unsigned s_off[FIRE_FPT][4];
    __shared__ unsigned long long s_base;
    const unsigned long long below = (1ull << lane) - 1ull;
    // +1 iteration space for the side slot (key == Long.MIN_VALUE)
    for (uint64_t b0 = (uint64_t)blockIdx.x * CH; b0 < cap + 1; b0 += (uint64_t)gridDim.x * CH) {
        unsigned flags = 0;
        unsigned pre[FIRE_FPT];
        // every slot's key and first two accumulator words load before any is tested (one round trip per chunk,
        // not two per slot); indices past the table read the side slot, words past the entry its last word
        int64_t kw[FIRE_FPT], aw[FIRE_FPT][2];
        const int w2 = NW >= 2 ? 2 : 1;
#pragma unroll
        for (int j = 0; j < FIRE_FPT; ++j) {
            const uint64_t i = b0 + (uint64_t)j * 256 + threadIdx.x;
            const int64_t *e = fire_entry(t, cap, p.stride, i <= cap ? i : cap);
            kw[j] = e[0];
            aw[j][0] = e[1];
            aw[j][1] = e[w2];
        }
#pragma unroll
        for (int j = 0; j < FIRE_FPT; ++j) {
            uint64_t i = b0 + (uint64_t)j * 256 + threadIdx.x;
            bool occ = false;
            if (i <= cap) {
                occ = i < cap ? kw[j] != GWO_EMPTY_KEY : kw[j] != 0;
                if (occ && live_word >= 0) {
                    const int64_t lv = live_word == 0 ? aw[j][0] : (live_word == 1 && NW >= 2 ? aw[j][1]
                                                                     : fire_entry(t, cap, p.stride, i)[1 + live_word]);
                    occ = lv > 0;
                }
            }
            if (occ) flags |= 1u << j;
            const unsigned long long m = __ballot(occ);
            pre[j] = (unsigned)__popcll(m & below);
            if (lane == 0) s_off[j][wid] = (unsigned)__popcll(m);
        }
        __syncthreads();
        if (threadIdx.x == 0) {   // (round, wave)-major exclusive offsets, one reservation for the chunk
            unsigned run = 0;
            for (int j = 0; j < FIRE_FPT; ++j)
                for (int w = 0; w < 4; ++w) {
                    const unsigned c = s_off[j][w];
                    s_off[j][w] = run;
                    run += c;
                }
            s_base = run ? atomicAdd(o.count, (unsigned long long)run) : 0ull;
        }
        __syncthreads();
        const unsigned long long base = s_base;
        for (int j = 0; j < FIRE_FPT; ++j) {
            if (!(flags >> j & 1u)) continue;
            uint64_t i = b0 + (uint64_t)j * 256 + threadIdx.x;
            const unsigned long long pos = base + s_off[j][wid] + pre[j];
            int64_t *e = (int64_t *)fire_entry(t, cap, p.stride, i);
            int64_t acc[GWO_MAX_WORDS];
#pragma unroll
            for (int w = 0; w < GWO_MAX_WORDS; ++w)
                if (w < NW) acc[w] = w < 2 ? aw[j][w] : e[1 + w];
            if ((long long)pos < o.cap) {
                o.key[pos] = i < cap ? kw[j] : GWO_EMPTY_KEY;
                o.start[pos] = start;
                o.end[pos] = end;
                write_results(p, rp, acc, o, pos);
            }
            if (reset) {
                e[0] = i < cap ? GWO_EMPTY_KEY : 0;
                for (int w = 0; w < NW; ++w) e[1 + w] = p.ident[w];
            }
        }
        __syncthreads();   // s_off / s_base are rewritten by the next chunk
    }
}

// Fill a fresh table with EMPTY keys and identity accumulators.
__global__ __launch_bounds__(256) void fill_kernel(int64_t *base, uint64_t words, AccPlan p) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
        int w = (int)(i % (uint64_t)p.stride);
        base[i] = w == 0 ? GWO_EMPTY_KEY : (w - 1 < p.nwords ? p.ident[w - 1] : 0);
    }
}

__global__ __launch_bounds__(256) void rehash_kernel(TableDesc src, uint64_t cap, TableDesc dst, AccPlan p,
                                                     int live_word) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride) {
        int64_t *e = src.base + i * (uint64_t)p.stride;
        int64_t k = e[0];
        if (k == GWO_EMPTY_KEY) continue;
        if (live_word >= 0 && e[1 + live_word] <= 0) {   // dead ring entry: drop it
            for (int w = 0; w < p.nwords; ++w) e[1 + w] = p.ident[w];
            e[0] = GWO_EMPTY_KEY;
            continue;
        }
        bool claimed;
        int64_t *a = find_or_insert(dst, p.stride, k, claimed);
        count_claims(dst.occ, claimed);
        for (int w = 0; w < p.nwords; ++w) {
            a[w] = e[1 + w];
            e[1 + w] = p.ident[w];
        }
        e[0] = GWO_EMPTY_KEY;
    }
}

__device__ __forceinline__ const int64_t *table_find(const TableDesc &t, int stride, int64_t key) {
    if (!t.base) return nullptr;
    if (key == GWO_EMPTY_KEY) return t.side[0] != 0 ? t.side + 1 : nullptr;
    uint64_t slot = slot_hash(key) & t.mask;
    while (true) {
        const int64_t *e = t.base + slot * (uint64_t)stride;
        if (e[0] == key) return e + 1;
        if (e[0] == GWO_EMPTY_KEY) return nullptr;
        slot = (slot + 1) & t.mask;
    }
}

// Pane fold: dst (+/-)= src entry-wise.  Sliding windows: add an entering pane to / subtract a
// leaving pane from the running window total, or combine a window's panes (recompute strategy).
// existing == 1: only keys dst already holds (with live_word >= 0: holds live) take src's words -- a restored
// window's entries whose fire timer already fired join the window's next emission only for keys that have new
// records in it (WindowOperator re-registers the timer per (key, window) on a new element); existing == 2: only
// keys dst does not hold yet (the rest of those entries, after the emission).
__global__ __launch_bounds__(256) void fold_kernel(TableDesc src, uint64_t cap, TableDesc dst, AccPlan p, int sign,
                                                   int live_word, unsigned long long *live, int existing) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    long long dlive = 0;   // live entries this lane added (+) or retired (-): one add per wave at the end
    const uint64_t lane = threadIdx.x & 63, lim = (cap + 1 + 63) & ~63ull;   // whole waves iterate together
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i - lane < lim; i += stride) {
        if (i > cap) continue;
        const int64_t *e;
        int64_t k;
        if (i < cap) {
            e = src.base + i * (uint64_t)p.stride;
            k = e[0];
            if (k == GWO_EMPTY_KEY) continue;
        } else {
            if (src.side[0] == 0) continue;
            e = src.side;
            k = GWO_EMPTY_KEY;
        }
        int64_t *a;
        if (existing == 1) {
            a = (int64_t *)table_find(dst, p.stride, k);
            if (!a || (live_word >= 0 && __hip_atomic_load(a + live_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= 0))
                continue;
        } else {
            bool claimed;
            a = find_or_insert(dst, p.stride, k, claimed);
            count_claims(dst.occ, claimed);
            if (existing == 2 && !claimed) continue;
        }
        for (int w = 0; w < p.nwords; ++w) {
            int64_t x = e[1 + w];
            if (sign < 0) x = (int64_t)(0ull - (uint64_t)x);   // ACC_ADD_I64 only: wrap-around inverse
            if (w == live_word) {
                unsigned long long old = atomicAdd((unsigned long long *)(a + w), (unsigned long long)x);
                long long nw = (long long)(old + (unsigned long long)x);
                if ((long long)old <= 0 && nw > 0) dlive++;
                else if ((long long)old > 0 && nw <= 0) dlive--;
            } else {
                atomic_combine(a + w, p.op[w], x);
            }
        }
    }
    if (live) wave_add_signed(live, dlive);
}

// ------------------------------------------------------------------------------------------------
// utility kernels
// ------------------------------------------------------------------------------------------------
__global__ void key_groups_kernel(const int64_t *keys, int64_t n, int kind, int max_par, int par, int32_t *kg,
                                  int32_t *op) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int32_t g = key_group(keys[i], kind, max_par);
        if (kg) kg[i] = g;
        if (op) op[i] = g * par / max_par;  // KeyGroupRangeAssignment.java:118-119
    }
}

// String keys: JDK String.hashCode (h = 31 * h + c over UTF-16 code units, wrapping) -> murmur -> key group.
// One lane per string (keys are short; a long one just loops).
__global__ void key_groups_utf16_kernel(const uint16_t *chars, const int64_t *offsets, int64_t n, int max_par, int par,
                                        int32_t *hash, int32_t *kg, int32_t *op) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t h = 0;
        for (int64_t c = offsets[i], e = offsets[i + 1]; c < e; ++c) h = 31u * h + (uint32_t)chars[c];
        const int32_t m = murmur_hash((int32_t)h);
        const int32_t g = (max_par & (max_par - 1)) == 0 ? (m & (max_par - 1)) : m % max_par;
        if (hash) hash[i] = (int32_t)h;
        if (kg) kg[i] = g;
        if (op) op[i] = g * par / max_par;  // KeyGroupRangeAssignment.java:118-119
    }
}

__global__ void window_starts_kernel(const int64_t *ts, int64_t n, int64_t off, int64_t size, double inv,
                                     int64_t *out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = window_start_f(ts[i], off, size, inv);
}

// Counter-based splitmix64 source (identical definition in oracle/gen.py):
//   u(s, g) = fmix64(seed + s * 0xD1B54A32D192ED03 + (g + 1) * 0x9E3779B97F4A7C15)
__device__ __forceinline__ uint64_t sm_u(uint64_t seed, uint64_t s, uint64_t g) {
    uint64_t z = seed + s * 0xD1B54A32D192ED03ull + (g + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void generate_kernel(uint64_t seed, int64_t first, int64_t total, int64_t nkeys, int64_t span,
                                int64_t disorder, int64_t t0, int64_t vrange, int vf64, int key_mode, int64_t n,
                                int64_t *key, int64_t *ts, int64_t *val) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t g = (uint64_t)(first + i);
        int64_t k;
        if (key_mode == 1) {  // YSB: ad_id uniform over 10*nkeys ads, campaign = ad_id % nkeys
            k = (int64_t)((sm_u(seed, 0, g) % (uint64_t)(10 * nkeys)) % (uint64_t)nkeys);
        } else {
            k = (int64_t)(sm_u(seed, 0, g) % (uint64_t)nkeys);
        }
        key[i] = k;
        int64_t jitter = disorder > 0 ? (int64_t)(sm_u(seed, 2, g) % (uint64_t)disorder) : 0;
        // (g * span) / total without overflow for g, span < 2^63: split the product
        int64_t q = (int64_t)g / total, r = (int64_t)g % total;
        int64_t base_t = q * span + (int64_t)(((__int128)r * span) / total);
        ts[i] = t0 + base_t + jitter;
        if (val) {
            uint64_t u = sm_u(seed, 1, g);
            if (vf64) {
                double d = (double)(u % (uint64_t)vrange) + (double)(sm_u(seed, 3, g) >> 11) * (1.0 / 9007199254740992.0);
                val[i] = __double_as_longlong(d);
            } else {
                val[i] = (int64_t)(u % (uint64_t)vrange);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static inline int grid_for(int64_t n, int per_thread = 1, int cap = 4096) {
    int64_t g = (n + 256LL * per_thread - 1) / (256LL * per_thread);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// ------------------------------------------------------------------------------------------------
// Per-element re-fire (allowedLateness > 0, tumbling): a record whose window already fired but is not
// yet cleaned up is added to the window state and EventTimeTrigger.onElement FIREs at once, emitting
// the window's contents including it (WindowOperator.java:393-406, EventTimeTrigger.java:37-45).  Every
// record of such a (key, window) in a batch is a re-fire, so re-fire j's row is
//   state before the batch  (+)  the batch's re-fire values of that (key, window) up to j, arrival order.
// Device steps: order-preserving compaction of the re-fire records, find-or-claim of their entries
// (reading the state before the batch), a stable radix sort by entry, and a segmented scan that emits
// the rows.  The batch's ordinary insert then adds the same records to the tables.
// ------------------------------------------------------------------------------------------------
#define RF_BLOCKS 256
#define RF_THREADS 256

// Re-fire (record, window) pairs of record i: tumbling, its window if inside the directory (0 or 1);
// sliding, every fired-but-not-cleaned window of the record (u = the first, the rest consecutive).
__device__ __forceinline__ int refire_pairs(const int64_t *ts, int64_t i, const WindowGeom &g, long long dir_base,
                                           int dir_len, long long &u) {
    u = 0;
    if (classify(ts[i], g, u) != REC_REFIRE) return 0;
    if (g.sliding) {
        long long ja, jb;
        slide_refire_windows(ts[i], g, ja, jb);
        u = ja;
        return (int)(jb - ja + 1);
    }
    return u - dir_base >= 0 && u - dir_base < dir_len;
}

// per block: re-fire pairs of its contiguous share of the batch
__global__ __launch_bounds__(RF_THREADS) void refire_count_kernel(const int64_t *__restrict__ ts, int64_t n,
                                                                  WindowGeom g, long long dir_base, int dir_len,
                                                                  uint32_t *blk) {
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
    unsigned c = 0;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += RF_THREADS) {
        long long u;
        c += (unsigned)refire_pairs(ts, i, g, dir_base, dir_len, u);
    }
    unsigned total;
    (void)block_exclusive_scan(c, &total);
    if (threadIdx.x == 0) blk[blockIdx.x] = total;
}

// writes the re-fire pairs of each block's share in arrival order (a record's windows ascending):
// r_idx (batch index), r_u (window)
__global__ __launch_bounds__(RF_THREADS) void refire_write_kernel(const int64_t *__restrict__ ts, int64_t n,
                                                                  WindowGeom g, long long dir_base, int dir_len,
                                                                  const uint32_t *blk, int64_t *r_idx,
                                                                  long long *r_u) {
    __shared__ unsigned s_base;
    if (threadIdx.x == 0) {
        unsigned b = 0;
        for (unsigned x = 0; x < blockIdx.x; ++x) b += blk[x];
        s_base = b;
    }
    __syncthreads();
    unsigned base = s_base;
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
    for (int64_t i0 = b0; i0 < b1; i0 += RF_THREADS) {
        const int64_t i = i0 + threadIdx.x;
        long long u = 0;
        const int c = i < b1 ? refire_pairs(ts, i, g, dir_base, dir_len, u) : 0;
        unsigned total;
        const unsigned at = block_exclusive_scan((unsigned)c, &total);
        for (int x = 0; x < c; ++x) {
            r_idx[base + at + x] = i;
            r_u[base + at + x] = u + x;
        }
        base += total;
    }
}

// Sliding: pair q's entry is (key, window); its sort key is key slot * nj + (window - j0), the key slot
// from a scratch table of the batch's re-fire keys (slot words hold key ^ 2^63, 0 = free; the empty-key
// marker itself takes slot cap).  `before` = the window's state before the batch: its panes' entries
// for the key, combined (the panes are the pane directory [pane_base, pane_base + pane_len)).

__global__ __launch_bounds__(RF_THREADS) void slide_refire_slot_kernel(
    const int64_t *__restrict__ key, const int64_t *r_idx, const long long *r_u, int64_t m, AccPlan p, WindowGeom g,
    unsigned long long *keytab, uint64_t kmask, long long j0, uint32_t nj, const TableDesc *__restrict__ pdir,
    long long pane_base, long long pane_len, const TableDesc *__restrict__ wdir, uint32_t *r_slot, int64_t *before) {
    const int64_t om = jsub(g.offset, fdiv_floor(g.offset, g.slide, g.inv_slide) * g.slide);
    const long long panes = g.size / g.unit;
    for (int64_t j = (int64_t)blockIdx.x * RF_THREADS + threadIdx.x; j < m; j += (int64_t)gridDim.x * RF_THREADS) {
        const int64_t k = key[r_idx[j]];
        uint64_t ks = kmask + 1;
        if (k != GWO_EMPTY_KEY) {
            const unsigned long long enc = (unsigned long long)k ^ 0x8000000000000000ull;
            ks = slot_hash(k) & kmask;
            while (true) {
                const unsigned long long prev = atomicCAS(&keytab[ks], 0ull, enc);
                if (prev == 0ull || prev == enc) break;
                ks = (ks + 1) & kmask;
            }
        }
        const long long w = r_u[j];
        r_slot[j] = (uint32_t)(ks * nj + (uint64_t)(w - j0));
        int64_t acc[GWO_MAX_WORDS];
        for (int x = 0; x < p.nwords; ++x) acc[x] = p.ident[x];
        const int64_t start = (int64_t)((uint64_t)w * (uint64_t)g.slide + (uint64_t)om);
        const long long u0 = fdiv_floor(jsub(start, g.unit_off_mod), g.unit, g.inv_unit);
        for (long long u = u0; u < u0 + panes; ++u) {
            const long long d = u - pane_base;
            if (d < 0 || d >= pane_len) continue;
            const int64_t *e = table_find(pdir[d], p.stride, k);
            if (e)
                for (int x = 0; x < p.nwords; ++x) acc[x] = combine(p.op[x], acc[x], e[x]);
        }
        if (wdir)   // the window's entries restored from a per-window savepoint (pending and fired ones)
            for (int h = 0; h < 2; ++h) {
                const int64_t *e = table_find(wdir[2 * (w - j0) + h], p.stride, k);
                if (e)
                    for (int x = 0; x < p.nwords; ++x) acc[x] = combine(p.op[x], acc[x], e[x]);
            }
        for (int x = 0; x < p.nwords; ++x) before[j * GWO_MAX_WORDS + x] = acc[x];
    }
}

// find-or-claim each re-fire record's entry; sort key = the entry's global slot, before = its words
__global__ __launch_bounds__(RF_THREADS) void refire_slot_kernel(const int64_t *__restrict__ key, const int64_t *r_idx,
                                                                 const long long *r_u, int64_t m, AccPlan p,
                                                                 const TableDesc *__restrict__ dir, long long dir_base,
                                                                 const uint64_t *slot_off, uint32_t *r_slot,
                                                                 int64_t *before) {
    for (int64_t j0 = (int64_t)blockIdx.x * RF_THREADS; j0 < m; j0 += (int64_t)gridDim.x * RF_THREADS) {
        const int64_t j = j0 + threadIdx.x;
        bool claimed = false;
        unsigned long long *occ = nullptr;
        if (j < m) {
            const int d = (int)(r_u[j] - dir_base);
            const TableDesc t = dir[d];
            const int64_t k = key[r_idx[j]];
            int64_t *acc = find_or_insert(t, p.stride, k, claimed);
            occ = t.occ;
            const uint64_t local = k == GWO_EMPTY_KEY ? t.mask + 1 : (uint64_t)(acc - 1 - t.base) / (uint64_t)p.stride;
            r_slot[j] = (uint32_t)(slot_off[d] + local);
            for (int w = 0; w < p.nwords; ++w) before[j * GWO_MAX_WORDS + w] = acc[w];
        }
        count_claims(occ, claimed);
    }
}

// One workgroup: segmented inclusive scan of the sorted re-fire records (segment = entry) in chunks of
// 1024, each row = before (+) prefix, written to rows [base, base + m) of the output.
__global__ __launch_bounds__(1024) void refire_emit_kernel(const int64_t *__restrict__ key,
                                                           const int64_t *__restrict__ val, const int64_t *r_idx,
                                                           const long long *r_u, int64_t m, const uint32_t *skey,
                                                           const uint32_t *spay, const int64_t *before, AccPlan p,
                                                           ResultPlan rp, int64_t unit, int64_t unit_off_mod,
                                                           int64_t span, OutCols o) {
    __shared__ int64_t s_x[1024][GWO_MAX_WORDS];
    __shared__ uint32_t s_slot[1024];
    __shared__ uint8_t s_flag[1024];
    __shared__ unsigned long long s_base;
    __shared__ uint32_t c_slot;
    __shared__ int64_t c_x[GWO_MAX_WORDS];
    const int t = threadIdx.x, NW = p.nwords;
    if (t == 0) {
        s_base = atomicAdd(o.count, (unsigned long long)m);
        c_slot = 0xffffffffu;
    }
    __syncthreads();
    for (int64_t q0 = 0; q0 < m; q0 += 1024) {
        const int64_t q = q0 + t;
        const bool live = q < m;
        const uint32_t j = live ? spay[q] : 0u;
        const uint32_t sl = live ? skey[q] : 0xfffffffeu;
        const int64_t vb = live && val ? val[r_idx[j]] : 0;
        int64_t x[GWO_MAX_WORDS];
        for (int w = 0; w < NW; ++w) x[w] = lift_word(p, w, vb);
        s_slot[t] = sl;
        __syncthreads();
        // a segment starts where the entry changes (element 0: against the previous chunk's last entry)
        uint8_t f = t == 0 ? (sl != c_slot) : (sl != s_slot[t - 1]);
        if (t == 0 && !f)   // continues the previous chunk's segment: fold its running value in first
            for (int w = 0; w < NW; ++w) x[w] = combine(p.op[w], c_x[w], x[w]);
        for (int w = 0; w < NW; ++w) s_x[t][w] = x[w];
        s_flag[t] = f;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            int64_t y[GWO_MAX_WORDS];
            uint8_t fy = 1;
            if (t >= off && !s_flag[t]) {
                fy = s_flag[t - off];
                for (int w = 0; w < NW; ++w) y[w] = s_x[t - off][w];
            }
            __syncthreads();
            if (t >= off && !s_flag[t]) {
                for (int w = 0; w < NW; ++w) s_x[t][w] = combine(p.op[w], y[w], s_x[t][w]);
                s_flag[t] = fy;
            }
            __syncthreads();
        }
        if (live) {
            int64_t acc[GWO_MAX_WORDS];
            for (int w = 0; w < NW; ++w) acc[w] = combine(p.op[w], before[(int64_t)j * GWO_MAX_WORDS + w], s_x[t][w]);
            const unsigned long long pos = s_base + (unsigned long long)q;
            if ((long long)pos < o.cap) {
                const int64_t start = (int64_t)((uint64_t)r_u[j] * (uint64_t)unit + (uint64_t)unit_off_mod);
                o.key[pos] = key[r_idx[j]];
                o.start[pos] = start;
                o.end[pos] = (int64_t)((uint64_t)start + (uint64_t)span);
                write_results(p, rp, acc, o, pos);
            }
        }
        __syncthreads();
        const int last = (int)min((int64_t)1023, m - 1 - q0);
        if (t == last) {
            c_slot = s_slot[t];
            for (int w = 0; w < NW; ++w) c_x[w] = s_x[t][w];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// Restore of table state (the heap backend's per-(key, namespace) entries, CopyOnWriteStateMapSnapshot.java:
// 127-129): raw accumulator words, so a restore continues exactly (collection: gwo_snapshot.hip).
// ------------------------------------------------------------------------------------------------
// Rows whose key group is outside [kg_lo, kg_hi] belong to another subtask (rescaling) and are skipped.
__global__ __launch_bounds__(256) void restore_kernel(const int64_t *key, const int64_t *wstart, const int64_t *words,
                                                      int64_t n, AccPlan p, WindowGeom g,
                                                      const TableDesc *__restrict__ dir, long long dir_base,
                                                      int dir_len) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x; j0 < n; j0 += stride) {
        const int64_t j = j0 + threadIdx.x;
        bool claimed = false;
        unsigned long long *occ = nullptr;
        if (j < n) {
            const int64_t k = key[j];
            const int32_t kg = key_group(k, g.key_kind, g.max_par);
            const long long d = fdiv_floor(jsub(wstart[j], g.unit_off_mod), g.unit, g.inv_unit) - dir_base;
            if (kg >= g.kg_lo && kg <= g.kg_hi && d >= 0 && d < dir_len) {
                const TableDesc t = dir[d];
                int64_t *acc = find_or_insert(t, p.stride, k, claimed);
                occ = t.occ;
                for (int w = 0; w < p.nwords; ++w) atomic_combine(acc + w, p.op[w], words[j * p.nwords + w]);
            }
        }
        count_claims(occ, claimed);
    }
}

void launch_restore(const int64_t *key, const int64_t *wstart, const int64_t *words, int64_t n, const AccPlan &p,
                    const WindowGeom &g, const TableDesc *dir, long long dir_base, int dir_len, hipStream_t s) {
    hipLaunchKernelGGL(restore_kernel, dim3(grid_for(n, 1, 4096)), dim3(256), 0, s, key, wstart, words, n, p, g, dir,
                       dir_base, dir_len);
}

void launch_refire_collect(const int64_t *ts, int64_t n, const WindowGeom &g, long long dir_base, int dir_len,
                           uint32_t *blk, int64_t *r_idx, long long *r_u, hipStream_t s) {
    hipLaunchKernelGGL(refire_count_kernel, dim3(RF_BLOCKS), dim3(RF_THREADS), 0, s, ts, n, g, dir_base, dir_len, blk);
    hipLaunchKernelGGL(refire_write_kernel, dim3(RF_BLOCKS), dim3(RF_THREADS), 0, s, ts, n, g, dir_base, dir_len, blk,
                       r_idx, r_u);
}

void launch_refire_slots(const int64_t *key, const int64_t *r_idx, const long long *r_u, int64_t m, const AccPlan &p,
                         const TableDesc *dir, long long dir_base, const uint64_t *slot_off, uint32_t *r_slot,
                         int64_t *before, hipStream_t s) {
    int blocks = (int)std::min<int64_t>(1024, (m + RF_THREADS - 1) / RF_THREADS);
    hipLaunchKernelGGL(refire_slot_kernel, dim3(std::max(blocks, 1)), dim3(RF_THREADS), 0, s, key, r_idx, r_u, m, p,
                       dir, dir_base, slot_off, r_slot, before);
}

void launch_refire_emit(const int64_t *key, const int64_t *val, const int64_t *r_idx, const long long *r_u, int64_t m,
                        const uint32_t *skey, const uint32_t *spay, const int64_t *before, const AccPlan &p,
                        const ResultPlan &rp, int64_t unit, int64_t unit_off_mod, int64_t span, OutCols o,
                        hipStream_t s) {
    hipLaunchKernelGGL(refire_emit_kernel, dim3(1), dim3(1024), 0, s, key, val, r_idx, r_u, m, skey, spay, before, p, rp,
                       unit, unit_off_mod, span, o);
}

void launch_slide_refire_slots(const int64_t *key, const int64_t *r_idx, const long long *r_u, int64_t m,
                               const AccPlan &p, const WindowGeom &g, unsigned long long *keytab, uint64_t kmask,
                               long long j0, uint32_t nj, const TableDesc *pdir, long long pane_base,
                               long long pane_len, const TableDesc *wdir, uint32_t *r_slot, int64_t *before,
                               hipStream_t s) {
    int blocks = (int)std::min<int64_t>(1024, (m + RF_THREADS - 1) / RF_THREADS);
    hipLaunchKernelGGL(slide_refire_slot_kernel, dim3(std::max(blocks, 1)), dim3(RF_THREADS), 0, s, key, r_idx, r_u, m,
                       p, g, keytab, kmask, j0, nj, pdir, pane_base, pane_len, wdir, r_slot, before);
}

// Copies nw device words into a host-mapped readback block, sequence word last (the host spins on it instead of a
// copy and a stream synchronisation).  Agent-scope loads: the words were written by earlier kernels' atomics.
__global__ __launch_bounds__(64) void publish_words_kernel(const unsigned long long *src, int nw,
                                                           unsigned long long *rb, unsigned long long seq) {
    for (int t = threadIdx.x; t < nw; t += 64)
        rb_put(&rb[t], __hip_atomic_load(&src[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    rb_publish(&rb[nw], seq);
}

void launch_publish_words(const unsigned long long *src, int nw, unsigned long long *rb, unsigned long long seq,
                          hipStream_t s) {
    hipLaunchKernelGGL(publish_words_kernel, dim3(1), dim3(64), 0, s, src, nw, rb, seq);
}

// One word into device memory, in stream order (a value travelling in the launch's arguments instead of a copy from
// host memory).
__global__ __launch_bounds__(64) void put_word_kernel(unsigned long long *dst, unsigned long long v) {
    if (threadIdx.x == 0) *dst = v;
}

void launch_put_word(unsigned long long *dst, unsigned long long v, hipStream_t s) {
    hipLaunchKernelGGL(put_word_kernel, dim3(1), dim3(64), 0, s, dst, v);
}

void launch_scan(const int64_t *key, const int64_t *ts, int64_t n, const WindowGeom &g, long long hist_base,
                 BatchStats *stats, int64_t *side_key, int64_t *side_ts, int64_t *side_val, const int64_t *val,
                 unsigned long long *side_count, long long side_cap, int side_enabled, unsigned long long *shards,
                 hipStream_t s, const ScanSpec *spec) {
    ScanSpec sp{};
    if (spec) sp = *spec;
    hipLaunchKernelGGL(scan_kernel, dim3(grid_for(n, 4, 2048)), dim3(256), 0, s, key, ts, val, n, g, hist_base,
                       stats, side_key, side_ts, side_val, side_count, side_cap, side_enabled, shards, sp);
}

void launch_insert(const int64_t *key, const int64_t *ts, const void *val, int64_t n, const WindowGeom &g,
                   const AccPlan &plan, const TableDesc *dir, long long dir_base, int dir_len, int preagg,
                   BatchStats *st, const RingDesc &ring, hipStream_t s, const uint32_t *go) {
    unsigned long long *partials = &st->partials;
    const int64_t *v = (const int64_t *)val;
    if (preagg && plan.nwords <= PREAGG_WORDS) {
        int grid = (int)((n + PREAGG_TILE - 1) / PREAGG_TILE);
        if (grid > 2048) grid = 2048;
        if (grid < 1) grid = 1;
        hipLaunchKernelGGL(insert_preagg_kernel, dim3(grid), dim3(256), 0, s, key, ts, v, n, g, plan, dir, dir_base,
                           dir_len, st, partials, ring);
    } else {
        int grid = grid_for(n, 1, 8192);
        hipLaunchKernelGGL(insert_direct_kernel, dim3(grid), dim3(256), 0, s, key, ts, v, n, g, plan, dir, dir_base,
                           dir_len, st, ring, go);
    }
}

void launch_fire(const TableDesc &t, uint64_t cap, const AccPlan &plan, const ResultPlan &rp, int64_t start,
                 int64_t end, OutCols out, int reset, int live_word, hipStream_t s) {
    int grid = grid_for((int64_t)cap + 1, FIRE_FPT, 4096);
    hipLaunchKernelGGL(fire_kernel, dim3(grid), dim3(256), 0, s, t, cap, plan, rp, start, end, out, reset, live_word);
}

void launch_fill(int64_t *base, uint64_t cap, const AccPlan &plan, hipStream_t s) {
    uint64_t words = cap * (uint64_t)plan.stride;
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for((int64_t)words, 4, 8192)), dim3(256), 0, s, base, words, plan);
}

void launch_rehash(const TableDesc &src, uint64_t src_cap, const TableDesc &dst, const AccPlan &plan,
                   hipStream_t s) {
    int grid = grid_for((int64_t)src_cap, 1, 8192);
    hipLaunchKernelGGL(rehash_kernel, dim3(grid), dim3(256), 0, s, src, src_cap, dst, plan, -1);
}

void launch_rehash_live(const TableDesc &src, uint64_t src_cap, const TableDesc &dst, const AccPlan &plan,
                        int live_word, hipStream_t s) {
    int grid = grid_for((int64_t)src_cap, 1, 8192);
    hipLaunchKernelGGL(rehash_kernel, dim3(grid), dim3(256), 0, s, src, src_cap, dst, plan, live_word);
}

void launch_fold(const TableDesc &src, uint64_t src_cap, const TableDesc &dst, const AccPlan &plan, int sign,
                 int live_word, unsigned long long *live, hipStream_t s, int existing) {
    int grid = grid_for((int64_t)src_cap + 1, 1, 8192);
    hipLaunchKernelGGL(fold_kernel, dim3(grid), dim3(256), 0, s, src, src_cap, dst, plan, sign, live_word, live,
                       existing);
}

// Rows (key, nwords raw words; row-major) combined into one table: a restored sliding window's entries.
__global__ __launch_bounds__(256) void rows_insert_kernel(const int64_t *key, const int64_t *words, int64_t n,
                                                          TableDesc t, AccPlan p) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool claimed;
        int64_t *a = find_or_insert(t, p.stride, key[i], claimed);
        count_claims(t.occ, claimed);
        for (int w = 0; w < p.nwords; ++w) atomic_combine(a + w, p.op[w], words[i * p.nwords + w]);
    }
}

void launch_rows_insert(const int64_t *key, const int64_t *words, int64_t n, const TableDesc &t, const AccPlan &p,
                        hipStream_t s) {
    hipLaunchKernelGGL(rows_insert_kernel, dim3(grid_for(n, 1, 4096)), dim3(256), 0, s, key, words, n, t, p);
}

void launch_key_groups(const int64_t *keys, int64_t n, int key_kind, int max_par, int par, int32_t *kg,
                       int32_t *op, hipStream_t s) {
    hipLaunchKernelGGL(key_groups_kernel, dim3(grid_for(n, 4)), dim3(256), 0, s, keys, n, key_kind, max_par, par,
                       kg, op);
}

void launch_key_groups_utf16(const uint16_t *chars, const int64_t *offsets, int64_t n, int max_par, int par,
                             int32_t *hash, int32_t *kg, int32_t *op, hipStream_t s) {
    hipLaunchKernelGGL(key_groups_utf16_kernel, dim3(grid_for(n, 1)), dim3(256), 0, s, chars, offsets, n, max_par, par,
                       hash, kg, op);
}

void launch_window_starts(const int64_t *ts, int64_t n, int64_t offset, int64_t size, int64_t *out,
                          hipStream_t s) {
    hipLaunchKernelGGL(window_starts_kernel, dim3(grid_for(n, 4)), dim3(256), 0, s, ts, n, offset, size,
                       1.0 / (double)size, out);
}

void launch_generate(uint64_t seed, int64_t first, int64_t total, int64_t nkeys, int64_t span, int64_t disorder,
                     int64_t t0, int64_t vrange, int vf64, int key_mode, int64_t n, int64_t *key, int64_t *ts,
                     void *val, hipStream_t s) {
    hipLaunchKernelGGL(generate_kernel, dim3(grid_for(n, 4, 8192)), dim3(256), 0, s, seed, first, total, nkeys,
                       span, disorder, t0, vrange, vf64, key_mode, n, key, ts, (int64_t *)val);
}

size_t gather_lds_bytes(int S, int nwords) { return (size_t)CB_NU * S * (1 + nwords) * 8 + 64 * 8; }
int gather_tile() { return CB_TILE; }
int gather_stat_words() { return CB_SHARDS * CS_WORDS; }

void launch_gather(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const WindowGeom &g,
                   const AccPlan &p, const CombineArgs &a, int grid, BatchStats *st, int64_t *side_key, int64_t *side_ts,
                   int64_t *side_val, unsigned long long *side_count, long long side_cap, int side_enabled,
                   hipStream_t s) {
    GatherArgs A{key, ts, val, n, g, p, a, st, side_key, side_ts, side_val, side_count, side_cap, side_enabled};
#define GATHER(NWT) \
    hipLaunchKernelGGL(gather_kernel<NWT>, dim3(grid), dim3(CB_THREADS), gather_lds_bytes(a.S, p.nwords), s, A)
    switch (p.nwords) {
        case 1: GATHER(1); break;
        case 2: GATHER(2); break;
        case 3: GATHER(3); break;
        case 4: GATHER(4); break;
        default: GATHER(0); break;
    }
#undef GATHER
}

void launch_merge(const int64_t *key, const int64_t *ts, const int64_t *val, const WindowGeom &g, const AccPlan &p,
                  const CombineArgs &a, int G, uint64_t novf, const TableDesc *dir, long long dir_base, int dir_len,
                  const RingDesc &ring, const uint32_t *go, hipStream_t s) {
    const int64_t runs = (G + CB_MERGE_RUN - 1) / CB_MERGE_RUN;
    int64_t dump_threads = (int64_t)CB_NU * a.S * runs;
    dump_threads = (dump_threads + 255) / 256 * 256;
    const int64_t total = dump_threads + (int64_t)novf;
    hipLaunchKernelGGL(merge_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, key, ts, val, g, p, a, G,
                       dump_threads, novf, dir, dir_base, dir_len, ring, go);
}

}  // namespace gwo
