// gwo_log.hip -- log-structured window state for high-cardinality tumbling windows.
//
// The reference keeps one accumulator per (key, window) in a heap hash map and updates it per
// record (HeapAggregatingState.add, HeapAggregatingState.java:96-109; StateTable.transform,
// heap/StateTable.java:194-202).  On MI355X a random read-modify-write of a 32-B entry in an
// 8-GB table costs a 64-128-B line round trip per record, and device-scope atomics execute at the
// memory side (tools/micro_table.hip).  For windows that receive about as many distinct keys as
// records (config C4: 166M records -> 81M (key, window) pairs) this path defers the aggregation to
// the window's fire instead:
//
//   per batch  log_part   (K1) classify every record (WindowOperator.java:386-427), check its key
//                         group, count late records / route them to the side output, and group the
//                         accepted (key, value) pairs of a 3584-record tile by (window, coarse digit)
//                         in LDS; each group is appended with one cursor reservation to its bucket
//                         of the batch buffer (fixed-capacity buckets, overflow -> exact rerun)
//              log_split  (pass 2) one workgroup per 3584-record chunk of a bucket groups it by the
//                         fine partition bits in LDS and appends each group to its partition of the
//                         window's new segment (fixed-capacity partitions, overflow -> rerun)
//   at fire    log_fire   one workgroup per partition folds the partition's records from every
//                         segment of the window into an LDS hash table and emits one row per key
//                         (WindowOperator.onEventTime + emitWindowContents, WindowOperator.java:430-473,546-550)
//
// Every HBM byte moves as a coalesced stream or as a run of consecutive 16-B records; the only
// random accesses are LDS.
#include "gwo_device.h"
#include "gwo_log.h"

namespace gwo {

typedef long long ll2 __attribute__((ext_vector_type(2)));

enum LogClass : int { L_ACCEPT = 0, L_LATE = 1, L_SKIP = 2, L_REFIRE = 3, L_BAD_TS = 4 };

// Tumbling classification, WindowOperator.java:386-427 + TumblingEventTimeWindows.java:68-81.
__device__ __forceinline__ int log_classify(int64_t ts, const WindowGeom &g, long long &unit) {
    if (ts == GWO_LONG_MIN) return L_BAD_TS;
    int64_t start = window_start_f(ts, g.offset, g.size, g.inv_size);
    int64_t max_ts = jsub(jadd(start, g.size), 1);
    if (cleanup_time(max_ts, g.lateness) <= g.wm) return jadd(ts, g.lateness) <= g.wm ? L_LATE : L_SKIP;
    if (max_ts <= g.wm) return L_REFIRE;
    unit = fdiv_floor(start, g.size, g.inv_size);
    return L_ACCEPT;
}

// Exclusive prefix over nb (<= 1024) LDS counters s_cnt -> s_off; thread t owns the `per`
// consecutive counters [t*per, t*per+per).  Returns the total.  All threads call it; ends
// synchronised, so s_off is complete on return.
__device__ __forceinline__ uint32_t tile_offsets(const uint32_t *s_cnt, uint32_t *s_off, int nb, uint32_t loc[4],
                                                 int per) {
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int b = threadIdx.x * per + q;
        loc[q] = (q < per && b < nb) ? s_cnt[b] : 0u;
        sum += loc[q];
    }
    uint32_t total;
    uint32_t ex = block_exclusive_scan(sum, &total);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int b = threadIdx.x * per + q;
        if (q < per && b < nb) s_off[b] = ex;
        ex += loc[q];
    }
    __syncthreads();   // every thread reads other threads' s_off next
    return total;
}

// ------------------------------------------------------------------------------------------------
// K1 log_part: batch -> batch buffer, grouped by bucket b = (window - base) * 256 + coarse digit.
// Bucket b owns records [b*cap, (b+1)*cap) of the buffer; cursor[b*LOG_CUR_STRIDE] ends as its record
// count (also when it exceeds cap: those records are not written and the host reruns).
// ------------------------------------------------------------------------------------------------
template <bool HASV>
__global__ __launch_bounds__(LOG_K1_THREADS) void log_part_kernel(
    const int64_t *__restrict__ key, const int64_t *__restrict__ ts, const int64_t *__restrict__ val, int64_t n,
    int64_t stride, WindowGeom g, long long base, int nunits, unsigned long long *__restrict__ cursor, uint64_t cap,
    int64_t *__restrict__ tmp, BatchStats *st, int64_t *side_key, int64_t *side_ts, int64_t *side_val,
    unsigned long long *side_count, long long side_cap, int side_enabled) {
    constexpr int W = HASV ? 2 : 1;
    __shared__ __attribute__((aligned(16))) int64_t s_rec[LOG_TILE * W];
    __shared__ uint16_t s_bk[LOG_TILE];
    __shared__ uint32_t s_cnt[LOG_NU * 256];
    __shared__ uint32_t s_off[LOG_NU * 256];
    __shared__ long long s_min[LOG_K1_THREADS / 64], s_max[LOG_K1_THREADS / 64];
    const int nb = nunits * 256;
    const int per = (nb + LOG_K1_THREADS - 1) / LOG_K1_THREADS;   // counters owned per thread (<= 4)
    const int tid = threadIdx.x;
    long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000LL;
    unsigned long long acc = 0, late = 0, refire = 0, bad_ts = 0, out = 0, bad_kg = 0;
    int64_t kk[LOG_K1_PER], vv[LOG_K1_PER], tt[LOG_K1_PER];
    // unconditional loads of a tile (lanes past the end re-read the tile's first record and are
    // discarded); the next tile's loads are issued before this tile's write phase
    auto load_tile = [&](int64_t tile) {
#pragma unroll
        for (int j = 0; j < LOG_K1_PER; ++j) {
            int64_t i = tile + j * LOG_K1_THREADS + tid;
            i = i < n ? i : (tile < n ? tile : 0);
            tt[j] = __builtin_nontemporal_load(ts + i * stride);
            kk[j] = __builtin_nontemporal_load(key + i * stride);
            vv[j] = HASV ? __builtin_nontemporal_load(val + i * stride) : 0;
        }
    };
    const int64_t tstride = (int64_t)gridDim.x * LOG_TILE;
    if ((int64_t)blockIdx.x * LOG_TILE < n) load_tile((int64_t)blockIdx.x * LOG_TILE);
    for (int64_t tile = (int64_t)blockIdx.x * LOG_TILE; tile < n; tile += tstride) {
        for (int i = tid; i < nb; i += LOG_K1_THREADS) s_cnt[i] = 0;
        __syncthreads();
        uint32_t code[LOG_K1_PER];
#pragma unroll
        for (int j = 0; j < LOG_K1_PER; ++j) {
            int64_t i = tile + j * LOG_K1_THREADS + tid;
            code[j] = 0xffffffffu;
            if (i >= n) continue;
            long long u = 0;
            int c = log_classify(tt[j], g, u);
            if (c == L_ACCEPT) {
                int64_t k = kk[j];
                int32_t kg = key_group(k, g.key_kind, g.max_par);
                if (kg < g.kg_lo || kg > g.kg_hi) {
                    bad_kg++;
                    st->bad_kg_key = k;
                }
                acc++;
                mn = u < mn ? u : mn;
                mx = u > mx ? u : mx;
                long long w = u - base;
                if (w >= 0 && w < nunits) {
                    uint32_t b = (uint32_t)(w * 256 + (int)(part_hash(k) >> 56));
                    uint32_t r = atomicAdd(&s_cnt[b], 1u);
                    code[j] = (b << 16) | r;
                } else {
                    out++;
                }
            } else if (c == L_LATE) {
                late++;
                if (side_enabled) {
                    unsigned long long pos = atomicAdd(side_count, 1ull);
                    if ((long long)pos < side_cap) {
                        side_key[pos] = kk[j];
                        side_ts[pos] = tt[j];
                        side_val[pos] = val ? val[i * stride] : 0;
                    }
                }
            } else if (c == L_REFIRE) {
                refire++;
            } else if (c == L_BAD_TS) {
                bad_ts++;
            }
        }
        __syncthreads();
        uint32_t loc[4];
        const uint32_t total = tile_offsets(s_cnt, s_off, nb, loc, per);
        // reserve each bucket's run (the atomics' round trip overlaps the LDS scatter below);
        // s_cnt[b] becomes the run's first record in the bucket
        unsigned long long at[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int b = tid * per + q;
            at[q] = 0;
            if (q < per && loc[q]) at[q] = atomicAdd(&cursor[(size_t)b * LOG_CUR_STRIDE], (unsigned long long)loc[q]);
        }
#pragma unroll
        for (int j = 0; j < LOG_K1_PER; ++j) {
            if (code[j] == 0xffffffffu) continue;
            uint32_t b = code[j] >> 16;
            uint32_t pos = s_off[b] + (code[j] & 0xffffu);
            if (HASV) {
                ll2 r2 = {kk[j], vv[j]};
                *(ll2 *)&s_rec[2 * pos] = r2;
            } else {
                s_rec[pos] = kk[j];
            }
            s_bk[pos] = (uint16_t)b;
        }
        if (tile + tstride < n) load_tile(tile + tstride);   // next tile in flight during the writes
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int b = tid * per + q;
            if (q < per && loc[q]) s_cnt[b] = (uint32_t)(at[q] < cap ? at[q] : cap);
        }
        __syncthreads();
        for (uint32_t p = tid; p < total; p += LOG_K1_THREADS) {
            uint32_t b = s_bk[p];
            if (b >= (uint32_t)nb) continue;   // defensive: never a write outside the buffer
            uint64_t q = (uint64_t)s_cnt[b] + (p - s_off[b]);
            if (q < cap) {
                int64_t *dst = tmp + ((uint64_t)b * cap + q) * W;
                if (HASV) *(ll2 *)dst = *(const ll2 *)&s_rec[2 * p];
                else *dst = s_rec[p];
            }
        }
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) {
        long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    wave_atomic_add(&st->accepted, acc);
    wave_atomic_add(&st->late, late);
    wave_atomic_add(&st->refire, refire);
    wave_atomic_add(&st->bad_ts, bad_ts);
    wave_atomic_add(&st->hist_out, out);
    wave_atomic_add(&st->bad_kg, bad_kg);
    const int lane = tid & 63, wid = tid >> 6;
    if (lane == 0) {
        s_min[wid] = mn;
        s_max[wid] = mx;
    }
    __syncthreads();
    if (tid == 0) {
        long long a = s_min[0], b = s_max[0];
        for (int w = 1; w < LOG_K1_THREADS / 64; ++w) {
            a = s_min[w] < a ? s_min[w] : a;
            b = s_max[w] > b ? s_max[w] : b;
        }
        if (a != 0x7fffffffffffffffLL) {
            atomicMin(&st->min_idx, a);
            atomicMax(&st->max_idx, b);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Pass 2 log_split: workgroup = one LOG_TILE chunk of one bucket (window w, coarse digit d).
// Partition p = top lp bits of part_hash = d * F + f, F = 2^(lp-8).  Partition p of the segment owns
// records [seg_base + f*pcap, + pcap); cnt[p] is its cursor (ends as its count, overflow -> rerun).
// ------------------------------------------------------------------------------------------------
template <bool HASV>
__global__ __launch_bounds__(LOG_TILE_THREADS) void log_split_kernel(const int64_t *__restrict__ tmp,
                                                                     const LogBucket *__restrict__ bk, int nb,
                                                                     const LogSegDesc *__restrict__ segs,
                                                                     unsigned *overflow) {
    constexpr int W = HASV ? 2 : 1;
    __shared__ __attribute__((aligned(16))) int64_t s_rec[LOG_TILE * W];
    __shared__ uint16_t s_bk[LOG_TILE];
    __shared__ uint32_t s_cnt[1024];
    __shared__ uint32_t s_off[1024];
    __shared__ int s_c;
    const int tid = threadIdx.x;
    // this chunk's bucket: the largest c with bk[c].chunk0 <= blockIdx.x (one parallel load of the
    // nb chunk prefixes into LDS, then a binary search there)
    for (int c = tid; c < nb; c += LOG_TILE_THREADS) s_off[c] = bk[c].chunk0;
    __syncthreads();
    if (tid == 0) {
        int lo = 0, hi = nb;
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (s_off[mid] <= blockIdx.x) lo = mid;
            else hi = mid;
        }
        s_c = lo;
    }
    __syncthreads();
    const int c = s_c;
    const LogBucket B = bk[c];
    const uint32_t chunk = blockIdx.x - B.chunk0;
    const int w = c >> 8, d = c & 255;
    const LogSegDesc S = segs[w];
    const int lp = S.lp, fb = lp - 8, F = 1 << fb;
    if (chunk == 0)
        for (int f = tid; f < F; f += LOG_TILE_THREADS) S.off[d * F + f] = B.seg_base + (uint32_t)f * B.pcap;
    for (int f = tid; f < F; f += LOG_TILE_THREADS) s_cnt[f] = 0;
    __syncthreads();
    const uint32_t begin = chunk * LOG_TILE;
    const uint32_t m = min((uint32_t)LOG_TILE, B.n - begin);
    int64_t kk[LOG_TILE_PER], vv[LOG_TILE_PER];
    uint32_t code[LOG_TILE_PER];
    // unconditional loads (a lane past the end re-reads the chunk's first record): no branch per load
#pragma unroll
    for (int j = 0; j < LOG_TILE_PER; ++j) {
        uint32_t i = j * LOG_TILE_THREADS + tid;
        const int64_t *src = tmp + (B.src + begin + (i < m ? i : 0u)) * W;
        if (HASV) {
            ll2 r2 = __builtin_nontemporal_load((const ll2 *)src);
            kk[j] = r2.x;
            vv[j] = r2.y;
        } else {
            kk[j] = __builtin_nontemporal_load(src);
            vv[j] = 0;
        }
    }
#pragma unroll
    for (int j = 0; j < LOG_TILE_PER; ++j) {
        uint32_t i = j * LOG_TILE_THREADS + tid;
        code[j] = 0xffffffffu;
        if (i < m) {
            uint32_t f = (uint32_t)(part_hash(kk[j]) >> (64 - lp)) & (uint32_t)(F - 1);
            uint32_t r = atomicAdd(&s_cnt[f], 1u);
            code[j] = (f << 16) | r;
        }
    }
    __syncthreads();
    const int per = F <= LOG_TILE_THREADS ? 1 : F / LOG_TILE_THREADS;
    uint32_t loc[4];
    const uint32_t total = tile_offsets(s_cnt, s_off, F, loc, per);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int f = tid * per + q;
        if (q < per && f < F && loc[q]) {
            uint32_t at = atomicAdd(&S.cnt[d * F + f], loc[q]);
            if (at + loc[q] > B.pcap) atomicOr(overflow, 1u);
            s_cnt[f] = at;
        }
    }
#pragma unroll
    for (int j = 0; j < LOG_TILE_PER; ++j) {
        if (code[j] == 0xffffffffu) continue;
        uint32_t f = code[j] >> 16;
        uint32_t pos = s_off[f] + (code[j] & 0xffffu);
        if (HASV) {
            ll2 r2 = {kk[j], vv[j]};
            *(ll2 *)&s_rec[2 * pos] = r2;
        } else {
            s_rec[pos] = kk[j];
        }
        s_bk[pos] = (uint16_t)f;
    }
    __syncthreads();
    for (uint32_t p = tid; p < total; p += LOG_TILE_THREADS) {
        uint32_t f = s_bk[p];
        if (f >= (uint32_t)F) continue;   // defensive: never a write outside the segment
        uint32_t q = s_cnt[f] + (p - s_off[f]);
        if (q < B.pcap) {
            int64_t *dst = S.rec + (uint64_t)(B.seg_base + f * B.pcap + q) * W;
            if (HASV) *(ll2 *)dst = *(const ll2 *)&s_rec[2 * p];
            else *dst = s_rec[p];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// log_fire: persistent workgroups, each folding partitions p = blockIdx.x, + gridDim.x, ...
// (WindowOperator.onEventTime + emitWindowContents, WindowOperator.java:430-473, 546-550) into an LDS
// hash table (key -> accumulator words) and emitting one row per key.
// Fast path (a partition of <= FIRE_RCAP records, held in registers by the prefetch):
//   1. every record finds or claims its key's slot (LDS CAS per probe);
//   2. the claiming record initialises the slot's words with plain stores;
//   3. the key's other records combine atomically -- so a key's first record costs no word atomics
//      (the per-word 64-bit LDS atomics were the fold's bottleneck);
//   4. the table is swept, rows placed in (round, wave, lane) order so each store instruction writes
//      one contiguous run, one row-counter reservation per partition, slots reset as they are read.
// The next partition's segment offsets and records are loaded while the current one is folded and
// emitted, so a workgroup exposes about one HBM round trip per partition.  Slow path (more records
// than the prefetch holds, or more keys than the table): rounds over disjoint ranges of a second
// group of hash bits with direct loads (the range halves until it fits), so no key is lost.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void lds_combine64(int64_t *dst, int op, int64_t x) {
    switch (op) {
        case ACC_ADD_I64: atomicAdd((unsigned long long *)dst, (unsigned long long)x); break;
        case ACC_ADD_F64: atomicAdd((double *)dst, __longlong_as_double(x)); break;
        case ACC_MIN_I64: atomicMin((long long *)dst, (long long)x); break;
        default: atomicMax((long long *)dst, (long long)x); break;
    }
}

__device__ __forceinline__ void emit_results(const ResultPlan &rp, const int64_t *acc, int accs, const OutCols &o,
                                             unsigned long long pos) {
    for (int a = 0; a < rp.naggs; ++a) {
        int w = rp.word[a];
        int64_t r;
        switch (rp.kind[a]) {
            case 2:
            case 3: r = rp.value_is_f64 ? f64_from_order_key(acc[w * accs]) : acc[w * accs]; break;
            case 4: {
                double s = rp.value_is_f64 ? __longlong_as_double(acc[w * accs]) : (double)acc[w * accs];
                r = __double_as_longlong(s / (double)acc[(w + 1) * accs]);
                break;
            }
            default: r = acc[w * accs]; break;
        }
        o.res[a][pos] = r;
    }
}

struct FireCtx {
    int64_t *key;                 // LDS table: [cap] keys, then nwords x [cap] words (SoA)
    int64_t *acc;
    int64_t *side;                // key == Long.MIN_VALUE: [flag, words...]
    unsigned *used, *fail;
    int cap;
    unsigned limit;
};

// Folds one record into the LDS table; a key that finds no slot (or overfills it) sets *fail.
__device__ __forceinline__ void fire_insert(const FireCtx &c, const AccPlan &p, int64_t k, uint64_t h, int64_t v) {
    int64_t *acc;
    int accs;
    if (k == GWO_EMPTY_KEY) {
        c.side[0] = 1;
        acc = c.side + 1;
        accs = 1;
    } else {
        int slot = (int)(h & (uint64_t)(c.cap - 1)), probes = 0;
        while (true) {
            unsigned long long prev = atomicCAS((unsigned long long *)&c.key[slot], (unsigned long long)GWO_EMPTY_KEY,
                                                (unsigned long long)k);
            if ((int64_t)prev == GWO_EMPTY_KEY) {
                if (atomicAdd(c.used, 1u) >= c.limit) *c.fail = 1;
                break;
            }
            if ((int64_t)prev == k) break;
            slot = (slot + 1) & (c.cap - 1);
            if (++probes >= c.cap) {
                *c.fail = 1;
                return;
            }
        }
        acc = c.acc + slot;
        accs = c.cap;
    }
    for (int w = 0; w < p.nwords; ++w) lds_combine64(acc + w * accs, p.op[w], lift_word(p, w, v));
}

// Resets every slot, the side slot and the flags (caller synchronises).
__device__ __forceinline__ void fire_clear(const FireCtx &c, const AccPlan &p) {
    for (int i = threadIdx.x; i < c.cap; i += LOG_FIRE_THREADS) {
        c.key[i] = GWO_EMPTY_KEY;
        for (int w = 0; w < p.nwords; ++w) c.acc[w * c.cap + i] = p.ident[w];
    }
    if (threadIdx.x <= GWO_MAX_WORDS) c.side[threadIdx.x] = threadIdx.x == 0 ? 0 : p.ident[threadIdx.x - 1];
    if (threadIdx.x == 0) {
        *c.used = 0;
        *c.fail = 0;
    }
}

// Emits every occupied slot (one output reservation per workgroup) and resets the table as it goes.
// Ends synchronised.
__device__ __forceinline__ void fire_emit(const FireCtx &c, const AccPlan &p, const ResultPlan &rp, int64_t start,
                                          int64_t end, const OutCols &o) {
    unsigned cnt = 0;
    for (int i = threadIdx.x; i < c.cap; i += LOG_FIRE_THREADS) cnt += c.key[i] != GWO_EMPTY_KEY;
    const bool side = threadIdx.x == 0 && c.side[0] != 0;
    cnt += side;
    unsigned long long pos = block_reserve(cnt, o.count);
    if (side) {
        if ((long long)pos < o.cap) {
            o.key[pos] = GWO_EMPTY_KEY;
            o.start[pos] = start;
            o.end[pos] = end;
            emit_results(rp, c.side + 1, 1, o, pos);
        }
        pos++;
    }
    for (int i = threadIdx.x; i < c.cap; i += LOG_FIRE_THREADS) {
        int64_t k = c.key[i];
        if (k == GWO_EMPTY_KEY) continue;
        if ((long long)pos < o.cap) {
            o.key[pos] = k;
            o.start[pos] = start;
            o.end[pos] = end;
            emit_results(rp, c.acc + i, c.cap, o, pos);
        }
        pos++;
        c.key[i] = GWO_EMPTY_KEY;
        for (int w = 0; w < p.nwords; ++w) c.acc[w * c.cap + i] = p.ident[w];
    }
    __syncthreads();
    if (threadIdx.x <= GWO_MAX_WORDS) c.side[threadIdx.x] = threadIdx.x == 0 ? 0 : p.ident[threadIdx.x - 1];
    if (threadIdx.x == 0) {
        *c.used = 0;
        *c.fail = 0;
    }
    __syncthreads();
}

typedef __attribute__((address_space(1))) const ll2 g_ll2;
typedef __attribute__((address_space(1))) const int64_t g_i64;

// One output row from NW register words.  Every loop has a compile-time trip count (unrolled), so
// the plan fields and the result-column pointers are read from kernel arguments once, outside the
// caller's loops, and no register array is indexed at run time.
template <int NW>
__device__ __forceinline__ void emit_row(const ResultPlan &rp, const int64_t (&acc)[NW], const OutCols &o,
                                         unsigned long long pos, int64_t k, int64_t start, int64_t end) {
    o.key[pos] = k;
    o.start[pos] = start;
    o.end[pos] = end;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        if (a >= rp.naggs) break;
        const int wi = rp.word[a];
        int64_t x = acc[0], y = acc[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
            if (w == wi) x = acc[w];
            if (w == wi + 1) y = acc[w];
        }
        int64_t r;
        switch (rp.kind[a]) {
            case 2:
            case 3: r = rp.value_is_f64 ? f64_from_order_key(x) : x; break;
            case 4: {
                double s = rp.value_is_f64 ? __longlong_as_double(x) : (double)x;
                r = __double_as_longlong(s / (double)y);
                break;
            }
            default: r = x; break;
        }
        o.res[a][pos] = r;
    }
}

template <int NW>
__global__ __launch_bounds__(LOG_FIRE_THREADS) void log_fire_kernel(const LogSegDesc *__restrict__ segs, int nseg,
                                                                    uint32_t nparts, int cap_log2, int has_val,
                                                                    AccPlan p, ResultPlan rp, int64_t start,
                                                                    int64_t end, OutCols o,
                                                                    unsigned long long *overflow) {
    extern __shared__ __attribute__((aligned(16))) int64_t s_dyn[];   // the LDS hash table (key, words; SoA)
    __shared__ int64_t s_side[GWO_MAX_WORDS + 1];
    __shared__ unsigned s_used, s_fail;
    __shared__ uint32_t s_beg[2][LOG_MAX_SEGS + 1];   // flattened record space of a partition: segment s
    __shared__ uint32_t s_src[2][LOG_MAX_SEGS];       //   covers [s_beg[s], s_beg[s+1]) from record s_src[s]
    __shared__ const int64_t *s_rp[LOG_MAX_SEGS];
    __shared__ uint32_t s_wrows[8][LOG_FIRE_THREADS / 64];   // rows per (sweep round, wave), then prefixes
    __shared__ unsigned long long s_rbase;
    __shared__ uint32_t s_side_pos;
    const int tid = threadIdx.x;
    const int cap = 1 << cap_log2;
    FireCtx c{s_dyn, s_dyn + cap, s_side, &s_used, &s_fail, cap, (unsigned)(cap - (cap >> 3))};
    uint32_t part = blockIdx.x;
    if (part >= nparts) return;
    for (int s = tid; s < nseg; s += LOG_FIRE_THREADS) s_rp[s] = segs[s].rec;
    fire_clear(c, p);   // the first publish() synchronises

    // segment ranges of a partition -> s_beg[b] / s_src[b] (all threads; ends synchronised)
    auto publish = [&](int b, uint32_t cnt, uint32_t off) {
        uint32_t tot;
        uint32_t ex = block_exclusive_scan(cnt, &tot);
        if (tid < nseg) {
            s_beg[b][tid] = ex;
            s_src[b][tid] = off;
        }
        if (tid == 0) s_beg[b][nseg] = tot;
        __syncthreads();
    };
    // register prefetch of a partition's records (only when they all fit); global (not flat) loads,
    // so LDS waits in between do not wait for them
    int64_t rk[FIRE_RPT], rv[FIRE_RPT];
    auto prefetch = [&](int b) {
        const uint32_t total = s_beg[b][nseg];
        const bool fits = total <= (uint32_t)FIRE_RCAP;
        const int64_t *addr[FIRE_RPT];
        int segr[FIRE_RPT];
        if (nseg <= 32) {   // segment of record i = number of segment starts <= i (broadcast LDS reads)
#pragma unroll
            for (int r = 0; r < FIRE_RPT; ++r) segr[r] = 0;
            for (int sg = 1; sg < nseg; ++sg) {
                const uint32_t bs = s_beg[b][sg];
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r) segr[r] += (uint32_t)(tid + r * LOG_FIRE_THREADS) >= bs;
            }
        } else {
            int seg = 0;
#pragma unroll
            for (int r = 0; r < FIRE_RPT; ++r) {
                const uint32_t i = tid + r * LOG_FIRE_THREADS;
                while (i < total && i >= s_beg[b][seg + 1]) seg++;
                segr[r] = seg;
            }
        }
#pragma unroll
        for (int r = 0; r < FIRE_RPT; ++r) {
            const uint32_t i = tid + r * LOG_FIRE_THREADS;
            addr[r] = s_rp[0];
            if (fits && i < total) {
                const int sg = segr[r];
                addr[r] = s_rp[sg] + (uint64_t)(s_src[b][sg] + (i - s_beg[b][sg])) * (has_val ? 2 : 1);
            }
        }
#pragma unroll
        for (int r = 0; r < FIRE_RPT; ++r) {
            if (has_val) {
                ll2 r2 = __builtin_nontemporal_load((g_ll2 *)addr[r]);
                rk[r] = r2.x;
                rv[r] = r2.y;
            } else {
                rk[r] = __builtin_nontemporal_load((g_i64 *)addr[r]);
                rv[r] = 0;
            }
        }
    };

    uint32_t a_cnt = 0, a_off = 0;
    if (tid < nseg) {
        a_cnt = segs[tid].cnt[part];
        a_off = segs[tid].off[part];
    }
    int buf = 0;
    publish(buf, a_cnt, a_off);
    prefetch(buf);
    while (true) {
        const uint32_t total = s_beg[buf][nseg];
        const uint32_t nxt = part + gridDim.x;
        const bool more = nxt < nparts;
        // next partition's segment offsets: in flight while this one is folded
        a_cnt = 0;
        a_off = 0;
        if (more && tid < nseg) {
            a_cnt = segs[tid].cnt[nxt];
            a_off = segs[tid].off[nxt];
        }
        bool fast = total <= (uint32_t)FIRE_RCAP;
        if (fast) {
            // phase 1: every record finds (or claims) its key's slot; one LDS CAS per probe
            int slot[FIRE_RPT];
            unsigned claimed = 0, pending = 0;
#pragma unroll
            for (int r = 0; r < FIRE_RPT; ++r) {
                const uint32_t i = tid + r * LOG_FIRE_THREADS;
                slot[r] = -1;
                if (i < total) {
                    const int64_t k = rk[r];
                    if (k == GWO_EMPTY_KEY) {
                        slot[r] = -2;
                    } else {
                        int sl = (int)(part_hash(k) & (uint64_t)(cap - 1));
                        for (int probes = 0; probes < cap; ++probes) {
                            unsigned long long prev = atomicCAS((unsigned long long *)&c.key[sl],
                                                                (unsigned long long)GWO_EMPTY_KEY, (unsigned long long)k);
                            if ((int64_t)prev == GWO_EMPTY_KEY || (int64_t)prev == k) {
                                claimed |= (unsigned)((int64_t)prev == GWO_EMPTY_KEY) << r;
                                slot[r] = sl;
                                break;
                            }
                            sl = (sl + 1) & (cap - 1);
                        }
                        if (slot[r] == -1) pending = 1;
                    }
                }
            }
            if (pending) s_fail = 1;   // table full
            {
                unsigned nc = (unsigned)__popc(claimed);
                for (int o2 = 32; o2 > 0; o2 >>= 1) nc += __shfl_xor(nc, o2);
                if ((tid & 63) == 0 && nc) atomicAdd(&s_used, nc);
            }
            __syncthreads();
            fast = s_fail == 0 && s_used <= c.limit;
            __syncthreads();
            if (fast) {
                // phase 2: the claiming record initialises its slot with plain stores
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r) {
                    if (!((claimed >> r) & 1u)) continue;
#pragma unroll
                    for (int w = 0; w < NW; ++w) c.acc[w * cap + slot[r]] = lift_word(p, w, rv[r]);
                }
                __syncthreads();
                // phase 3: the other records of a key combine atomically (about half of them in C4)
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r) {
                    if (slot[r] == -1 || ((claimed >> r) & 1u)) continue;
                    int64_t *acc;
                    int accs;
                    if (slot[r] == -2) {
                        s_side[0] = 1;
                        acc = s_side + 1;
                        accs = 1;
                    } else {
                        acc = c.acc + slot[r];
                        accs = cap;
                    }
#pragma unroll
                    for (int w = 0; w < NW; ++w) lds_combine64(acc + w * accs, p.op[w], lift_word(p, w, rv[r]));
                }
                __syncthreads();
            } else {
                fire_clear(c, p);   // back to a clean table for the slow path
                __syncthreads();
            }
        }
        if (!fast) {
            // slow path: hash-table rounds over disjoint ranges of hash bits 12..43, direct loads
            if (tid == 0) atomicAdd(overflow + 1, 1ull);   // slow-path partitions (statistics)
            fire_clear(c, p);
            __syncthreads();
            const uint64_t kAll = 1ull << 32;
            uint64_t lo = 0, width = kAll;
            while (lo < kAll) {
                const uint64_t hi = lo + width < kAll ? lo + width : kAll;
                const bool ranged = width < kAll;
                int seg = 0;
                for (uint32_t i = tid; i < total; i += LOG_FIRE_THREADS) {
                    while (i >= s_beg[buf][seg + 1]) seg++;
                    const int64_t *q = s_rp[seg] + (uint64_t)(s_src[buf][seg] + (i - s_beg[buf][seg])) * (has_val ? 2 : 1);
                    const int64_t k = q[0];
                    const uint64_t h = part_hash(k);
                    if (ranged) {
                        uint64_t sub = (uint32_t)(h >> 12);
                        if (sub < lo || sub >= hi) continue;
                    }
                    fire_insert(c, p, k, h, has_val ? q[1] : 0);
                }
                __syncthreads();
                const bool failed = s_fail != 0;
                __syncthreads();
                if (failed) {
                    fire_clear(c, p);
                    __syncthreads();
                    width >>= 1;
                    if (width == 0) {
                        if (tid == 0) atomicAdd(overflow, 1ull);
                        break;
                    }
                    continue;
                }
                fire_emit(c, p, rp, start, end, o);
                lo = hi;
            }
        }
        if (more) {
            publish(buf ^ 1, a_cnt, a_off);
            prefetch(buf ^ 1);   // in flight during this partition's fold and emit
        }
        if (fast) {
            // emit: thread t sweeps slots t + m*512; rows are placed in (m, wave, lane) order, so each
            // store instruction writes one contiguous run; slots are reset as they are read
            constexpr int NWAVES = LOG_FIRE_THREADS / 64;
            const int lane = tid & 63, wave = tid >> 6;
            const int rounds = cap / LOG_FIRE_THREADS;
            for (int m = 0; m < rounds; ++m) {
                const unsigned long long bal = __ballot(c.key[m * LOG_FIRE_THREADS + tid] != GWO_EMPTY_KEY);
                if (lane == 0) s_wrows[m][wave] = (uint32_t)__popcll(bal);
            }
            __syncthreads();
            if (tid == 0) {   // exclusive prefix over (round, wave), then one reservation per partition
                uint32_t run = 0;
                for (int m = 0; m < rounds; ++m)
                    for (int w = 0; w < NWAVES; ++w) {
                        uint32_t t = s_wrows[m][w];
                        s_wrows[m][w] = run;
                        run += t;
                    }
                s_side_pos = run;
                run += s_side[0] != 0;
                s_rbase = run ? atomicAdd(o.count, (unsigned long long)run) : 0ull;
            }
            __syncthreads();
            const unsigned long long rbase = s_rbase;
            for (int m = 0; m < rounds; ++m) {
                const int sl = m * LOG_FIRE_THREADS + tid;
                const int64_t k = c.key[sl];
                const bool occ = k != GWO_EMPTY_KEY;
                const unsigned long long bal = __ballot(occ);
                if (!occ) continue;
                int64_t acc[NW];
#pragma unroll
                for (int w = 0; w < NW; ++w) acc[w] = c.acc[w * cap + sl];
                c.key[sl] = GWO_EMPTY_KEY;   // words need no reset: the next claimer overwrites them
                const unsigned long long pos =
                    rbase + s_wrows[m][wave] + (unsigned long long)__popcll(bal & ((1ull << lane) - 1ull));
                if ((long long)pos < o.cap) emit_row<NW>(rp, acc, o, pos, k, start, end);
            }
            if (tid == 0 && s_side[0] != 0) {
                int64_t acc[NW];
#pragma unroll
                for (int w = 0; w < NW; ++w) acc[w] = s_side[1 + w];
                const unsigned long long pos = rbase + s_side_pos;
                if ((long long)pos < o.cap) emit_row<NW>(rp, acc, o, pos, GWO_EMPTY_KEY, start, end);
            }
            __syncthreads();
            if (tid <= GWO_MAX_WORDS) s_side[tid] = tid == 0 ? 0 : p.ident[tid - 1];
            if (tid == 0) {
                s_used = 0;
                s_fail = 0;
            }
            __syncthreads();
        }
        if (!more) break;
        part = nxt;
        buf ^= 1;
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
void launch_log_part(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, int64_t stride,
                     const WindowGeom &g,
                     long long base, int nunits, int has_val, unsigned long long *cursor, uint64_t cap,
                     int64_t *tmp, BatchStats *st, int64_t *side_key, int64_t *side_ts, int64_t *side_val,
                     unsigned long long *side_count, long long side_cap, int side_enabled, hipStream_t s) {
    int64_t grid = (n + LOG_TILE - 1) / LOG_TILE;
    grid = grid < 1 ? 1 : (grid > 2048 ? 2048 : grid);
    if (has_val)
        hipLaunchKernelGGL(log_part_kernel<true>, dim3((int)grid), dim3(LOG_K1_THREADS), 0, s, key, ts, val, n, stride, g,
                           base, nunits, cursor, cap, tmp, st, side_key, side_ts, side_val, side_count, side_cap,
                           side_enabled);
    else
        hipLaunchKernelGGL(log_part_kernel<false>, dim3((int)grid), dim3(LOG_K1_THREADS), 0, s, key, ts, val, n, stride, g,
                           base, nunits, cursor, cap, tmp, st, side_key, side_ts, side_val, side_count, side_cap,
                           side_enabled);
}

__global__ __launch_bounds__(1024) void log_collect_kernel(unsigned long long *cursor, int nb, BatchStats *st,
                                                          unsigned long long *rb) {
    constexpr int SW = (int)(sizeof(BatchStats) / 8);
    unsigned long long *sw = (unsigned long long *)st;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        rb[b] = cursor[(size_t)b * LOG_CUR_STRIDE];
        cursor[(size_t)b * LOG_CUR_STRIDE] = 0;
    }
    unsigned long long w = 0;
    if (threadIdx.x < SW) {
        w = sw[threadIdx.x];
        rb[LOG_NU * 256 + threadIdx.x] = w;
    }
    __syncthreads();
    if (threadIdx.x < SW) sw[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        st->min_idx = 0x7fffffffffffffffLL;
        st->max_idx = (long long)0x8000000000000000LL;
    }
}

void launch_log_collect(unsigned long long *cursor, int nb, BatchStats *stats, unsigned long long *rb, hipStream_t s) {
    hipLaunchKernelGGL(log_collect_kernel, dim3(1), dim3(1024), 0, s, cursor, nb, stats, rb);
}

void launch_log_split(const int64_t *tmp, int has_val, const LogBucket *buckets, int nb, int nunits,
                      const LogSegDesc *segs, unsigned *overflow, uint32_t nchunks, hipStream_t s) {
    (void)nunits;
    if (nchunks == 0) return;
    if (has_val)
        hipLaunchKernelGGL(log_split_kernel<true>, dim3(nchunks), dim3(LOG_TILE_THREADS), 0, s, tmp, buckets, nb, segs,
                           overflow);
    else
        hipLaunchKernelGGL(log_split_kernel<false>, dim3(nchunks), dim3(LOG_TILE_THREADS), 0, s, tmp, buckets, nb,
                           segs, overflow);
}

// The fire's LDS hash table: 64 KiB of (1 + nwords) * 8 B slots (power of two).
int log_fire_cap_log2(int nwords) {
    int bytes_per = (1 + nwords) * 8;
    int c = 0;
    while ((2 << c) * bytes_per <= 64 * 1024) c++;
    return c;
}

void launch_log_fire(const LogSegDesc *segs, int nseg, int lp, int has_val, const AccPlan &plan,
                     const ResultPlan &rp, int64_t start, int64_t end, OutCols out, unsigned long long *overflow,
                     int cus, int max_per_cu, hipStream_t s) {
    if (nseg <= 0 || nseg > LOG_MAX_SEGS) return;   // nothing to fold (the host never asks; defensive)
    int cl = log_fire_cap_log2(plan.nwords);
    size_t lds = (size_t)(1 + plan.nwords) * 8 << cl;
    uint32_t parts = 1u << lp;
    // persistent grid: two 64-KiB-LDS workgroups per CU, or fewer to leave room for concurrent kernels
    const uint32_t groups = (uint32_t)cus * (uint32_t)(max_per_cu < 2 ? max_per_cu : 2);
    uint32_t grid = parts < groups ? parts : groups;
#define GWO_FIRE_NW(NW)                                                                                          \
    case NW:                                                                                                     \
        hipLaunchKernelGGL(log_fire_kernel<NW>, dim3(grid), dim3(LOG_FIRE_THREADS), lds, s, segs, nseg, parts, cl, \
                           has_val, plan, rp, start, end, out, overflow);                                        \
        break;
    switch (plan.nwords) {
        GWO_FIRE_NW(1)
        GWO_FIRE_NW(2)
        GWO_FIRE_NW(3)
        GWO_FIRE_NW(4)
        GWO_FIRE_NW(5)
        GWO_FIRE_NW(6)
        GWO_FIRE_NW(7)
        default: GWO_FIRE_NW(8)
    }
#undef GWO_FIRE_NW
}

}  // namespace gwo
