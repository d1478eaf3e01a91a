// gwo_log.hip -- log-structured window state for high-cardinality tumbling windows.
//
// The reference keeps one accumulator per (key, window) in a heap hash map and updates it per
// record (HeapAggregatingState.add, HeapAggregatingState.java:96-109; StateTable.transform,
// heap/StateTable.java:194-202).  On MI355X a random read-modify-write of a 32-B entry in an
// 8-GB table costs a 64-128-B line round trip per record, and device-scope atomics execute at the
// memory side (tools/micro_table.hip: 8 G updates/s for sum/min/max).  For windows that receive
// about as many distinct keys as records (config C4: 166M records -> 81M (key, window) pairs),
// this path defers the aggregation to the window's fire instead:
//
//   per batch  log_scan   classify + late accounting + key-group check + a (window, coarse digit)
//                         histogram (coarse digit = top 8 bits of the partition hash)
//              log_pass1  scatter accepted (key, value) pairs into a batch buffer grouped by
//                         (window, coarse digit); one cursor reservation per tile and bucket
//              log_pass2  one workgroup per coarse bucket splits it by the fine partition bits
//                         into the window's new segment and writes the segment's offsets
//   at fire    log_fire   one workgroup per partition folds the partition's records from every
//                         segment of the window into an LDS hash table and emits one row per key
//                         (WindowOperator.onEventTime + emitWindowContents, WindowOperator.java:430-473,546-550)
//
// Every byte moved is a coalesced or run-length-grouped stream; the only random accesses are LDS.
#include "gwo_device.h"
#include "gwo_log.h"

namespace gwo {

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

// ------------------------------------------------------------------------------------------------
// log_scan: per-batch statistics + (unit, coarse digit) histogram for units [base, base+LOG_UNITS)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void log_scan_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                       const int64_t *__restrict__ val, int64_t n, WindowGeom g,
                                                       long long base, BatchStats *st, unsigned *chist,
                                                       int64_t *side_key, int64_t *side_ts, int64_t *side_val,
                                                       unsigned long long *side_count, long long side_cap,
                                                       int side_enabled) {
    __shared__ unsigned s_c[LOG_UNITS * 256];
    __shared__ long long s_min[4], s_max[4];
    for (int i = threadIdx.x; i < LOG_UNITS * 256; i += blockDim.x) s_c[i] = 0;
    __syncthreads();
    long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000LL;
    unsigned long long acc = 0, late = 0, refire = 0, bad_ts = 0, out = 0, bad_kg = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        long long u = 0;
        int c = log_classify(ts[i], g, u);
        if (c == L_ACCEPT) {
            int64_t k = key[i];
            int32_t kg = key_group(k, g.key_kind, g.max_par);
            if (kg < g.kg_lo || kg > g.kg_hi) {
                bad_kg++;
                st->bad_kg_key = k;
            }
            acc++;
            mn = u < mn ? u : mn;
            mx = u > mx ? u : mx;
            long long b = u - base;
            if (b >= 0 && b < LOG_UNITS) atomicAdd(&s_c[b * 256 + (int)(part_hash(k) >> 56)], 1u);
            else out++;
        } else if (c == L_LATE) {
            late++;
            if (side_enabled) {
                unsigned long long pos = atomicAdd(side_count, 1ull);
                if ((long long)pos < side_cap) {
                    side_key[pos] = key[i];
                    side_ts[pos] = ts[i];
                    side_val[pos] = val ? val[i] : 0;
                }
            }
        } else if (c == L_REFIRE) {
            refire++;
        } else if (c == L_BAD_TS) {
            bad_ts++;
        }
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
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        s_min[wid] = mn;
        s_max[wid] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        long long a = s_min[0], b = s_max[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            a = s_min[w] < a ? s_min[w] : a;
            b = s_max[w] > b ? s_max[w] : b;
        }
        if (a != 0x7fffffffffffffffLL) {
            atomicMin(&st->min_idx, a);
            atomicMax(&st->max_idx, b);
        }
    }
    for (int i = threadIdx.x; i < LOG_UNITS * 256; i += blockDim.x)
        if (s_c[i]) atomicAdd(&chist[i], s_c[i]);
}

// ------------------------------------------------------------------------------------------------
// log_pass1: records -> batch buffer grouped by coarse bucket b = (unit - base) * 256 + digit.
// A tile of P1_TILE records counts its buckets in LDS, reserves each bucket's run with one device
// atomic on the bucket cursor, then writes every record at cursor + rank.
// ------------------------------------------------------------------------------------------------
#define P1_PER 32
#define P1_TILE (256 * P1_PER)

__global__ __launch_bounds__(256) void log_pass1_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                        const int64_t *__restrict__ val, int64_t n, WindowGeom g,
                                                        long long base, int nunits,
                                                        unsigned long long *__restrict__ cursor,
                                                        int64_t *__restrict__ tkey, int64_t *__restrict__ tval) {
    __shared__ unsigned s_cnt[LOG_UNITS * 256];
    __shared__ unsigned long long s_pos[LOG_UNITS * 256];
    __shared__ uint16_t s_b[P1_TILE];
    const int nb = nunits * 256;
    for (int i = threadIdx.x; i < nb; i += 256) s_cnt[i] = 0;
    __syncthreads();
    for (int64_t tile = (int64_t)blockIdx.x * P1_TILE; tile < n; tile += (int64_t)gridDim.x * P1_TILE) {
#pragma unroll 4
        for (int j = 0; j < P1_PER; ++j) {
            int64_t i = tile + j * 256 + threadIdx.x;
            uint16_t b = 0xffff;
            if (i < n) {
                long long u = 0;
                if (log_classify(ts[i], g, u) == L_ACCEPT) {
                    long long w = u - base;
                    if (w >= 0 && w < nunits) {
                        b = (uint16_t)(w * 256 + (int)(part_hash(key[i]) >> 56));
                        atomicAdd(&s_cnt[b], 1u);
                    }
                }
            }
            s_b[j * 256 + threadIdx.x] = b;
        }
        __syncthreads();
        for (int b = threadIdx.x; b < nb; b += 256) {
            unsigned c = s_cnt[b];
            if (c) {
                s_pos[b] = atomicAdd(&cursor[b], (unsigned long long)c);
                s_cnt[b] = 0;
            }
        }
        __syncthreads();
#pragma unroll 4
        for (int j = 0; j < P1_PER; ++j) {
            uint16_t b = s_b[j * 256 + threadIdx.x];
            if (b == 0xffff) continue;
            int64_t i = tile + j * 256 + threadIdx.x;
            unsigned long long pos = s_pos[b] + atomicAdd(&s_cnt[b], 1u);
            tkey[pos] = key[i];
            if (tval) tval[pos] = val[i];
        }
        __syncthreads();
        for (int b = threadIdx.x; b < nb; b += 256) s_cnt[b] = 0;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// log_pass2: one workgroup per coarse bucket -> the window's segment, ordered by partition.
// Partition p = top lp bits of the partition hash; coarse digit d = top 8 bits.  lp <= 8: a
// partition is 2^(8-lp) whole coarse buckets (copy); lp > 8: the bucket splits into 2^(lp-8)
// partitions by a counting sort.  Also writes the segment's partition offsets.
// ------------------------------------------------------------------------------------------------
#define P2_THREADS 512
#define P2_MAXF 1024   // lp <= 18

__global__ __launch_bounds__(P2_THREADS) void log_pass2_kernel(const int64_t *__restrict__ tkey,
                                                               const int64_t *__restrict__ tval,
                                                               const unsigned long long *__restrict__ cbase,
                                                               const LogSegDesc *__restrict__ segs) {
    __shared__ unsigned s_hist[P2_MAXF];
    __shared__ unsigned s_pre[P2_MAXF];
    const int c = blockIdx.x;
    const int w = c >> 8, d = c & 255;
    const LogSegDesc sd = segs[w];
    if (!sd.off) return;   // no records of this window in the chunk
    const int lp = sd.lp;
    const unsigned long long lo = cbase[c], hi = cbase[c + 1], wbase = cbase[w * 256];
    const uint32_t rel = (uint32_t)(lo - wbase);
    if (lp <= 8) {
        const int sh = 8 - lp;
        if (threadIdx.x == 0) {
            if ((d & ((1 << sh) - 1)) == 0) sd.off[d >> sh] = rel;
            if (d == 255) sd.off[1u << lp] = (uint32_t)(hi - wbase);
        }
        for (unsigned long long i = lo + threadIdx.x; i < hi; i += P2_THREADS) {
            unsigned long long o = i - wbase;
            sd.key[o] = tkey[i];
            if (sd.val) sd.val[o] = tval[i];
        }
        return;
    }
    const int fb = lp - 8, F = 1 << fb;
    for (int f = threadIdx.x; f < F; f += P2_THREADS) s_hist[f] = 0;
    __syncthreads();
    for (unsigned long long i0 = lo + threadIdx.x; i0 < hi; i0 += 4 * P2_THREADS) {
        int64_t kk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            unsigned long long i = i0 + u * P2_THREADS;
            kk[u] = i < hi ? tkey[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * P2_THREADS < hi) atomicAdd(&s_hist[(int)(part_hash(kk[u]) >> (64 - lp)) & (F - 1)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {   // F <= 1024: serial scan is a few microseconds at most
        unsigned run = 0;
        for (int f = 0; f < F; ++f) {
            s_pre[f] = run;
            run += s_hist[f];
            s_hist[f] = 0;
        }
    }
    __syncthreads();
    for (int f = threadIdx.x; f < F; f += P2_THREADS) sd.off[(size_t)d * F + f] = rel + s_pre[f];
    if (d == 255 && threadIdx.x == 0) sd.off[(size_t)256 * F] = (uint32_t)(hi - wbase);
    for (unsigned long long i0 = lo + threadIdx.x; i0 < hi; i0 += 4 * P2_THREADS) {
        int64_t kk[4], vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            unsigned long long i = i0 + u * P2_THREADS;
            kk[u] = i < hi ? tkey[i] : 0;
            vv[u] = (i < hi && tval) ? tval[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (i0 + u * P2_THREADS >= hi) break;
            int f = (int)(part_hash(kk[u]) >> (64 - lp)) & (F - 1);
            unsigned long long o = rel + s_pre[f] + atomicAdd(&s_hist[f], 1u);
            sd.key[o] = kk[u];
            if (sd.val) sd.val[o] = vv[u];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// log_fire: one workgroup per partition.  Folds the partition's records from every segment of the
// window into an LDS hash table (key -> accumulator words), then emits one output row per key.
// A partition holding more records than 3/4 of the table is folded in rounds over a second set of
// hash bits, so the table can never overflow for non-adversarial keys; an overflow is reported.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void lds_combine64(int64_t *dst, int op, int64_t x) {
    switch (op) {
        case ACC_ADD_I64: atomicAdd((unsigned long long *)dst, (unsigned long long)x); break;
        case ACC_ADD_F64: atomicAdd((double *)dst, __longlong_as_double(x)); break;
        case ACC_MIN_I64: atomicMin((long long *)dst, (long long)x); break;
        default: atomicMax((long long *)dst, (long long)x); break;
    }
}

__device__ __forceinline__ void emit_results(const AccPlan &p, const ResultPlan &rp, const int64_t *acc, int accs,
                                             const OutCols &o, unsigned long long pos) {
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


__device__ __forceinline__ void lds_insert(int64_t *s_key, int64_t *s_acc, int64_t *s_side, int cap, const AccPlan &p,
                                           int64_t k, uint64_t h, int64_t v, unsigned *fail) {
    int64_t *acc;
    int accs;
    if (k == GWO_EMPTY_KEY) {
        s_side[0] = 1;
        acc = s_side + 1;
        accs = 1;
    } else {
        int slot = (int)(h & (uint64_t)(cap - 1)), probes = 0;
        while (true) {
            unsigned long long prev = atomicCAS((unsigned long long *)&s_key[slot], (unsigned long long)GWO_EMPTY_KEY,
                                                (unsigned long long)k);
            if ((int64_t)prev == GWO_EMPTY_KEY || (int64_t)prev == k) break;
            slot = (slot + 1) & (cap - 1);
            if (++probes >= cap) {
                *fail = 1;
                return;
            }
        }
        acc = s_acc + slot;
        accs = cap;
    }
    for (int w = 0; w < p.nwords; ++w) lds_combine64(acc + w * accs, p.op[w], lift_word(p, w, v));
}

__global__ __launch_bounds__(LOG_FIRE_THREADS) void log_fire_kernel(const LogSegDesc *__restrict__ segs, int nseg,
                                                                    int lp, int cap_log2, AccPlan p, ResultPlan rp,
                                                                    int64_t start, int64_t end, OutCols o,
                                                                    unsigned long long *overflow) {
    extern __shared__ int64_t s_tab[];   // [cap] keys, then nwords x [cap] accumulator words (SoA)
    __shared__ int64_t s_side[GWO_MAX_WORDS + 1];   // key == Long.MIN_VALUE: [flag, words...]
    __shared__ unsigned s_fail;
    __shared__ uint32_t s_beg[LOG_MAX_SEGS + 1];      // flattened record space: segment s covers
    __shared__ uint32_t s_src[LOG_MAX_SEGS];          //   [s_beg[s], s_beg[s+1]) starting at offset s_src[s]
    const int cap = 1 << cap_log2;
    const int NW = p.nwords;
    int64_t *s_key = s_tab;
    int64_t *s_acc = s_tab + cap;
    const uint32_t part = blockIdx.x;
    // prologue: every segment's slice of this partition, loaded in parallel
    uint32_t cnt_s = 0;
    if (threadIdx.x < (unsigned)nseg) {
        const uint32_t *off = segs[threadIdx.x].off;
        uint32_t a = off[part], b = off[part + 1];
        s_src[threadIdx.x] = a;
        cnt_s = b - a;
    }
    if (threadIdx.x == 0) s_fail = 0;
    uint32_t seg_total;
    uint32_t excl = block_exclusive_scan(cnt_s, &seg_total);
    if (threadIdx.x < (unsigned)nseg) s_beg[threadIdx.x] = excl;
    if (threadIdx.x == 0) s_beg[nseg] = seg_total;
    __syncthreads();
    const uint32_t total = s_beg[nseg];
    if (total == 0) return;
    int rbits = 0;
    while ((total >> rbits) > (uint32_t)(cap * 3 / 4)) rbits++;   // rounds = 2^rbits
    for (int round = 0; round < (1 << rbits); ++round) {
        for (int i = threadIdx.x; i < cap; i += LOG_FIRE_THREADS) {
            s_key[i] = GWO_EMPTY_KEY;
            for (int w = 0; w < NW; ++w) s_acc[w * cap + i] = p.ident[w];
        }
        if (threadIdx.x <= GWO_MAX_WORDS) s_side[threadIdx.x] = threadIdx.x == 0 ? 0 : p.ident[threadIdx.x - 1];
        __syncthreads();
        // records in flattened order, 4 loads in flight per thread
        int seg = 0;
        for (uint32_t i0 = threadIdx.x; i0 < total; i0 += 4 * LOG_FIRE_THREADS) {
            int64_t kk[4], vv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint32_t i = i0 + u * LOG_FIRE_THREADS;
                kk[u] = 0;
                vv[u] = 0;
                if (i < total) {
                    while (i >= s_beg[seg + 1]) seg++;
                    const LogSegDesc &sd = segs[seg];
                    uint32_t o_ = s_src[seg] + (i - s_beg[seg]);
                    kk[u] = sd.key[o_];
                    if (sd.val) vv[u] = sd.val[o_];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (i0 + u * LOG_FIRE_THREADS >= total) break;
                uint64_t h = part_hash(kk[u]);
                if (rbits && (int)((h >> 24) & ((1u << rbits) - 1)) != round) continue;
                lds_insert(s_key, s_acc, s_side, cap, p, kk[u], h, vv[u], &s_fail);
            }
        }
        __syncthreads();
        // emit: occupied slots, one output reservation per workgroup
        unsigned cnt = 0;
        for (int i = threadIdx.x; i < cap; i += LOG_FIRE_THREADS) cnt += s_key[i] != GWO_EMPTY_KEY;
        bool side = threadIdx.x == 0 && s_side[0] != 0;
        cnt += side;
        unsigned long long pos = block_reserve(cnt, o.count);
        if (side) {
            if ((long long)pos < o.cap) {
                o.key[pos] = GWO_EMPTY_KEY;
                o.start[pos] = start;
                o.end[pos] = end;
                emit_results(p, rp, s_side + 1, 1, o, pos);
            }
            pos++;
        }
        for (int i = threadIdx.x; i < cap; i += LOG_FIRE_THREADS) {
            int64_t k = s_key[i];
            if (k == GWO_EMPTY_KEY) continue;
            if ((long long)pos < o.cap) {
                o.key[pos] = k;
                o.start[pos] = start;
                o.end[pos] = end;
                emit_results(p, rp, s_acc + i, cap, o, pos);
            }
            pos++;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && s_fail) atomicAdd(overflow, 1ull);
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
void launch_log_scan(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const WindowGeom &g,
                     long long base, BatchStats *st, unsigned *chist, int64_t *side_key, int64_t *side_ts,
                     int64_t *side_val, unsigned long long *side_count, long long side_cap, int side_enabled,
                     hipStream_t s) {
    int64_t grid = (n + 256LL * 16 - 1) / (256LL * 16);
    grid = grid < 1 ? 1 : (grid > 1024 ? 1024 : grid);
    hipLaunchKernelGGL(log_scan_kernel, dim3((int)grid), dim3(256), 0, s, key, ts, val, n, g, base, st, chist,
                       side_key, side_ts, side_val, side_count, side_cap, side_enabled);
}

void launch_log_pass1(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const WindowGeom &g,
                      long long base, int nunits, unsigned long long *cursor, int64_t *tkey, int64_t *tval,
                      hipStream_t s) {
    int64_t grid = (n + P1_TILE - 1) / P1_TILE;
    grid = grid < 1 ? 1 : (grid > 2048 ? 2048 : grid);
    hipLaunchKernelGGL(log_pass1_kernel, dim3((int)grid), dim3(256), 0, s, key, ts, val, n, g, base, nunits, cursor,
                       tkey, tval);
}

void launch_log_pass2(const int64_t *tkey, const int64_t *tval, const unsigned long long *cbase, int nunits,
                      const LogSegDesc *segs, hipStream_t s) {
    hipLaunchKernelGGL(log_pass2_kernel, dim3(nunits * 256), dim3(P2_THREADS), 0, s, tkey, tval, cbase, segs);
}

int log_fire_cap_log2(int nwords) {
    // table of 64 KiB: (1 + nwords) * 8 B per slot
    int bytes_per = (1 + nwords) * 8;
    int c = 0;
    while ((2 << c) * bytes_per <= 64 * 1024) c++;
    return c;
}

void launch_log_fire(const LogSegDesc *segs, int nseg, int lp, const AccPlan &plan, const ResultPlan &rp,
                     int64_t start, int64_t end, OutCols out, unsigned long long *overflow, hipStream_t s) {
    int cl = log_fire_cap_log2(plan.nwords);
    size_t lds = (size_t)(1 + plan.nwords) * 8 << cl;
    hipLaunchKernelGGL(log_fire_kernel, dim3(1u << lp), dim3(LOG_FIRE_THREADS), lds, s, segs, nseg, lp, cl, plan, rp,
                       start, end, out, overflow);
}

}  // namespace gwo
