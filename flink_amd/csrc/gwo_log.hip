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
#include "../../include/gwo.h"
#include "gwo_device.h"
#include "gwo_log.h"

namespace gwo {

typedef long long ll2 __attribute__((ext_vector_type(2)));

// Phase trace (built with -DGWO_KTRACE, run with GWO_KTRACE=1; diagnostics only): lane 0 of every K1 / fire
// workgroup accumulates shader-clock
// cycles per phase (s_memtime deltas between the phase's closing barriers) and adds them here at its end; the host
// prints the sums when the handle is destroyed.  Off: one scalar load per launch.
__device__ int g_kt_on;
__device__ unsigned long long g_kt[64];   // [0, 16): K1 phases, [16, 32): fire phases, [32]: K1 launches, [33]: fires
#define KT_K1 0
#define KT_FIRE 16
#ifdef GWO_KTRACE
struct KTrace {
    bool on;
    uint64_t t;
    uint64_t acc[10];
    __device__ __forceinline__ void start(bool en) {
        on = en;
        t = on ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll
        for (int i = 0; i < 10; ++i) acc[i] = 0;
    }
    __device__ __forceinline__ void stamp(int ph) {
        if (on) {
            const uint64_t n = __builtin_amdgcn_s_memtime();
#pragma unroll
            for (int i = 0; i < 10; ++i)
                if (i == ph) acc[i] += n - t;
            t = n;
        }
    }
    __device__ __forceinline__ void flush(int base) {
        if (on && (threadIdx.x & 63) == 0)
#pragma unroll
            for (int i = 0; i < 10; ++i)
                if (acc[i]) atomicAdd(&g_kt[base + i], acc[i]);
    }
};
#else   // the product build: no trace code or registers in the kernels (`make KTRACE=1` builds the traced library)
struct KTrace {
    static constexpr bool on = false;
    __device__ __forceinline__ void start(bool) {}
    __device__ __forceinline__ void stamp(int) {}
    __device__ __forceinline__ void flush(int) {}
};
#endif

enum LogClass : int { L_ACCEPT = 0, L_LATE = 1, L_SKIP = 2, L_REFIRE = 3, L_BAD_TS = 4, L_BAD_RANGE = 5 };

// Tumbling classification, WindowOperator.java:386-427 + TumblingEventTimeWindows.java:68-81.
// With a = ts - offset + size in [0, 2^52) (every timestamp within 142,000 years of the epoch):
// getWindowStartWithOffset = ts - a % size = offset + (q - 1) * size for q = floor(a / size), and the
// window index floor(start / size) = q - 1 - (offset < 0) since |offset| < size (the assigner's
// constructor check, TumblingEventTimeWindows.java:57-60) -- one small division instead of two full ones.
__device__ __forceinline__ int log_classify(int64_t ts, const WindowGeom &g, long long &unit) {
    if (ts == GWO_LONG_MIN) return L_BAD_TS;
    const int64_t a = jadd(jsub(ts, g.offset), g.size);
    // sliding panes (g.size = slide): Java's '%' gives a start > ts for ts - offset + slide < 0, outside the
    // pane restatement -- rejected loudly, as the table path does (gwo_kernels.hip classify)
    if (g.sliding && a < 0) return L_BAD_RANGE;
    int64_t start, u;
    if ((uint64_t)a < (1ull << 52)) {
        const int64_t q = fdiv_small(a, g.size, g.inv_size);
        start = g.offset + (q - 1) * g.size;
        u = q - 1 - (g.offset < 0 ? 1 : 0);
    } else {
        start = window_start_f(ts, g.offset, g.size, g.inv_size);
        u = fdiv_floor(start, g.size, g.inv_size);
    }
    int64_t max_ts = jsub(jadd(start, g.size), 1);
    if (cleanup_time(max_ts, g.lateness) <= g.wm) return jadd(ts, g.lateness) <= g.wm ? L_LATE : L_SKIP;
    unit = u;
    if (max_ts <= g.wm) return L_REFIRE;
    return L_ACCEPT;
}

// Inclusive prefix sum across a wave64 (DPP row shifts + row broadcasts; VALU only, no LDS).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return x;
}

// Exclusive prefix of v over a workgroup of T threads (DPP wave scans + one LDS round; VALU, no bpermute).
// *total = the workgroup sum.  The caller synchronises before the next call (s_w is reused).
template <int T>
__device__ __forceinline__ uint32_t block_excl_scan_dpp(uint32_t v, uint32_t *total) {
    __shared__ uint32_t s_w[T / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) s_w[wid] = incl;
    lds_barrier();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
        const uint32_t x = s_w[w];
        pre += w < wid ? x : 0u;
        tot += x;
    }
    *total = tot;
    return pre + incl - v;
}

// Exclusive prefix over nb (<= 4 * T) LDS counters s_cnt -> s_off; thread t owns the `per` consecutive counters
// [t*per, t*per+per) (their counts in loc, their offsets in lof).  Returns the total.  All T threads call it; ends
// synchronised, so s_off is complete on return.
template <int T>
__device__ __forceinline__ uint32_t tile_offsets(const uint32_t *s_cnt, uint32_t *s_off, int nb, uint32_t loc[4],
                                                 uint32_t lof[4], int per) {
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int b = threadIdx.x * per + q;
        loc[q] = (q < per && b < nb) ? s_cnt[b] : 0u;
        sum += loc[q];
    }
    uint32_t total;
    uint32_t ex = block_excl_scan_dpp<T>(sum, &total);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int b = threadIdx.x * per + q;
        lof[q] = ex;
        if (q < per && b < nb) s_off[b] = ex;
        ex += loc[q];
    }
    lds_barrier();   // every thread reads other threads' s_off next
    return total;
}

// Inclusive prefix of a 64-bit value over a K1 workgroup (LOG_K1_THREADS; wave shuffles + one LDS round);
// ends synchronised.  *total = the workgroup sum.
__device__ __forceinline__ unsigned long long block_k1_incl_scan64(unsigned long long v, unsigned long long *total) {
    constexpr int NWV = LOG_K1_THREADS / 64;
    __shared__ unsigned long long s_w[NWV];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(v, o);
        if (lane >= o) v += y;
    }
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
        pre += w < wid ? s_w[w] : 0ull;
        tot += s_w[w];
    }
    *total = tot;
    __syncthreads();
    return v + pre;
}

// K1's tail, run by its last workgroup (LOG_K1_THREADS threads; formerly a separate collect kernel): moves the bucket
// counts and batch statistics into the host-visible readback block (resetting cursors and statistics for the
// next K1), and plans pass 2 on the device -- per bucket the partition capacity (mean + 6 sigma + 4 of a
// Binomial(n_b, 1/F) partition, the host's group_capacity), the bucket's first record in its window's
// segment and its first pass-2 workgroup -- with each window's segment size and the workgroup total in the
// readback.  Speculative launches (ca.spec): the pass 2 already queued behind K1 runs the plan only if it
// is the batch's final plan -- no error, no bucket over its region capacity, the batch's first window inside
// the launch's window range, every segment within its carved capacity -- else it exits and the host takes over.
__device__ __forceinline__ void k1_plan_tail(unsigned long long *cursor, BatchStats *st, const CollectArgs &a,
                                          long long base, const LogRoute &rt) {
    constexpr int SW = (int)(sizeof(BatchStats) / 8);
    constexpr int K1_T0 = LOG_K1_THREADS - 32, K1_T1 = K1_T0 + K1_SW;   // threads past the statistics words
    static_assert(SW <= K1_T0 && K1_T1 + LOG_SHARDS + 1 <= LOG_K1_THREADS, "statistics words");
    __shared__ unsigned long long s_sw[SW];
    __shared__ unsigned s_bad;
    __shared__ unsigned long long s_maxreg;
    const int t = threadIdx.x;
    unsigned long long *sw = (unsigned long long *)st;
    if (t == 0) {
        s_bad = 0;
        s_maxreg = 0;
    }
    // the launch's bucket counts (cursors reset for the next K1): every exchange in flight before any is used
    unsigned long long cq[LOG_NU][LOG_XG];
#pragma unroll
    for (int q = 0; q < LOG_NU; ++q)
#pragma unroll
        for (int x = 0; x < LOG_XG; ++x)
            cq[q][x] = t < LOG_ND && q < a.nunits
                           ? atomicExch(&cursor[((size_t)(q * LOG_ND + t) * LOG_XG + x) * LOG_CUR_STRIDE], 0ull)
                           : 0ull;
    __shared__ unsigned long long s_rmax[2];
    if (t < 2) s_rmax[t] = 0;
    __syncthreads();
    if (rt.mode == 1)   // routed records per destination; the cursors start the next routed K1 at zero
        for (int p = t; p < rt.nranks; p += LOG_K1_THREADS) {
            const unsigned long long cn = atomicExch(&rt.cursor[(size_t)p * LOG_CUR_STRIDE], 0ull);
            const unsigned long long cw = atomicExch(&rt.cursor[(size_t)(LOG_RT_MAX + p) * LOG_CUR_STRIDE], 0ull);
            rt.count[2 * p] = cn;
            rt.count[2 * p + 1] = cw;
            atomicMax(&s_rmax[0], cn);   // the largest counts go to the readback: a region overflow is seen with the plan
            atomicMax(&s_rmax[1], cw);
        }
    __shared__ unsigned long long s_k1[K1_SW];
    if (t < SW) {   // read-and-reset through the same device-scope atomics the workgroups used
        const unsigned long long reset = t == 0 ? 0x7fffffffffffffffull : (t == 1 ? 0x8000000000000000ull : 0ull);
        s_sw[t] = atomicExch(&sw[t], reset);
    } else if (t >= K1_T0 && t < K1_T0 + K1_SW) {   // fold (and reset) the statistics shards
        const int f = t - K1_T0;
        const unsigned long long init = (f == K1S_MIN || f == K1S_NEXT) ? 0x7fffffffffffffffull
                                                                        : (f == K1S_MAX ? 0x8000000000000000ull : 0ull);
        const int kind = (f == K1S_MIN || f == K1S_NEXT) ? 1 : (f == K1S_MAX ? 2 : 0);
        s_k1[f] = xchg_fold<LOG_SHARDS>(&a.shard[f], LOG_CUR_STRIDE, init, kind);
    } else if (t >= K1_T1 && t < K1_T1 + LOG_SHARDS + 1) {   // arrival counters start the next K1 at zero
        atomicExch(&a.done[(t - K1_T1) * LOG_CUR_STRIDE], 0ull);
    }
    __syncthreads();
    if (t == 0) {
        BatchStats &W = *(BatchStats *)s_sw;
        W.min_idx = (long long)s_k1[K1S_MIN];
        W.max_idx = (long long)s_k1[K1S_MAX];
        W.accepted = s_k1[K1S_ACC];
        W.late = s_k1[K1S_LATE];
        W.refire = s_k1[K1S_REFIRE];
        W.bad_ts = s_k1[K1S_BADTS];
        W.bad_kg = s_k1[K1S_BADKG];
        W.hist_out = s_k1[K1S_HOUT];
        W.bad_range = s_k1[K1S_BADR];
        rb_put(&a.rb[LOG_RB_NEXT], s_k1[K1S_NEXT]);
    }
    __syncthreads();
    if (t < SW) rb_put(&a.rb[LOG_RB_STATS + t], s_sw[t]);
    const BatchStats &S = *(const BatchStats *)s_sw;
    unsigned long long chunk_run = 0;
    unsigned bad = 0;
    unsigned long long maxreg = 0;
#pragma unroll
    for (int q = 0; q < LOG_NU; ++q) {   // window q of the launch: bucket b = q * LOG_ND + t (digit t)
        if (q >= a.nunits) break;
        const bool dig = t < LOG_ND;
        const int b = q * LOG_ND + t;
        unsigned long long c[LOG_XG], n_b = 0;
#pragma unroll
        for (int x = 0; x < LOG_XG; ++x) c[x] = cq[q][x];
        uint32_t xoff[LOG_XG];
#pragma unroll
        for (int x = 0; x < LOG_XG; ++x) {
            xoff[x] = (uint32_t)n_b;
            n_b += c[x];
            maxreg = c[x] > maxreg ? c[x] : maxreg;
        }
        if (dig) rb_put(&a.rb[b], n_b);
        uint32_t pcap = 0, chunks = 0;
        unsigned long long seg = 0;
        if (n_b) {
            const int F = 1 << (a.lp[q] - LOG_DB);
            const double mean = (double)n_b / (double)F;
            pcap = (uint32_t)ceil(__dadd_rn(__dadd_rn(mean, __dmul_rn(6.0, sqrt(mean))), 4.0));
            seg = (unsigned long long)F * pcap;
            chunks = (uint32_t)((n_b + LOG_TILE - 1) / LOG_TILE);
        }
        unsigned long long seg_tot, chk_tot;
        const unsigned long long seg_incl = block_k1_incl_scan64(seg, &seg_tot);
        const unsigned long long chk_incl = block_k1_incl_scan64(chunks, &chk_tot);
        LogBucket B;
        B.n = (uint32_t)n_b;
#pragma unroll
        for (int x = 0; x < LOG_XG; ++x) B.xoff[x] = xoff[x];
        B.pcap = pcap;
        B.seg_base = (uint32_t)(seg_incl - seg);
        B.chunk0 = (uint32_t)(chunk_run + chk_incl - chunks);
        if (dig) a.bk[b] = B;
        if (t == 0) {
            rb_put(&a.rb[LOG_RB_SEG + q], seg_tot);
            if (a.spec && seg_tot > a.seg_cap[q]) bad = 1;
        }
        chunk_run += chk_tot;
    }
    if (maxreg > a.cap) bad = 1;           // K1 dropped records past a region: the host re-runs K1
    if (bad) atomicOr(&s_bad, 1u);
    if (maxreg) atomicMax(&s_maxreg, maxreg);
    __syncthreads();
    if (t == 0) {
        LogBucket E{};
        E.chunk0 = (uint32_t)chunk_run;
        a.bk[a.nunits * LOG_ND] = E;
        rb_put(&a.rb[LOG_RB_CHUNKS], chunk_run);
        const bool go = a.spec && !s_bad && S.bad_ts == 0 && S.bad_kg == 0 && S.refire == 0 && S.bad_range == 0 && S.accepted > 0 &&
                        S.min_idx >= base && S.min_idx < base + a.nunits && chunk_run < (1ull << 32);
        *a.go = go ? 1u : 0u;
        rb_put(&a.rb[LOG_RB_GO], go ? 1ull : 0ull);
        rb_put(&a.rb[LOG_RB_MAXREG], s_maxreg);
        rb_put(&a.rb[LOG_RB_RMAX], s_rmax[0]);
        rb_put(&a.rb[LOG_RB_RWMAX], s_rmax[1]);
    }
    if (t == 0 && a.t0) {
        rb_put(&a.rb[LOG_RB_T0], atomicAdd(a.t0, 0ull));
        rb_put(&a.rb[LOG_RB_T1], (unsigned long long)wall_clock64());
    }
    // the host spins on the sequence word: every other readback word must be visible first
    rb_publish(&a.rb[LOG_RB_SEQ], a.seq);
}

// ------------------------------------------------------------------------------------------------
// K1 log_part: batch -> batch buffer, grouped by bucket b = (window - base) * LOG_ND + coarse digit.
// Bucket b owns LOG_XG regions of cap records; workgroup w appends to region group x = w % LOG_XG at
// records [(b * LOG_XG + x) * cap, ...), whose cursor cursor[(b * LOG_XG + x) * LOG_CUR_STRIDE] ends as its
// record count (also when it exceeds cap: those records are not written and the host reruns).
// ------------------------------------------------------------------------------------------------
// ROUTE: the multi-GPU instance (LogRoute): records of other GPUs are routed (rt.mode 1) or skipped (2).
// TS32: `ts` holds int32 timestamps - th.tbase (records received in the 20-B wire format; S == 1).
// V2 (S == 1, 16-B aligned columns, even tile length): each lane loads two adjacent records per column with one
// 16-B load (8 B for int32 timestamps) -- record j of a thread is tile + (j / 2) * 2 * LOG_K1_THREADS + 2 * tid + j % 2.
// A pair straddling the end of the batch reads 8 B past it, inside the 16-B aligned granule of its first record.
#ifdef LOG_K1_WPE   // waves per SIMD the non-routed instances' registers are sized for (A/B of the workgroup shape)
#define K1_WPE_ATTR(R) __attribute__((amdgpu_num_vgpr(512 / LOG_K1_WPE)))   // (every instance: A/B only)
#else
#define K1_WPE_ATTR(R)
#endif
template <bool HASV, int S, bool ROUTE, bool TS32, bool V2>   // S: record stride in int64 words (1: SoA columns, 3: {key, ts, value}; 0: runtime)
#ifndef GWO_K1_ROUTE_WG
#define GWO_K1_ROUTE_WG 2   // routed instances: 2 workgroups per CU, with 52-140 B of spills per lane (1: no spills,
                            // one per CU -- routed K1 7-15 % slower, profiles/r06_experiments.txt)
#endif
__global__ __launch_bounds__(LOG_K1_THREADS, ROUTE ? GWO_K1_ROUTE_WG : 2) K1_WPE_ATTR(ROUTE) void log_part_kernel(
    const int64_t *__restrict__ key, const int64_t *__restrict__ ts, const int64_t *__restrict__ val, int64_t n,
    int64_t stride, WindowGeom g, long long base, int nunits, unsigned long long *__restrict__ cursor, uint64_t cap,
    int64_t *__restrict__ tmp, BatchStats *st, int64_t *side_key, int64_t *side_ts, int64_t *side_val,
    unsigned long long *side_count, long long side_cap, int side_enabled, CollectArgs ca, LogThr th, LogRoute rt,
    int tlen) {
    constexpr int W = HASV ? 2 : 1;
    KTrace kt;
    kt.start(__builtin_amdgcn_readfirstlane(threadIdx.x) < 64 && g_kt_on);   // wave 0, uniform (scalar registers)
    // K1 times itself: workgroup 0's start and the tail's end on the device wall clock (read back with the plan),
    // so profiling puts no event markers between K1 and pass 2 (each costs the stream ~5 us)
    if (blockIdx.x == 0 && threadIdx.x == 0 && ca.t0) atomicExch(ca.t0, (unsigned long long)wall_clock64());
    // the new segments' partition counters (pass 2's cursors) start at zero: pass 2 follows in stream order
    // (a route-only re-run follows a pass 2 that already used them)
    for (int w = 0; w < ((ROUTE && rt.mode == 3) ? 0 : ca.nunits); ++w) {
        uint4 *c4 = (uint4 *)ca.cnt[w];
        const uint32_t n4 = (1u << ca.lp[w]) / 4;
        for (uint32_t i = blockIdx.x * LOG_K1_THREADS + threadIdx.x; i < n4; i += gridDim.x * LOG_K1_THREADS)
            c4[i] = make_uint4(0, 0, 0, 0);
    }
    // tlen (<= LOG_K1_TILE) records per tile: the launcher sizes tiles so that every workgroup loops over the same
    // number of them (a last round of a few workgroups would cost a whole tile's latency).  One spare record slot
    // (index LOG_K1_TILE) takes the LDS writes of records that go nowhere, so the scatter needs no branch.
    __shared__ __attribute__((aligned(16))) int64_t s_rec[(LOG_K1_TILE + 1) * W];
    __shared__ uint16_t s_bk[LOG_K1_TILE + 1];
    __shared__ uint32_t s_rbase[ROUTE ? LOG_RT_MAX : 1];            // routed runs' first record in the region
    const int nb = nunits * LOG_ND;
    // dynamic LDS, sized for the launch's windows (2 workgroups per CU up to 2 windows): counters [0, nb), a spare
    // counter (nb) for records counted nowhere, routed counters per destination (ROUTE), then the offsets [nb]
    extern __shared__ uint32_t s_kdyn[];
    uint32_t *const s_cnt = s_kdyn;
    const int rc0 = nb + 1;                                          // first routed counter
    uint32_t *const s_off = s_kdyn + nb + 1 + (ROUTE ? LOG_RT_MAX : 0);
    const int nr = ROUTE ? rt.nranks : 0;
    const int per = (nb + LOG_K1_THREADS - 1) / LOG_K1_THREADS;   // counters owned per thread (<= 4)
    const int tid = threadIdx.x;
    const int xg = blockIdx.x % LOG_XG;                           // region group (an XCD under round-robin placement)
    const uint32_t cap32 = cap < 0xffffffffull ? (uint32_t)cap : 0xffffffffu;
    long long mn = 0x7fffffffffffffffLL, mx = (long long)0x8000000000000000LL;   // accepted windows (slow path)
    long long nx = 0x7fffffffffffffffLL;   // first accepted window after the launch's range (slow path)
    uint32_t wmask = 0;   // launch windows (bit jj) the inline path accepted records into
    unsigned acc = 0, late = 0, refire = 0, bad_ts = 0, out = 0, bad_kg = 0, bad_range = 0;   // per thread: < 2^32
    int64_t kk[LOG_K1_PER], vv[LOG_K1_PER], tt[LOG_K1_PER];
    static_assert(!V2 || (S == 1 && LOG_K1_PER % 2 == 0), "V2: SoA columns, pairs of records");
    // record j's position in the tile
    auto rec_pos = [&](int j) -> int {
        return V2 ? (j >> 1) * 2 * LOG_K1_THREADS + 2 * tid + (j & 1) : j * LOG_K1_THREADS + tid;
    };
    // unconditional loads of a tile (lanes past the end re-read the tile's first record and are
    // discarded); the next tile's loads are issued before this tile's write phase
    auto load_tile = [&](int64_t tile) {
        if (V2) {
#pragma unroll
            for (int j2 = 0; j2 < LOG_K1_PER / 2; ++j2) {
                const int p = j2 * 2 * LOG_K1_THREADS + 2 * tid;
                int64_t i = tile + p;
                i = (i < n && p < tlen) ? i : (tile < n ? tile : 0);   // (tile, n: even offsets of aligned columns)
                if (TS32) {
                    typedef int int2v __attribute__((ext_vector_type(2)));
                    const int2v t2 = __builtin_nontemporal_load((const int2v *)((const int32_t *)ts + i));
                    tt[2 * j2] = th.tbase + (int64_t)t2.x;
                    tt[2 * j2 + 1] = th.tbase + (int64_t)t2.y;
                } else {
                    const ll2 t2 = __builtin_nontemporal_load((const ll2 *)(ts + i));
                    tt[2 * j2] = t2.x;
                    tt[2 * j2 + 1] = t2.y;
                }
                const ll2 k2 = __builtin_nontemporal_load((const ll2 *)(key + i));
                kk[2 * j2] = k2.x;
                kk[2 * j2 + 1] = k2.y;
                if (HASV) {
                    const ll2 v2 = __builtin_nontemporal_load((const ll2 *)(val + i));
                    vv[2 * j2] = v2.x;
                    vv[2 * j2 + 1] = v2.y;
                } else {
                    vv[2 * j2] = vv[2 * j2 + 1] = 0;
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < LOG_K1_PER; ++j) {
                int64_t i = tile + j * LOG_K1_THREADS + tid;
                i = (i < n && j * LOG_K1_THREADS + tid < tlen) ? i : (tile < n ? tile : 0);
                const int64_t o = S ? i * S : i * stride;
                tt[j] = TS32 ? th.tbase + (int64_t)__builtin_nontemporal_load((const int32_t *)ts + o)
                             : __builtin_nontemporal_load(ts + o);
                kk[j] = __builtin_nontemporal_load(key + o);
                vv[j] = HASV ? __builtin_nontemporal_load(val + o) : 0;
            }
        }
    };
    const int64_t tstride = (int64_t)gridDim.x * tlen;
    // this workgroup's trash line (LOG_K1_TRASH_WORDS): the write phase's lanes without a record store there
    int64_t *const trash = (int64_t *)(cursor + LOG_CURSOR_WORDS) + (blockIdx.x % LOG_K1_GRID) * LOG_K1_TRASH_WG;
    if ((int64_t)blockIdx.x * tlen < n) load_tile((int64_t)blockIdx.x * tlen);
    // as many stores after the first tile's loads as every later tile's loads have after them (its predecessor's
    // write phase): the loop's waits are then counted the same on entry as on the back edge (the compiler takes the
    // smaller count where paths merge, and zero stores after the loads made each tile wait for all of its memory
    // operations -- the previous tile's store acknowledgements and the reservation atomics -- before the scatter)
#ifndef GWO_K1_NO_TRASH
#pragma unroll
    for (int j = 0; j < LOG_K1_TILE / LOG_K1_THREADS; ++j) {   // (distinct words: not merged into one store)
        if (HASV) *(ll2 *)(trash + 2 * j) = ll2{0, 0};
        else trash[2 * j] = 0;
    }
#endif
    // the launch's window bounds as scalars (a run-time index into the argument, th.bound[nunits], is a scalar load
    // per record, and its lgkmcnt wait also waited for the record's LDS atomic)
    const int64_t tb0 = th.bound[0], tb1 = th.bound[1], tb2 = th.bound[2], tb3 = th.bound[3];
    const int64_t tbh = nunits <= 1 ? tb1 : (nunits == 2 ? tb2 : (nunits == 3 ? tb3 : th.bound[4]));
    const bool tok = th.ok != 0;
    const uint32_t tcls = th.cls;
    // Every per-record step below is branch-free where it touches LDS: a record's LDS atomic or read inside an
    // `if` is waited for before the branch joins (its register is merged with the other path's value), which
    // serialised one LDS round trip per record (ISA of r03: 16 waits per tile in each of classify, scatter, write).
    for (int64_t tile = (int64_t)blockIdx.x * tlen; tile < n; tile += tstride) {
        for (int i = tid; i < rc0 + nr; i += LOG_K1_THREADS) s_kdyn[i] = 0;
        lds_barrier();
        kt.stamp(0);
        uint32_t code[LOG_K1_PER];   // (bucket or LOG_RT_B + destination) << 16 | rank; 0xffffffff: none
        uint32_t rank[LOG_K1_PER];
        uint32_t slow = 0;   // bit j: record j is classified out of line (below)
#pragma unroll
        for (int j = 0; j < LOG_K1_PER; ++j) {
            const int64_t i = tile + rec_pos(j);
            const bool in = i < n && rec_pos(j) < tlen;
            uint32_t ci = (uint32_t)nb;   // counter this record increments (nb: the spare)
            uint32_t cb = 0xffffu;        // its code's upper half (0xffff: none)
            bool local = in;
            if (ROUTE) {   // KeyGroupStreamPartitioner.selectChannel: another GPU's record is its owner's to classify
                const int dest = (int)(key_group(kk[j], g.key_kind, g.max_par) * rt.nranks / g.max_par);
                const bool remote = in && dest != rt.me;
                const bool fits = log_rt_fits(tt[j], rt.tbase);
                if (remote && (rt.mode == 1 || rt.mode == 3)) {
                    if (fits) {
                        ci = (uint32_t)(rc0 + dest);
                        cb = (uint32_t)(LOG_RT_B + dest);
                    } else {   // beyond the int32 timestamp range: a 24-B record in the wide region (rare)
                        const unsigned long long q =
                            atomicAdd(&rt.cursor[(size_t)(LOG_RT_MAX + dest) * LOG_CUR_STRIDE], 1ull);
                        if (q < rt.wcap) {
                            int64_t *w = log_rt_wide(rt.send, rt.rcap, rt.nranks, rt.wcap, dest) + q * 3;
                            w[0] = kk[j];
                            w[1] = tt[j];
                            w[2] = HASV ? vv[j] : 0;
                        }
                    }
                }
                local = in && !remote && rt.mode != 3;   // route-only re-run: the first K1 partitioned this GPU's records
            }
            // the common case, inline: a timestamp inside one of the launch's windows and that window open --
            // WindowOperator.java:386-427 decided once per window (LogThr), a few compares per record
            const int64_t t = tt[j];
            const int jj = (t >= tb1) + (t >= tb2) + (t >= tb3);
            const bool inl = tok & (t >= tb0) & (t < tbh) & (((tcls >> (2 * jj)) & 3u) == 0);   // (no short circuit)
            const bool take = local & inl;
            slow |= ((local & !inl) ? 1u : 0u) << j;
            const int64_t k = kk[j];
            if (!ROUTE && !th.full_range && take) {   // (routed: a record kept here is in range by construction)
                const int32_t kg = key_group(k, g.key_kind, g.max_par);
                if (kg < g.kg_lo || kg > g.kg_hi) {
                    bad_kg++;
                    atomicExch((unsigned long long *)&st->bad_kg_key, (unsigned long long)k);
                }
            }
            acc += take ? 1u : 0u;
            wmask |= (take ? 1u : 0u) << jj;
            const uint32_t b = (uint32_t)(jj * LOG_ND + (int)(digit_hash(k) >> (32 - LOG_DB)));
            ci = take ? b : ci;
            cb = take ? b : cb;
            rank[j] = atomicAdd(&s_kdyn[ci], 1u);   // every record: the 16 atomics in flight together
            code[j] = cb;
        }
#pragma unroll
        for (int j = 0; j < LOG_K1_PER; ++j) code[j] = code[j] == 0xffffu ? 0xffffffffu : (code[j] << 16) | rank[j];
        // everything else (late, re-fire and out-of-range records, Long.MIN_VALUE timestamps, extreme windows):
        // reloaded and classified in full by log_classify, one record at a time, outside the unrolled loop
#pragma unroll 1
        while (slow) {
            const int j = __builtin_ctz(slow);
            slow &= slow - 1;
            const int64_t i = tile + rec_pos(j);
            const int64_t o = S ? i * S : i * stride;
            const int64_t t = TS32 ? th.tbase + (int64_t)((const int32_t *)ts)[o] : ts[o], k = key[o];
            long long u = 0;
            int c = log_classify(t, g, u);
            // the sliding-log late pass: only records of panes already in the running total are taken
            if (th.only_refire) c = c == L_REFIRE ? L_ACCEPT : L_SKIP;
            if (c == L_ACCEPT) {
                if (!ROUTE && !th.full_range) {
                    const int32_t kg = key_group(k, g.key_kind, g.max_par);
                    if (kg < g.kg_lo || kg > g.kg_hi) {
                        bad_kg++;
                        atomicExch((unsigned long long *)&st->bad_kg_key, (unsigned long long)k);
                    }
                }
                acc++;
                mn = u < mn ? u : mn;
                mx = u > mx ? u : mx;
                const long long w = u - base;
                if (w >= 0 && w < nunits) {   // only without valid window bounds (th.ok == 0)
                    const uint32_t b = (uint32_t)(w * LOG_ND + (int)(digit_hash(k) >> (32 - LOG_DB)));
                    const uint32_t cd = (b << 16) | atomicAdd(&s_cnt[b], 1u);
#pragma unroll
                    for (int q = 0; q < LOG_K1_PER; ++q)   // code[j] without a run-time register index
                        if (q == j) code[q] = cd;
                } else {
                    out++;
                    if (w >= nunits) nx = u < nx ? u : nx;
                }
            } else if (c == L_LATE) {
                late++;
                if (side_enabled) {
                    const unsigned long long pos = atomicAdd(side_count, 1ull);
                    if ((long long)pos < side_cap) {
                        side_key[pos] = k;
                        side_ts[pos] = t;
                        side_val[pos] = val ? val[o] : 0;
                    }
                }
            } else if (c == L_REFIRE) {
                refire++;
            } else if (c == L_BAD_TS) {
                bad_ts++;
            } else if (c == L_BAD_RANGE) {
                bad_range++;
            }
            // (rare path) its loads complete here, so the compiler's wait tracking carries no pending load of this
            // path's registers into the common path (it had put an s_waitcnt vmcnt(0) into every tile's offsets scan)
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
        }
        kt.stamp(1);
        lds_barrier();
        kt.stamp(2);
        // reserve each bucket's run in this workgroup's region group, before the offsets scan, so that the
        // atomics' round trip overlaps the scan and the LDS scatter (q < per is uniform: no per-lane branch, so the
        // results are waited for only where they are used, after the next tile's loads are issued)
        unsigned long long at[4];   // (no initial value: a merge with one would wait for the atomic at the branch)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int b = tid * per + q;
#ifdef GWO_ABL_K1_NORET   // ablation (timing only: records land at made-up offsets): reservations not waited for
            if (q < per) {
                atomicAdd(&cursor[((size_t)b * LOG_XG + xg) * LOG_CUR_STRIDE], (unsigned long long)(b < nb ? s_cnt[b] : 0u));
                at[q] = ((unsigned long long)(tile / tlen) * 40ull) % (cap > 128 ? cap - 128 : 1);
            }
#else
            if (q < per) at[q] = atomicAdd(&cursor[((size_t)b * LOG_XG + xg) * LOG_CUR_STRIDE],
                                           (unsigned long long)(b < nb ? s_cnt[b] : 0u));
#endif
        }
        unsigned long long rat = 0;
        if (ROUTE && (rt.mode == 1 || rt.mode == 3) && tid < nr) {
            const uint32_t c = s_kdyn[rc0 + tid];
            rat = c ? atomicAdd(&rt.cursor[(size_t)tid * LOG_CUR_STRIDE], (unsigned long long)c) : 0ull;
        }
        uint32_t loc[4], lof[4];
        const uint32_t total = tile_offsets<LOG_K1_THREADS>(s_cnt, s_off, nb, loc, lof, per);
        if (ROUTE && (rt.mode == 1 || rt.mode == 3)) {
            if (tid < nr) s_rbase[tid] = rat < 0xffffffffull ? (uint32_t)rat : 0xffffffffu;   // (>= rcap: not written)
            lds_barrier();
        }
        kt.stamp(3);
        // scatter into LDS by bucket: every offset read in flight together, then the writes (records of no local
        // bucket write the spare slot)
        uint32_t pos[LOG_K1_PER];
#pragma unroll
        for (int j = 0; j < LOG_K1_PER; ++j) {
            const uint32_t b = code[j] >> 16;
            const bool lc = code[j] != 0xffffffffu && (!ROUTE || b < LOG_RT_B);
            pos[j] = s_off[lc ? b : 0u];
        }
#pragma unroll
        for (int j = 0; j < LOG_K1_PER; ++j) {
            const uint32_t b = code[j] >> 16;
            const bool lc = code[j] != 0xffffffffu && (!ROUTE || b < LOG_RT_B);
            const uint32_t ps = lc ? pos[j] + (code[j] & 0xffffu) : (uint32_t)LOG_K1_TILE;
            if (HASV) {
                ll2 r2 = {kk[j], vv[j]};
                *(ll2 *)&s_rec[2 * ps] = r2;
            } else {
                s_rec[ps] = kk[j];
            }
            s_bk[ps] = (uint16_t)b;
        }
        if (ROUTE && (rt.mode == 1 || rt.mode == 3)) {
#pragma unroll
            for (int j = 0; j < LOG_K1_PER; ++j) {   // routed: straight from registers into the destination's run
                const uint32_t b = code[j] >> 16;
                if (code[j] == 0xffffffffu || b < LOG_RT_B) continue;
                const uint32_t d = b - LOG_RT_B;
                const unsigned long long q = (unsigned long long)s_rbase[d] + (code[j] & 0xffffu);
                if (q < rt.rcap) {   // 20-B wire record: key, value, int32 ts - tbase (SoA per destination)
                    log_rt_keys(rt.send, rt.rcap, (int)d)[q] = kk[j];
                    log_rt_vals(rt.send, rt.rcap, (int)d)[q] = HASV ? vv[j] : 0;
                    log_rt_ts32(rt.send, rt.rcap, (int)d)[q] = (int32_t)(uint32_t)((uint64_t)tt[j] - (uint64_t)rt.tbase);
                }
            }
        }
        // next tile in flight during the writes: unconditional (past the end every lane re-reads record 0, one line),
        // so the write phase's waits count exactly these loads instead of waiting for all of them
        kt.stamp(4);   // (scatter)
#ifndef GWO_K1_DELTA_FIRST
        load_tile(tile + tstride);
#endif
        kt.stamp(7);   // (next tile's loads issued)
        // s_cnt[b] := the run's first region record - the bucket's tile offset, so the write phase finds a record's
        // destination with one read (mod 2^32: q = s_cnt[b] + p; at >= cap -> q >= cap, the run is dropped).  The
        // atomics precede the loads just issued: their wait is vmcnt(loads), in order, not a wait for the loads.
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int b = tid * per + q;
            if (q < per && loc[q]) s_cnt[b] = (at[q] < cap32 ? (uint32_t)at[q] : cap32) - lof[q];
        }
#ifdef GWO_K1_DELTA_FIRST   // (A/B: r03's order)
        load_tile(tile + tstride);
#endif
        kt.stamp(8);   // (the reservations' results in s_cnt)
        lds_barrier();
        kt.stamp(9);
        // write phase: straight-line code (a loop here made the compiler wait for every prefetched load first),
        // 4 records per thread per group with their LDS reads in flight together
#pragma unroll
        for (int p0 = 0; p0 < LOG_K1_TILE; p0 += 4 * LOG_K1_THREADS) {
            uint32_t bb[4], pp[4];
            ll2 rr[4];
            int64_t r1[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                pp[u] = (uint32_t)p0 + u * LOG_K1_THREADS + tid;
                const uint32_t pe = pp[u] < total ? pp[u] : (uint32_t)LOG_K1_TILE;
                bb[u] = s_bk[pe];
                if (HASV) rr[u] = *(const ll2 *)&s_rec[2 * pe];
                else r1[u] = s_rec[pe];
            }
            uint32_t dl[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) dl[u] = s_cnt[bb[u] < (uint32_t)nb ? bb[u] : 0u];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t q = dl[u] + pp[u];
                // every lane stores (exact wait counts): a lane without a record -- past the tile, a dropped run
                // (q >= cap), or bb >= nb (defensive: never a write outside the buffer) -- to the trash line
#ifdef GWO_ABL_K1_NOSTORE   // ablation (timing experiments only): the write phase's stores all to the trash line
                const bool ok = false;
#else
                const bool ok = pp[u] < total && bb[u] < (uint32_t)nb && q < cap32;
#endif
#ifdef GWO_K1_NO_TRASH   // (A/B: r03's predicated stores)
                if (ok) {
                    int64_t *dst = tmp + (((uint64_t)bb[u] * LOG_XG + xg) * cap + q) * W;
                    if (HASV) *(ll2 *)dst = rr[u];
                    else *dst = r1[u];
                }
#else
                int64_t *dst = ok ? tmp + (((uint64_t)bb[u] * LOG_XG + xg) * cap + q) * W : trash;
                if (HASV) *(ll2 *)dst = rr[u];
                else *dst = r1[u];
#endif
            }
        }
        lds_barrier();
        kt.stamp(5);
    }
    if (wmask) {
        const long long lo = base + __builtin_ctz(wmask), hi = base + 31 - __builtin_clz(wmask);
        mn = lo < mn ? lo : mn;
        mx = hi > mx ? hi : mx;
    }
    // workgroup statistics -> shard blockIdx % LOG_SHARDS (zero words skipped)
    unsigned long long v[K1_SW] = {(unsigned long long)mn, (unsigned long long)mx, acc, late, refire, bad_ts, bad_kg,
                                   out, bad_range, (unsigned long long)nx};
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const long long a = __shfl_xor((long long)v[K1S_MIN], o), b = __shfl_xor((long long)v[K1S_MAX], o);
        const long long c = __shfl_xor((long long)v[K1S_NEXT], o);
        v[K1S_MIN] = a < (long long)v[K1S_MIN] ? (unsigned long long)a : v[K1S_MIN];
        v[K1S_MAX] = b > (long long)v[K1S_MAX] ? (unsigned long long)b : v[K1S_MAX];
        v[K1S_NEXT] = c < (long long)v[K1S_NEXT] ? (unsigned long long)c : v[K1S_NEXT];

#pragma unroll
        for (int f = K1S_ACC; f < K1S_NEXT; ++f) v[f] += __shfl_xor(v[f], o);
    }
    __shared__ unsigned long long s_st[LOG_K1_THREADS / 64][K1_SW];
    const int lane = tid & 63, wid = tid >> 6;
    if (lane == 0)
#pragma unroll
        for (int f = 0; f < K1_SW; ++f) s_st[wid][f] = v[f];
    __syncthreads();
    if (tid < K1_SW) {
        unsigned long long r = s_st[0][tid];
        for (int w = 1; w < LOG_K1_THREADS / 64; ++w) {
            const unsigned long long x = s_st[w][tid];
            if (tid == K1S_MIN || tid == K1S_NEXT) r = (long long)x < (long long)r ? x : r;
            else if (tid == K1S_MAX) r = (long long)x > (long long)r ? x : r;
            else r += x;
        }
        unsigned long long *sh = ca.shard + (blockIdx.x % LOG_SHARDS) * LOG_CUR_STRIDE + tid;
        if (tid == K1S_MIN || tid == K1S_NEXT) {
            if ((long long)r != 0x7fffffffffffffffLL) atomicMin((long long *)sh, (long long)r);
        } else if (tid == K1S_MAX) {
            if ((long long)r != (long long)0x8000000000000000LL) atomicMax((long long *)sh, (long long)r);
        } else if (r) {
            atomicAdd(sh, r);
        }
    }
    // the last workgroup to finish plans pass 2: every workgroup's atomics are complete before its arrival
    // is counted (each wave drains its memory operations).  Arrivals are counted per shard; the last arrival of
    // a shard counts the shard.  Everything the tail reads was written by device-scope read-modify-write
    // atomics, coherent across XCDs; the records reach pass 2 through the kernel boundary -- so no release
    // fence, which on gfx950 writes back the XCD's whole L2 once per workgroup.
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    kt.stamp(6);
    if (kt.on && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_kt[32], 1ull);
    kt.flush(KT_K1);
    if (tid == 0) {
        const unsigned sh = blockIdx.x % LOG_SHARDS;
        const unsigned members = (gridDim.x - sh + LOG_SHARDS - 1) / LOG_SHARDS;
        const unsigned nsh = gridDim.x < LOG_SHARDS ? gridDim.x : LOG_SHARDS;
        bool last = false;
        if (atomicAdd(&ca.done[sh * LOG_CUR_STRIDE], 1ull) == members - 1)
            last = atomicAdd(&ca.done[LOG_SHARDS * LOG_CUR_STRIDE], 1ull) == nsh - 1;
        s_last = last;
    }
    __syncthreads();
    if (s_last) {
        if (ca.reset_rows && tid == 0) *ca.reset_rows = 0;
        if (ROUTE && rt.mode == 3) {   // route-only re-run: counts out, cursors and arrival counters reset; no plan
            for (int p = tid; p < rt.nranks; p += LOG_K1_THREADS) {
                rt.count[2 * p] = atomicExch(&rt.cursor[(size_t)p * LOG_CUR_STRIDE], 0ull);
                rt.count[2 * p + 1] = atomicExch(&rt.cursor[(size_t)(LOG_RT_MAX + p) * LOG_CUR_STRIDE], 0ull);
            }
            if (tid < LOG_SHARDS + 1) atomicExch(&ca.done[tid * LOG_CUR_STRIDE], 0ull);
            return;
        }
        LogRoute r = rt;
        if (!ROUTE) r.mode = 0;
        k1_plan_tail(cursor, st, ca, base, r);
    }
}

// ------------------------------------------------------------------------------------------------
// Pass 2 log_split: workgroup = one LOG_TILE chunk of one bucket (window w, coarse digit d).
// Partition p = top lp bits of digit_hash = d * F + f, F = 2^(lp-8).  Partition p of the segment owns
// records [seg_base + f*pcap, + pcap); cnt[p] is its cursor (ends as its count, overflow -> rerun).
// ------------------------------------------------------------------------------------------------
template <bool HASV>
__global__ __launch_bounds__(LOG_TILE_THREADS) void log_split_kernel(const int64_t *__restrict__ tmp, uint64_t cap,
                                                                     const LogBucket *__restrict__ bk, int nb,
                                                                     const LogSegSet segs,
                                                                     unsigned *overflow, const unsigned *go) {
    constexpr int W = HASV ? 2 : 1;
    // speculative launch: an upper bound of workgroups, behind K1 in stream order -- run only the plan
    if (go && (*go == 0u || blockIdx.x >= bk[nb].chunk0)) return;
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
    const int w = c >> LOG_DB, d = c & (LOG_ND - 1);
    const LogSegDesc S = segs.s[w];
    const int lp = S.lp, fb = lp - LOG_DB, F = 1 << fb;
    if (chunk == 0)
        for (int f = tid; f < F; f += LOG_TILE_THREADS) S.off[d * F + f] = B.seg_base + (uint32_t)f * B.pcap;
    for (int f = tid; f < F; f += LOG_TILE_THREADS) s_cnt[f] = 0;
    __syncthreads();
    const uint32_t begin = chunk * LOG_TILE;
    const uint32_t m = min((uint32_t)LOG_TILE, B.n - begin);
    int64_t kk[LOG_TILE_PER], vv[LOG_TILE_PER];
    uint32_t code[LOG_TILE_PER];
    // unconditional loads (a lane past the end re-reads the chunk's first record): no branch per load; record v
    // of the bucket is record v - xoff[x] of region group x, the last group with xoff[x] <= v
#pragma unroll
    for (int j = 0; j < LOG_TILE_PER; ++j) {
        uint32_t i = j * LOG_TILE_THREADS + tid;
        const uint32_t v = begin + (i < m ? i : 0u);
        int x = 0;
#pragma unroll
        for (int y = 1; y < LOG_XG; ++y) x += v >= B.xoff[y];
        const int64_t *src = tmp + (((uint64_t)c * LOG_XG + x) * cap + (v - B.xoff[x])) * W;
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
            uint32_t f = (uint32_t)(digit_hash(kk[j]) >> (32 - lp)) & (uint32_t)(F - 1);
            uint32_t r = atomicAdd(&s_cnt[f], 1u);
            code[j] = (f << 16) | r;
        }
    }
    __syncthreads();
    const int per = F <= LOG_TILE_THREADS ? 1 : F / LOG_TILE_THREADS;
    uint32_t loc[4], lof[4];
    const uint32_t total = tile_offsets<LOG_TILE_THREADS>(s_cnt, s_off, F, loc, lof, per);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int f = tid * per + q;
        if (q < per && f < F && loc[q]) {
            uint32_t at = atomicAdd(&S.cnt[d * F + f], loc[q]);
            // host-mapped flag: a system-scope store (write-through, no cache between it and the host), issued before
            // the kernel ends -- the host reads it after a later readback in stream order (log_resolve_split)
            if (at + loc[q] > B.pcap) __hip_atomic_store(overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

// Folds a partial accumulator (restored from a checkpoint: raw words, already lifted) into the LDS table.
__device__ __forceinline__ void fire_insert_words(const FireCtx &c, const AccPlan &p, int64_t k, uint64_t h,
                                                  const int64_t *words) {
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
    for (int w = 0; w < p.nwords; ++w) lds_combine64(acc + w * accs, p.op[w], words[w]);
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
typedef __attribute__((address_space(1))) const uint32_t g_u32;

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

// Result columns of one row from NW accumulator words (ResultPlan: value, f64 order key, avg).
// row_results on a plan held in scalars (the fire's emit: the plan loaded where it is used, see P5)
template <int NW>
__device__ __forceinline__ void row_results_s(int naggs, const int (&kind)[4], const int (&word)[4], int f64,
                                              const int64_t (&acc)[NW], int64_t (&res)[4]) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        if (a >= naggs) break;
        const int wi = word[a];
        int64_t x = acc[0], y = acc[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
            if (w == wi) x = acc[w];
            if (w == wi + 1) y = acc[w];
        }
        switch (kind[a]) {
            case 2:
            case 3: res[a] = f64 ? f64_from_order_key(x) : x; break;
            case 4: {
                double s = f64 ? __longlong_as_double(x) : (double)x;
                res[a] = __double_as_longlong(s / (double)y);
                break;
            }
            default: res[a] = x; break;
        }
    }
}
template <int NW>
__device__ __forceinline__ void row_results(const ResultPlan &rp, const int64_t (&acc)[NW], int64_t (&res)[4]) {
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
        switch (rp.kind[a]) {
            case 2:
            case 3: res[a] = rp.value_is_f64 ? f64_from_order_key(x) : x; break;
            case 4: {
                double s = rp.value_is_f64 ? __longlong_as_double(x) : (double)x;
                res[a] = __double_as_longlong(s / (double)y);
                break;
            }
            default: res[a] = x; break;
        }
    }
}

// Value of the other lane of the pair (2m, 2m+1): DPP quad_perm [1,0,3,2].
__device__ __forceinline__ int dpp_swap_pair(int x) { return __builtin_amdgcn_mov_dpp(x, 0xb1, 0xf, 0xf, false); }
__device__ __forceinline__ int64_t dpp_swap_pair64(int64_t x) {
    const int lo = dpp_swap_pair((int)(uint32_t)x), hi = dpp_swap_pair((int)(uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int64_t word_combine(int op, int64_t a, int64_t b) {
    switch (op) {
        case ACC_ADD_I64: return (int64_t)((uint64_t)a + (uint64_t)b);
        case ACC_ADD_F64: return __double_as_longlong(__longlong_as_double(a) + __longlong_as_double(b));
        case ACC_MIN_I64: return b < a ? b : a;
        default: return b > a ? b : a;
    }
}

// Slot hash of the fire's election table: two 32-bit multiplies with other multipliers than digit_hash
// (whose top bits picked the partition); the top bits index the table, lower bits give the probe step.
__device__ __forceinline__ uint32_t slot_mix(int64_t k) {
    return (uint32_t)k * 0x9E3779B1u + (uint32_t)((uint64_t)k >> 32) * 0x85EBCA77u;
}

// Election table word: leader record index (low 12 bits) | records of its key so far << 12.  Free: all ones.
#define FIRE_FREE 0xffffffffu
#define FIRE_ONE (1u << 12)

// PART: the checkpoint instance -- restored partial accumulators (after gwo_restore) and slow-path-only folds
// (gwo_snapshot's raw-word rows); a separate instance, so the watermark fire carries none of their code or registers.
// HV: the records carry values (16-B records; keys only: 8 B) -- a compile-time choice, since a load into registers
// chosen at run time between two widths merges the two definitions and waits for the load on the spot (the register
// prefetch of the next partition had waited for each of its 7 loads in turn).
// The fire's arguments, one struct: the kernel reads it through the kernarg segment pointer (offset 0), so the emit can
// load the plan and the output columns where it uses them (see P5).
struct FireArgs {
    const LogSegDesc *segs;
    int nseg;
    uint32_t nparts;
    int cap_log2;
    int has_val;
    AccPlan p;
    ResultPlan rp;
    int64_t start, end;
    OutCols o;
    unsigned long long *overflow;
    int slow_only;
    LogSegDesc partial;
    uint32_t *plist;
    uint32_t *pcount;
    // direct != 0 (int64 values, COUNT/SUM/MIN/MAX results only: no AVG, no float64): each result column is one of the
    // run's count, sum, min, max or the constant 1, chosen per aggregate by sel (4 bits each: 0 n, 1 sum, 2 min, 3 max,
    // 4 one) -- the emit selects without the plan's per-word and per-kind dispatch (fire_direct_sel)
    int32_t direct;
    uint32_t sel;
};
typedef __attribute__((address_space(4))) const FireArgs KFireArgs;   // in the (constant) kernarg segment

// FireArgs.direct / .sel for a plan: every aggregate's result column is one accumulator word as it is (int64 values,
// kinds COUNT, SUM, MIN, MAX) and each such word is the run's count, sum, min, max or the constant 1.
static void fire_direct_sel(const AccPlan &p, const ResultPlan &rp, int32_t *direct, uint32_t *sel) {
    *direct = 0;
    *sel = 0;
    if (p.value_is_f64 || rp.value_is_f64) return;
    uint32_t s = 0;
    for (int a = 0; a < rp.naggs; ++a) {
        if (rp.kind[a] == GWO_AGG_AVG) return;
        const int w = rp.word[a];
        if (w < 0 || w >= p.nwords) return;
        uint32_t c;
        if (p.src[w] == SRC_ONE) c = p.op[w] == ACC_ADD_I64 ? 0u : 4u;
        else if (p.src[w] != SRC_VALUE) return;
        else if (p.op[w] == ACC_ADD_I64) c = 1u;
        else if (p.op[w] == ACC_MIN_I64) c = 2u;
        else if (p.op[w] == ACC_MAX_I64) c = 3u;
        else return;
        s |= c << (4 * a);
    }
    *direct = 1;
    *sel = s;
}

template <int NW, bool PART, bool HV>
__global__ __launch_bounds__(LOG_FIRE_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4))) void log_fire_kernel(FireArgs A) {
    const LogSegDesc *__restrict__ segs = A.segs;
    const int nseg = A.nseg;
    const uint32_t nparts = A.nparts;
    const int cap_log2 = A.cap_log2;
    const int has_val_arg = A.has_val;
    const AccPlan &p = A.p;
    const ResultPlan &rp = A.rp;
    const int64_t start = A.start, end = A.end;
    const OutCols &o = A.o;
    unsigned long long *const overflow = A.overflow;
    const int slow_only = A.slow_only;
    const LogSegDesc &partial = A.partial;
    uint32_t *const plist = A.plist;
    uint32_t *const pcount = A.pcount;
    // Dynamic LDS (FIRE_LDS bytes).  Fast path:
    //   s_key [FIRE_RCAP] int64   record keys (record i = r * 512 + tid), then leader keys by row ordinal
    //   s_val [FIRE_RCAP] int64   values grouped by key (after the election; overlays s_own)
    //   s_own [FIRE_OWN]  uint32  election table: slot -> leader record | key's record count << 12 (overlays
    //                             s_val and the head of s_cnt; dead once the leaders have read their counts)
    //   s_cnt [FIRE_RCAP] uint32  per-leader record counts -> offsets -> (offset | count << 16) by ordinal
    // Slow path: the same bytes hold a FireCtx hash table (key + words, SoA, 2^cap_log2 slots).
    (void)has_val_arg;
    constexpr int has_val = HV ? 1 : 0;
    extern __shared__ __attribute__((aligned(16))) int64_t s_dyn[];
    int64_t *const s_key = s_dyn;
    int64_t *const s_val = s_dyn + FIRE_RCAP;
    uint32_t *const s_own = (uint32_t *)(s_dyn + FIRE_RCAP);
    uint32_t *const s_cnt = (uint32_t *)(s_dyn + 2 * FIRE_RCAP);
    __shared__ int64_t s_side[GWO_MAX_WORDS + 1];
    __shared__ unsigned s_used, s_fail;
    __shared__ uint32_t s_beg[LOG_MAX_SEGS + 1];   // flattened record space of a partition: segment s
    __shared__ uint32_t s_src[LOG_MAX_SEGS];       //   covers [s_beg[s], s_beg[s+1]) from record s_src[s]
    __shared__ const int64_t *s_rp[LOG_MAX_SEGS];
    __shared__ uint16_t s_cseg[FIRE_RCAP / 64];    // segment of record 64 c (chunks starting below the total)
    __shared__ uint32_t s_wsum[FIRE_RPT * (LOG_FIRE_THREADS / 64)];   // per-(r, wave) sums -> prefixes
    __shared__ uint32_t s_tot, s_rows;
    __shared__ uint32_t s_pw[LOG_FIRE_THREADS / 64 + 1];
    __shared__ unsigned long long s_rbase;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cap = 1 << cap_log2;
    FireCtx c{s_dyn, s_dyn + cap, s_side, &s_used, &s_fail, cap, (unsigned)(cap - (cap >> 3))};
    // !PART: the watermark fire's fast path only -- a partition it cannot hold is appended to plist (count *pcount)
    // and folded by the PART instance launched right behind it over that list (plist set: partitions plist[i]), so
    // the fast instance carries none of the slow path's code or registers (its scalars had spilled to VGPR lanes:
    // a v_readlane per use)
    const bool listed = PART && plist != nullptr;
    const uint32_t npi = listed ? *pcount : nparts;
    uint32_t pi = blockIdx.x;
    if (pi >= npi) return;
    uint32_t part = listed ? plist[pi] : pi;
    KTrace kt;
    kt.start(__builtin_amdgcn_readfirstlane(threadIdx.x) < 64 && g_kt_on);   // wave 0, uniform (scalar registers)
    for (int s = tid; s < nseg; s += LOG_FIRE_THREADS) s_rp[s] = segs[s].rec;
    if (tid <= GWO_MAX_WORDS) s_side[tid] = tid == 0 ? 0 : p.ident[tid - 1];
    if (tid == 0) {
        s_used = 0;
        s_fail = 0;
    }

    // Barriers in the fast path are LDS-only (lds_barrier): the next partition's records, the row reservation and
    // the emitted rows stay in flight across them (__syncthreads() drained every load, store and atomic each time).
    // segment ranges of a partition -> s_beg / s_src (all threads; ends synchronised)
    // (a DPP scan with the workgroup size fixed at compile time: block_exclusive_scan reads blockDim,
    // which costs a dispatch-packet load and a vmcnt(0) wait on everything in flight)
    auto publish = [&](uint32_t cnt, uint32_t off) {
        const uint32_t incl_c = wave_incl_scan(cnt);
        if (lane == 63) s_pw[wave] = incl_c;
        lds_barrier();
        if (tid == 0) {
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < LOG_FIRE_THREADS / 64; ++w) {
                const uint32_t t = s_pw[w];
                s_pw[w] = run;
                run += t;
            }
            s_pw[LOG_FIRE_THREADS / 64] = run;
        }
        lds_barrier();
        if (tid < nseg) {
            const uint32_t b = s_pw[wave] + incl_c - cnt;
            s_beg[tid] = b;
            s_src[tid] = off;
            // the chunks of 64 records that start inside this segment (the fast path's records only)
            const uint32_t e = b + cnt < (uint32_t)FIRE_RCAP ? b + cnt : (uint32_t)FIRE_RCAP;
            for (uint32_t ch = (b + 63) >> 6; (ch << 6) < e; ++ch) s_cseg[ch] = (uint16_t)tid;
        }
        if (tid == 0) s_beg[nseg] = s_pw[LOG_FIRE_THREADS / 64];
        lds_barrier();
    };
    // register prefetch of a partition's records (only when they all fit); global (not flat) loads,
    // so LDS waits in between do not wait for them
    int64_t rk[FIRE_RPT], rv[FIRE_RPT];
    // Always issued (a lane with nothing to fetch re-reads a valid record): a branch around the loads would merge
    // them with a second definition of rk/rv, and that copy waits for the loads (measured: fire 1.71 -> 1.95 ms).
    auto prefetch = [&](bool on) {   // (called after publish: s_rp is complete)
        const int64_t *const dflt = (PART && nseg == 0) ? partial.rec : s_rp[0];
        const uint32_t total = s_beg[nseg];
        const bool fits = on && total <= (uint32_t)FIRE_RCAP;
        const int64_t *addr[FIRE_RPT];
        int segr[FIRE_RPT];
        if (fits) {   // segment of record i: its 64-record chunk's first record's segment, then the (few) starts
                      // between (record i's chunk is a wave's run: one broadcast read)
#pragma unroll
            for (int r = 0; r < FIRE_RPT; ++r) {
                const uint32_t i = tid + r * LOG_FIRE_THREADS;
                int seg = 0;
                if (i < total) {
                    seg = s_cseg[i >> 6];
                    while (i >= s_beg[seg + 1]) seg++;
                }
                segr[r] = seg;
            }
        } else {
            int seg = 0;
#pragma unroll
            for (int r = 0; r < FIRE_RPT; ++r) {
                const uint32_t i = tid + r * LOG_FIRE_THREADS;
                while (i < total && i >= s_beg[seg + 1]) seg++;
                segr[r] = seg;
            }
        }
#pragma unroll
        for (int r = 0; r < FIRE_RPT; ++r) {
            const uint32_t i = tid + r * LOG_FIRE_THREADS;
            addr[r] = dflt;
            if (fits && i < total) {
                const int sg = segr[r];
                addr[r] = s_rp[sg] + (uint64_t)(s_src[sg] + (i - s_beg[sg])) * (has_val ? 2 : 1);
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

    // thread s < nseg keeps segment s's count / offset arrays (loaded once)
    g_u32 *seg_cnt = nullptr, *seg_off = nullptr;
    uint32_t a_cnt = 0, a_off = 0;
    if (tid < nseg) {
        seg_cnt = (g_u32 *)segs[tid].cnt;
        seg_off = (g_u32 *)segs[tid].off;
        a_cnt = seg_cnt[part];
        a_off = seg_off[part];
    }
    publish(a_cnt, a_off);
    prefetch(!(PART && slow_only));
    while (true) {
        const uint32_t total = s_beg[nseg];
        const uint32_t nxt_i = pi + gridDim.x;
        const bool more = nxt_i < npi;
        const uint32_t nxt = listed ? (more ? plist[nxt_i] : 0u) : nxt_i;
        // next partition's segment offsets: in flight while this one is folded (issued after the fast
        // path's first use of rk/rv, so waiting for the prefetch does not wait for them too)
        auto load_next = [&]() {
            a_cnt = 0;
            a_off = 0;
            if (more && tid < nseg) {
                a_cnt = seg_cnt[nxt];
                a_off = seg_off[nxt];
            }
        };
        unsigned long long rbase_lane0 = 0;   // wave 0 lane 0: the row reservation, consumed after P4
        bool fast = !(PART && slow_only) && total <= (uint32_t)FIRE_RCAP;
        if (fast) {
            // P0: record keys into LDS; free election table; zero counts
#pragma unroll
            for (int r = 0; r < FIRE_RPT; ++r) {
                const uint32_t i = r * LOG_FIRE_THREADS + tid;
                if (i < total) s_key[i] = rk[r];
            }
            load_next();
            for (int q = tid; q < FIRE_OWN / 4; q += LOG_FIRE_THREADS)
                ((uint4 *)s_own)[q] = make_uint4(FIRE_FREE, FIRE_FREE, FIRE_FREE, FIRE_FREE);
            if (tid == 0) s_rows = 0;
            lds_barrier();
            kt.stamp(0);
            // P1: claim or join, no barrier per probe round.  Every record of a key walks the same slot
            // sequence (double hashing on slot_mix).  A compare-and-swap of a free slot makes the record its
            // key's leader (count 1, rank 0); a slot whose leader holds the same key is joined by one add of
            // FIRE_ONE, whose return value is the record's rank among its key's records; a slot of another key
            // sends the record on.  The table never fills (8192 slots, <= 3584 keys), so every record ends.
            // sl[r]: probe slot while pending; then a leader's own slot, or a follower's leader record.
            uint32_t sl[FIRE_RPT], rank[FIRE_RPT];
            unsigned pend = 0, leader = 0;
#pragma unroll
            for (int r = 0; r < FIRE_RPT; ++r) {
                const uint32_t i = r * LOG_FIRE_THREADS + tid;
                sl[r] = slot_mix(rk[r]) >> (32 - FIRE_OWN_LOG2);
                rank[r] = 0;
                if (i < total) pend |= 1u << r;
            }
            while (pend) {   // per wave: ends when its lanes' records are all placed
                uint32_t prev[FIRE_RPT];
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r)
                    prev[r] = ((pend >> r) & 1u)
                                  ? atomicCAS(&s_own[sl[r]], FIRE_FREE, (r * LOG_FIRE_THREADS + tid) | FIRE_ONE)
                                  : FIRE_FREE;
                unsigned join = 0;
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r) {
                    if (!((pend >> r) & 1u)) continue;
                    if (prev[r] == FIRE_FREE) {   // claimed: this record leads its key
                        leader |= 1u << r;   // (sl[r] stays its slot)
                        pend &= ~(1u << r);
                    } else if (s_key[prev[r] & (FIRE_ONE - 1)] == rk[r]) {
                        join |= 1u << r;
                    } else {
                        const uint32_t step = ((slot_mix(rk[r]) >> 4) & (FIRE_OWN - 1)) | 1u;
                        sl[r] = (sl[r] + step) & (FIRE_OWN - 1);
                    }
                }
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r)
                    if ((join >> r) & 1u) rank[r] = atomicAdd(&s_own[sl[r]], FIRE_ONE) >> 12;
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r)
                    if ((join >> r) & 1u) sl[r] = prev[r] & (FIRE_ONE - 1);
                pend &= ~join;
            }
            {   // the partition's rows = its leaders: counted per wave now, so the row reservation is issued before P3
                uint32_t nl = 0;
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r) nl += (uint32_t)__popcll(__ballot((leader >> r) & 1u));
                if (lane == 0 && nl) atomicAdd(&s_rows, nl);
            }
            kt.stamp(1);
            lds_barrier();
            // the row reservation's round trip overlaps P3-P4 (consumed at P4b)
            if (tid == 0) rbase_lane0 = atomicAdd(o.count, (unsigned long long)s_rows);
            kt.stamp(2);
            {
                // P3: exclusive scan over record ids of (count | 1 << 16) at leaders -> each leader's
                // first value offset (low half) and row ordinal (high half).
                // (records in thread-major order -- thread t's FIRE_RPT records, then thread t + 1's: a serial prefix
                // per thread and one wave scan, instead of a wave scan per register slot)
                uint32_t xl[FIRE_RPT];   // exclusive prefix within the thread (one array live across the barriers)
                uint32_t run = 0;
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r) {   // (an unconditional read: a read under a branch is waited at the join)
#if FIRE_P3_BCAST   // followers read word 0 (their value is unused): one broadcast address instead of scattered ones
                    const uint32_t ow = s_own[((leader >> r) & 1u) ? sl[r] : 0u];
#else
                    const uint32_t ow = s_own[sl[r]];   // followers: sl = a record index, a valid slot too
#endif
                    const uint32_t x = ((leader >> r) & 1u) ? ((ow >> 12) | 0x10000u) : 0u;
                    xl[r] = run;
                    run += x;
                }
                const uint32_t incl = wave_incl_scan(run);
                if (lane == 63) s_wsum[wave] = incl;
                lds_barrier();
                if (wave == 0) {
                    constexpr int NS = LOG_FIRE_THREADS / 64;
                    const uint32_t w = lane < NS ? s_wsum[lane] : 0u;
                    const uint32_t wi = wave_incl_scan(w);
                    if (lane < NS) s_wsum[lane] = wi - w;
                    const uint32_t tot = __shfl(wi, 63);
                    if (lane == 0) s_tot = tot;
                }
                lds_barrier();
                const uint32_t tbase = s_wsum[wave] + incl - run;   // this thread's first record's prefix
                uint32_t lo[FIRE_RPT];   // leaders: value offset | row ordinal << 16
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r) {
                    const uint32_t i = r * LOG_FIRE_THREADS + tid;
                    const uint32_t pre = tbase + xl[r];
                    lo[r] = pre;
                    if ((leader >> r) & 1u) s_cnt[i] = pre & 0xffffu;
                }
                lds_barrier();
                // P4: values grouped by key, in row order (the election table is dead).  Every follower's read of its
                // leader's offset is issued before any write (reads unconditional: leaders read entry 0).
                if (has_val) {
                    uint32_t lof[FIRE_RPT];
#pragma unroll
                    for (int r = 0; r < FIRE_RPT; ++r) lof[r] = s_cnt[((leader >> r) & 1u) ? 0u : sl[r]];
#pragma unroll
                    for (int r = 0; r < FIRE_RPT; ++r) {
                        const uint32_t i = r * LOG_FIRE_THREADS + tid;
                        const uint32_t off = ((leader >> r) & 1u) ? (lo[r] & 0xffffu) : lof[r];
                        const uint32_t at = off + rank[r];
                        if (i < total && at < (uint32_t)FIRE_RCAP) s_val[at] = rv[r];
                    }
                }
                lds_barrier();
                // P4b: by row ordinal, the row's first value offset (a row's value count is the next row's offset
                // minus its own; s_cnt[rows] = total) and its key (every read of s_key by record is done)
#pragma unroll
                for (int r = 0; r < FIRE_RPT; ++r)
                    if ((leader >> r) & 1u) {
                        s_cnt[lo[r] >> 16] = lo[r] & 0xffffu;
                        s_key[lo[r] >> 16] = rk[r];
                    }
                if (tid == 0) {
                    s_cnt[s_tot >> 16] = s_tot & 0xffffu;
                    s_rbase = rbase_lane0;   // the atomic's round trip overlapped P4
                }
                kt.stamp(3);
            }
        }
        // (the fast path loaded them in P0).  Every partition the fast path did not take -- also a small one in a
        // slow-only fold (a restored window's fire, a checkpoint's or a lateness migration's fold): keyed on the
        // total instead, a workgroup's second small partition republished its first one's ranges (rows of one
        // partition twice, another's lost, once a window had more partitions than the grid's 2 per CU)
        if (!fast) load_next();
        if constexpr (!PART) {
            if (!fast && tid == 0) {   // for the slow instance
                plist[atomicAdd(pcount, 1u)] = part;
                atomicAdd(overflow + 1, 1ull);   // slow-path partitions (statistics)
            }
        } else if (!fast) {
            // slow path: hash-table rounds over disjoint ranges of hash bits 12..43, direct loads
            if (tid == 0 && !listed) atomicAdd(overflow + 1, 1ull);   // slow-path partitions (statistics)
            __syncthreads();
            fire_clear(c, p);
            __syncthreads();
            const uint64_t kAll = 1ull << 32;
            uint64_t lo = 0, width = kAll;
            while (lo < kAll) {
                const uint64_t hi = lo + width < kAll ? lo + width : kAll;
                const bool ranged = width < kAll;
                int seg = 0;
                for (uint32_t i = tid; i < total; i += LOG_FIRE_THREADS) {
                    while (i >= s_beg[seg + 1]) seg++;
                    const int64_t *q = s_rp[seg] + (uint64_t)(s_src[seg] + (i - s_beg[seg])) * (has_val ? 2 : 1);
                    const int64_t k = q[0];
                    const uint64_t h = part_hash(k);
                    if (ranged) {
                        uint64_t sub = (uint32_t)(h >> 12);
                        if (sub < lo || sub >= hi) continue;
                    }
                    fire_insert(c, p, k, h, has_val ? q[1] : 0);
                }
                if (PART && partial.rec) {   // restored accumulators of this partition (raw words, combined as they are)
                    const uint32_t pc = partial.cnt[part], po = partial.off[part];
                    for (uint32_t i = tid; i < pc; i += LOG_FIRE_THREADS) {
                        const int64_t *q = partial.rec + (uint64_t)(po + i) * (1 + p.nwords);
                        const int64_t k = q[0];
                        const uint64_t h = part_hash(k);
                        if (ranged) {
                            uint64_t sub = (uint32_t)(h >> 12);
                            if (sub < lo || sub >= hi) continue;
                        }
                        fire_insert_words(c, p, k, h, q + 1);
                    }
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
        // (synchronises: the fast path's (offset, count) words and s_rbase are visible)
        if (more) publish(a_cnt, a_off);
        else lds_barrier();
        // unconditional, so the loads land straight in rk/rv (no loop-carried copy that would wait for
        // them): in flight during this partition's emit and the next one's election
        prefetch(more && !(PART && slow_only));
        kt.stamp(4);
        if (fast) {
            // P5: one row per leader, in ordinal order.  Each lane takes two consecutive ordinals, so that its rows
            // are a 16-B-aligned pair of global rows (lane t: ordinals 2t - sh, 2t + 1 - sh with sh = rbase & 1) and
            // it stores each column of both with one 16-B store (8-B stores are issue-bound at about half the
            // bandwidth; r03 paired lanes with DPP swaps instead, which cost a fifth of this phase's VALU).  A row
            // whose partner is outside the partition's run is stored alone, 8 B per column.
            const uint32_t rows = s_tot >> 16;
            const unsigned long long rbase = s_rbase;
            const int sh = (int)(rbase & 1ull);
            // one row's key and results; reads unconditional (from row 0 for a lane without a row: no LDS read waits
            // at a branch join)
            // the plan and the output columns, loaded here (scalar loads from the kernarg segment, behind an opaque
            // copy of its pointer, once per partition) instead of held in scalar registers across the persistent
            // loop: they spilled to VGPR lanes, a v_readlane per use.  (The kernarg segment is constant memory, so no
            // store is taken to alias them.)
            KFireArgs *KA = (KFireArgs *)__builtin_amdgcn_kernarg_segment_ptr();
            asm volatile("" : "+s"(KA));
            int64_t *const okey = KA->o.key, *const ostart = KA->o.start, *const oend = KA->o.end;
            int64_t *ores[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) ores[a] = KA->o.res[a];
            const long long ocap = KA->o.cap;
            const int64_t wstart = KA->start, wend = KA->end;
            int pop[NW], psrc[NW];
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                pop[w] = KA->p.op[w];
                psrc[w] = KA->p.src[w];
            }
            const int vf64 = KA->p.value_is_f64;
            const int naggs = KA->rp.naggs, rf64 = KA->rp.value_is_f64;
            int rkind[4], rword[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                rkind[a] = KA->rp.kind[a];
                rword[a] = KA->rp.word[a];
            }
            auto fold_row = [&](int q, bool valid, int64_t &k, int64_t (&res)[4]) {
                const uint32_t qc = valid ? (uint32_t)q : 0u;
                const uint32_t off = s_cnt[qc], nxt = s_cnt[qc + 1];
                k = s_key[qc];
                const uint32_t n = valid ? nxt - off : 0u;
                // the run's count, sum and min/max (of the values, or of their Double.compareTo order keys for
                // float64): its first 4 values read together, the rest (rare) in a loop; the plan's words are read
                // off them afterwards
                int64_t si = 0, mn = 0x7fffffffffffffffLL, mx = (int64_t)0x8000000000000000LL;
                double sf = 0.0;
                if (has_val) {
                    int64_t v4[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const uint32_t ix = off + t < (uint32_t)FIRE_RCAP ? off + t : 0u;
                        v4[t] = s_val[ix];
                    }
                    if (vf64) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const bool in = (uint32_t)t < n;
                            const int64_t v = v4[t], ok = f64_order_key(v);
                            sf += in ? __longlong_as_double(v) : 0.0;
                            mn = (in && ok < mn) ? ok : mn;
                            mx = (in && ok > mx) ? ok : mx;
                        }
                        for (uint32_t t = 4; t < n; ++t) {
                            const int64_t v = s_val[off + t], ok = f64_order_key(v);
                            sf += __longlong_as_double(v);
                            mn = ok < mn ? ok : mn;
                            mx = ok > mx ? ok : mx;
                        }
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const bool in = (uint32_t)t < n;
                            const int64_t v = v4[t];
                            si = (int64_t)((uint64_t)si + (uint64_t)(in ? v : 0));
                            mn = (in && v < mn) ? v : mn;
                            mx = (in && v > mx) ? v : mx;
                        }
                        for (uint32_t t = 4; t < n; ++t) {
                            const int64_t v = s_val[off + t];
                            si = (int64_t)((uint64_t)si + (uint64_t)v);
                            mn = v < mn ? v : mn;
                            mx = v > mx ? v : mx;
                        }
                    }
                }
                int64_t acc[NW];
#pragma unroll
                for (int w = 0; w < NW; ++w) {
                    switch (pop[w]) {
                        case ACC_ADD_I64: acc[w] = psrc[w] == SRC_ONE ? (int64_t)n : si; break;
                        case ACC_ADD_F64: acc[w] = __double_as_longlong(sf); break;
                        case ACC_MIN_I64: acc[w] = psrc[w] == SRC_ONE ? 1 : mn; break;
                        default: acc[w] = psrc[w] == SRC_ONE ? 1 : mx; break;
                    }
                }
                row_results_s<NW>(naggs, rkind, rword, rf64, acc, res);
            };
            // the direct plan (int64 COUNT/SUM/MIN/MAX: FireArgs.direct): the run's count, sum, min and max, then a
            // branch-free select per result column -- no per-word or per-kind dispatch per row
            const bool direct = KA->direct != 0;
            const uint32_t dsel = KA->sel;
            auto fold_row_direct = [&](int q, bool valid, int64_t &k, int64_t (&res)[4]) {
                const uint32_t qc = valid ? (uint32_t)q : 0u;
                const uint32_t off = s_cnt[qc], nxt = s_cnt[qc + 1];
                k = s_key[qc];
                const uint32_t n = valid ? nxt - off : 0u;
                int64_t si = 0, mn = 0x7fffffffffffffffLL, mx = (int64_t)0x8000000000000000LL;
                if (has_val) {
                    // the run's first FIRE_EMIT_V values, unclamped (adjacent reads pair into ds_read2_b64): off <=
                    // FIRE_RCAP, and s_val[FIRE_RCAP ..] is the s_own / s_cnt area, inside the allocation (values past
                    // n are unused); the rest in a loop, which a wave runs as long as its longest run
                    int64_t v4[FIRE_EMIT_V];
#pragma unroll
                    for (int t = 0; t < FIRE_EMIT_V; ++t) v4[t] = s_val[off + t];
#pragma unroll
                    for (int t = 0; t < FIRE_EMIT_V; ++t) {
                        const bool in = (uint32_t)t < n;
                        const int64_t v = v4[t];
                        si = (int64_t)((uint64_t)si + (uint64_t)(in ? v : 0));
                        mn = (in && v < mn) ? v : mn;
                        mx = (in && v > mx) ? v : mx;
                    }
                    for (uint32_t t = FIRE_EMIT_V; t < n; ++t) {
                        const int64_t v = s_val[off + t];
                        si = (int64_t)((uint64_t)si + (uint64_t)v);
                        mn = v < mn ? v : mn;
                        mx = v > mx ? v : mx;
                    }
                }
                // the selector is wave-uniform: these branches do not diverge (a mask-and-or selection measured 3 %
                // slower per fire, profiles/r06_experiments.txt)
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    const uint32_t c = (dsel >> (4 * a)) & 15u;
                    res[a] = c == 0u ? (int64_t)n : c == 1u ? si : c == 2u ? mn : c == 3u ? mx : (int64_t)1;
                }
            };
            for (int base = 0; base < (int)rows + sh; base += 2 * LOG_FIRE_THREADS) {
                const int q0 = base + 2 * tid - sh, q1 = q0 + 1;
                const bool v0 = q0 >= 0 && q0 < (int)rows, v1 = q1 < (int)rows;
                if (!v0 && !v1) continue;
                int64_t k0, k1, r0[4] = {0, 0, 0, 0}, r1[4] = {0, 0, 0, 0};
                if (direct) {
                    fold_row_direct(q0, v0, k0, r0);
                    fold_row_direct(q1, v1, k1, r1);
                } else {
                    fold_row(q0, v0, k0, r0);
                    fold_row(q1, v1, k1, r1);
                }
                const unsigned long long pb = rbase + (unsigned long long)(long long)q0;   // even: the pair's first row
#ifdef GWO_ABL_FIRE_NOSTORE   // ablation (timing experiments only): the emit without its global stores
                if (pb != ~0ull) continue;
#endif
                if (v0 && v1 && (long long)pb + 1 < ocap) {
                    *(ll2 *)(okey + pb) = ll2{k0, k1};
                    *(ll2 *)(ostart + pb) = ll2{wstart, wstart};
                    *(ll2 *)(oend + pb) = ll2{wend, wend};
#pragma unroll
                    for (int a = 0; a < 4; ++a)
                        if (a < naggs) *(ll2 *)(ores[a] + pb) = ll2{r0[a], r1[a]};
                } else {   // a row alone (first or last of the partition's run)
                    const unsigned long long pos = v0 ? pb : pb + 1;
                    if ((long long)pos < ocap) {
                        okey[pos] = v0 ? k0 : k1;
                        ostart[pos] = wstart;
                        oend[pos] = wend;
#pragma unroll
                        for (int a = 0; a < 4; ++a)
                            if (a < naggs) ores[a][pos] = v0 ? r0[a] : r1[a];
                    }
                }
            }
            lds_barrier();   // the next partition overwrites s_key / s_cnt
            kt.stamp(5);
        }
        if (!more) break;
        pi = nxt_i;
        part = nxt;
    }
    if (kt.on && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_kt[33], 1ull);
    kt.flush(KT_FIRE);
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
// GWO_K1_V2=0: K1 loads one record per lane per column (A/B of the 16-B pair loads)
static bool getenv_k1_v2() {
    static const int on = getenv("GWO_K1_V2") ? atoi(getenv("GWO_K1_V2")) : 1;
    return on != 0;
}

void launch_log_part(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, int64_t stride,
                     const WindowGeom &g,
                     long long base, int nunits, int has_val, unsigned long long *cursor, uint64_t cap,
                     int64_t *tmp, BatchStats *st, int64_t *side_key, int64_t *side_ts, int64_t *side_val,
                     unsigned long long *side_count, long long side_cap, int side_enabled, const CollectArgs &ca,
                     const LogThr &thr, const LogRoute &rt, hipStream_t s) {
    // rounds = tiles per workgroup at full tiles; then the tile length that gives every workgroup that many
    // (16.67M records: 8 rounds of 4070 records instead of 9 rounds for most workgroups and a 10th for 42)
    const int64_t grid = log_k1_grid(n);
    const int64_t rounds = (n + grid * LOG_K1_TILE - 1) / (grid * LOG_K1_TILE);
    int64_t tl = rounds > 0 ? (n + grid * rounds - 1) / (grid * rounds) : LOG_K1_TILE;
    tl = tl < 1 ? 1 : (tl > LOG_K1_TILE ? LOG_K1_TILE : tl);
    const bool route = rt.mode != 0 && stride == 1;
    const size_t dyn = ((size_t)2 * nunits * LOG_ND + 1 + (route ? LOG_RT_MAX : 0)) * sizeof(uint32_t);
    // 16-B loads of record pairs: SoA columns aligned to 16 B (8 B for int32 timestamps), tiles of an even length
    const bool v2 = stride == 1 && ((uintptr_t)key & 15) == 0 && (!has_val || ((uintptr_t)val & 15) == 0) &&
                    ((uintptr_t)ts & (thr.ts32 ? 7 : 15)) == 0 && getenv_k1_v2();
    if (v2) tl = (tl + 1) & ~(int64_t)1;
#define GWO_K1(HV, S, R, T32, VV)                                                                              \
    hipLaunchKernelGGL((log_part_kernel<HV, S, R, T32, VV>), dim3((int)grid), dim3(LOG_K1_THREADS), dyn, s, key, ts, \
                       val, n, stride, g, base, nunits, cursor, cap, tmp, st, side_key, side_ts, side_val, side_count, \
                       side_cap, side_enabled, ca, thr, rt, (int)tl)
#define GWO_K1S(HV, R, T32)                  \
    do {                                     \
        if (v2) GWO_K1(HV, 1, R, T32, true); \
        else GWO_K1(HV, 1, R, T32, false);   \
    } while (0)
    if (route) {   // routing: the first K1 over a batch's own columns (and its route-only re-run)
        if (has_val) GWO_K1S(true, true, false);
        else GWO_K1S(false, true, false);
    } else if (thr.ts32) {               // received 20-B wire records (SoA columns, int32 timestamps)
        if (has_val) GWO_K1S(true, false, true);
        else GWO_K1S(false, false, true);
    } else if (has_val) {
        if (stride == 1) GWO_K1S(true, false, false);
        else if (stride == 3) GWO_K1(true, 3, false, false, false);
        else GWO_K1(true, 0, false, false, false);
    } else {
        if (stride == 1) GWO_K1S(false, false, false);
        else if (stride == 3) GWO_K1(false, 3, false, false, false);
        else GWO_K1(false, 0, false, false, false);
    }
#undef GWO_K1S
#undef GWO_K1
}

void launch_log_split(const int64_t *tmp, uint64_t cap, int has_val, const LogBucket *buckets, int nb,
                      const LogSegSet &segs, unsigned *overflow, uint32_t nchunks, const unsigned *go, hipStream_t s) {
    if (nchunks == 0) return;
    if (has_val)
        hipLaunchKernelGGL(log_split_kernel<true>, dim3(nchunks), dim3(LOG_TILE_THREADS), 0, s, tmp, cap, buckets, nb,
                           segs, overflow, go);
    else
        hipLaunchKernelGGL(log_split_kernel<false>, dim3(nchunks), dim3(LOG_TILE_THREADS), 0, s, tmp, cap, buckets, nb,
                           segs, overflow, go);
}

int log_k1_grid(int64_t n) {
    int64_t grid = (n + LOG_K1_TILE - 1) / LOG_K1_TILE;
    return (int)(grid < 1 ? 1 : (grid > LOG_K1_GRID ? LOG_K1_GRID : grid));
}

void warm_log_kernels(int nwords, int has_val, hipStream_t s) {
    const AccPlan p{};
    const ResultPlan rp{};
    const OutCols o{};
    const int cl = log_fire_cap_log2(nwords);
    size_t lds = (size_t)(1 + nwords) * 8 << cl;
    if (lds < (size_t)FIRE_LDS) lds = FIRE_LDS;
    FireArgs fa{};   // no partitions: every workgroup returns at once
    fa.cap_log2 = cl;
    fa.has_val = has_val;
    fa.p = p;
    fa.rp = rp;
    fa.o = o;
#define GWO_WARM_NW(NW)                                                                                            \
    case NW:                                                                                                       \
        if (has_val) {                                                                                             \
            hipLaunchKernelGGL((log_fire_kernel<NW, false, true>), dim3(1), dim3(LOG_FIRE_THREADS), lds, s, fa);      \
            hipLaunchKernelGGL((log_fire_kernel<NW, true, true>), dim3(1), dim3(LOG_FIRE_THREADS), lds, s, fa);       \
        } else {                                                                                                   \
            hipLaunchKernelGGL((log_fire_kernel<NW, false, false>), dim3(1), dim3(LOG_FIRE_THREADS), lds, s, fa);     \
            hipLaunchKernelGGL((log_fire_kernel<NW, true, false>), dim3(1), dim3(LOG_FIRE_THREADS), lds, s, fa);      \
        }                                                                                                          \
        break;
    switch (nwords) {
        GWO_WARM_NW(1)
        GWO_WARM_NW(2)
        GWO_WARM_NW(3)
        GWO_WARM_NW(4)
        GWO_WARM_NW(5)
        GWO_WARM_NW(6)
        GWO_WARM_NW(7)
        default: GWO_WARM_NW(8)
    }
#undef GWO_WARM_NW
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
                     int cus, int max_per_cu, int slow_only, const LogSegDesc &partial, uint32_t *slow_list,
                     uint32_t *slow_cnt, hipStream_t s) {
    if (nseg < 0 || nseg > LOG_MAX_SEGS || (nseg == 0 && !partial.rec)) return;   // nothing to fold (defensive)
    static_assert(FIRE_OWN * 4 <= FIRE_RCAP * 12 && FIRE_OWN == (1 << FIRE_OWN_LOG2) && FIRE_RCAP <= 4096 &&
                      FIRE_OWN > FIRE_RCAP, "fire fast-path layout");
    int cl = log_fire_cap_log2(plan.nwords);
    size_t lds = (size_t)(1 + plan.nwords) * 8 << cl;
    if (lds < (size_t)FIRE_LDS) lds = FIRE_LDS;
    uint32_t parts = 1u << lp;
    // persistent grid: two 64-KiB-LDS workgroups per CU, or fewer to leave room for concurrent kernels
    const uint32_t groups = (uint32_t)cus * (uint32_t)(max_per_cu < 2 ? max_per_cu : 2);
    uint32_t grid = parts < groups ? parts : groups;
    // the watermark fire: the fast instance lists the partitions it cannot hold, the slow instance folds that list
    const bool listed = !(partial.rec || slow_only);
    if (listed) (void)hipMemsetAsync(slow_cnt, 0, 4, s);
    FireArgs fa{};
    fa.segs = segs;
    fa.nseg = nseg;
    fa.nparts = parts;
    fa.cap_log2 = cl;
    fa.has_val = has_val;
    fa.p = plan;
    fa.rp = rp;
    fa.start = start;
    fa.end = end;
    fa.o = out;
    fa.overflow = overflow;
    fa.partial = partial;
    fa.pcount = slow_cnt;
    static const bool direct_on = getenv("GWO_FIRE_DIRECT") == nullptr || atoi(getenv("GWO_FIRE_DIRECT")) != 0;
    if (direct_on) fire_direct_sel(plan, rp, &fa.direct, &fa.sel);
    FireArgs fs = fa;            // the slow instance: over the fast instance's list, or every partition
    fa.slow_only = 0;
    fa.plist = slow_list;
    fs.slow_only = listed ? 1 : slow_only;
    fs.plist = listed ? slow_list : nullptr;
#define GWO_FIRE_NW(NW)                                                                                          \
    case NW:                                                                                                     \
        if (has_val) {                                                                                           \
            if (listed)                                                                                          \
                hipLaunchKernelGGL((log_fire_kernel<NW, false, true>), dim3(grid), dim3(LOG_FIRE_THREADS), lds, s, fa); \
            hipLaunchKernelGGL((log_fire_kernel<NW, true, true>), dim3(grid), dim3(LOG_FIRE_THREADS), lds, s, fs);   \
        } else {                                                                                                 \
            if (listed)                                                                                          \
                hipLaunchKernelGGL((log_fire_kernel<NW, false, false>), dim3(grid), dim3(LOG_FIRE_THREADS), lds, s, fa); \
            hipLaunchKernelGGL((log_fire_kernel<NW, true, false>), dim3(grid), dim3(LOG_FIRE_THREADS), lds, s, fs);  \
        }                                                                                                        \
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

// Phase trace switch and report (GWO_KTRACE=1; diagnostics only).
void ktrace_enable(int on) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kt_on), &on, sizeof(int));
}

void ktrace_report() {
    unsigned long long v[64];
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_kt), sizeof(v)) != hipSuccess) return;
    const double k1 = v[32] ? (double)v[32] : 1.0, fi = v[33] ? (double)v[33] : 1.0;
    fprintf(stderr, "[ktrace] K1 launches %llu, per launch per workgroup (Mcycles, summed over workgroups):\n", v[32]);
    const char *kn[10] = {"zero+loop", "classify", "slow+barrier", "reserve+offsets", "scatter", "write", "stats",
                          "load issue", "reserved delta", "barrier"};
    for (int i = 0; i < 10; ++i) fprintf(stderr, "  K1 %-18s %10.3f\n", kn[i], v[i] / k1 / 1e6);
    const char *fn[6] = {"P0 keys/table", "P1 claim", "P1 barrier", "P3-P4b", "publish+prefetch", "P5 emit"};
    fprintf(stderr, "[ktrace] fires %llu, per fire (Mcycles, summed over workgroups):\n", v[33]);
    for (int i = 0; i < 6; ++i) fprintf(stderr, "  fire %-18s %10.3f\n", fn[i], v[16 + i] / fi / 1e6);
    for (int i = 0; i < 64; ++i) v[i] = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kt), v, sizeof(v));
}

}  // namespace gwo
