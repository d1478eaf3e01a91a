// gwo_slog.hip -- the window step of sliding windows over logged panes (gwo_slog.h).
//
// WindowOperator.onEventTime + emitWindowContents (WindowOperator.java:430-473, 546-550) for every key of
// sliding window J at once: the running total of window J-1 (R, partitioned by the top lp bits of
// digit_hash, one HBM region per partition), the records of the pane that enters J and -- negated --
// of the pane that leaves it, folded per partition in an LDS hash table; then every key whose count is
// positive emits J's row and is written back as R' (keys whose count fell to zero leave the state:
// the reference's window for that key holds no element, so it emits nothing).  All words are int64
// sums (AggregateFunction add of SumFunction/CountAggregate/AverageAggregate; wrap-around as Java long),
// an abelian group, so the result is bit-identical to summing the window's panes.
//
// The LDS table is made of 8-slot buckets.  R' is written bucket by bucket with a byte per bucket (entries,
// overflow flag), so the next step puts each entry of R straight into its bucket: the running total -- about
// three quarters of a step's records at C3 -- costs no hash, probe or atomic; only the panes' records search
// the table (bucket reads, one CAS to claim a new key, word atomics).  (Hashing and probing every entry made
// the step VALU-issue bound: ~33K VALU instructions per wave, LDS bank conflicts 54 % of the LDS cycles.)
//
// One persistent workgroup of 256 threads takes partitions p = blockIdx.x, + gridDim.x, ...; every HBM
// access is a run of consecutive records (R_p, the segments' partition slices, R'_p, the rows).  A partition
// with more keys than the table holds is folded in rounds over disjoint ranges of a second hash (each round
// re-reads the partition's inputs; its R' is then written unstructured), so no key is ever lost.
#include "../../include/gwo.h"
#include "gwo_device.h"
#include "gwo_slog.h"

namespace gwo {

#ifndef GWO_SLOG_J
#define GWO_SLOG_J 4
#endif
constexpr int SLOG_J = GWO_SLOG_J;   // records per thread per pass (the loads of a pass are all in flight together)

typedef __attribute__((address_space(1))) const int64_t g_i64;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

size_t slog_lds_bytes(int cap_log2, int nwords) { return ((size_t)1 << cap_log2) * (size_t)(1 + nwords) * 8; }
int slog_table_log2(int nwords) { return slog_cap_log2_for(nwords); }

// Bucket of a key: a multiplicative hash of both halves, independent of the partition bits (digit_hash) and of lp,
// so a partition split keeps every key's bucket.
__device__ __forceinline__ uint32_t slog_bucket(int64_t k, int nbits) {
    return ((uint32_t)k * 0x9E3779B1u + (uint32_t)((uint64_t)k >> 32) * 0x85EBCA77u) >> (32 - nbits);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// LDS position of table slot s (bucket s >> 3, slot s & 7 of it): the slot index within the bucket is XORed with bits
// 2-4 of the bucket.  A bucket is 64 B, so without it slot i of every bucket falls on one of only 4 bank pairs and
// a wave searching 64 random buckets reads 16-way conflicted; with it slot i spreads over all 32 (and the sweep's
// thread-contiguous slots, 8-way conflicted at a 32-B lane stride, spread too).  A bucket's slots stay in its 64 B.
__device__ __forceinline__ int slot_lds(int s) { return s ^ ((s >> 5) & 7); }

__device__ __forceinline__ int64_t lds_key(const int64_t *s_key, int slot) {
    return __hip_atomic_load(&s_key[slot_lds(slot)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Find or claim key k's slot.  The search reads whole buckets (8 LDS reads, one round trip) from the key's home
// bucket on, and ends at the first bucket that has a free slot and no overflow flag (a key displaced past a
// bucket set that bucket's flag when it found the bucket full); a new key is claimed, with one CAS, in the first
// free slot the search met -- every lane claiming k targets the same slot, so a key is never claimed twice (a
// failed CAS restarts the search).  -1: the side slot (k == Long.MIN_VALUE, the free marker); -2: table full.
__device__ __forceinline__ int slog_find(int64_t *s_key, uint8_t *s_ovf, int NB, int nbits, int64_t k,
                                         unsigned &claims) {
    if (k == GWO_EMPTY_KEY) return -1;
    const int home = (int)slog_bucket(k, nbits);
    for (int attempt = 0; attempt < 64; ++attempt) {
        int b = home, ff = -1;
        for (int steps = 0; steps < NB; ++steps) {
            int64_t kb[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) kb[i] = lds_key(s_key, b * 8 + i);
            int hit = -1, fr = -1;
#pragma unroll
            for (int i = 7; i >= 0; --i) {
                if (kb[i] == k) hit = i;
                if (kb[i] == GWO_EMPTY_KEY) fr = i;
            }
            if (hit >= 0) return b * 8 + hit;
            if (fr >= 0 && ff < 0) ff = b * 8 + fr;
            if (fr >= 0 && !s_ovf[b]) break;
            if (fr < 0) s_ovf[b] = 1;   // full: a key placed beyond it is displaced past it
            b = (b + 1) & (NB - 1);
        }
        if (ff < 0) return -2;
        const unsigned long long prev = atomicCAS((unsigned long long *)&s_key[slot_lds(ff)], (unsigned long long)GWO_EMPTY_KEY,
                                                  (unsigned long long)k);
        if ((int64_t)prev == GWO_EMPTY_KEY) {
            claims++;
            return ff;
        }
        if ((int64_t)prev == k) return ff;
    }
    return -2;
}

#if GWO_SLOG_CHECK
// The diagnostic build's violation record (gwo_slog.h SlogCheck): the first one's details, every one counted.
__device__ __noinline__ void slog_violation(unsigned long long *v, int what, uint64_t p, uint64_t idx, uint64_t bound,
                                            uint64_t width, int lp_in, int lp_out) {
    if (atomicAdd(&v[0], 1ull) == 0ull) {
        v[1] = (unsigned long long)what;
        v[2] = p;
        v[3] = idx;
        v[4] = bound;
        v[5] = width;
        v[6] = (unsigned long long)lp_in;
        v[7] = (unsigned long long)lp_out;
    }
}
#define SLOG_CHK(ok, what, idx, bound) \
    (((ok)) ? true : (slog_violation(a.chk.viol, (what), p, (uint64_t)(idx), (uint64_t)(bound), width, lp_in, a.out.lp), false))
#else
#define SLOG_CHK(ok, what, idx, bound) true
#endif

#ifndef GWO_SLOG_SLOTS
#define GWO_SLOG_SLOTS 1   // R' carries each entry's table slot: the next step places R_p without the bucket bytes
#endif
#ifndef GWO_SLOG_WPE
#define GWO_SLOG_WPE 4   // waves per SIMD the registers are sized for (4: 128 VGPRs, 4 workgroups per CU)
#endif
template <int NW>
__global__ __launch_bounds__(slog_threads_for(NW)) __attribute__((amdgpu_waves_per_eu(GWO_SLOG_WPE, GWO_SLOG_WPE))) void slog_fire_kernel(SlogArgs a) {
    constexpr int TH = slog_threads_for(NW);   // SLOG_THREADS, or 512 with GWO_SLOG_BIG's larger tables
    extern __shared__ __attribute__((aligned(16))) int64_t s_dyn[];
    const int T = 1 << a.cap_log2, NB = T >> 3, nbits = a.cap_log2 - 3, SPT = T / TH;
    int64_t *const s_key = s_dyn;       // [T]
    int64_t *const s_w = s_dyn + T;     // [NW][T]
    __shared__ int64_t s_side[1 + GWO_MAX_WORDS];   // key == Long.MIN_VALUE: [present, words]
    __shared__ unsigned s_used, s_fail, s_rn;
    // the partition's record inputs as one flattened record space: range r covers [s_beg[r], s_beg[r + 1]) from
    // record s_src[r] of s_ptr[r]; range 0 is R_p when it is unstructured (else empty: its entries are placed)
    __shared__ const int64_t *s_ptr[SLOG_MAX_SEGS + 1];
    __shared__ uint32_t s_beg[SLOG_MAX_SEGS + 2], s_src[SLOG_MAX_SEGS + 1];
    __shared__ int32_t s_meta[SLOG_MAX_SEGS + 1];   // stride | words-to-load << 8 | raw << 12 | filter << 13 | neg << 14
    __shared__ uint8_t s_ovf[SLOG_MAX_NB];          // the fold's overflow flags (R's, and those its inserts set)
#if !GWO_SLOG_SLOTS
    __shared__ uint8_t s_map[SLOG_MAX_NB * 9];      // R_p entry -> its bucket (a bucket holds <= 8 + the side entry)
    __shared__ uint16_t s_pre[SLOG_MAX_NB];         // first R_p entry of each bucket
#endif
    __shared__ uint8_t s_ovo[2][SLOG_MAX_NB];       // R''s, recomputed from the keys' displacement by the sweep
    __shared__ unsigned s_wsum[TH / 64];
    __shared__ unsigned s_qn[2];          // R' entries written so far for the partition's (one or two) outputs
    __shared__ unsigned long long s_rowbase;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lp_in = a.in.lp, split = a.out.lp - a.in.lp;   // 0 or 1
    const uint32_t P = 1u << lp_in;
    const int RW = 1 + NW;
    const unsigned limit = (unsigned)(T - (T >> 3));
    const int side_bucket = (int)slog_bucket(GWO_EMPTY_KEY, nbits);
    unsigned long long st_live = 0, st_maxp = 0, st_rovf = 0, st_neg = 0, st_lds = 0, st_slow = 0;

    for (int i = tid; i < T; i += TH) s_key[i] = GWO_EMPTY_KEY;
    for (int i = tid; i < T * NW; i += TH) s_w[i] = 0;
    if (tid <= GWO_MAX_WORDS) s_side[tid] = 0;
    if (tid < SLOG_MAX_NB) {
        s_ovo[0][tid] = 0;
        s_ovo[1][tid] = 0;
        s_ovf[tid] = 0;
    }
    if (tid == 0) {
        s_used = 0;
        s_fail = 0;
    }
    __syncthreads();

    if (a.dbg && tid == 0 && blockIdx.x < SLOG_DBG_BLOCKS) a.dbg[SLOG_DBG_PHASES + 2 * blockIdx.x] = wall_clock64();
    int pn = 0;
    auto stamp = [&](int ph) {
        if (a.dbg && blockIdx.x == 0 && tid == 0 && pn < 32) a.dbg[pn * 8 + ph] = wall_clock64();
    };
    for (uint32_t p = blockIdx.x; p < P; p += gridDim.x, ++pn) {
        stamp(0);
        // ---- the partition's ranges: each segment's slice (its partition p >> (lp_in - lp_s), filtered by the top
        // lp_in bits when the segment is coarser), and R_p's entry count ----
        if (wave == 0) {
            uint32_t c = 0, src = 0;
            const int r = lane;
            if (r == 0) {
                uint32_t rn = ((g_u32 *)a.in.cnt)[p];
#if GWO_SLOG_CHECK
                {   // R_p's region and slot column inside their allocations (else: recorded, R_p read as empty)
                    uint64_t width = 0;
                    const uint32_t n = rn & ~SLOG_UNSTRUCT;
                    bool ok = SLOG_CHK(n <= a.in.rcap, SLC_IN_REC, n, a.in.rcap);
                    if (ok && n) ok = SLOG_CHK((uint64_t)(p + 1) * a.in.rcap * RW <= a.chk.in_rec, SLC_IN_REC,
                                               (uint64_t)(p + 1) * a.in.rcap * RW, a.chk.in_rec);
                    if (ok && n && !(rn & SLOG_UNSTRUCT))
                        ok = SLOG_CHK((uint64_t)(p + 1) * a.in.rcap <= a.chk.in_slot, SLC_IN_SLOT,
                                      (uint64_t)(p + 1) * a.in.rcap, a.chk.in_slot);
                    if (!ok) rn = 0;
                }
#endif
                s_rn = rn;
                c = (rn & SLOG_UNSTRUCT) ? (rn & ~SLOG_UNSTRUCT) : 0u;
                s_ptr[0] = a.in.rec + (uint64_t)p * a.in.rcap * RW;
                s_meta[0] = 1 | (NW << 8) | (1 << 12) | (1 << 15);   // SoA columns of rcap words
            } else if (r <= a.nseg) {
                // the descriptor from the kernarg segment (a run-time index into the by-value argument would copy
                // it into scratch memory)
                typedef __attribute__((address_space(4))) const SlogArgs KSlogArgs;
                KSlogArgs *ka = (KSlogArgs *)__builtin_amdgcn_kernarg_segment_ptr();
                asm volatile("" : "+s"(ka));
                SlogSeg sg;
                sg.rec = ka->seg[r - 1].rec;
                sg.off = ka->seg[r - 1].off;
                sg.cnt = ka->seg[r - 1].cnt;
                sg.lp = ka->seg[r - 1].lp;
                sg.sign = ka->seg[r - 1].sign;
                sg.fmt = ka->seg[r - 1].fmt;
                sg.nrec = ka->seg[r - 1].nrec;
                const int d = lp_in - sg.lp;   // >= 0 (the host never gives a finer segment)
                const uint32_t q = p >> d;
                c = ((g_u32 *)sg.cnt)[q];
                src = ((g_u32 *)sg.off)[q];
                // a partition's run never reaches past the segment's carve: only a step queued behind a pass 2 whose
                // partition overflowed sees a larger count (its uncapped cursor) -- that step is redone (slog_step)
                if (sg.nrec) {
                    const uint32_t room = src < sg.nrec ? sg.nrec - src : 0u;
#if GWO_SLOG_CHECK
                    uint64_t width = 0;
                    if (c > room) (void)SLOG_CHK(false, SLC_SEG_CNT, (uint64_t)src + c, sg.nrec);
#endif
                    c = c < room ? c : room;
                }
                s_ptr[r] = sg.rec;
                const int stride = sg.fmt ? RW : (a.has_val ? 2 : 1);
                const int nl = sg.fmt ? NW : (a.has_val ? 1 : 0);
                s_meta[r] = stride | (nl << 8) | (sg.fmt << 12) | ((d > 0) << 13) | ((sg.sign < 0) << 14);
            }
            uint32_t incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (r <= a.nseg) {
                s_beg[r] = incl - c;
                s_src[r] = src;
            }
            if (r == a.nseg) s_beg[r + 1] = incl;
            if (r == 0) {
                s_qn[0] = 0;
                s_qn[1] = 0;
            }
        }
        __syncthreads();
        stamp(1);
        const bool structured = !(s_rn & SLOG_UNSTRUCT);
        const int nr = a.nseg + 1;
        const uint32_t total = s_beg[nr];
        uint64_t lo = 0, width = 1ull << 32;
        bool slow = false;
        while (lo < (1ull << 32)) {
            const uint64_t hi = lo + width < (1ull << 32) ? lo + width : (1ull << 32);
            const bool ranged = width < (1ull << 32);
            auto in_range = [&](int64_t k) {
                const uint64_t sub = (uint32_t)part_hash(k);
                return !ranged || (sub >= lo && sub < hi);
            };
            unsigned claims = 0;
#if GWO_SLOG_SLOTS
            // ---- R_p placed (structured): every entry at the table slot it had (R''s slot column), thread t loads
            // entries t, t + 256, ... (coalesced SoA columns); the overflow flags are rebuilt from the entries' own
            // displacement (every bucket from a key's home to its slot's bucket was full when it was claimed) --
            // one round trip, no bucket bytes, scan or map ----
            {
                const uint32_t rcount = structured ? (s_rn & ~SLOG_UNSTRUCT) : 0u;
                const int64_t *col = a.in.rec + (uint64_t)p * a.in.rcap * RW;   // keys[rcap], then each word's column
                const uint16_t *scol = a.in.slot + (uint64_t)p * a.in.rcap;
                unsigned placed = 0;
                for (uint32_t base = 0; base < rcount; base += TH * 4) {
                    int64_t ek[4], ew[4][NW];
                    uint32_t es[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t i = base + j * TH + tid;
                        ek[j] = 0;
                        es[j] = 0xffffu;
#pragma unroll
                        for (int w = 0; w < NW; ++w) ew[j][w] = 0;
                        if (i >= rcount) continue;
                        ek[j] = __builtin_nontemporal_load((g_i64 *)col + i);
                        es[j] = scol[i];
#pragma unroll
                        for (int w = 0; w < NW; ++w)
                            ew[j][w] = __builtin_nontemporal_load((g_i64 *)col + (uint64_t)(1 + w) * a.in.rcap + i);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t i = base + j * TH + tid;
                        if (i >= rcount || !in_range(ek[j])) continue;
                        if (ek[j] == GWO_EMPTY_KEY) {   // Long.MIN_VALUE: the side slot
                            s_side[0] = 1;
#pragma unroll
                            for (int w = 0; w < NW; ++w) s_side[1 + w] = ew[j][w];
                            continue;
                        }
                        if (!SLOG_CHK(es[j] < (uint32_t)T, SLC_SLOT_RANGE, es[j], T)) continue;
                        const int sl = (int)(es[j] & (uint32_t)(T - 1));
                        const int slot = slot_lds(sl);
#if GWO_SLOG_CHECK
                        {   // two entries of R_p at one slot: the slot column is inconsistent
                            const unsigned long long prev = atomicCAS((unsigned long long *)&s_key[slot],
                                                                      (unsigned long long)GWO_EMPTY_KEY, (unsigned long long)ek[j]);
                            if (!SLOG_CHK((int64_t)prev == GWO_EMPTY_KEY, SLC_SLOT_RANGE, ((uint64_t)sl << 32) | i, 0xdead))
                                continue;
                        }
#endif
                        s_key[slot] = ek[j];
#pragma unroll
                        for (int w = 0; w < NW; ++w) s_w[w * T + slot] = ew[j][w];
                        const int bs = sl >> 3;
                        for (int bb = (int)slog_bucket(ek[j], nbits); bb != bs; bb = (bb + 1) & (NB - 1)) s_ovf[bb] = 1;
                        placed++;
                    }
                }
                claims += placed;
            }
#else
            // ---- R_p placed into its buckets (structured): the bucket bytes give each entry's bucket (an LDS map
            // entry -> bucket), then thread t loads entries t, t + 256, ... -- coalesced SoA columns ----
            {
                uint32_t c = 0;
                const uint32_t rcount = structured ? (s_rn & ~SLOG_UNSTRUCT) : 0u;
                if (tid < NB) {
                    const uint32_t byte = rcount ? ((g_u8 *)a.in.bkt)[(size_t)p * NB + tid] : 0u;
                    c = byte & 15u;
                    s_ovf[tid] = (uint8_t)((byte >> 4) & 1u);
                }
                uint32_t incl = c;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o);
                    if (lane >= o) incl += y;
                }
                if (lane == 63) s_wsum[wave] = incl;
                __syncthreads();
                uint32_t pre = incl - c;
                for (int w = 0; w < wave; ++w) pre += s_wsum[w];
                if (tid < NB) {
                    s_pre[tid] = (uint16_t)pre;
                    for (uint32_t j = 0; j < c; ++j) s_map[pre + j] = (uint8_t)tid;
                }
                __syncthreads();
                const int64_t *col = a.in.rec + (uint64_t)p * a.in.rcap * RW;   // keys[rcap], then each word's column
                unsigned placed = 0;
                for (uint32_t base = 0; base < rcount; base += TH * 4) {
                    int64_t ek[4], ew[4][NW];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t i = base + j * TH + tid;
                        ek[j] = 0;
#pragma unroll
                        for (int w = 0; w < NW; ++w) ew[j][w] = 0;
                        if (i >= rcount) continue;
                        ek[j] = __builtin_nontemporal_load((g_i64 *)col + i);
#pragma unroll
                        for (int w = 0; w < NW; ++w)
                            ew[j][w] = __builtin_nontemporal_load((g_i64 *)col + (uint64_t)(1 + w) * a.in.rcap + i);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t i = base + j * TH + tid;
                        if (i >= rcount || !in_range(ek[j])) continue;
                        if (ek[j] == GWO_EMPTY_KEY) {   // Long.MIN_VALUE: the side slot
                            s_side[0] = 1;
#pragma unroll
                            for (int w = 0; w < NW; ++w) s_side[1 + w] = ew[j][w];
                            continue;
                        }
                        const uint32_t b = s_map[i];
                        const int slot = slot_lds((int)(b * 8 + (i - s_pre[b])));
                        s_key[slot] = ek[j];
#pragma unroll
                        for (int w = 0; w < NW; ++w) s_w[w * T + slot] = ew[j][w];
                        placed++;
                    }
                }
                claims += placed;
            }
#endif
            __syncthreads();
            stamp(2);
            // ---- fold: the segments' records (and R_p when unstructured), SLOG_J per thread, loads in flight ----
            for (uint32_t base = 0; base < total; base += TH * SLOG_J) {
                int64_t rk[SLOG_J], rw[SLOG_J][NW];
                int rr[SLOG_J];
                // every record's range and address first (LDS only), then every load: global (not flat) loads,
                // so the LDS waits in between do not wait for them
                const int64_t *ea[SLOG_J];
                int nlj[SLOG_J];
#pragma unroll
                for (int j = 0; j < SLOG_J; ++j) {
                    const uint32_t i = base + j * TH + tid;
                    rr[j] = -1;
                    ea[j] = s_ptr[0];
                    nlj[j] = 0;
                    if (i >= total) continue;
                    int r = 0;
                    for (int q = 1; q < nr; ++q) r += i >= s_beg[q];
                    const int m = s_meta[r];
                    ea[j] = s_ptr[r] + (uint64_t)(s_src[r] + (i - s_beg[r])) * (uint32_t)(m & 0xff);
                    nlj[j] = ((m >> 8) & 0xf) | (((m >> 15) & 1) << 4);
                    rr[j] = r;
                }
#pragma unroll
                for (int j = 0; j < SLOG_J; ++j) {
                    rk[j] = 0;
#pragma unroll
                    for (int w = 0; w < NW; ++w) rw[j][w] = 0;
                    if (rr[j] < 0) continue;
                    rk[j] = __builtin_nontemporal_load((g_i64 *)ea[j]);
                    const uint64_t wstride = (nlj[j] >> 4) ? a.in.rcap : 1u;   // R's SoA columns, or record words
#pragma unroll
                    for (int w = 0; w < NW; ++w)
                        if (w < (nlj[j] & 0xf))
                            rw[j][w] = __builtin_nontemporal_load((g_i64 *)ea[j] + (uint64_t)(1 + w) * wstride);
                }
#pragma unroll
                for (int j = 0; j < SLOG_J; ++j) {
                    if (rr[j] < 0) continue;
                    const int m = s_meta[rr[j]];
                    const int64_t k = rk[j];
                    if (((m >> 13) & 1) && (digit_hash(k) >> (32 - lp_in)) != p) continue;
                    if (!in_range(k)) continue;
                    const int slot = slog_find(s_key, s_ovf, NB, nbits, k, claims);
                    if (slot == -2) {
                        s_fail = 1;
                        continue;
                    }
                    int64_t *dst = slot >= 0 ? s_w + slot_lds(slot) : s_side + 1;
                    const int ds = slot >= 0 ? T : 1;
                    if (slot < 0) s_side[0] = 1;
                    const bool raw = (m >> 12) & 1, neg = (m >> 14) & 1;
#pragma unroll
                    for (int w = 0; w < NW; ++w) {
                        int64_t x = raw ? rw[j][w] : lift_word(a.p, w, rw[j][0]);
                        x = neg ? (int64_t)(0ull - (uint64_t)x) : x;
                        atomicAdd((unsigned long long *)(dst + w * ds), (unsigned long long)x);
                    }
                }
            }
            const unsigned long long cw = wave_sum_u64(claims);
            if (lane == 0 && cw) atomicAdd(&s_used, (unsigned)cw);
            __syncthreads();
            const bool failed = s_fail != 0 || s_used > limit;
            __syncthreads();
            stamp(3);
            if (failed) {   // more keys in range than the table holds: reset, halve the range
                for (int i = tid; i < T; i += TH) s_key[i] = GWO_EMPTY_KEY;
                for (int i = tid; i < T * NW; i += TH) s_w[i] = 0;
                if (tid <= GWO_MAX_WORDS) s_side[tid] = 0;
                if (GWO_SLOG_SLOTS && tid < NB) s_ovf[tid] = 0;
                if (tid == 0) {
                    s_used = 0;
                    s_fail = 0;
                }
                __syncthreads();
                slow = true;
                width >>= 1;
                if (width == 0) {
                    st_lds++;
                    break;
                }
                continue;
            }
            // ---- sweep: thread t takes slots [t * SPT, (t + 1) * SPT) (one bucket part), so R' comes out bucket by
            // bucket; live keys -> rows of window J and R'; every slot reset for the next fold ----
            const bool out_struct = !slow;   // range rounds write R' unstructured
            const int b_t = (tid * SPT) >> 3;   // this thread's bucket
            uint32_t cnt0 = 0, cnt1 = 0, code = 0;   // code bit 2i: slot i live, bit 2i+1: its output half
            for (int i = 0; i < SPT; ++i) {
                const int s = slot_lds(tid * SPT + i);
                const int64_t k = s_key[s];
                if (k == GWO_EMPTY_KEY) continue;
                const int64_t c = s_w[a.count_word * T + s];
                if (c < 0) st_neg++;
                if (c <= 0) {   // the key left the window: its slot is simply reset
                    s_key[s] = GWO_EMPTY_KEY;
#pragma unroll
                    for (int w = 0; w < NW; ++w) s_w[w * T + s] = 0;
                    continue;
                }
                const uint32_t half = split ? (digit_hash(k) >> (31 - lp_in)) & 1u : 0u;
                code |= (1u | (half << 1)) << (2 * i);
                if (half) cnt1++;
                else cnt0++;
                // a key displaced from its home bucket: every bucket it passed is flagged in its output table
                const int home = (int)slog_bucket(k, nbits);
                for (int bb = home; bb != b_t; bb = (bb + 1) & (NB - 1)) s_ovo[half][bb] = 1;
            }
            // the side entry (Long.MIN_VALUE) goes out with its bucket, before that bucket's slots
            bool side_live = false;
            uint32_t side_half = 0;
            if (tid == (side_bucket * 8) / SPT && s_side[0]) {
                const int64_t c = s_side[1 + a.count_word];
                if (c < 0) st_neg++;
                if (c > 0) {
                    side_live = true;
                    side_half = split ? (digit_hash(GWO_EMPTY_KEY) >> (31 - lp_in)) & 1u : 0u;
                    if (side_half) cnt1++;
                    else cnt0++;
                }
            }
            // workgroup scan of (cnt0, cnt1) packed in one word (each < 2^16)
            const uint32_t v = cnt0 | (cnt1 << 16);
            uint32_t incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (lane == 63) s_wsum[wave] = incl;
            __syncthreads();   // (also: every s_ovo flag is set)
            stamp(6);
            uint32_t pre = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < TH / 64; ++w) {
                const uint32_t x = s_wsum[w];
                pre += w < wave ? x : 0u;
                tot += x;
            }
            const uint32_t ex = pre + incl - v;   // this thread's first positions (low: half 0, high: half 1)
            const uint32_t tot0 = tot & 0xffffu, tot1 = tot >> 16;
            if (tid == 0)
                s_rowbase = (a.mode & 4) ? (unsigned long long)p * 700ull   // (diagnostic: no reservation)
                            : (a.emit && tot0 + tot1) ? atomicAdd(a.o.count, (unsigned long long)(tot0 + tot1)) : 0ull;
            const uint32_t qb0 = s_qn[0], qb1 = s_qn[1];
            const uint32_t qout0 = split ? 2 * p : p;
            // R''s bucket bytes: the first thread of each bucket sums the bucket's threads (consecutive lanes)
            if (out_struct && !GWO_SLOG_SLOTS) {
                uint32_t bc = v;
                for (int o = 1; o < 8 / SPT; o <<= 1) bc += __shfl_xor(bc, o);
                if (((tid * SPT) & 7) == 0) {
                    uint8_t *ob = a.out.bkt + (size_t)qout0 * NB + b_t;
                    ob[0] = (uint8_t)((bc & 0xffffu) | ((uint32_t)s_ovo[0][b_t] << 4));
                    if (split) ob[NB] = (uint8_t)((bc >> 16) | ((uint32_t)s_ovo[1][b_t] << 4));
                }
            }
            // pass A: R' (needs no row base), while thread 0's row reservation is in flight
            {
                uint32_t at0 = ex & 0xffffu, at1 = ex >> 16;
                auto put = [&](int64_t k, const int64_t *wp, int ws, uint32_t half, uint32_t lslot) {
                    const uint32_t qpos = (half ? qb1 + at1++ : qb0 + at0++);
                    if (qpos >= a.out.rcap || (a.mode & 8)) return;
#if GWO_SLOG_CHECK
                    if (!SLOG_CHK((qout0 + half) < (1u << a.out.lp), SLC_PART, qout0 + half, 1u << a.out.lp)) return;
                    if (!SLOG_CHK((uint64_t)(qout0 + half + 1) * a.out.rcap * RW <= a.chk.out_rec, SLC_OUT_REC,
                                  (uint64_t)(qout0 + half + 1) * a.out.rcap * RW, a.chk.out_rec)) return;
                    if (!SLOG_CHK((uint64_t)(qout0 + half + 1) * a.out.rcap <= a.chk.out_slot, SLC_OUT_SLOT,
                                  (uint64_t)(qout0 + half + 1) * a.out.rcap, a.chk.out_slot)) return;
#endif
                    int64_t *col = a.out.rec + (uint64_t)(qout0 + half) * a.out.rcap * RW;   // SoA columns
                    col[qpos] = k;
                    if (GWO_SLOG_SLOTS) a.out.slot[(uint64_t)(qout0 + half) * a.out.rcap + qpos] = (uint16_t)lslot;
#pragma unroll
                    for (int w = 0; w < NW; ++w) col[(uint64_t)(1 + w) * a.out.rcap + qpos] = wp[w * ws];
                };
                if (side_live) put(GWO_EMPTY_KEY, s_side + 1, 1, side_half, 0xffffu);
                for (int i = 0; i < SPT; ++i) {
                    if (!((code >> (2 * i)) & 1u)) continue;
                    const int sl = slot_lds(tid * SPT + i);
                    put(s_key[sl], s_w + sl, T, (code >> (2 * i + 1)) & 1u, (uint32_t)(tid * SPT + i));
                }
            }
            __syncthreads();   // s_rowbase is published; every read of s_qn and s_ovo is done
            stamp(7);
            // pass B: rows (the partition's run: half-0 keys first), slots reset for the next fold
            {
                const unsigned long long rowbase = s_rowbase;
                uint32_t at0 = ex & 0xffffu, at1 = ex >> 16;
                auto row = [&](int64_t k, const int64_t *wp, int ws, uint32_t half) {
                    const uint32_t ord = half ? tot0 + at1++ : at0++;
                    const unsigned long long r = rowbase + ord;
                    if (!a.emit || (long long)r >= a.o.cap || (a.mode & 16)) return;
                    int64_t acc[NW];
#pragma unroll
                    for (int w = 0; w < NW; ++w) acc[w] = wp[w * ws];
                    a.o.key[r] = k;
                    a.o.start[r] = a.start;
                    a.o.end[r] = a.end;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        if (g >= a.rp.naggs) break;
                        const int wi = a.rp.word[g];
                        int64_t x = acc[0], y = acc[0];
#pragma unroll
                        for (int w = 1; w < NW; ++w) {
                            if (w == wi) x = acc[w];
                            if (w == wi + 1) y = acc[w];
                        }
                        a.o.res[g][r] = a.rp.kind[g] == GWO_AGG_AVG ? __double_as_longlong((double)x / (double)y) : x;
                    }
                };
                if (side_live) row(GWO_EMPTY_KEY, s_side + 1, 1, side_half);
                for (int i = 0; i < SPT; ++i) {
                    if (!((code >> (2 * i)) & 1u)) continue;
                    const int sl = slot_lds(tid * SPT + i);
                    row(s_key[sl], s_w + sl, T, (code >> (2 * i + 1)) & 1u);
                    s_key[sl] = GWO_EMPTY_KEY;
#pragma unroll
                    for (int w = 0; w < NW; ++w) s_w[w * T + sl] = 0;
                }
            }
            __syncthreads();   // every read of s_side is done
            if (tid == 0) {
                s_qn[0] = qb0 + tot0;
                s_qn[1] = qb1 + tot1;
                s_used = 0;
            }
            if (tid <= GWO_MAX_WORDS) s_side[tid] = 0;
            if (tid < NB) {
                s_ovo[0][tid] = 0;
                s_ovo[1][tid] = 0;
                if (GWO_SLOG_SLOTS) s_ovf[tid] = 0;
            }
            stamp(4);
            __syncthreads();
            lo = hi;
        }
        if (slow) st_slow++;
        if (tid == 0) {
            const uint32_t n0 = s_qn[0], n1 = s_qn[1];
            const uint32_t q0 = split ? 2 * p : p;
            const uint32_t flag = slow ? SLOG_UNSTRUCT : 0u;
            a.out.cnt[q0] = (n0 < a.out.rcap ? n0 : (uint32_t)a.out.rcap) | flag;
            if (split) a.out.cnt[q0 + 1] = (n1 < a.out.rcap ? n1 : (uint32_t)a.out.rcap) | flag;
            if (n0 > a.out.rcap || n1 > a.out.rcap) st_rovf++;
            st_live += n0 + n1;
            const unsigned long long mq = n0 > n1 ? n0 : n1;
            st_maxp = mq > st_maxp ? mq : st_maxp;
        }
        __syncthreads();   // s_beg / s_qn / s_rn are rewritten for the next partition
        stamp(5);
    }
    if (a.dbg && tid == 0 && blockIdx.x < SLOG_DBG_BLOCKS) a.dbg[SLOG_DBG_PHASES + 2 * blockIdx.x + 1] = wall_clock64();
    // statistics -> shard blockIdx % SLOG_SHARDS
    const unsigned long long nl = wave_sum_u64(st_neg);
    if (lane == 0 && nl) atomicAdd(&a.stat[(blockIdx.x % SLOG_SHARDS) * SLOG_STAT_STRIDE + SLS_NEG], nl);
    if (tid == 0) {
        unsigned long long *sh = a.stat + (blockIdx.x % SLOG_SHARDS) * SLOG_STAT_STRIDE;
        if (st_live) atomicAdd(sh + SLS_LIVE, st_live);
        if (st_maxp) atomicMax(sh + SLS_MAXP, st_maxp);
        if (st_rovf) atomicAdd(sh + SLS_ROVF, st_rovf);
        if (st_lds) atomicAdd(sh + SLS_LDS, st_lds);
        if (st_slow) atomicAdd(sh + SLS_SLOW, st_slow);
    }
}

// The window step's statistics: the shards folded (sums; SLS_MAXP a max) into a host-mapped block, sequence word
// last, and reset for the next step -- one wave behind the step instead of a memset, a copy and a stream
// synchronisation (the host spins on the block).
__global__ __launch_bounds__(64) void slog_stat_publish_kernel(unsigned long long *stat, unsigned long long *rb,
                                                               unsigned long long seq) {
    const int t = threadIdx.x;
    if (t < SLS_WORDS) {
        unsigned long long x[SLOG_SHARDS];
#pragma unroll
        for (int q = 0; q < SLOG_SHARDS; ++q) x[q] = atomicExch(&stat[q * SLOG_STAT_STRIDE + t], 0ull);
        unsigned long long acc = 0;
#pragma unroll
        for (int q = 0; q < SLOG_SHARDS; ++q) acc = t == SLS_MAXP ? (x[q] > acc ? x[q] : acc) : acc + x[q];
        rb_put(&rb[t], acc);
    }
    rb_publish(&rb[SLS_WORDS], seq);
}

void launch_slog_stat_publish(unsigned long long *stat, unsigned long long *rb, unsigned long long seq, hipStream_t s) {
    hipLaunchKernelGGL(slog_stat_publish_kernel, dim3(1), dim3(64), 0, s, stat, rb, seq);
}

// Persistent grid: every workgroup resident at once (the occupancy of the instance at this LDS size, per CU, times
// the CUs given as `groups`), so no workgroup waits for another to finish before it starts its partitions.
void launch_slog_fire(const SlogArgs &a, int cus, hipStream_t s) {
    const size_t lds = slog_lds_bytes(a.cap_log2, a.p.nwords);
    const uint32_t P = 1u << a.in.lp;
#define GWO_SLOG(NW)                                                                                    \
    case NW: {                                                                                          \
        static int occ[16] = {};                                                                        \
        int &per_cu = occ[a.cap_log2 & 15];                                                             \
        if (!per_cu && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, slog_fire_kernel<NW>, slog_threads_for(NW), \
                                                                    lds) != hipSuccess)                \
            per_cu = 1;                                                                                 \
        if (per_cu < 1) per_cu = 1;                                                                     \
        const uint32_t groups = (uint32_t)cus * (uint32_t)per_cu;                                       \
        const int grid = (int)(P < groups ? P : groups);                                                \
        hipLaunchKernelGGL(slog_fire_kernel<NW>, dim3(grid), dim3(slog_threads_for(NW)), lds, s, a);     \
        break;                                                                                          \
    }
    switch (a.p.nwords) {
        GWO_SLOG(1)
        GWO_SLOG(2)
        GWO_SLOG(3)
        GWO_SLOG(4)
        GWO_SLOG(5)
        GWO_SLOG(6)
        GWO_SLOG(7)
        GWO_SLOG(8)
        default: break;
    }
#undef GWO_SLOG
}

}  // namespace gwo
