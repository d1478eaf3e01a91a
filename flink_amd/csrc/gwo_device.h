// gwo_device.h -- gfx950 device helpers: Java integer semantics, Flink's hash functions,
// window arithmetic and the HBM hash-table primitives.  Included only by .hip translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gwo_internal.h"
#include "gwo_hash.h"

namespace gwo {

#define GWO_LONG_MIN ((int64_t)0x8000000000000000LL)
#define GWO_LONG_MAX ((int64_t)0x7fffffffffffffffLL)

// Java long arithmetic wraps; do it in unsigned to keep the compiler from assuming no overflow.
__device__ __host__ __forceinline__ int64_t jadd(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a + (uint64_t)b);
}
__device__ __host__ __forceinline__ int64_t jsub(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a - (uint64_t)b);
}
// Java '%' on longs (truncating; C++ '%' has the same semantics).  b > 0.
__device__ __host__ __forceinline__ int64_t jrem(int64_t a, int64_t b) { return a % b; }

// TimeWindow.getWindowStartWithOffset, TimeWindow.java:270-272 (Java '%' quirk included).
__device__ __host__ __forceinline__ int64_t window_start(int64_t ts, int64_t off, int64_t size) {
    return jsub(ts, jrem(jadd(jsub(ts, off), size), size));
}

__device__ __host__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

// floor(a / d) for d > 0, exact for every int64 a, without the ~150-instruction 64-bit integer
// division: a double-precision reciprocal estimate, one refinement on the (small) remainder, and
// exact integer corrections.  Products wrap, which is harmless because the true remainder fits.
__device__ __forceinline__ int64_t fdiv_floor(int64_t a, int64_t d, double inv) {
    double x = (double)a * inv;
    x = x > 9.2e18 ? 9.2e18 : (x < -9.2e18 ? -9.2e18 : x);
    int64_t q = (int64_t)x;
    int64_t r = jsub(a, (int64_t)((uint64_t)q * (uint64_t)d));
    q += (int64_t)((double)r * inv);
    r = jsub(a, (int64_t)((uint64_t)q * (uint64_t)d));
    while (r < 0) {
        q -= 1;
        r = jadd(r, d);
    }
    while (r >= d) {
        q += 1;
        r = jsub(r, d);
    }
    return q;
}
// Java '%' (truncating) for d > 0 via fdiv_floor.
__device__ __forceinline__ int64_t jrem_f(int64_t a, int64_t d, double inv) {
    int64_t fm = jsub(a, (int64_t)((uint64_t)fdiv_floor(a, d, inv) * (uint64_t)d));   // floorMod in [0, d)
    return (a < 0 && fm != 0) ? fm - d : fm;
}
// TimeWindow.getWindowStartWithOffset with the fast remainder (TimeWindow.java:270-272).
__device__ __forceinline__ int64_t window_start_f(int64_t ts, int64_t off, int64_t size, double inv) {
    return jsub(ts, jrem_f(jadd(jsub(ts, off), size), size, inv));
}

// floor(a / d) for 0 <= a < 2^52 and d > 0: the double estimate is within 1 of the quotient, so one
// exact correction step suffices (about 10 instructions instead of fdiv_floor's 40).
__device__ __forceinline__ int64_t fdiv_small(int64_t a, int64_t d, double inv) {
    const double two52 = 4503599627370496.0;
    const double af = __longlong_as_double(a | 0x4330000000000000LL) - two52;   // exact: a < 2^52
    const double qf = trunc(af * inv);
    int64_t q = __double_as_longlong(qf + two52) & 0x000FFFFFFFFFFFFFLL;        // exact: 0 <= qf < 2^52
    const int64_t r = a - q * d;
    q += (int64_t)(r >= d) - (int64_t)(r < 0);
    return q;
}

// WindowOperator.cleanupTime (WindowOperator.java:639-646): maxTs + lateness, Long.MAX_VALUE on overflow.
__device__ __host__ __forceinline__ int64_t cleanup_time(int64_t max_ts, int64_t lateness) {
    int64_t c = jadd(max_ts, lateness);
    return c >= max_ts ? c : GWO_LONG_MAX;
}

// ---- table hashing -------------------------------------------------------------------------------
// Slot hash (independent of the key-group hash so that a shard's table is not biased).
__device__ __forceinline__ uint64_t slot_hash(int64_t key) {
    uint64_t k = (uint64_t)key ^ 0x9E3779B97F4A7C15ull;
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// Partition hash of the log-structured state (gwo_log.hip): a bijective 64-bit mix, different from
// slot_hash.  Top 8 bits = coarse digit, top lp bits = partition, low bits = LDS slot.
__device__ __forceinline__ uint64_t part_hash(int64_t key) {
    uint64_t z = (uint64_t)key + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Double.compareTo total order as a signed int64 key (doubleToLongBits canonicalises NaN).
__device__ __host__ __forceinline__ int64_t f64_order_key(int64_t bits) {
    if ((bits & 0x7ff0000000000000LL) == 0x7ff0000000000000LL && (bits & 0x000fffffffffffffLL) != 0)
        bits = 0x7ff8000000000000LL;
    return bits >= 0 ? bits : (bits ^ 0x7fffffffffffffffLL);
}
__device__ __host__ __forceinline__ int64_t f64_from_order_key(int64_t k) {
    return k >= 0 ? k : (k ^ 0x7fffffffffffffffLL);
}

__device__ __forceinline__ int64_t lift_word(const AccPlan &p, int w, int64_t vbits) {
    switch (p.src[w]) {
        case SRC_ONE: return 1;
        case SRC_ORDER: return f64_order_key(vbits);
        default: return vbits;
    }
}

// Atomic combine into a global (HBM) word -- device scope.
__device__ __forceinline__ void atomic_combine(int64_t *dst, int op, int64_t x) {
    switch (op) {
        case ACC_ADD_I64: atomicAdd((unsigned long long *)dst, (unsigned long long)x); break;
        case ACC_ADD_F64: atomicAdd((double *)dst, __longlong_as_double(x)); break;
        case ACC_MIN_I64: atomicMin((long long *)dst, (long long)x); break;
        default: atomicMax((long long *)dst, (long long)x); break;
    }
}

// Plain (non-atomic) combine.
__device__ __forceinline__ int64_t combine(int op, int64_t a, int64_t b) {
    switch (op) {
        case ACC_ADD_I64: return jadd(a, b);
        case ACC_ADD_F64: return __double_as_longlong(__longlong_as_double(a) + __longlong_as_double(b));
        case ACC_MIN_I64: return a < b ? a : b;
        default: return a > b ? a : b;
    }
}

// Find the entry of `key` in table t, claiming a free slot if absent.  Returns the entry's
// accumulator words; `claimed` is set when this call took a new slot.  Linear probing; the table
// never fills (host keeps load <= 0.7).  Occupancy is NOT counted here: callers pass `claimed`
// to count_claims() at a point where the whole wave has re-converged.
__device__ __forceinline__ int64_t *find_or_insert(const TableDesc &t, int stride, int64_t key, bool &claimed) {
    claimed = false;
    if (key == GWO_EMPTY_KEY) {
        if (__hip_atomic_load(t.side, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            if (atomicCAS((unsigned long long *)t.side, 0ull, 1ull) == 0ull) claimed = true;
        }
        return t.side + 1;
    }
    uint64_t slot = slot_hash(key) & t.mask;
    while (true) {
        int64_t *e = t.base + slot * (uint64_t)stride;
        // Within a kernel a slot's key only goes EMPTY -> key, so a possibly stale read is safe: a stale EMPTY
        // is settled by the CAS (which returns the current key), any other key is final.  Workgroup scope keeps
        // the probe in the caches instead of bypassing them to the coherence point.
        int64_t cur = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == key) return e + 1;
        if (cur == GWO_EMPTY_KEY) {
            unsigned long long prev =
                atomicCAS((unsigned long long *)e, (unsigned long long)GWO_EMPTY_KEY, (unsigned long long)key);
            if ((int64_t)prev == GWO_EMPTY_KEY) {
                claimed = true;
                return e + 1;
            }
            if ((int64_t)prev == key) return e + 1;
        }
        slot = (slot + 1) & t.mask;
    }
}

// Occupancy counters are GWO_OCC_SHARDS words on separate 64-B lines (host sums them); a workgroup
// adds to shard blockIdx % GWO_OCC_SHARDS, so one hot word never serialises a whole launch.
__device__ __forceinline__ void occ_add(unsigned long long *occ, unsigned long long n) {
    atomicAdd(occ + (blockIdx.x & (GWO_OCC_SHARDS - 1)) * GWO_OCC_SHARD_STRIDE, n);
}

// Adds the claims of the active lanes to their tables' occupancy: one atomic per (wave, table).
__device__ __forceinline__ void count_claims(unsigned long long *occ, bool claimed) {
    unsigned long long m = __ballot(claimed);
    const int lane = threadIdx.x & 63;
    while (m) {
        int leader = __ffsll((long long)m) - 1;
        unsigned long long *p = (unsigned long long *)__shfl((long long)occ, leader);
        bool mine = claimed && occ == p;
        unsigned long long peers = __ballot(mine);
        if (lane == leader) occ_add(p, (unsigned long long)__popcll(peers));
        if (mine) claimed = false;
        m &= ~peers;
    }
}

// Workgroup-wide exclusive prefix of v (blockDim.x a multiple of 64, <= 1024) plus ONE atomicAdd of
// the workgroup total on *ctr: returns this thread's first output position.  Used by every kernel
// that stream-compacts rows into a shared output, so a launch issues one atomic per workgroup
// chunk, not one per lane or per wave.  Must be called by all threads of the workgroup.
__device__ __forceinline__ unsigned long long block_reserve(unsigned v, unsigned long long *ctr) {
    __shared__ unsigned s_wave[16];
    __shared__ unsigned long long s_base;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    unsigned incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        unsigned y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_wave[wid] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned run = 0;
        for (int w = 0; w < nw; ++w) {
            unsigned t = s_wave[w];
            s_wave[w] = run;
            run += t;
        }
        s_base = run ? atomicAdd(ctr, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    unsigned long long r = s_base + s_wave[wid] + (incl - v);
    __syncthreads();   // s_wave / s_base are reused by the next call
    return r;
}

// Workgroup-wide exclusive prefix sum of v (all threads call it); *total gets the sum.
// Workgroup barrier for LDS hand-offs only: this wave's LDS operations complete, then s_barrier -- no memory fence.
// __syncthreads() lowers to a workgroup release + acquire fence, which on gfx950 waits vmcnt(0) whenever a global
// store or atomic may be pending: every load, store and atomic in flight (a prefetch, a row reservation, a tile's
// output) drained at each barrier.  Use only where the barrier orders LDS accesses, never global memory.
// Arrival of this workgroup at the end of its grid, from thread 0 once every statistic of the workgroup has completed
// (vmcnt): true for the last workgroup.  Arrivals are counted per shard (blockIdx % ARR_SHARDS, a 128-B line each) and
// the last of a shard counts the shard, so an address takes about gridDim / 16 + 16 adds instead of gridDim
// (device-scope atomics on one address serialise at ~12 ns each: ~3 us for the last of 256 workgroups).  ctr:
// ARR_WORDS words, zero at launch and left zero (each counter is reset by its last arriver).
// (ARR_SHARDS, ARR_WORDS: gwo_internal.h)
__device__ __forceinline__ bool grid_arrive_last(unsigned long long *ctr) {
    const unsigned q = blockIdx.x % ARR_SHARDS;
    const unsigned members = (gridDim.x - q + ARR_SHARDS - 1) / ARR_SHARDS;
    const unsigned nsh = gridDim.x < ARR_SHARDS ? gridDim.x : ARR_SHARDS;
    if (atomicAdd(&ctr[q * 16], 1ull) != members - 1) return false;
    atomicExch(&ctr[q * 16], 0ull);   // every member of the shard has arrived: free for the next launch
    if (atomicAdd(&ctr[ARR_SHARDS * 16], 1ull) != nsh - 1) return false;
    atomicExch(&ctr[ARR_SHARDS * 16], 0ull);
    return true;
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ unsigned block_exclusive_scan(unsigned v, unsigned *total) {
    __shared__ unsigned s_w[17];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    unsigned incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        unsigned y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned run = 0;
        for (int w = 0; w < nw; ++w) {
            unsigned t = s_w[w];
            s_w[w] = run;
            run += t;
        }
        s_w[16] = run;
    }
    __syncthreads();
    unsigned r = s_w[wid] + incl - v;
    *total = s_w[16];
    __syncthreads();
    return r;
}

// Wave-level sum for counters: one atomic per wave.
__device__ __forceinline__ void wave_atomic_add(unsigned long long *dst, unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, v);
}

// Host-mapped readback blocks (coherent host memory the host spins on).  Every word goes out as a system-scope
// store, written through the L2 (sc0 sc1), so that the waves' own store counters order the words before the
// sequence word: a system-scope release fence instead writes back the XCD's whole L2 (measured 4.6 us in the
// combine gather's tail, ~3 us at K1's end).
__device__ __forceinline__ void rb_put(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The workgroup's readback words are complete (each wave waits for its stores) before thread 0 writes the
// sequence word.  Called by every thread of the workgroup.
__device__ __forceinline__ void rb_publish(unsigned long long *seq_word, unsigned long long seq) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) rb_put(seq_word, seq);
}

// Read-and-reset of N statistics shards (word p[q * stride], q < N) folded with kind 0 sum, 1 signed min,
// 2 signed max.  Every exchange is issued before the first result is used: a device-scope atomic is a
// round trip of ~1 us, and a fold between them (branches on the kind) serialised N of them per call.
template <int N>
__device__ __forceinline__ unsigned long long xchg_fold(unsigned long long *p, size_t stride, unsigned long long init,
                                                        int kind) {
    unsigned long long x[N];
#pragma unroll
    for (int q = 0; q < N; ++q) x[q] = atomicExch(p + q * stride, init);
    long long r = (long long)init;
#pragma unroll
    for (int q = 0; q < N; ++q) {
        const long long v = (long long)x[q];
        const long long s = (long long)((unsigned long long)r + (unsigned long long)v);
        const long long lo = v < r ? v : r, hi = v > r ? v : r;
        r = kind == 0 ? s : (kind == 1 ? lo : hi);
    }
    return (unsigned long long)r;
}

}  // namespace gwo
