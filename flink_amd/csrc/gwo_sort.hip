// gwo_sort.hip -- stable LSD radix sort of (uint32 key, uint32 payload) pairs for gfx950.
//
// Used to group a batch's records by session-state slot while keeping arrival order inside each
// group (MergingWindowSet semantics depend on arrival order once late records exist).  Digits of DB
// bits (8, or 10 for keys of at most 20 bits: a session table of up to 2^19 slots sorts in two passes instead
// of three -- each pass is three launches of a latency-bound size); per pass: block histograms (digit-major) ->
// one-workgroup exclusive scan -> stable scatter.  Stability inside a block: each 256-record sub-tile is ranked
// with wave ballots (lanes with the same digit, lower lane id) plus per-wave digit counts in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gwo_device.h"

namespace gwo {

#define RS_TILE 4096
#define RS_THREADS 256

template <int DB>
__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const uint32_t *__restrict__ keys, int64_t n, int shift,
                                                             uint32_t *__restrict__ block_hist, int nblocks, int tile) {
    constexpr int BINS = 1 << DB;
    __shared__ uint32_t h[BINS];
    for (int b = threadIdx.x; b < BINS; b += RS_THREADS) h[b] = 0;
    __syncthreads();
    int64_t base = (int64_t)blockIdx.x * tile;
    for (int j = threadIdx.x; j < tile; j += RS_THREADS) {
        int64_t i = base + j;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & (BINS - 1)], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < BINS; b += RS_THREADS)
        block_hist[(int64_t)b * nblocks + blockIdx.x] = h[b];  // digit-major
}

// exclusive scan of m entries by one workgroup: each thread sums a contiguous segment, one workgroup scan of the
// segment sums, then each thread writes its segment's prefixes (one pass over the data, two barriers)
__global__ __launch_bounds__(1024) void rs_scan_kernel(uint32_t *__restrict__ data, int64_t m) {
    const int64_t per = (m + 1023) / 1024;
    const int64_t b = (int64_t)threadIdx.x * per, e = b + per < m ? b + per : m;
    uint32_t sum = 0;
    for (int64_t i = b; i < e; ++i) sum += data[i];
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, &total);
    for (int64_t i = b; i < e; ++i) {
        const uint32_t v = data[i];
        data[i] = run;
        run += v;
    }
}

// FUSED (few blocks): `offsets` holds the raw block histograms and every block derives its own starting
// positions from them (digit totals over all blocks, exclusive over digits, plus the earlier blocks' counts of
// the digit) -- no separate scan launch.  Otherwise `offsets` is the scanned histogram.
template <int DB, bool FUSED>
__global__ __launch_bounds__(RS_THREADS) void rs_scatter_kernel(const uint32_t *__restrict__ keys,
                                                                const uint32_t *__restrict__ vals, int64_t n,
                                                                int shift, const uint32_t *__restrict__ offsets,
                                                                int nblocks, uint32_t *__restrict__ okeys,
                                                                uint32_t *__restrict__ ovals, int tile) {
    constexpr int BINS = 1 << DB;
    __shared__ uint32_t run[BINS];              // running position per digit for this block
    __shared__ uint32_t wcnt[RS_THREADS / 64][BINS];
    if constexpr (FUSED) {   // thread t owns digits [t * DPT, (t + 1) * DPT)
        constexpr int DPT = BINS / RS_THREADS;
        static_assert(DPT * RS_THREADS == BINS, "whole digits per thread");
        uint32_t tot[DPT], pre[DPT], sum = 0;
#pragma unroll
        for (int c = 0; c < DPT; ++c) {
            const uint32_t *h = offsets + (int64_t)(threadIdx.x * DPT + c) * nblocks;
            tot[c] = 0;
            pre[c] = 0;
#pragma unroll 16
            for (int j = 0; j < nblocks; ++j) {   // unrolled: 16 loads in flight, not one round trip per block
                const uint32_t x = h[j];
                tot[c] += x;
                pre[c] += j < (int)blockIdx.x ? x : 0u;
            }
            sum += tot[c];
        }
        uint32_t all;
        uint32_t at = block_exclusive_scan(sum, &all);
#pragma unroll
        for (int c = 0; c < DPT; ++c) {
            run[threadIdx.x * DPT + c] = at + pre[c];
            at += tot[c];
        }
    } else {
        for (int b = threadIdx.x; b < BINS; b += RS_THREADS) run[b] = offsets[(int64_t)b * nblocks + blockIdx.x];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1;
    const int64_t base = (int64_t)blockIdx.x * tile;
    // the block's keys and payloads load before the first sub-tile is ranked (one round trip, not one per sub-tile)
    constexpr int SUBS = RS_TILE / RS_THREADS;
    uint32_t kq[SUBS], vq[SUBS];
#pragma unroll
    for (int q = 0; q < SUBS; ++q) {
        const int64_t i = base + q * RS_THREADS + threadIdx.x;
        const bool ok = q * RS_THREADS < tile && i < n;
        kq[q] = ok ? keys[i] : 0u;
        vq[q] = ok ? (vals ? vals[i] : (uint32_t)i) : 0u;
    }
#pragma unroll
    for (int q = 0; q < SUBS; ++q) {
        if (q * RS_THREADS >= tile) break;
        for (int b = threadIdx.x; b < BINS; b += RS_THREADS)
            for (int w = 0; w < RS_THREADS / 64; ++w) wcnt[w][b] = 0;
        __syncthreads();
        const int64_t i = base + q * RS_THREADS + threadIdx.x;
        bool valid = i < n;
        uint32_t k = kq[q];
        uint32_t d = (k >> shift) & (BINS - 1);
        // lanes of this wave holding the same digit
        uint64_t same = __ballot(valid);
        for (int b = 0; b < DB; ++b) {
            uint64_t bb = __ballot(((d >> b) & 1) != 0);
            same &= ((d >> b) & 1) ? bb : ~bb;
        }
        uint32_t rank = (uint32_t)__popcll(same & lt);
        if (valid && rank == 0) wcnt[wid][d] = (uint32_t)__popcll(same);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[d] + rank;
            for (int w = 0; w < wid; ++w) pos += wcnt[w][d];
            okeys[pos] = k;
            ovals[pos] = vq[q];
        }
        __syncthreads();
        // advance running positions by this sub-tile's digit totals
        for (int b = threadIdx.x; b < BINS; b += RS_THREADS) {
            uint32_t tot = 0;
            for (int w = 0; w < RS_THREADS / 64; ++w) tot += wcnt[w][b];
            run[b] += tot;
        }
        __syncthreads();
    }
}

// Sorts keys[0..n) stably by their low key_bits bits; payload = vals (or the original index when vals == nullptr).
// tmp buffers: k1/v1/k2/v2 of n entries each, hist of 256*ceil(n/4096) entries (1024*.. with digit_bits 10).
// The result lands in (k1, v1) or (k2, v2): returns 0 for (k1, v1), 1 for (k2, v2).
int radix_sort_pairs(const uint32_t *keys, const uint32_t *vals, int64_t n, int key_bits, uint32_t *k1,
                     uint32_t *v1, uint32_t *k2, uint32_t *v2, uint32_t *hist, hipStream_t s, int digit_bits,
                     int64_t hist_cap) {
    int nblocks = (int)((n + RS_TILE - 1) / RS_TILE);
    if (nblocks < 1) nblocks = 1;
    const int db = digit_bits == 10 && key_bits > 8 && key_bits <= 20 ? 10 : 8;
    const int64_t bins = (int64_t)1 << db;
    if (hist_cap <= 0) hist_cap = bins * nblocks;   // the documented minimum
    // small sorts (at most 64 blocks, the histogram in room): two launches per pass, each block deriving its
    // offsets from the raw histograms; tiles shrink while that holds -- a block's scatter is a chain of
    // tile / 256 ranked sub-tiles
    int tile = RS_TILE;
    const bool fused = nblocks <= 64 && bins * nblocks <= hist_cap;
    while (fused && tile > RS_THREADS) {
        const int64_t nb = (n + tile / 2 - 1) / (tile / 2);
        if (nb > 64 || bins * nb > hist_cap) break;
        tile /= 2;
        nblocks = (int)(nb < 1 ? 1 : nb);
    }
    const uint32_t *ik = keys;
    const uint32_t *iv = vals;
    uint32_t *ok = k1, *ov = v1;
    int which = 0;
    for (int shift = 0; shift < key_bits; shift += db) {
        if (db == 10) {
            hipLaunchKernelGGL(rs_hist_kernel<10>, dim3(nblocks), dim3(RS_THREADS), 0, s, ik, n, shift, hist, nblocks,
                               tile);
            if (fused) {
                hipLaunchKernelGGL((rs_scatter_kernel<10, true>), dim3(nblocks), dim3(RS_THREADS), 0, s, ik, iv, n,
                                   shift, hist, nblocks, ok, ov, tile);
            } else {
                hipLaunchKernelGGL(rs_scan_kernel, dim3(1), dim3(1024), 0, s, hist, (int64_t)1024 * nblocks);
                hipLaunchKernelGGL((rs_scatter_kernel<10, false>), dim3(nblocks), dim3(RS_THREADS), 0, s, ik, iv, n,
                                   shift, hist, nblocks, ok, ov, tile);
            }
        } else {
            hipLaunchKernelGGL(rs_hist_kernel<8>, dim3(nblocks), dim3(RS_THREADS), 0, s, ik, n, shift, hist, nblocks,
                               tile);
            if (fused) {
                hipLaunchKernelGGL((rs_scatter_kernel<8, true>), dim3(nblocks), dim3(RS_THREADS), 0, s, ik, iv, n,
                                   shift, hist, nblocks, ok, ov, tile);
            } else {
                hipLaunchKernelGGL(rs_scan_kernel, dim3(1), dim3(1024), 0, s, hist, (int64_t)256 * nblocks);
                hipLaunchKernelGGL((rs_scatter_kernel<8, false>), dim3(nblocks), dim3(RS_THREADS), 0, s, ik, iv, n,
                                   shift, hist, nblocks, ok, ov, tile);
            }
        }
        ik = ok;
        iv = ov;
        which = ok == k1 ? 0 : 1;
        ok = (ok == k1) ? k2 : k1;
        ov = (ov == v1) ? v2 : v1;
    }
    return which;
}

}  // namespace gwo
