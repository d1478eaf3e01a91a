// gwo_sort.hip -- stable LSD radix sort of (uint32 key, uint32 payload) pairs for gfx950.
//
// Used to group a batch's records by session-state slot while keeping arrival order inside each
// group (MergingWindowSet semantics depend on arrival order once late records exist).  8-bit
// digits; per pass: block histograms (digit-major) -> one-workgroup exclusive scan -> stable
// scatter.  Stability inside a block: each 256-record sub-tile is ranked with wave ballots
// (lanes with the same digit, lower lane id) plus per-wave digit counts in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gwo {

#define RS_TILE 4096
#define RS_THREADS 256
#define RS_BINS 256

__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const uint32_t *__restrict__ keys, int64_t n, int shift,
                                                             uint32_t *__restrict__ block_hist, int nblocks) {
    __shared__ uint32_t h[RS_BINS];
    h[threadIdx.x] = 0;
    __syncthreads();
    int64_t base = (int64_t)blockIdx.x * RS_TILE;
    for (int j = threadIdx.x; j < RS_TILE; j += RS_THREADS) {
        int64_t i = base + j;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xff], 1u);
    }
    __syncthreads();
    block_hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];  // digit-major
}

// exclusive scan of m entries by one workgroup
__global__ __launch_bounds__(1024) void rs_scan_kernel(uint32_t *__restrict__ data, int64_t m) {
    __shared__ uint32_t s[1024];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < m; base += 1024) {
        int64_t i = base + threadIdx.x;
        uint32_t v = i < m ? data[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            uint32_t t = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        uint32_t incl = s[threadIdx.x];
        if (i < m) data[i] = carry + incl - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += incl;
        __syncthreads();
    }
}

__global__ __launch_bounds__(RS_THREADS) void rs_scatter_kernel(const uint32_t *__restrict__ keys,
                                                                const uint32_t *__restrict__ vals, int64_t n,
                                                                int shift, const uint32_t *__restrict__ offsets,
                                                                int nblocks, uint32_t *__restrict__ okeys,
                                                                uint32_t *__restrict__ ovals) {
    __shared__ uint32_t run[RS_BINS];              // running position per digit for this block
    __shared__ uint32_t wcnt[RS_THREADS / 64][RS_BINS];
    run[threadIdx.x] = offsets[(int64_t)threadIdx.x * nblocks + blockIdx.x];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1;
    int64_t base = (int64_t)blockIdx.x * RS_TILE;
    for (int sub = 0; sub < RS_TILE; sub += RS_THREADS) {
        for (int w = 0; w < RS_THREADS / 64; ++w) wcnt[w][threadIdx.x] = 0;
        __syncthreads();
        int64_t i = base + sub + threadIdx.x;
        bool valid = i < n;
        uint32_t k = valid ? keys[i] : 0;
        uint32_t d = (k >> shift) & 0xff;
        // lanes of this wave holding the same digit
        uint64_t same = __ballot(valid);
        for (int b = 0; b < 8; ++b) {
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
            ovals[pos] = vals ? vals[i] : (uint32_t)i;
        }
        __syncthreads();
        // advance running positions by this sub-tile's digit totals
        uint32_t tot = 0;
        for (int w = 0; w < RS_THREADS / 64; ++w) tot += wcnt[w][threadIdx.x];
        run[threadIdx.x] += tot;
        __syncthreads();
    }
}

// Sorts keys[0..n) stably; payload = vals (or the original index when vals == nullptr).
// tmp buffers: k1/v1/k2/v2 of n entries each, hist of 256*ceil(n/4096) entries.
// The result lands in (k1, v1) or (k2, v2): returns 0 for (k1, v1), 1 for (k2, v2).
int radix_sort_pairs(const uint32_t *keys, const uint32_t *vals, int64_t n, int key_bits, uint32_t *k1,
                     uint32_t *v1, uint32_t *k2, uint32_t *v2, uint32_t *hist, hipStream_t s) {
    int nblocks = (int)((n + RS_TILE - 1) / RS_TILE);
    if (nblocks < 1) nblocks = 1;
    const uint32_t *ik = keys;
    const uint32_t *iv = vals;
    uint32_t *ok = k1, *ov = v1;
    int which = 0;
    for (int shift = 0; shift < key_bits; shift += 8) {
        hipLaunchKernelGGL(rs_hist_kernel, dim3(nblocks), dim3(RS_THREADS), 0, s, ik, n, shift, hist, nblocks);
        hipLaunchKernelGGL(rs_scan_kernel, dim3(1), dim3(1024), 0, s, hist, (int64_t)RS_BINS * nblocks);
        hipLaunchKernelGGL(rs_scatter_kernel, dim3(nblocks), dim3(RS_THREADS), 0, s, ik, iv, n, shift, hist, nblocks,
                           ok, ov);
        ik = ok;
        iv = ov;
        which = ok == k1 ? 0 : 1;
        ok = (ok == k1) ? k2 : k1;
        ov = (ov == v1) ? v2 : v1;
    }
    return which;
}

}  // namespace gwo
