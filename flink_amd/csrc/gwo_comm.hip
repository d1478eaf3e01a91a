// gwo_comm.hip -- keyBy shuffle kernels for the multi-GPU path.
//
// Reference: KeyGroupStreamPartitioner.selectChannel (SJ/runtime/partitioner/
// KeyGroupStreamPartitioner.java:51-58) = computeOperatorIndexForKeyGroup(assignToKeyGroup(key))
// (KeyGroupRangeAssignment.java:48-73, 118-119).  Records are grouped by destination GPU with a
// stable one-digit radix pass (gwo_sort.hip's kernels, digit = destination) so each source
// rank's records reach their owner in arrival order, packed as 24-byte {key, ts, value} records
// for one ncclSend per peer, and unpacked to columns on the receiving side.
#include "gwo_device.h"

namespace gwo {

__global__ __launch_bounds__(256) void dest_kernel(const int64_t *__restrict__ key, int64_t n, int kind, int max_par,
                                                   int nranks, uint32_t *__restrict__ dest) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        int32_t kg = key_group(key[i], kind, max_par);
        dest[i] = (uint32_t)(kg * nranks / max_par);
    }
}

__global__ __launch_bounds__(256) void pack_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                   const int64_t *__restrict__ val, const uint32_t *__restrict__ perm,
                                                   int64_t n, int64_t *__restrict__ out) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += step) {
        uint32_t i = perm[j];
        out[3 * j] = key[i];
        out[3 * j + 1] = ts[i];
        out[3 * j + 2] = val ? val[i] : 0;
    }
}

__global__ __launch_bounds__(256) void unpack_kernel(const int64_t *__restrict__ in, int64_t n, int64_t *__restrict__ key,
                                                     int64_t *__restrict__ ts, int64_t *__restrict__ val) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += step) {
        key[j] = in[3 * j];
        ts[j] = in[3 * j + 1];
        val[j] = in[3 * j + 2];
    }
}

// per-destination counts (nranks <= 256)
__global__ __launch_bounds__(256) void dest_count_kernel(const uint32_t *__restrict__ dest, int64_t n,
                                                         unsigned long long *__restrict__ counts) {
    __shared__ unsigned long long c[256];
    c[threadIdx.x] = 0;
    __syncthreads();
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) atomicAdd(&c[dest[i]], 1ull);
    __syncthreads();
    if (c[threadIdx.x]) atomicAdd(&counts[threadIdx.x], c[threadIdx.x]);
}

static inline int cgrid(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

void launch_dest(const int64_t *key, int64_t n, int kind, int max_par, int nranks, uint32_t *dest, hipStream_t s) {
    hipLaunchKernelGGL(dest_kernel, dim3(cgrid(n)), dim3(256), 0, s, key, n, kind, max_par, nranks, dest);
}
void launch_dest_count(const uint32_t *dest, int64_t n, unsigned long long *counts, hipStream_t s) {
    hipLaunchKernelGGL(dest_count_kernel, dim3(cgrid(n)), dim3(256), 0, s, dest, n, counts);
}
void launch_pack(const int64_t *key, const int64_t *ts, const int64_t *val, const uint32_t *perm, int64_t n,
                 int64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(pack_kernel, dim3(cgrid(n)), dim3(256), 0, s, key, ts, val, perm, n, out);
}
void launch_unpack(const int64_t *in, int64_t n, int64_t *key, int64_t *ts, int64_t *val, hipStream_t s) {
    hipLaunchKernelGGL(unpack_kernel, dim3(cgrid(n)), dim3(256), 0, s, in, n, key, ts, val);
}

}  // namespace gwo

namespace gwo {

// ------------------------------------------------------------------------------------------------
// route: the batch form of KeyGroupStreamPartitioner.selectChannel for order-insensitive window
// state (tumbling/sliding).  A 2048-record tile is grouped by destination operator index in LDS
// (counting sort), each destination's run is reserved with one atomic on that destination's cursor
// (one per 128-B line) in a fixed-capacity region of the send buffer, and written as contiguous
// 24-B {key, ts, value} records -- word-wise, so each store instruction writes one contiguous run.
// A cursor ends as the destination's record count; a count above the capacity means those records
// were not written and the caller re-runs with a larger capacity.
// ------------------------------------------------------------------------------------------------
#define RT_PER 8
#define RT_THREADS 256
#define RT_TILE (RT_PER * RT_THREADS)
#define RT_CUR_STRIDE 16

__global__ __launch_bounds__(RT_THREADS) void route_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                           const int64_t *__restrict__ val, int64_t n, int kind,
                                                           int max_par, int nranks,
                                                           unsigned long long *__restrict__ cursor, uint64_t cap,
                                                           int64_t *__restrict__ send) {
    __shared__ __attribute__((aligned(16))) int64_t s_rec[3 * RT_TILE];
    __shared__ uint8_t s_dst[RT_TILE];
    __shared__ uint32_t s_cnt[256], s_off[257];
    __shared__ uint32_t s_pos[256];
    const int tid = threadIdx.x;
    for (int64_t tile = (int64_t)blockIdx.x * RT_TILE; tile < n; tile += (int64_t)gridDim.x * RT_TILE) {
        s_cnt[tid] = 0;
        __syncthreads();
        int64_t kk[RT_PER], tt[RT_PER], vv[RT_PER];
        uint32_t code[RT_PER];
#pragma unroll
        for (int j = 0; j < RT_PER; ++j) {
            int64_t i = tile + j * RT_THREADS + tid;
            i = i < n ? i : tile;   // unconditional loads; lanes past the end are discarded
            kk[j] = __builtin_nontemporal_load(key + i);
            tt[j] = __builtin_nontemporal_load(ts + i);
            vv[j] = val ? __builtin_nontemporal_load(val + i) : 0;
        }
#pragma unroll
        for (int j = 0; j < RT_PER; ++j) {
            const int64_t i = tile + j * RT_THREADS + tid;
            code[j] = 0xffffffffu;
            if (i < n) {
                const uint32_t d = (uint32_t)(key_group(kk[j], kind, max_par) * nranks / max_par);
                code[j] = (d << 16) | atomicAdd(&s_cnt[d], 1u);
            }
        }
        __syncthreads();
        // exclusive prefix over the (<= 256) destinations, one reservation per non-empty destination
        const uint32_t c = tid < nranks ? s_cnt[tid] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(c, &tot);
        unsigned long long at = 0;
        if (c) at = atomicAdd(&cursor[(size_t)tid * RT_CUR_STRIDE], (unsigned long long)c);
        s_off[tid] = ex;
        if (tid == 0) s_off[256] = tot;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RT_PER; ++j) {
            if (code[j] == 0xffffffffu) continue;
            const uint32_t d = code[j] >> 16;
            const uint32_t pos = s_off[d] + (code[j] & 0xffffu);
            s_rec[3 * pos] = kk[j];
            s_rec[3 * pos + 1] = tt[j];
            s_rec[3 * pos + 2] = vv[j];
            s_dst[pos] = (uint8_t)d;
        }
        if (c) s_pos[tid] = (uint32_t)(at < cap ? at : cap);
        __syncthreads();
        // word-wise copy-out: word w of the tile belongs to record w / 3
        for (uint32_t w = tid; w < 3 * tot; w += RT_THREADS) {
            const uint32_t r = w / 3, f = w - 3 * r;
            const uint32_t d = s_dst[r];
            const uint64_t q = (uint64_t)s_pos[d] + (r - s_off[d]);
            if (q < cap) send[((uint64_t)d * cap + q) * 3 + f] = s_rec[w];
        }
        __syncthreads();
    }
}

// counts[p] = cursor[p * RT_CUR_STRIDE]; resets the cursors for the next launch
__global__ void route_collect_kernel(unsigned long long *cursor, int nranks, unsigned long long *counts) {
    for (int p = threadIdx.x; p < nranks; p += blockDim.x) {
        counts[p] = cursor[(size_t)p * RT_CUR_STRIDE];
        cursor[(size_t)p * RT_CUR_STRIDE] = 0;
    }
}

void launch_route(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, int kind, int max_par,
                  int nranks, unsigned long long *cursor, uint64_t cap, int64_t *send, hipStream_t s) {
    int64_t grid = (n + RT_TILE - 1) / RT_TILE;
    grid = grid < 1 ? 1 : (grid > 4096 ? 4096 : grid);
    hipLaunchKernelGGL(route_kernel, dim3((int)grid), dim3(RT_THREADS), 0, s, key, ts, val, n, kind, max_par, nranks,
                       cursor, cap, send);
}

void launch_route_collect(unsigned long long *cursor, int nranks, unsigned long long *counts, hipStream_t s) {
    hipLaunchKernelGGL(route_collect_kernel, dim3(1), dim3(256), 0, s, cursor, nranks, counts);
}

size_t route_cursor_bytes() { return (size_t)256 * RT_CUR_STRIDE * 8; }

}  // namespace gwo
