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
