// micro_table.hip -- gfx950 microbenchmark of the access patterns a keyed window-state table can
// use (DESIGN.md §4 records the numbers).  Table: CAP entries of 32 B (key + 3 accumulator words),
// 16.7M updates per launch (one C4 watermark interval), uniformly random entries.
//
//   stream    read 24 B/record input only (HBM streaming reference)
//   rmw       plain 32-B load + plain 32-B store per update (exclusive ownership assumed)
//   atom3     atomic key load + 3 device-scope atomics (add, min, max) per update
//   atom3wg   the same with workgroup-scope atomics
//   cas       one device-scope atomicCAS per update
//   rmw_sorted  rmw, but updates grouped by 8-MB table region (partitioned insert)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

struct E4 {
    int64_t w[4];
};

__global__ void k_stream(const int64_t *a, const int64_t *b, const int64_t *c, int64_t n, int64_t *out) {
    int64_t s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        s += a[i] ^ b[i] ^ c[i];
    if (s == 42) out[0] = s;
}

__global__ void k_rmw(const int64_t *key, const int64_t *val, int64_t n, E4 *t, uint64_t mask) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t s = mix((uint64_t)key[i]) & mask;
        int64_t v = val[i];
        E4 e = t[s];
        e.w[0] = key[i];
        e.w[1] += v;
        e.w[2] = e.w[2] < v ? e.w[2] : v;
        e.w[3] = e.w[3] > v ? e.w[3] : v;
        t[s] = e;
    }
}

__global__ void k_atom3(const int64_t *key, const int64_t *val, int64_t n, E4 *t, uint64_t mask) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t s = mix((uint64_t)key[i]) & mask;
        int64_t v = val[i];
        int64_t *e = t[s].w;
        int64_t cur = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == 12345) continue;
        atomicAdd((unsigned long long *)(e + 1), (unsigned long long)v);
        atomicMin((long long *)(e + 2), (long long)v);
        atomicMax((long long *)(e + 3), (long long)v);
    }
}

__global__ void k_atom3wg(const int64_t *key, const int64_t *val, int64_t n, E4 *t, uint64_t mask) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t s = mix((uint64_t)key[i]) & mask;
        int64_t v = val[i];
        int64_t *e = t[s].w;
        int64_t cur = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 12345) continue;
        __hip_atomic_fetch_add(e + 1, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_min(e + 2, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_max(e + 3, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

__global__ void k_cas(const int64_t *key, int64_t n, E4 *t, uint64_t mask, unsigned long long *won) {
    unsigned long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t s = mix((uint64_t)key[i]) & mask;
        unsigned long long prev = atomicCAS((unsigned long long *)t[s].w, 0ull, (unsigned long long)key[i]);
        c += prev == 0;
    }
    if (c == 0xffffffffull) atomicAdd(won, c);
}

// records pre-grouped by region: block b handles records [off[b], off[b+1])
__global__ void k_rmw_sorted(const int64_t *key, const int64_t *val, const int64_t *off, E4 *t, uint64_t mask) {
    int64_t lo = off[blockIdx.x], hi = off[blockIdx.x + 1];
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        uint64_t s = mix((uint64_t)key[i]) & mask;
        int64_t v = val[i];
        E4 e = t[s];
        e.w[0] = key[i];
        e.w[1] += v;
        e.w[2] = e.w[2] < v ? e.w[2] : v;
        e.w[3] = e.w[3] > v ? e.w[3] : v;
        t[s] = e;
    }
}

__global__ void k_gen(int64_t *key, int64_t *val, int64_t n, uint64_t nkeys, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        key[i] = (int64_t)(mix(seed + (uint64_t)i * 0x9E3779B97F4A7C15ull) % nkeys);
        val[i] = (int64_t)(mix(seed ^ (uint64_t)i) % 1000);
    }
}

int main(int argc, char **argv) {
    int64_t n = argc > 1 ? atoll(argv[1]) : 16666666;
    int log_cap = argc > 2 ? atoi(argv[2]) : 28;
    uint64_t cap = 1ull << log_cap, mask = cap - 1;
    int64_t *key, *val, *ts, *sk, *sv, *off, *dummy;
    E4 *t;
    unsigned long long *won;
    CHECK(hipMalloc(&key, n * 8));
    CHECK(hipMalloc(&val, n * 8));
    CHECK(hipMalloc(&ts, n * 8));
    CHECK(hipMalloc(&sk, n * 8));
    CHECK(hipMalloc(&sv, n * 8));
    CHECK(hipMalloc(&dummy, 64));
    CHECK(hipMalloc(&won, 64));
    CHECK(hipMalloc(&t, cap * sizeof(E4)));
    CHECK(hipMemset(t, 0, cap * sizeof(E4)));
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, key, val, n, (uint64_t)100000000, 42ull);
    CHECK(hipMemcpy(ts, key, n * 8, hipMemcpyDeviceToDevice));
    // host-side grouping by region for rmw_sorted
    const int log_regions = 10;
    const int R = 1 << log_regions;
    std::vector<int64_t> hk(n), hv(n);
    CHECK(hipMemcpy(hk.data(), key, n * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hv.data(), val, n * 8, hipMemcpyDeviceToHost));
    auto hmix = [](uint64_t k) {
        k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33; return k;
    };
    std::vector<int64_t> cnt(R + 1, 0);
    for (int64_t i = 0; i < n; ++i) cnt[((hmix(hk[i]) & mask) >> (log_cap - log_regions)) + 1]++;
    for (int r = 0; r < R; ++r) cnt[r + 1] += cnt[r];
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1), gk(n), gv(n);
    for (int64_t i = 0; i < n; ++i) {
        int r = (int)((hmix(hk[i]) & mask) >> (log_cap - log_regions));
        gk[pos[r]] = hk[i];
        gv[pos[r]] = hv[i];
        pos[r]++;
    }
    CHECK(hipMalloc(&off, (R + 1) * 8));
    CHECK(hipMemcpy(off, cnt.data(), (R + 1) * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(sk, gk.data(), n * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(sv, gv.data(), n * 8, hipMemcpyHostToDevice));
    CHECK(hipDeviceSynchronize());

    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    int grid = 256 * 8;
    auto timeit = [&](const char *name, auto fn) {
        fn();
        CHECK(hipDeviceSynchronize());
        const int reps = 5;
        CHECK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) fn();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        printf("%-12s n=%lld cap=2^%d  %8.3f ms  %7.2f G upd/s  %7.1f ns/wave-upd\n", name, (long long)n, log_cap, ms,
               n / ms / 1e6, ms * 1e6 / n);
        fflush(stdout);
    };
    timeit("stream24", [&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, key, val, ts, n, dummy); });
    timeit("rmw", [&] { hipLaunchKernelGGL(k_rmw, dim3(grid), dim3(256), 0, 0, key, val, n, t, mask); });
    timeit("rmw_g64k", [&] { hipLaunchKernelGGL(k_rmw, dim3(65536), dim3(256), 0, 0, key, val, n, t, mask); });
    timeit("rmw_sorted", [&] { hipLaunchKernelGGL(k_rmw_sorted, dim3(R), dim3(256), 0, 0, sk, sv, off, t, mask); });
    timeit("atom3", [&] { hipLaunchKernelGGL(k_atom3, dim3(grid), dim3(256), 0, 0, key, val, n, t, mask); });
    timeit("atom3wg", [&] { hipLaunchKernelGGL(k_atom3wg, dim3(grid), dim3(256), 0, 0, key, val, n, t, mask); });
    timeit("cas", [&] { hipLaunchKernelGGL(k_cas, dim3(grid), dim3(256), 0, 0, key, n, t, mask, won); });
    return 0;
}
