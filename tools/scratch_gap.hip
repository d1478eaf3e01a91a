// Dispatch cost of kernel shapes behind a small plain kernel: N pairs on one stream, timed with events.  B is a
// plain kernel, one with a private segment (scratch), one of 1024-thread workgroups, one with 64 KB of dynamic LDS,
// or 1024 threads + 64 KB LDS (C2's gather shape).  Prints us per pair.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_plain(int *p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1;
}
__global__ void k_scratch(int *p, int n, int j) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    volatile int a[8];   // dynamically indexed: a private segment
    for (int q = 0; q < 8; ++q) a[q] = i + q;
    if (i < n) p[i] += a[(i + j) & 7];
}
__global__ __launch_bounds__(1024) void k_plain2(int *p, int n, int j) {
    extern __shared__ int s[];
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < 0) s[threadIdx.x] = i;   // (never: the LDS is only allocated)
    if (i < n) p[i] += j;
}

int main() {
    const int n = 1 << 20, iters = 2000;
    int *p;
    if (hipMalloc(&p, n * 4) != hipSuccess) return 1;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const char *names[5] = {"plain 256      ", "scratch        ", "1024 threads   ", "64 KB LDS      ", "1024 + 64 KB   "};
    for (int mode = 0; mode < 5; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(a, s);
            for (int it = 0; it < iters; ++it) {
                hipLaunchKernelGGL(k_plain, dim3(n / 256), dim3(256), 0, s, p, n);
                if (mode == 1) hipLaunchKernelGGL(k_scratch, dim3(n / 256), dim3(256), 0, s, p, n, it);
                else {
                    const int t = (mode == 2 || mode == 4) ? 1024 : 256;
                    const size_t lds = (mode == 3 || mode == 4) ? 65536 : 0;
                    hipLaunchKernelGGL(k_plain2, dim3(n / t), dim3(t), lds, s, p, n, it);
                }
            }
            (void)hipEventRecord(b, s);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("plain + %s: %.2f us per pair\n", names[mode], ms * 1000 / iters);
        }
    }
    return 0;
}
