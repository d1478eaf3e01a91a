// slog_lab.hip -- data movement of the C3 window step alone: per partition, read R_p's SoA columns
// (key + 2 words), write R'_p's columns and the partition's rows (key, start, end, result) at a reserved offset -- no
// hash table, no fold.  Bounds what the window step can reach with its layout.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/slog_lab.hip -o tools/slog_lab
// usage: tools/slog_lab [partitions=16384] [entries=545] [rcap=704] [workgroups_per_cu=4]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

// mode bits: 1 read R, 2 write R', 4 write rows, 8 reserve rows with an atomic
__global__ __launch_bounds__(256) void mover(const int64_t *__restrict__ R, int64_t *__restrict__ Rp, int64_t *k_out,
                                             int64_t *s_out, int64_t *e_out, int64_t *r_out, unsigned long long *ctr,
                                             int P, int rcap, int n, int mode) {
    __shared__ unsigned long long s_base;
    const int tid = threadIdx.x;
    for (int p = blockIdx.x; p < P; p += gridDim.x) {
        const int64_t *in = R + (size_t)p * rcap * 3;
        int64_t *out = Rp + (size_t)p * rcap * 3;
        int64_t k[4], w0[4], w1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = tid + j * 256;
            k[j] = w0[j] = w1[j] = i;
            if ((mode & 1) && i < n) {
                k[j] = __builtin_nontemporal_load(in + i);
                w0[j] = __builtin_nontemporal_load(in + rcap + i);
                w1[j] = __builtin_nontemporal_load(in + 2 * rcap + i);
            }
        }
        if (tid == 0) s_base = (mode & 8) ? atomicAdd(ctr, (unsigned long long)n) : (unsigned long long)p * n;
        __syncthreads();
        const unsigned long long base = s_base;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = tid + j * 256;
            if (i >= n) continue;
            if (mode & 2) {
                out[i] = k[j];
                out[rcap + i] = w0[j];
                out[2 * rcap + i] = w1[j];
            }
            if (mode & 4) {
                k_out[base + i] = k[j];
                s_out[base + i] = 1000;
                e_out[base + i] = 2000;
                r_out[base + i] = w0[j] + w1[j];
            }
        }
        __syncthreads();
    }
}

int main(int argc, char **argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 16384, n = argc > 2 ? atoi(argv[2]) : 545,
              rcap = argc > 3 ? atoi(argv[3]) : 704, wpc = argc > 4 ? atoi(argv[4]) : 4;
    if (n > 1024 || n > rcap) return 1;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    int64_t *R, *Rp, *ko, *so, *eo, *ro;
    unsigned long long *ctr;
    const size_t rb = (size_t)P * rcap * 3 * 8, ob = (size_t)P * n * 8;
    CK(hipMalloc(&R, rb));
    CK(hipMalloc(&Rp, rb));
    CK(hipMalloc(&ko, ob));
    CK(hipMalloc(&so, ob));
    CK(hipMalloc(&eo, ob));
    CK(hipMalloc(&ro, ob));
    CK(hipMalloc(&ctr, 8));
    CK(hipMemset(R, 1, rb));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = cus * wpc;
    const int modes[] = {1, 3, 7, 15, 5, 13, 2, 6};
    const char *names[] = {"read R", "read R + write R'", "read + R' + rows", "read + R' + rows + atomic",
                           "read + rows", "read + rows + atomic", "write R' only", "write R' + rows"};
    for (int m = 0; m < 8; ++m) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipMemset(ctr, 0, 8));
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(mover, dim3(grid), dim3(256), 0, 0, R, Rp, ko, so, eo, ro, ctr, P, rcap, n, modes[m]);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        const double bytes = ((modes[m] & 1) ? (double)P * n * 24 : 0) + ((modes[m] & 2) ? (double)P * n * 24 : 0) +
                             ((modes[m] & 4) ? (double)P * n * 32 : 0);
        printf("%-28s %8.1f us  %7.0f MB  %6.2f TB/s\n", names[m], best * 1e3, bytes / 1e6, bytes / (best * 1e-3) / 1e12);
    }
    return 0;
}
