// k1_bench.hip -- gfx950 microbenchmark of the log layout's K1 write strategies, one C4 batch:
// 16.67M records (key uniform in [0, 1e8), one 1-s interval of event time, every record accepted into one
// window), grouped into 256 coarse buckets (top 8 bits of digit_hash) in bucket regions of the batch buffer.
// Not part of the library; it decides which variant the product's log_part_kernel uses.
//
//   stream  read 24 B, write 16 B per record, contiguous (the byte mix's streaming reference)
//   v0      the product's scheme: tile 256 x PER, LDS counting sort, one cursor reservation per (tile, bucket),
//           each tile's run written from LDS (runs of ~PER*256/256 records at unaligned starts)
//   half    the same reservations for a 256 x 14 tile, but the LDS scatter + write done in NH parts (LDS/NH)
//   wc      write-combining chunks: a workgroup owns one open CH-record chunk per bucket and appends each tile's
//           run where the last one ended (partial lines completed by the same workgroup); reservations in whole
//           chunks; a chunk's fill is recorded (the workgroup's last chunk per bucket ends partly filled)
//
// Every variant's bucket contents are checked (count, key sum, value sum per bucket) against the host.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef long long ll2 __attribute__((ext_vector_type(2)));
static constexpr int NB = 256;
static constexpr int CSTR = 16;   // cursor stride (one per 128-B line)

__host__ __device__ inline uint32_t digit_hash(int64_t key) {
    return (uint32_t)key * 0xCC9E2D51u + (uint32_t)((uint64_t)key >> 32) * 0x1B873593u;
}
__host__ __device__ inline uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void gen(int64_t *k, int64_t *t, int64_t *v, int64_t n, int64_t t0) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        k[i] = (int64_t)(mix(2 * i) % 100000000ull);
        t[i] = t0 + (int64_t)(mix(2 * i + 1) % 1000ull);
        v[i] = (int64_t)(mix(3 * i + 7) % 1000ull);
    }
}

__global__ __launch_bounds__(256) void stream_kernel(const int64_t *__restrict__ k, const int64_t *__restrict__ t,
                                                     const int64_t *__restrict__ v, int64_t n, int64_t w0,
                                                     int64_t *__restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ts = __builtin_nontemporal_load(t + i);
        ll2 r = {__builtin_nontemporal_load(k + i), __builtin_nontemporal_load(v + i)};
        if (ts >= w0) *(ll2 *)(out + 2 * i) = r;
    }
}

__device__ __forceinline__ unsigned scan256(unsigned v, unsigned *total) {
    __shared__ unsigned s_w[5];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        unsigned y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    unsigned pre = 0;
    for (int w = 0; w < wid; ++w) pre += s_w[w];
    *total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    return pre + incl - v;
}

// v0 / half: PER records per thread per tile, written in NH parts.  MODE 0: one reservation per (tile, bucket)
// (slots = records).  MODE 1: write-combining chunks of CH records (cursor counts chunks).
template <int PER, int NH, int MODE, int CH, int STATS = 0>
__global__ __launch_bounds__(256) void k1_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                 const int64_t *__restrict__ val, int64_t n, int64_t w0, int64_t w1,
                                                 unsigned long long *__restrict__ cursor, uint64_t cap,
                                                 int64_t *__restrict__ out, uint8_t *__restrict__ fill,
                                                 uint32_t nchk, unsigned long long *__restrict__ stats) {
    constexpr int TILE = 256 * PER;
    constexpr int HP = PER / NH;
    static_assert(PER % NH == 0, "parts");
    __shared__ __attribute__((aligned(16))) int64_t s_rec[256 * HP * 2];
    __shared__ uint8_t s_bk[256 * HP];
    __shared__ uint32_t s_cnt[NH][NB];
    __shared__ uint32_t s_off[NB];
    __shared__ unsigned long long s_base[NB];
    __shared__ uint32_t s_avail[NB];
    __shared__ unsigned long long s_base2[NB];
    const int tid = threadIdx.x;
    // write-combining state of bucket tid (thread tid owns bucket tid)
    uint32_t pos = CH;                // position in the open chunk (CH: none open)
    unsigned long long cb = 0;        // open chunk
    int64_t kk[PER], vv[PER], tt[PER];
    auto load_tile = [&](int64_t tile) {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            int64_t i = tile + j * 256 + tid;
            i = i < n ? i : tile;
            tt[j] = __builtin_nontemporal_load(ts + i);
            kk[j] = __builtin_nontemporal_load(key + i);
            vv[j] = __builtin_nontemporal_load(val + i);
        }
    };
    const int64_t tstride = (int64_t)gridDim.x * TILE;
    if ((int64_t)blockIdx.x * TILE < n) load_tile((int64_t)blockIdx.x * TILE);
    for (int64_t tile = (int64_t)blockIdx.x * TILE; tile < n; tile += tstride) {
#pragma unroll
        for (int h = 0; h < NH; ++h) s_cnt[h][tid] = 0;
        __syncthreads();
        uint32_t code[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int64_t i = tile + j * 256 + tid;
            code[j] = 0xffffffffu;
            if (i < n && tt[j] >= w0 && tt[j] < w1) {
                const uint32_t b = digit_hash(kk[j]) >> 24;
                code[j] = (b << 16) | atomicAdd(&s_cnt[j / HP][b], 1u);
            }
        }
        __syncthreads();
        uint32_t c = 0, ch[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            ch[h] = s_cnt[h][tid];
            c += ch[h];
        }
        unsigned long long a0 = 0, a1 = 0;   // run address of rank r: r < avail ? a0 + r : a1 + r
        uint32_t avail = 0;
        if (MODE == 0) {
            a0 = c ? atomicAdd(&cursor[tid * CSTR], (unsigned long long)c) : 0ull;
            avail = c;
        } else {
            avail = CH - pos;
            if (c > avail) {
                const uint32_t k = (c - avail + CH - 1) / CH;
                const unsigned long long nc = atomicAdd(&cursor[tid * CSTR], (unsigned long long)k);
                a0 = cb * CH + pos;
                a1 = nc * CH - avail;
                // the old chunk is full now (fill stays CH); the last new chunk is the open one
                cb = nc + k - 1;
                pos = c - avail - (k - 1) * CH;
            } else {
                a0 = cb * CH + pos;
                pos += c;
            }
        }
        uint32_t before = 0;   // records of bucket tid in earlier parts
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            unsigned total;
            const unsigned ex = scan256(ch[h], &total);
            s_off[tid] = ex;
            // part h of the run: ranks [before, before + ch[h])
            s_base[tid] = a0 + before;
            s_base2[tid] = a1 + before;
            s_avail[tid] = avail > before ? avail - before : 0;
            before += ch[h];
            __syncthreads();
#pragma unroll
            for (int jj = 0; jj < HP; ++jj) {
                const int j = h * HP + jj;
                if (code[j] == 0xffffffffu) continue;
                const uint32_t b = code[j] >> 16;
                const uint32_t p = s_off[b] + (code[j] & 0xffffu);
                ll2 r2 = {kk[j], vv[j]};
                *(ll2 *)&s_rec[2 * p] = r2;
                s_bk[p] = (uint8_t)b;
            }
            if (h == NH - 1 && tile + tstride < n) load_tile(tile + tstride);
            __syncthreads();
            for (uint32_t p = tid; p < total; p += 256) {
                const uint32_t b = s_bk[p];
                const uint32_t r = p - s_off[b];
                const unsigned long long q = MODE == 0 ? s_base[b] + r : (r < s_avail[b] ? s_base[b] + r : s_base2[b] + r);
                if (q < cap) *(ll2 *)(out + ((uint64_t)b * cap + q) * 2) = *(const ll2 *)&s_rec[2 * p];
            }
            __syncthreads();
        }
    }
    if (MODE == 1 && pos < CH && cb < nchk) fill[(size_t)tid * nchk + cb] = (uint8_t)pos;
    if (STATS == 1) {   // the r02 product's end: per-wave atomics on one word, one arrival counter
        unsigned long long acc = PER;
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if ((tid & 63) == 0) atomicAdd(&stats[0], acc);
        if (tid == 0) {
            atomicMin((long long *)&stats[16], (long long)blockIdx.x);
            atomicMax((long long *)&stats[32], (long long)blockIdx.x);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) atomicAdd(&stats[48], 1ull);
    } else if (STATS == 2) {   // sharded: one atomic per workgroup per word, 16 shards; two-level arrival
        if (tid == 0) {
            const int sh = blockIdx.x % 16;
            atomicAdd(&stats[64 + sh * 16], (unsigned long long)PER * 256);
            atomicMin((long long *)&stats[64 + sh * 16 + 1], (long long)blockIdx.x);
            atomicMax((long long *)&stats[64 + sh * 16 + 2], (long long)blockIdx.x);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const unsigned sh = blockIdx.x % 16, members = (gridDim.x - sh + 15) / 16;
            if (atomicAdd(&stats[512 + sh * 16], 1ull) == members - 1) atomicAdd(&stats[768], 1ull);
        }
    }
}

// per-bucket (count, key sum, value sum) of the batch buffer; slots valid per fill (MODE 1)
__global__ void check_kernel(const int64_t *out, uint64_t cap, const unsigned long long *cursor, int mode, int ch,
                             const uint8_t *fill, uint32_t nchk, unsigned long long *res) {
    const int b = blockIdx.x;
    unsigned long long slots = cursor[b * CSTR] * (mode ? ch : 1);
    if (slots > cap) slots = cap;
    unsigned long long c = 0, sk = 0, sv = 0;
    for (unsigned long long s = threadIdx.x; s < slots; s += blockDim.x) {
        if (mode && (s % ch) >= fill[(size_t)b * nchk + s / ch]) continue;
        c++;
        sk += (unsigned long long)out[((uint64_t)b * cap + s) * 2];
        sv += (unsigned long long)out[((uint64_t)b * cap + s) * 2 + 1];
    }
    atomicAdd(&res[b * 3], c);
    atomicAdd(&res[b * 3 + 1], sk);
    atomicAdd(&res[b * 3 + 2], sv);
}

struct Bufs {
    int64_t *k, *t, *v, *out;
    unsigned long long *cur, *res, *stats;
    uint8_t *fill;
    int64_t n;
    uint64_t cap;
    uint32_t nchk;
};

typedef void (*Launch)(const Bufs &, int grid, hipStream_t);

template <int PER, int NH, int MODE, int CH, int STATS = 0>
void launch(const Bufs &B, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k1_kernel<PER, NH, MODE, CH, STATS>), dim3(grid), dim3(256), 0, s, B.k, B.t, B.v, B.n,
                       (int64_t)0, (int64_t)1000000, B.cur, B.cap, B.out, B.fill, B.nchk, B.stats);
}

static std::vector<unsigned long long> host_ref;

static double run(const char *name, Launch L, const Bufs &B, int grid, int mode, int ch, int reps) {
    hipStream_t s = 0;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    double tot = 0;
    for (int r = 0; r < reps + 3; ++r) {
        CHECK(hipMemsetAsync(B.cur, 0, NB * CSTR * 8, s));
        if (mode) CHECK(hipMemsetAsync(B.fill, ch, (size_t)NB * B.nchk, s));
        CHECK(hipEventRecord(e0, s));
        L(B, grid, s);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) tot += ms;
    }
    CHECK(hipMemset(B.res, 0, NB * 3 * 8));
    hipLaunchKernelGGL(check_kernel, dim3(NB), dim3(256), 0, 0, B.out, B.cap, B.cur, mode, ch, B.fill, B.nchk, B.res);
    std::vector<unsigned long long> got(NB * 3), curs(NB * CSTR);
    CHECK(hipMemcpy(got.data(), B.res, NB * 3 * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(curs.data(), B.cur, NB * CSTR * 8, hipMemcpyDeviceToHost));
    bool ok = got == host_ref;
    unsigned long long slots = 0;
    for (int b = 0; b < NB; ++b) slots += curs[b * CSTR] * (mode ? ch : 1);
    const double us = tot / reps * 1e3;
    printf("%-24s grid %5d  %8.1f us  %6.2f TB/s (40 B/rec)  slots/records %.3f  %s\n", name, grid, us,
           B.n * 40.0 / (us * 1e-6) / 1e12, (double)slots / B.n, ok ? "OK" : "MISMATCH");
    fflush(stdout);
    return us;
}

int main() {
    Bufs B{};
    B.n = 16666666;
    const uint64_t per_b = B.n / NB;
    B.cap = (per_b + per_b / 3 + 4096) & ~63ull;   // room for the write-combining holes
    B.nchk = (uint32_t)(B.cap / 8);
    CHECK(hipMalloc(&B.k, B.n * 8));
    CHECK(hipMalloc(&B.t, B.n * 8));
    CHECK(hipMalloc(&B.v, B.n * 8));
    CHECK(hipMalloc(&B.out, (size_t)NB * B.cap * 16 > (size_t)B.n * 16 ? (size_t)NB * B.cap * 16 : (size_t)B.n * 16));
    CHECK(hipMalloc(&B.cur, NB * CSTR * 8));
    CHECK(hipMalloc(&B.res, NB * 3 * 8));
    CHECK(hipMalloc(&B.stats, 1024 * 8));
    CHECK(hipMemset(B.stats, 0, 1024 * 8));
    CHECK(hipMalloc(&B.fill, (size_t)NB * B.nchk));
    hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, B.k, B.t, B.v, B.n, (int64_t)500000);
    CHECK(hipDeviceSynchronize());
    {
        std::vector<int64_t> k(B.n), v(B.n);
        CHECK(hipMemcpy(k.data(), B.k, B.n * 8, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(v.data(), B.v, B.n * 8, hipMemcpyDeviceToHost));
        host_ref.assign(NB * 3, 0);
        for (int64_t i = 0; i < B.n; ++i) {
            const uint32_t b = digit_hash(k[i]) >> 24;
            host_ref[b * 3]++;
            host_ref[b * 3 + 1] += (unsigned long long)k[i];
            host_ref[b * 3 + 2] += (unsigned long long)v[i];
        }
    }
    {   // streaming reference
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        double tot = 0;
        for (int r = 0; r < 13; ++r) {
            CHECK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, 0, B.k, B.t, B.v, B.n, (int64_t)0, B.out);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3) tot += ms;
        }
        const double us = tot / 10 * 1e3;
        printf("%-24s grid %5d  %8.1f us  %6.2f TB/s (40 B/rec)\n", "stream", 4096, us, B.n * 40.0 / (us * 1e-6) / 1e12);
    }
    const int reps = 10;
    run("v0 per14", launch<14, 1, 0, 1>, B, 512, 0, 1, reps);
    run("v0 per14 stats/wave", launch<14, 1, 0, 1, 1>, B, 512, 0, 1, reps);
    run("v0 per14 stats/shard", launch<14, 1, 0, 1, 2>, B, 512, 0, 1, reps);
    run("half per14/2", launch<14, 2, 0, 1>, B, 1024, 0, 1, reps);
    run("half per14/2 st/shard", launch<14, 2, 0, 1, 2>, B, 1024, 0, 1, reps);
    run("wc per14 ch64", launch<14, 1, 1, 64>, B, 512, 1, 64, reps);
    run("wc per14 ch64", launch<14, 1, 1, 64>, B, 256, 1, 64, reps);
    run("wc per14 ch32", launch<14, 1, 1, 32>, B, 256, 1, 32, reps);
    return 0;
}
