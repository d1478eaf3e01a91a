// k1_lab.hip -- gfx950 microbenchmark of K1 (the log layout's batch partition kernel) pipelining
// variants on one C4 batch: 16.67M records (key uniform in [0, 1e8), one 1-s interval, every record accepted
// into one window), grouped into 256 coarse buckets (top 8 bits of digit_hash) in bucket regions.  Not part of
// the library: it decides how the product's log_part_kernel is built.
//
//   stream   read 24 B, write 16 B per record, contiguous (the byte mix's streaming reference)
//   lds      the product's scheme: tile THREADS x PER, LDS counting sort, one reservation per (tile, bucket),
//            each tile's runs written from LDS; the next tile's loads issued after the scatter (one register set)
//   pipe     the same, two register sets: tile t+1's loads are issued before tile t is classified, so they have
//            the whole tile's processing to arrive
//   V2       16-B loads of record pairs (two adjacent records per lane per column)
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
static constexpr int TAILCAP = 4096;   // wc: records of a bucket region reserved for the workgroups' final carries
// cursor words: main cursors [0, 512) x CSTR, wc tail cursors [512, 768) x CSTR, statistics [768, 784) x CSTR, then
// the trash lines

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
    for (int64_t i = 2 * (blockIdx.x * (int64_t)blockDim.x + threadIdx.x); i < n; i += 2 * (int64_t)gridDim.x * blockDim.x) {
        const ll2 ts = __builtin_nontemporal_load((const ll2 *)(t + i));
        const ll2 kk = __builtin_nontemporal_load((const ll2 *)(k + i));
        const ll2 vv = __builtin_nontemporal_load((const ll2 *)(v + i));
        if (ts.x >= w0) *(ll2 *)(out + 2 * i) = ll2{kk.x, vv.x};
        if (ts.y >= w0) *(ll2 *)(out + 2 * i + 2) = ll2{kk.y, vv.y};
    }
}

template <int T>
__device__ __forceinline__ unsigned block_excl_scan(unsigned v, unsigned *total) {
    __shared__ unsigned s_w[T / 64 + 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        unsigned y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    unsigned pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
        pre += w < wid ? s_w[w] : 0u;
        tot += s_w[w];
    }
    *total = tot;
    __syncthreads();
    return pre + incl - v;
}

// Record j of a thread in a tile: V2 -- pairs (j / 2) of adjacent records; else one record per lane per column.
template <int T, bool V2>
__device__ __forceinline__ int rpos(int j, int tid) {
    return V2 ? (j >> 1) * 2 * T + 2 * tid + (j & 1) : j * T + tid;
}

template <int T, int PER, bool V2>
struct Regs {
    int64_t k[PER], t[PER], v[PER];
    __device__ __forceinline__ void load(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n,
                                         int64_t tile, int tid) {
        if (V2) {
#pragma unroll
            for (int j2 = 0; j2 < PER / 2; ++j2) {
                int64_t i = tile + j2 * 2 * T + 2 * tid;
                i = i < n ? i : (tile < n ? tile : 0);
                const ll2 t2 = __builtin_nontemporal_load((const ll2 *)(ts + i));
                const ll2 k2 = __builtin_nontemporal_load((const ll2 *)(key + i));
                const ll2 v2 = __builtin_nontemporal_load((const ll2 *)(val + i));
                t[2 * j2] = t2.x;
                t[2 * j2 + 1] = t2.y;
                k[2 * j2] = k2.x;
                k[2 * j2 + 1] = k2.y;
                v[2 * j2] = v2.x;
                v[2 * j2 + 1] = v2.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                int64_t i = tile + j * T + tid;
                i = i < n ? i : (tile < n ? tile : 0);
                t[j] = __builtin_nontemporal_load(ts + i);
                k[j] = __builtin_nontemporal_load(key + i);
                v[j] = __builtin_nontemporal_load(val + i);
            }
        }
    }
};

// One tile: classify + count (LDS atomics), reserve runs (one device atomic per bucket), scan, scatter to LDS,
// [next loads: caller's hook], write runs.
template <int T, int PER, bool V2, int NBX, bool CLS, class Hook>
__device__ __forceinline__ void k1_tile(const Regs<T, PER, V2> &R, int64_t tile, int64_t n, int64_t w0, int64_t w1,
                                        unsigned long long *__restrict__ cursor, uint64_t cap,
                                        int64_t *__restrict__ out, int64_t *s_rec, uint8_t *s_bk, uint8_t *s_bh, uint32_t *s_cnt,
                                        uint32_t *s_off, int64_t *trash, unsigned &acc, unsigned &wmask,
                                        Hook hook) {
    constexpr int TILE = T * PER;
    constexpr int NB = NBX;
    constexpr int BPT = NB / T > 0 ? NB / T : 1;   // buckets per thread
    const int tid = threadIdx.x;
    for (int b = tid; b <= NB; b += T) s_cnt[b] = 0;
    __syncthreads();
    uint32_t code[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int64_t i = tile + rpos<T, V2>(j, tid);
        bool take;
        uint32_t b;
        if (CLS) {   // the product's classification: window bounds compares, class bits, a second window's buckets
            const int64_t t = R.t[j];
            const int jj = (t >= w1) + 0;
            take = i < n && t >= w0 && t < w1 + (w1 - w0) && ((0u >> (2 * jj)) & 3u) == 0;
            acc += take ? 1u : 0u;
            wmask |= (take ? 1u : 0u) << jj;
            b = (uint32_t)(jj * 256 + (int)(digit_hash(R.k[j]) >> 24));
        } else {
            take = i < n && R.t[j] >= w0 && R.t[j] < w1;
            b = digit_hash(R.k[j]) >> 24;
        }
        const uint32_t r = atomicAdd(&s_cnt[take ? b : NB], 1u);   // (NB: a spare counter)
        code[j] = take ? (b << 16) | r : 0xffffffffu;
    }
    __syncthreads();
    unsigned long long at[BPT];
    uint32_t c[BPT];
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int b = tid * BPT + q;
        c[q] = b < NB ? s_cnt[b] : 0u;
        if (b < NB) at[q] = atomicAdd(&cursor[(b & 255) * CSTR + (b >> 8) * 256 * CSTR], (unsigned long long)c[q]);
    }
    uint32_t csum = 0;
#pragma unroll
    for (int q = 0; q < BPT; ++q) csum += c[q];
    unsigned total;
    uint32_t ex = block_excl_scan<T>(tid * BPT < NB ? csum : 0u, &total);
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int b = tid * BPT + q;
        if (b < NB) s_off[b] = ex;
        ex += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const bool ok = code[j] != 0xffffffffu;
        const uint32_t b = ok ? code[j] >> 16 : 0u;
        const uint32_t p = ok ? s_off[b] + (code[j] & 0xffffu) : (uint32_t)TILE;
        *(ll2 *)&s_rec[2 * p] = ll2{R.k[j], R.v[j]};
        s_bk[p] = (uint8_t)b;
        if (NB > 256) s_bh[p] = (uint8_t)(b >> 8);
    }
    hook();
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int b = tid * BPT + q;
        if (b < NB) s_cnt[b] = (uint32_t)(at[q] < cap ? at[q] : cap) - s_off[b];
    }
    __syncthreads();
    // fixed trip count, every lane stores (lanes without a record to the trash line): exact wait counts
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t p = j * T + tid;
        const uint32_t pe = p < total ? p : (uint32_t)TILE;
        const uint32_t b = s_bk[pe] | (NB > 256 ? ((uint32_t)s_bh[pe] << 8) : 0u);
        const uint32_t q = s_cnt[b] + p;
        const bool ok = p < total && q < cap;
        int64_t *dst = ok ? out + ((uint64_t)(b & 255) * cap + q) * 2 : trash + 2 * j;
        *(ll2 *)dst = *(const ll2 *)&s_rec[2 * pe];
    }
    __syncthreads();
}

template <int T, int PER, bool V2, bool PIPE, int WPS, int NBX = 256, bool CLS = false, bool STATS = false>
__global__ __launch_bounds__(T, WPS) void k1_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                    const int64_t *__restrict__ val, int64_t n, int64_t w0, int64_t w1,
                                                    unsigned long long *__restrict__ cursor, uint64_t cap,
                                                    int64_t *__restrict__ out) {
    constexpr int TILE = T * PER;
    __shared__ __attribute__((aligned(16))) int64_t s_rec[(TILE + 1) * 2];
    __shared__ uint8_t s_bk[TILE + 1];
    __shared__ uint8_t s_bhx[NBX > 256 ? TILE + 1 : 1];
    __shared__ uint32_t s_cnt[NBX + 1];
    __shared__ uint32_t s_off[NBX];
    uint8_t *s_bh = s_bhx;
    unsigned acc = 0, wmask = 0;
    const int tid = threadIdx.x;
    const int64_t tstride = (int64_t)gridDim.x * TILE;
    int64_t tile = (int64_t)blockIdx.x * TILE;
    int64_t *const trash = (int64_t *)(cursor + 1024 * CSTR) + (size_t)blockIdx.x * 2 * PER;
    if (!PIPE) {
        Regs<T, PER, V2> R;
        R.load(key, ts, val, n, tile, tid);
        for (; tile < n; tile += tstride) {
            k1_tile<T, PER, V2, NBX, CLS>(R, tile, n, w0, w1, cursor, cap, out, s_rec, s_bk, s_bh, s_cnt, s_off, trash, acc, wmask,
                                [&]() { R.load(key, ts, val, n, tile + tstride, tid); });
        }
    } else {
        Regs<T, PER, V2> A, B;
        A.load(key, ts, val, n, tile, tid);
        for (; tile < n; tile += 2 * tstride) {
            B.load(key, ts, val, n, tile + tstride, tid);
            k1_tile<T, PER, V2, NBX, CLS>(A, tile, n, w0, w1, cursor, cap, out, s_rec, s_bk, s_bh, s_cnt, s_off, trash, acc, wmask, []() {});
            if (tile + tstride >= n) break;
            A.load(key, ts, val, n, tile + 2 * tstride, tid);
            k1_tile<T, PER, V2, NBX, CLS>(B, tile + tstride, n, w0, w1, cursor, cap, out, s_rec, s_bk, s_bh, s_cnt, s_off, trash, acc, wmask, []() {});
        }
    }
    if (STATS) {
        unsigned long long a = acc;
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
        if ((tid & 63) == 0) atomicAdd(&cursor[(768 + blockIdx.x % 16) * CSTR], a + wmask);
    }
}


// ---- wc: write-combining with per-bucket carries (full 128-B lines only) -----------------------------------------
// One workgroup per CU (T threads, PER records each, two register sets: tile t+1's loads issued before tile t is
// classified).  Per bucket the workgroup keeps up to 7 records (its carry) in LDS; a tile's records of bucket b
// follow its carry, the whole 8-record lines of that sequence are written (one reservation per bucket per tile, in
// lines), the rest becomes the new carry.  At the end every carry goes to the bucket's tail region (records).
// Every store is a full, aligned 128-B line: 8 consecutive lanes x 16 B.
template <int T, int PER, int NBX, bool CLS>
__global__ __launch_bounds__(T, 1) void wc_kernel(const int64_t *__restrict__ key, const int64_t *__restrict__ ts,
                                                  const int64_t *__restrict__ val, int64_t n, int64_t w0, int64_t w1,
                                                  unsigned long long *__restrict__ cursor, uint64_t cap,
                                                  int64_t *__restrict__ out) {
    constexpr int TILE = T * PER;
    constexpr int NB_ = NBX;
    constexpr int BPT = (NB_ + T - 1) / T;
    __shared__ __attribute__((aligned(16))) int64_t s_rec[(TILE + 1) * 2];
    __shared__ __attribute__((aligned(16))) int64_t s_car[NB_ * 8 * 2];   // carries: bucket b's records at [8b, 8b + c_b)
    __shared__ uint16_t s_lb[TILE / 8 + NB_ + 1];   // line -> bucket
    __shared__ uint32_t s_cnt[NB_ + 1];            // tile counts -> (after the scan) line base of each bucket
    __shared__ uint32_t s_off[NB_];                // first s_rec record of each bucket
    __shared__ uint8_t s_cc[NB_];                  // carry counts
    __shared__ uint32_t s_gl[NB_];                 // reserved line index (global, per bucket) for this tile
    __shared__ unsigned s_tl;
    const int tid = threadIdx.x;
    for (int b = tid; b < NB_; b += T) s_cc[b] = 0;
    const int64_t tstride = (int64_t)gridDim.x * TILE;
    int64_t *const trash = (int64_t *)(cursor + 1024 * CSTR) + (size_t)blockIdx.x * 2 * 64;   // (unused: never dropped)
    Regs<T, PER, true> A, B;
    auto tile_fn = [&](const Regs<T, PER, true> &R, int64_t tile) {
        for (int b = tid; b <= NB_; b += T) s_cnt[b] = 0;
        __syncthreads();
        uint32_t code[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int64_t i = tile + rpos<T, true>(j, tid);
            bool take;
            uint32_t b;
            if (CLS) {
                const int64_t t = R.t[j];
                const int jj = (t >= w1) + 0;
                take = i < n && t >= w0 && t < w1 + (w1 - w0);
                b = (uint32_t)(jj * 256 + (int)(digit_hash(R.k[j]) >> 24));
            } else {
                take = i < n && R.t[j] >= w0 && R.t[j] < w1;
                b = digit_hash(R.k[j]) >> 24;
            }
            const uint32_t r = atomicAdd(&s_cnt[take ? b : NB_], 1u);
            code[j] = take ? (b << 16) | r : 0xffffffffu;
        }
        __syncthreads();
        // per bucket: lines = (carry + count) / 8, one reservation (in lines) when there are any
        uint32_t cnt[BPT], cc[BPT], ln[BPT];
        unsigned long long at[BPT];
        uint32_t lsum = 0, rsum = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid * BPT + q;
            cnt[q] = b < NB_ ? s_cnt[b] : 0u;
            cc[q] = b < NB_ ? s_cc[b] : 0u;
            ln[q] = (cnt[q] + cc[q]) >> 3;
            at[q] = 0;
            if (b < NB_) at[q] = atomicAdd(&cursor[(b & 255) * CSTR + (b >> 8) * 256 * CSTR], (unsigned long long)ln[q] * 8);
            lsum += ln[q];
            rsum += cnt[q];
        }
        unsigned ltot, rtot;
        uint32_t lex = block_excl_scan<T>(lsum, &ltot);
        uint32_t rex = block_excl_scan<T>(rsum, &rtot);
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid * BPT + q;
            if (b < NB_) {
                s_off[b] = rex;
                s_cnt[b] = lex;   // first local line of bucket b
                for (uint32_t l = 0; l < ln[q]; ++l) s_lb[lex + l] = (uint16_t)b;
            }
            lex += ln[q];
            rex += cnt[q];
        }
        __syncthreads();
        // scatter the tile's records by bucket
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const bool ok = code[j] != 0xffffffffu;
            const uint32_t b = ok ? code[j] >> 16 : 0u;
            const uint32_t p = ok ? s_off[b] + (code[j] & 0xffffu) : (uint32_t)TILE;
            *(ll2 *)&s_rec[2 * p] = ll2{R.k[j], R.v[j]};
        }
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid * BPT + q;
            if (b < NB_) s_gl[b] = (uint32_t)(at[q] < cap ? at[q] : cap) / 8;
        }
        __syncthreads();
        // write whole lines: lane = (line, slot); virtual position v of bucket b's (carry ++ tile records)
        const uint32_t lines = ltot;
        for (uint32_t x = tid; x < lines * 8; x += T) {
            const uint32_t l = x >> 3, sl = x & 7;
            const uint32_t b = s_lb[l];
            const uint32_t v = (l - s_cnt[b]) * 8 + sl;
            const uint32_t c = s_cc[b];
            const ll2 r = v < c ? *(const ll2 *)&s_car[(b * 8 + v) * 2] : *(const ll2 *)&s_rec[2 * (s_off[b] + v - c)];
            const uint64_t q = (uint64_t)(s_gl[b] + (l - s_cnt[b])) * 8 + sl;
            int64_t *dst = q < cap - TAILCAP ? out + ((uint64_t)(b & 255) * cap + q) * 2 : trash;
            *(ll2 *)dst = r;
        }
        __syncthreads();
        // new carries: the records after the last whole line (from the tile's records when a line was written)
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            const int b = tid * BPT + q;
            if (b >= NB_) continue;
            const uint32_t tot = cnt[q] + cc[q], keep = tot & 7u;
            if (ln[q] == 0) {   // no line: the carry grows by the tile's records
                for (uint32_t i = 0; i < cnt[q]; ++i)
                    *(ll2 *)&s_car[(b * 8 + cc[q] + i) * 2] = *(const ll2 *)&s_rec[2 * (s_off[b] + i)];
            } else {
                for (uint32_t i = 0; i < keep; ++i)
                    *(ll2 *)&s_car[(b * 8 + i) * 2] = *(const ll2 *)&s_rec[2 * (s_off[b] + (tot - keep + i) - cc[q])];
            }
            s_cc[b] = (uint8_t)keep;
        }
        __syncthreads();
    };
    int64_t tile = (int64_t)blockIdx.x * TILE;
    A.load(key, ts, val, n, tile, tid);
    for (; tile < n; tile += 2 * tstride) {
        B.load(key, ts, val, n, tile + tstride, tid);
        tile_fn(A, tile);
        if (tile + tstride >= n) break;
        A.load(key, ts, val, n, tile + 2 * tstride, tid);
        tile_fn(B, tile + tstride);
    }
    // carries -> each bucket's tail region, the last TAILCAP records of its region (tail cursors at 512 * CSTR)
    for (int b = tid; b < NB_; b += T) {
        const uint32_t c = s_cc[b];
        if (!c) continue;
        const unsigned long long base = atomicAdd(&cursor[(512 + (b & 255)) * CSTR], (unsigned long long)c);
        for (uint32_t i = 0; i < c; ++i)
            *(ll2 *)(out + ((uint64_t)(b & 255) * cap + (cap - TAILCAP) + base + i) * 2) = *(const ll2 *)&s_car[(b * 8 + i) * 2];
    }
}

// per-bucket (count, key sum, value sum) of the batch buffer
__global__ void check_kernel(const int64_t *out, uint64_t cap, const unsigned long long *cursor,
                             unsigned long long *res) {
    const int b = blockIdx.x;
    unsigned long long slots = cursor[b * CSTR], tail = cursor[(512 + b) * CSTR];
    if (slots > cap) slots = cap;
    unsigned long long c = 0, sk = 0, sv = 0;
    for (unsigned long long s = threadIdx.x; s < slots; s += blockDim.x) {
        c++;
        sk += (unsigned long long)out[((uint64_t)b * cap + s) * 2];
        sv += (unsigned long long)out[((uint64_t)b * cap + s) * 2 + 1];
    }
    for (unsigned long long s = threadIdx.x; s < tail && s < TAILCAP; s += blockDim.x) {
        c++;
        sk += (unsigned long long)out[((uint64_t)b * cap + cap - TAILCAP + s) * 2];
        sv += (unsigned long long)out[((uint64_t)b * cap + cap - TAILCAP + s) * 2 + 1];
    }
    atomicAdd(&res[b * 3], c);
    atomicAdd(&res[b * 3 + 1], sk);
    atomicAdd(&res[b * 3 + 2], sv);
}

struct Bufs {
    int64_t *k, *t, *v, *out;
    unsigned long long *cur, *res;
    int64_t n;
    uint64_t cap;
};

typedef void (*Launch)(const Bufs &, int grid, hipStream_t);

template <int T, int PER, bool V2, bool PIPE, int WPS, int NBX = 256, bool CLS = false, bool STATS = false>
void launch(const Bufs &B, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k1_kernel<T, PER, V2, PIPE, WPS, NBX, CLS, STATS>), dim3(grid), dim3(T), 0, s, B.k, B.t, B.v, B.n, (int64_t)0,
                       (int64_t)1000000, B.cur, B.cap, B.out);
}

template <int T, int PER, int NBX, bool CLS>
void launch_wc(const Bufs &B, int grid, hipStream_t s) {
    hipLaunchKernelGGL((wc_kernel<T, PER, NBX, CLS>), dim3(grid), dim3(T), 0, s, B.k, B.t, B.v, B.n, (int64_t)0,
                       (int64_t)1000000, B.cur, B.cap, B.out);
}

static std::vector<unsigned long long> host_ref;

static double run(const char *name, Launch L, const Bufs &B, int grid, int reps) {
    hipStream_t s = 0;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    double tot = 0;
    for (int r = 0; r < reps + 3; ++r) {
        CHECK(hipMemsetAsync(B.cur, 0, 1024 * CSTR * 8, s));
        CHECK(hipEventRecord(e0, s));
        L(B, grid, s);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) tot += ms;
    }
    CHECK(hipMemset(B.res, 0, NB * 3 * 8));
    hipLaunchKernelGGL(check_kernel, dim3(NB), dim3(256), 0, 0, B.out, B.cap, B.cur, B.res);
    std::vector<unsigned long long> got(NB * 3);
    CHECK(hipMemcpy(got.data(), B.res, NB * 3 * 8, hipMemcpyDeviceToHost));
    const bool ok = got == host_ref;
    const double us = tot / reps * 1e3;
    printf("%-28s grid %5d  %8.1f us  %6.2f TB/s (40 B/rec)  %s\n", name, grid, us, B.n * 40.0 / (us * 1e-6) / 1e12,
           ok ? "OK" : "MISMATCH");
    fflush(stdout);
    return us;
}

int main(int argc, char **argv) {
    Bufs B{};
    B.n = 16666666;
    const uint64_t per_b = B.n / NB;
    B.cap = (per_b + per_b / 8 + 4096) & ~63ull;
    CHECK(hipMalloc(&B.k, B.n * 8 + 64));
    CHECK(hipMalloc(&B.t, B.n * 8 + 64));
    CHECK(hipMalloc(&B.v, B.n * 8 + 64));
    CHECK(hipMalloc(&B.out, (size_t)NB * B.cap * 16 > (size_t)B.n * 16 ? (size_t)NB * B.cap * 16 : (size_t)B.n * 16));
    CHECK(hipMalloc(&B.cur, 1024 * CSTR * 8 + 4096 * 2 * 64 * 8));   // cursors, stats, then trash lines
    CHECK(hipMalloc(&B.res, NB * 3 * 8));
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
        printf("%-28s grid %5d  %8.1f us  %6.2f TB/s (40 B/rec)\n", "stream", 4096, us, B.n * 40.0 / (us * 1e-6) / 1e12);
    }
    const int reps = 10;
    run("lds 256x16 V2", launch<256, 16, true, false, 2>, B, 512, reps);
    run("lds 256x16 V2 nb512 cls st", launch<256, 16, true, false, 2, 512, true, true>, B, 512, reps);
    run("pipe 512x8 V2", launch<512, 8, true, true, 2>, B, 256, reps);
    run("pipe 512x8 V2 nb512 cls st", launch<512, 8, true, true, 2, 512, true, true>, B, 256, reps);
    run("wc 512x8", launch_wc<512, 8, 256, false>, B, 256, reps);
    run("wc 512x8 nb512 cls", launch_wc<512, 8, 512, true>, B, 256, reps);
    run("wc 1024x4 nb512 cls", launch_wc<1024, 4, 512, true>, B, 256, reps);
    return 0;
}
