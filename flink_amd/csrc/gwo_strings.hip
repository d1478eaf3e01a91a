// gwo_strings.hip -- the String-key dictionary (kernels; host side: gwo_strings.cpp).
//
// A String-keyed stream is keyed by the String itself (KeyGroupRangeAssignment.java:60-73 hashes
// String.hashCode; the heap state table keys entries by the String).  The window kernels key their tables by
// int64, so a handle interns every distinct String into an HBM dictionary and keys the state by its id:
//   id = (uint32)String.hashCode << 32 | sequence number
// -- the high half is what every key-group computation reads (gwo_hash.h key_hash_code, kind 2).
//
// Dictionary: open-addressed slots of 8 words, keyed by a 64-bit fingerprint of the UTF-16 code units; the
// code units themselves sit in an append-only arena.  A batch is interned in three launches, so no lane ever
// waits on another lane's write:
//   claim    every record claims (or finds) its fingerprint's slot; for a slot not yet published, the
//            smallest record index wins it (atomicMax of ~index)
//   publish  each winner takes a sequence number and arena space, copies its code units, publishes the id
//   resolve  every record reads its slot's id and compares its code units with the arena's copy: a mismatch
//            is a true fingerprint collision, counted so the host rejects the batch (never a wrong key)
#include "gwo_device.h"
#include "gwo_strings.h"

namespace gwo {

// JDK String.hashCode (h = 31 * h + c, wrapping) and a 64-bit fingerprint (FNV-1a over code units, then the
// splitmix64 finaliser, never 0) of one String.
__device__ __forceinline__ void string_hashes(const uint16_t *chars, int64_t b, int64_t e, uint32_t &h, uint64_t &fp) {
    uint32_t hc = 0;
    uint64_t x = 0xcbf29ce484222325ull;
    for (int64_t i = b; i < e; ++i) {
        const uint32_t u = chars[i];
        hc = 31u * hc + u;
        x = (x ^ u) * 0x100000001b3ull;
    }
    x ^= (uint64_t)(e - b) * 0x9E3779B97F4A7C15ull;
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    h = hc;
    fp = x | 1ull;
}

__device__ __forceinline__ uint64_t dict_probe(const DictDesc &d, uint64_t fp) {
    uint64_t s = (fp >> 7) & d.mask;
    while (true) {
        unsigned long long *w = d.slots + s * DS_WORDS;
        const unsigned long long prev = atomicCAS(&w[DS_FP], 0ull, (unsigned long long)fp);
        if (prev == 0ull || prev == fp) return s;
        s = (s + 1) & d.mask;
    }
}

__global__ __launch_bounds__(256) void dict_claim_kernel(const uint16_t *__restrict__ chars,
                                                         const int64_t *__restrict__ offsets, int64_t n, DictDesc d,
                                                         uint32_t *rec_slot, uint32_t *rec_hash) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += step) {
        uint32_t h;
        uint64_t fp;
        string_hashes(chars, offsets[r], offsets[r + 1], h, fp);
        const uint64_t s = dict_probe(d, fp);
        unsigned long long *w = d.slots + s * DS_WORDS;
        if (__hip_atomic_load(&w[DS_PUB], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
            atomicMax(&w[DS_WIN], ~(unsigned long long)r);   // the smallest record index wins
        rec_slot[r] = (uint32_t)s;
        rec_hash[r] = h;
    }
}

__global__ __launch_bounds__(256) void dict_publish_kernel(const uint16_t *__restrict__ chars,
                                                           const int64_t *__restrict__ offsets, int64_t n, DictDesc d,
                                                           const uint32_t *rec_slot, const uint32_t *rec_hash) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += step) {
        unsigned long long *w = d.slots + (uint64_t)rec_slot[r] * DS_WORDS;
        if (w[DS_PUB] != 0 || w[DS_WIN] != ~(unsigned long long)r) continue;
        const int64_t b = offsets[r], len = offsets[r + 1] - b;
        const unsigned long long seq = atomicAdd(&d.ctr[0], 1ull);
        const unsigned long long at = atomicAdd(&d.ctr[1], (unsigned long long)len);
        if (seq >= d.idx_cap || at + (uint64_t)len > d.arena_cap) {   // the host sizes both: cannot happen
            atomicAdd(&d.ctr[3], 1ull);
            continue;
        }
        for (int64_t i = 0; i < len; ++i) d.arena[at + i] = chars[b + i];
        d.idx_off[seq] = (int64_t)at;
        d.idx_len[seq] = len;
        w[DS_ID] = ((unsigned long long)rec_hash[r] << 32) | seq;
        w[DS_OFF] = at;
        w[DS_LEN] = (unsigned long long)len;
        w[DS_PUB] = 1;
    }
}

__global__ __launch_bounds__(256) void dict_resolve_kernel(const uint16_t *__restrict__ chars,
                                                           const int64_t *__restrict__ offsets, int64_t n, DictDesc d,
                                                           const uint32_t *rec_slot, int64_t *ids) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += step) {
        const unsigned long long *w = d.slots + (uint64_t)rec_slot[r] * DS_WORDS;
        const int64_t b = offsets[r], len = offsets[r + 1] - b;
        bool same = w[DS_PUB] != 0 && (int64_t)w[DS_LEN] == len;
        for (int64_t i = 0; same && i < len; ++i) same = d.arena[w[DS_OFF] + i] == chars[b + i];
        if (!same) atomicAdd(&d.ctr[2], 1ull);
        ids[r] = (int64_t)w[DS_ID];
    }
}

// Growth: every published slot re-inserted by fingerprint into the (zeroed) larger table.
__global__ __launch_bounds__(256) void dict_rehash_kernel(const unsigned long long *old_slots, uint64_t old_cap,
                                                          DictDesc d) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < (int64_t)old_cap; s += step) {
        const unsigned long long *o = old_slots + (uint64_t)s * DS_WORDS;
        if (o[DS_FP] == 0) continue;
        unsigned long long *w = d.slots + dict_probe(d, o[DS_FP]) * DS_WORDS;
        for (int i = 1; i < DS_WORDS; ++i) w[i] = o[i];
    }
}

static inline int dict_grid(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

void launch_dict_intern(const uint16_t *chars, const int64_t *offsets, int64_t n, const DictDesc &d,
                        uint32_t *rec_slot, uint32_t *rec_hash, int64_t *ids, hipStream_t s) {
    hipLaunchKernelGGL(dict_claim_kernel, dim3(dict_grid(n)), dim3(256), 0, s, chars, offsets, n, d, rec_slot, rec_hash);
    hipLaunchKernelGGL(dict_publish_kernel, dim3(dict_grid(n)), dim3(256), 0, s, chars, offsets, n, d, rec_slot,
                       rec_hash);
    hipLaunchKernelGGL(dict_resolve_kernel, dim3(dict_grid(n)), dim3(256), 0, s, chars, offsets, n, d, rec_slot, ids);
}

void launch_dict_rehash(const unsigned long long *old_slots, uint64_t old_cap, const DictDesc &d, hipStream_t s) {
    hipLaunchKernelGGL(dict_rehash_kernel, dim3(dict_grid((int64_t)old_cap)), dim3(256), 0, s, old_slots, old_cap, d);
}

}  // namespace gwo
