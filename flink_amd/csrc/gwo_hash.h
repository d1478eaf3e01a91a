// gwo_hash.h -- Flink's key hashing (bit-exact) and the log layout's partition digit hash, shared by the
// gfx950 kernels and the host runtime (checkpoint restore groups rows on the host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gwo {

// ---- Flink hashing (bit-exact) -----------------------------------------------------------------
__device__ __host__ inline int32_t long_hash_code(int64_t v) {  // JDK Long.hashCode
    return (int32_t)(uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32));
}
// kind 0 Long, 1 Integer, 2 String: a String key travels as its dictionary id, whose high 32 bits are the
// String.hashCode (gwo_strings.hip)
__device__ __host__ inline int32_t key_hash_code(int64_t v, int kind) {
    return kind == 1 ? (int32_t)v : kind == 2 ? (int32_t)(uint32_t)((uint64_t)v >> 32) : long_hash_code(v);
}
__device__ __host__ inline int32_t bit_mix(int32_t in) {  // MathUtils.java:191-198
    uint32_t x = (uint32_t)in;
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 13;
    x *= 0xc2b2ae35u;
    x ^= x >> 16;
    return (int32_t)x;
}
__device__ __host__ inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __host__ inline int32_t murmur_hash(int32_t code) {  // MathUtils.java:134-154
    uint32_t c = (uint32_t)code;
    c *= 0xcc9e2d51u;
    c = rotl32(c, 15);
    c *= 0x1b873593u;
    c = rotl32(c, 13);
    c = c * 5u + 0xe6546b64u;
    c ^= 4u;
    int32_t r = bit_mix((int32_t)c);
    if (r >= 0) return r;
    if (r != (int32_t)0x80000000) return -r;
    return 0;
}
// KeyGroupRangeAssignment.java:60-73 (murmur_hash is non-negative, so a power-of-two maxParallelism --
// the default 128 and every C4 setting -- is a mask, not a 32-bit division)
__device__ __host__ inline int32_t key_group(int64_t key, int kind, int32_t max_par) {
    const int32_t m = murmur_hash(key_hash_code(key, kind));
    return (max_par & (max_par - 1)) == 0 ? (m & (max_par - 1)) : m % max_par;
}

// Partition digit hash of the log layout (K1 and pass 2; the fire never recomputes a record's
// partition): two 32-bit multiplies whose sum's top bits carry every key bit, ~4 instructions instead of
// part_hash's ~24.  Independent of the fire's election hash (gwo_log.hip slot_mix: other multipliers).
// A skewed key set only costs capacity re-runs and slow-path partitions, never a wrong result.
__device__ __host__ inline uint32_t digit_hash(int64_t key) {
    return (uint32_t)key * 0xCC9E2D51u + (uint32_t)((uint64_t)key >> 32) * 0x1B873593u;
}

}  // namespace gwo
