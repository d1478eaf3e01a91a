/*
 * jsem.h -- Java semantics shared by the C restatements of WindowOperator (oracle/window_oracle*.c) -- TEST INFRASTRUCTURE.
 * Long arithmetic wraps (two's complement); MathUtils.murmurHash / bitMix (flink-core/.../util/MathUtils.java:
 * 134-198); KeyGroupRangeAssignment.assignToKeyGroup over Long.hashCode (flink-runtime/.../state/
 * KeyGroupRangeAssignment.java:60-73); WindowOperator.cleanupTime (WindowOperator.java:639-646).
 */
#ifndef ORACLE_JSEM_H
#define ORACLE_JSEM_H
#include <stdint.h>

#define LMIN ((int64_t)0x8000000000000000LL)
#define LMAX ((int64_t)0x7fffffffffffffffLL)

static inline int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

static inline int32_t bit_mix(int32_t in) {
    uint32_t x = (uint32_t)in;
    x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
    return (int32_t)x;
}
static inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline int32_t murmur(int32_t code) {
    uint32_t c = (uint32_t)code;
    c *= 0xcc9e2d51u; c = rotl(c, 15); c *= 0x1b873593u; c = rotl(c, 13); c = c * 5u + 0xe6546b64u; c ^= 4u;
    int32_t r = bit_mix((int32_t)c);
    if (r >= 0) return r;
    if (r != (int32_t)0x80000000) return -r;
    return 0;
}
static inline int32_t key_group(int64_t k, int32_t maxp) {
    return murmur((int32_t)(uint32_t)((uint64_t)k ^ ((uint64_t)k >> 32))) % maxp;
}
static inline int64_t cleanup_time(int64_t max_ts, int64_t lateness) {
    int64_t c = jadd(max_ts, lateness);
    return c >= max_ts ? c : LMAX;
}

/* TimeWindow.getWindowStartWithOffset (TimeWindow.java:271-273): Java's truncating '%' */
static inline int64_t window_start(int64_t t, int64_t offset, int64_t size) {
    return jsub(t, jadd(jsub(t, offset), size) % size);
}

#endif
