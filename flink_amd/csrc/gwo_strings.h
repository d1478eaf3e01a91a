// gwo_strings.h -- the String-key dictionary shared by gwo_strings.hip (kernels) and gwo_strings.cpp (host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gwo {

enum : int { DS_FP = 0, DS_WIN = 1, DS_ID = 2, DS_OFF = 3, DS_LEN = 4, DS_PUB = 5, DS_WORDS = 8 };

struct DictDesc {
    unsigned long long *slots;   // cap * DS_WORDS words, zero = free
    uint64_t mask;
    uint16_t *arena;             // code units of every interned String
    uint64_t arena_cap;
    int64_t *idx_off;            // per sequence number: arena offset and length (the id -> String map)
    int64_t *idx_len;
    uint64_t idx_cap;
    unsigned long long *ctr;     // [0] Strings, [1] arena units used, [2] collisions, [3] capacity misses
};

void launch_dict_intern(const uint16_t *chars, const int64_t *offsets, int64_t n, const DictDesc &d,
                        uint32_t *rec_slot, uint32_t *rec_hash, int64_t *ids, hipStream_t s);
void launch_dict_rehash(const unsigned long long *old_slots, uint64_t old_cap, const DictDesc &d, hipStream_t s);

}  // namespace gwo
