// gwo_strings.cpp -- host side of the String-key dictionary (kernels and layout: gwo_strings.hip / .h).
//
// The dictionary lives in HBM; the host keeps a mirror of the id -> String map (the arena and the per-id
// offsets, appended after every batch that interned new Strings) so that output, side-output and checkpoint
// rows can be turned back into Strings without a device round trip (gwo_key_strings).
#include <algorithm>
#include <cstring>
#include <vector>

#include "gwo_handle.h"
#include "gwo_strings.h"

namespace gwo {

struct StrDict {
    DevBuf slots, arena, idx_off, idx_len, ctr, rec_slot, rec_hash, ids, chars, offsets;
    uint64_t cap = 0, count = 0, arena_used = 0, arena_cap = 0, idx_cap = 0;
    std::vector<uint16_t> h_arena;   // mirror of arena[0, arena_used)
    std::vector<int64_t> h_off, h_len;   // mirror of idx_off / idx_len [0, count)
    DictDesc desc() const {
        DictDesc d;
        d.slots = (unsigned long long *)slots.ptr;
        d.mask = cap - 1;
        d.arena = (uint16_t *)arena.ptr;
        d.arena_cap = arena_cap;
        d.idx_off = (int64_t *)idx_off.ptr;
        d.idx_len = (int64_t *)idx_len.ptr;
        d.idx_cap = idx_cap;
        d.ctr = (unsigned long long *)ctr.ptr;
        return d;
    }
};

void Handle::dict_free() {
    if (!dict) return;
    for (DevBuf *b : {&dict->slots, &dict->arena, &dict->idx_off, &dict->idx_len, &dict->ctr, &dict->rec_slot,
                      &dict->rec_hash, &dict->ids, &dict->chars, &dict->offsets})
        b->release();
    delete dict;
    dict = nullptr;
}

// Grows a device buffer that holds `used` bytes of live data to at least `need` bytes, keeping the data.
static gwo_status grow_keep(Handle &h, DevBuf &b, size_t used, size_t need) {
    if (b.bytes >= need) return GWO_OK;
    DevBuf nb;
    size_t bytes = std::max(need, b.bytes * 2);
    GWO_TRY(h.dalloc(&nb.ptr, bytes));
    nb.bytes = bytes;
    if (used) GWO_TRY(h.hipcheck(hipMemcpyAsync(nb.ptr, b.ptr, used, hipMemcpyDeviceToDevice, h.stream), "dict grow"));
    GWO_TRY(h.hipcheck(hipStreamSynchronize(h.stream), "dict grow"));
    b.release();
    b = nb;
    return GWO_OK;
}

// Interns n Strings (UTF-16 code units chars[offsets[i] .. offsets[i + 1])); *ids points at n device ids, valid
// until the next intern.
gwo_status Handle::intern_utf16(const uint16_t *chars, const int64_t *offsets, int64_t n, const int64_t **ids) {
    if (cfg.key_kind != GWO_KEY_STRING) return fail(GWO_ERR_INVALID_ARGUMENT, "String keys need key_kind GWO_KEY_STRING");
    if (!dict) dict = new StrDict();
    StrDict &D = *dict;
    // offsets on the device; every offset is validated on the host first (the claim, publish and resolve kernels
    // read chars[offsets[i] .. offsets[i + 1]) unchecked: an interior offset past offsets[n] would read beyond the
    // staged code units)
    int64_t first_last[2];
    const int64_t *d_off = offsets;
    const int64_t *h_off = offsets;
    std::vector<int64_t> off_copy;
    if (is_device_ptr(offsets)) {
        off_copy.resize((size_t)n + 1);
        GWO_TRY(hipcheck(copy_out(off_copy.data(), offsets, (size_t)(n + 1) * 8, stream), "offsets"));
        h_off = off_copy.data();
    }
    if (h_off[0] < 0) return fail(GWO_ERR_INVALID_ARGUMENT, "String key offsets must be non-negative and non-decreasing");
    for (int64_t i = 0; i < n; ++i)
        if (h_off[i + 1] < h_off[i])
            return fail(GWO_ERR_INVALID_ARGUMENT, "String key offsets must be non-negative and non-decreasing");
    first_last[0] = h_off[0];
    first_last[1] = h_off[n];
    if (!is_device_ptr(offsets)) {
        GWO_TRY(ensure_buf(D.offsets, (size_t)(n + 1) * 8));
        GWO_TRY(hipcheck(copy_in(D.offsets.ptr, offsets, (size_t)(n + 1) * 8, stream), "stage offsets"));
        d_off = (const int64_t *)D.offsets.ptr;
    }
    const uint64_t units = (uint64_t)first_last[1];
    const uint16_t *d_chars = chars;
    if (units > 0 && !is_device_ptr(chars)) {
        GWO_TRY(ensure_buf(D.chars, units * 2));
        GWO_TRY(hipcheck(copy_in(D.chars.ptr, chars, units * 2, stream), "stage chars"));
        d_chars = (const uint16_t *)D.chars.ptr;
    }
    // capacity: slots at load <= 1/2, arena and id index for every String of the batch being new
    if (D.count + (uint64_t)n >= (1ull << 32)) return fail(GWO_ERR_CAPACITY, "more than 2^32 distinct String keys");
    uint64_t ncap = std::max<uint64_t>(D.cap, 1024);
    while (2 * (D.count + (uint64_t)n) > ncap) ncap <<= 1;
    if (ncap != D.cap) {
        DevBuf ns;
        GWO_TRY(dalloc(&ns.ptr, ncap * DS_WORDS * 8));
        ns.bytes = ncap * DS_WORDS * 8;
        GWO_TRY(hipcheck(hipMemsetAsync(ns.ptr, 0, ns.bytes, stream), "dict slots"));
        if (!D.ctr.ptr) {
            GWO_TRY(ensure_buf(D.ctr, 32));
            GWO_TRY(hipcheck(hipMemsetAsync(D.ctr.ptr, 0, 32, stream), "dict counters"));
        }
        const uint64_t old_cap = D.cap;
        DevBuf old = D.slots;
        D.slots = ns;
        D.cap = ncap;
        if (old_cap) {
            launch_dict_rehash((const unsigned long long *)old.ptr, old_cap, D.desc(), stream);
            GWO_TRY(launch_ok("dict rehash"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "dict rehash"));
        }
        old.release();
    }
    GWO_TRY(grow_keep(*this, D.arena, D.arena_used * 2, (D.arena_used + units + 1) * 2));
    D.arena_cap = D.arena.bytes / 2;
    GWO_TRY(grow_keep(*this, D.idx_off, D.count * 8, (D.count + (uint64_t)n + 1) * 8));
    GWO_TRY(grow_keep(*this, D.idx_len, D.count * 8, (D.count + (uint64_t)n + 1) * 8));
    D.idx_cap = std::min(D.idx_off.bytes, D.idx_len.bytes) / 8;
    GWO_TRY(ensure_buf(D.rec_slot, (size_t)std::max<int64_t>(n, 1) * 4));
    GWO_TRY(ensure_buf(D.rec_hash, (size_t)std::max<int64_t>(n, 1) * 4));
    GWO_TRY(ensure_buf(D.ids, (size_t)std::max<int64_t>(n, 1) * 8));
    GWO_TRY(hipcheck(hipMemsetAsync((char *)D.ctr.ptr + 16, 0, 16, stream), "dict errors"));
    launch_dict_intern(d_chars, d_off, n, D.desc(), (uint32_t *)D.rec_slot.ptr, (uint32_t *)D.rec_hash.ptr,
                       (int64_t *)D.ids.ptr, stream);
    GWO_TRY(launch_ok("dict intern"));
    unsigned long long c[4];
    GWO_TRY(hipcheck(hipMemcpyAsync(c, D.ctr.ptr, 32, hipMemcpyDeviceToHost, stream), "dict counters"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "dict intern"));
    if (c[3]) return poison(GWO_ERR_HIP, "String dictionary: a new key found no room (sizing error)");
    // mirror the new Strings (also when the batch is rejected below: interned Strings stay valid)
    if (c[0] > D.count) {
        const uint64_t old_count = D.count, old_used = D.arena_used;
        D.h_off.resize(c[0]);
        D.h_len.resize(c[0]);
        D.h_arena.resize(c[1]);
        GWO_TRY(hipcheck(copy_out(D.h_off.data() + old_count, (int64_t *)D.idx_off.ptr + old_count,
                                  (c[0] - old_count) * 8, stream), "dict mirror"));
        GWO_TRY(hipcheck(copy_out(D.h_len.data() + old_count, (int64_t *)D.idx_len.ptr + old_count,
                                  (c[0] - old_count) * 8, stream), "dict mirror"));
        if (c[1] > old_used)
            GWO_TRY(hipcheck(copy_out(D.h_arena.data() + old_used, (uint16_t *)D.arena.ptr + old_used,
                                      (c[1] - old_used) * 2, stream), "dict mirror"));
        D.count = c[0];
        D.arena_used = c[1];
    }
    if (c[2]) return fail(GWO_ERR_UNSUPPORTED, "two distinct String keys share a 64-bit fingerprint (%llu records)",
                          c[2]);
    *ids = (const int64_t *)D.ids.ptr;
    return GWO_OK;
}

gwo_status Handle::key_strings(const int64_t *ids, int64_t n, int64_t *offsets_out, uint16_t *chars_out,
                               int64_t chars_cap, int64_t *chars_needed) {
    std::vector<int64_t> hid;
    const int64_t *src = ids;
    if (n > 0 && is_device_ptr(ids)) {
        hid.resize(n);
        GWO_TRY(hipcheck(copy_out(hid.data(), ids, (size_t)n * 8, stream), "ids"));   // (ordered behind this handle's fires)
        src = hid.data();
    }
    const uint64_t count = dict ? dict->count : 0;
    int64_t total = 0;
    offsets_out[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t seq = (uint64_t)src[i] & 0xffffffffull;
        if (seq >= count) return fail(GWO_ERR_INVALID_ARGUMENT, "id %lld is no String key of this handle", (long long)src[i]);
        total += dict->h_len[seq];
        offsets_out[i + 1] = total;
    }
    if (chars_needed) *chars_needed = total;
    if (!chars_out) return GWO_OK;
    if (chars_cap < total) return fail(GWO_ERR_CAPACITY, "key strings need %lld code units", (long long)total);
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t seq = (uint64_t)src[i] & 0xffffffffull;
        memcpy(chars_out + offsets_out[i], dict->h_arena.data() + dict->h_off[seq], (size_t)dict->h_len[seq] * 2);
    }
    return GWO_OK;
}

}  // namespace gwo
