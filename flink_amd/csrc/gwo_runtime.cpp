// gwo_runtime.cpp -- host side of the C ABI declared in include/gwo.h.
//
// One gwo_handle is one WindowOperator subtask (WindowOperator.java:100) whose keyed window state
// lives in HBM.  Host code here only does bookkeeping that the reference keeps in its timer
// service and state table directory: which per-window tables exist, their capacities, which fire
// at a watermark (InternalTimerServiceImpl.advanceWatermark, :268-278).  Every per-record and
// per-entry operation runs in the gfx950 kernels of gwo_kernels.hip / gwo_slide.hip / gwo_session.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/gwo.h"
#include "gwo_handle.h"
#include "gwo_log_state.h"

using namespace gwo;

namespace gwo {

const char *status_str(gwo_status s) {
    switch (s) {
        case GWO_OK: return "GWO_OK";
        case GWO_ERR_INVALID_ARGUMENT: return "GWO_ERR_INVALID_ARGUMENT";
        case GWO_ERR_NO_TIMESTAMP: return "GWO_ERR_NO_TIMESTAMP";
        case GWO_ERR_KEY_GROUP: return "GWO_ERR_KEY_GROUP";
        case GWO_ERR_OUT_OF_MEMORY: return "GWO_ERR_OUT_OF_MEMORY";
        case GWO_ERR_HIP: return "GWO_ERR_HIP";
        case GWO_ERR_UNSUPPORTED: return "GWO_ERR_UNSUPPORTED";
        case GWO_ERR_MERGE_LATE: return "GWO_ERR_MERGE_LATE";
        case GWO_ERR_COMM: return "GWO_ERR_COMM";
        case GWO_ERR_STATE: return "GWO_ERR_STATE";
        case GWO_ERR_CAPACITY: return "GWO_ERR_CAPACITY";
    }
    return "GWO_ERR_UNKNOWN";
}

gwo_status Handle::fail(gwo_status s, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = std::string(status_str(s)) + ": " + buf;
    return s;
}

gwo_status Handle::poison(gwo_status s, const char *what) {
    poisoned = true;
    poison_status = s;
    err = std::string(status_str(s)) + ": " + what;
    return s;
}

// ---- device memory -------------------------------------------------------------------------------
gwo_status Handle::dalloc(void **p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(GWO_ERR_OUT_OF_MEMORY, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    }
    return GWO_OK;
}

// Waits for an event by polling it (no blocking runtime wait: its wake-up latency varies widely
// between hosts, and the fire's completion is on the watermark's critical path).
gwo_status Handle::spin_event(hipEvent_t ev, const char *what) {
    while (true) {
        hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return GWO_OK;
        if (e != hipErrorNotReady) return hipcheck(e, what);
        for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
    }
}

gwo_status Handle::hipcheck(hipError_t e, const char *what) {
    if (e == hipSuccess) return GWO_OK;
    (void)hipGetLastError();
    return poison(GWO_ERR_HIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
}

gwo_status Handle::ensure_buf(DevBuf &b, size_t bytes) {
    if (b.bytes >= bytes) return GWO_OK;
    if (b.ptr) {
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "sync before realloc"));
        (void)hipFree(b.ptr);
        b.ptr = nullptr;
        b.bytes = 0;
    }
    size_t nb = std::max(bytes, b.bytes * 2);
    GWO_TRY(dalloc(&b.ptr, nb));
    b.bytes = nb;
    return GWO_OK;
}

// Counter slots for table occupancy (one device array, so one D2H copy reads all of them).
int Handle::take_counter() {
    for (size_t i = 0; i < counter_used.size(); ++i)
        if (!counter_used[i]) {
            counter_used[i] = 1;
            return (int)i;
        }
    return -1;
}

gwo_status Handle::alloc_table(uint64_t cap, Table &t) {
    // pool first: released tables are clean (fire/rehash reset every entry they touch)
    auto it = pool.find(cap);
    if (it != pool.end()) {
        t.base = it->second;
        pool.erase(it);
    } else {
        void *p = nullptr;
        size_t words = (size_t)cap * plan.stride + plan.stride;  // + side slot
        gwo_status s = dalloc(&p, words * 8);
        if (s != GWO_OK) {
            // return pooled memory to the allocator and retry once
            trim_pool();
            GWO_TRY(dalloc(&p, words * 8));
        }
        t.base = (int64_t *)p;
        launch_fill(t.base, cap + 1, plan, stream);  // side slot is entry `cap`: flag word 0 = EMPTY
        GWO_TRY(launch_ok("fill"));
        // the side slot's flag must read 0 (not EMPTY): reset its first word
        GWO_TRY(hipcheck(hipMemsetAsync(t.base + cap * plan.stride, 0, 8, stream), "side slot init"));
    }
    t.cap = cap;
    t.side = t.base + cap * plan.stride;
    t.counter = take_counter();
    if (t.counter < 0) return fail(GWO_ERR_OUT_OF_MEMORY, "too many live windows/panes (> %zu)", counter_used.size());
    t.occ = 0;
    return ctr_zero(t.counter);
}

gwo_status Handle::ctr_read(int c, uint64_t *v) {
    GWO_TRY(hipcheck(hipMemcpyAsync(h_counters + (size_t)c * GWO_OCC_WORDS, ctr(c), GWO_OCC_WORDS * 8,
                                    hipMemcpyDeviceToHost, stream), "occ"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "occ sync"));
    *v = ctr_host(c);
    return GWO_OK;
}

void Handle::release_table(Table &t) {
    if (t.counter >= 0) counter_used[t.counter] = 0;
    pool.emplace(t.cap, t.base);
    t.base = nullptr;
    t.counter = -1;
}

void Handle::trim_pool() {
    (void)hipStreamSynchronize(stream);
    for (auto &kv : pool) (void)hipFree(kv.second);
    pool.clear();
}

TableDesc Handle::desc(const Table &t) const {
    TableDesc d;
    d.base = t.base;
    d.side = t.side;
    d.occ = ctr(t.counter);
    d.mask = t.cap - 1;
    return d;
}

static uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Make sure table `u` can take `incoming` more entries at load <= kMaxLoad; grow by rehash.
gwo_status Handle::ensure_table(long long u, uint64_t incoming) {
    auto it = tables.find(u);
    uint64_t want_min = std::max<uint64_t>(kMinCap, next_pow2((uint64_t)((double)(incoming) / kInitLoad) + 1));
    if (cfg.expected_keys > 0)
        want_min = std::max<uint64_t>(want_min, next_pow2((uint64_t)((double)cfg.expected_keys / kInitLoad) + 1));
    if (it == tables.end()) {
        // a new window / pane starts at the size the last retired one grew to: a unit's records arrive over
        // several batches (disorder), and sizing by the first batch's share alone rehashes every unit once
        want_min = std::max<uint64_t>(want_min, recent_cap);
        Table t;
        GWO_TRY(alloc_table(want_min, t));
        // tumbling: a window created after the watermark passed its end only receives re-fire records
        // (EventTimeTrigger.onElement FIREs them; no maxTs timer, WindowOperator.java:393-410)
        if (cfg.assigner == GWO_ASSIGNER_TUMBLING &&
            (int64_t)((uint64_t)unit_start(u) + (uint64_t)cfg.size - 1) <= wm)
            t.fired = true;
        tables.emplace(u, t);
        return GWO_OK;
    }
    Table &t = it->second;
    if ((double)(t.occ + incoming) <= kMaxLoad * (double)t.cap) return GWO_OK;
    uint64_t ncap = next_pow2((uint64_t)((double)(t.occ + incoming) / kInitLoad) + 1);
    Table nt;
    GWO_TRY(alloc_table(ncap, nt));
    launch_rehash(desc(t), t.cap, desc(nt), plan, stream);
    GWO_TRY(launch_ok("rehash"));
    // the side slot moves by copy (flag + words)
    GWO_TRY(hipcheck(hipMemcpyAsync(nt.side, t.side, (size_t)plan.stride * 8, hipMemcpyDeviceToDevice, stream),
                     "side copy"));
    GWO_TRY(reset_side(t));
    // occupancy moves with the entries
    GWO_TRY(hipcheck(hipMemcpyAsync(ctr(nt.counter), ctr(t.counter), GWO_OCC_WORDS * 8, hipMemcpyDeviceToDevice, stream),
                     "occ copy"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "rehash"));
    nt.occ = t.occ;
    nt.fired = t.fired;
    release_table(t);
    it->second = nt;
    return GWO_OK;
}

gwo_status Handle::launch_ok(const char *what) { return hipcheck(hipGetLastError(), what); }

// side slot := [flag 0, identity words] (copied from the pinned identity entry built at init)
gwo_status Handle::reset_side(const Table &t) {
    return hipcheck(hipMemcpyAsync(t.side, h_ident_side, (size_t)plan.stride * 8, hipMemcpyHostToDevice, stream),
                    "side reset");
}

// Reads every live table's occupancy counter (one D2H copy).
gwo_status Handle::read_occupancy() {
    int hi = 0;
    for (auto &kv : tables) hi = std::max(hi, kv.second.counter + 1);
    for (auto &kv : rdone) hi = std::max(hi, kv.second.counter + 1);
    for (auto &kv : aux_tables) hi = std::max(hi, kv.counter + 1);
    if (hi == 0) return hipcheck(hipStreamSynchronize(stream), "occ sync");   // callers rely on the sync
    GWO_TRY(hipcheck(hipMemcpyAsync(h_counters, d_counters, (size_t)hi * GWO_OCC_WORDS * 8, hipMemcpyDeviceToHost, stream),
                     "occ"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "occ sync"));
    for (auto &kv : tables) kv.second.occ = ctr_host(kv.second.counter);
    for (auto &kv : rdone) kv.second.occ = ctr_host(kv.second.counter);
    for (auto &t : aux_tables) t.occ = ctr_host(t.counter);
    return GWO_OK;
}

gwo_status Handle::ensure_output(uint64_t extra) {
    if (out_count_dirty) {
        GWO_TRY(hipcheck(hipMemsetAsync(d_out_count, 0, 8, stream), "row counter"));
        out_count_dirty = false;
    }
    uint64_t need = out_rows + extra;
    if ((long long)need <= out.cap) return GWO_OK;
    uint64_t ncap = std::max<uint64_t>(need, (uint64_t)out.cap * 2);
    ncap = std::max<uint64_t>(ncap, 1 << 16);
    int ncols = 3 + rplan.naggs;
    int64_t *cols[7] = {};
    for (int c = 0; c < ncols; ++c) GWO_TRY(dalloc((void **)&cols[c], ncap * 8));
    int64_t *old[7] = {out.key, out.start, out.end, out.res[0], out.res[1], out.res[2], out.res[3]};
    for (int c = 0; c < ncols; ++c) {
        if (old[c] && out_rows)
            GWO_TRY(hipcheck(hipMemcpyAsync(cols[c], old[c], out_rows * 8, hipMemcpyDeviceToDevice, stream), "out grow"));
    }
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "out grow sync"));
    for (int c = 0; c < ncols; ++c)
        if (old[c]) (void)hipFree(old[c]);
    out.key = cols[0];
    out.start = cols[1];
    out.end = cols[2];
    for (int a = 0; a < 4; ++a) out.res[a] = a < rplan.naggs ? cols[3 + a] : nullptr;
    out.cap = (long long)ncap;
    return GWO_OK;
}

// ---- profiling ---------------------------------------------------------------------------------
void Handle::prof_begin(int k, hipStream_t s) {
    if (!profiling || !((prof_mask >> k) & 1u)) return;
    if (!s) s = stream;
    hipEvent_t a, b;
    if (event_pool.size() >= 2) {   // events are recycled: hipEventCreate costs microseconds per call
        a = event_pool.back();
        event_pool.pop_back();
        b = event_pool.back();
        event_pool.pop_back();
    } else {
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
    }
    (void)hipEventRecord(a, s);
    pending_events.push_back({k, a, b, 0});
}
void Handle::prof_end(int k, int64_t items, hipStream_t s) {
    if (!profiling || pending_events.empty()) return;
    if (!s) s = stream;
    auto &pe = pending_events.back();
    if (pe.kernel != k) return;
    (void)hipEventRecord(pe.b, s);
    pe.items = items;
}
gwo_status Handle::prof_collect() {
    if (pending_events.empty()) return GWO_OK;
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "prof sync"));
    if (fire_stream) GWO_TRY(hipcheck(hipStreamSynchronize(fire_stream), "prof sync"));
    if (cb_side) GWO_TRY(hipcheck(hipStreamSynchronize(cb_side), "prof sync"));
    if (logst && logst->split_stream) GWO_TRY(hipcheck(hipStreamSynchronize(logst->split_stream), "prof sync"));
    for (auto &pe : pending_events) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, pe.a, pe.b);
        kstats[pe.kernel].launches++;
        kstats[pe.kernel].ms += ms;
        kstats[pe.kernel].items += pe.items;
        event_pool.push_back(pe.a);
        event_pool.push_back(pe.b);
    }
    pending_events.clear();
    return GWO_OK;
}

// ---- input staging ----------------------------------------------------------------------------
bool is_device_ptr(const void *p) {
    if (!p) return true;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// Columns inside a device allocation seen earlier in the same call need no pointer query: a batch's columns are
// usually slices of one buffer (hipPointerGetAttributes is a runtime call per column).  The ranges are forgotten at
// every call (stage_inputs), so a range the caller freed between calls -- whose addresses a later host allocation
// may take -- is never trusted.
bool Handle::known_device(const void *p, size_t bytes) {
    const uintptr_t a = (uintptr_t)p;
    for (const auto &r : dev_ranges)
        if (a >= r.first && a + bytes <= r.second) return true;
    if (!is_device_ptr(p)) return false;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && size > 0) {
        if (dev_ranges.size() >= 8) dev_ranges.erase(dev_ranges.begin());
        dev_ranges.push_back({(uintptr_t)base, (uintptr_t)base + size});
    } else {
        (void)hipGetLastError();
    }
    return true;
}

gwo_status Handle::stage_inputs(const int64_t *key, const int64_t *ts, const void *val, int64_t n, const int64_t **dk,
                                const int64_t **dt, const int64_t **dv) {
    const void *src[3] = {key, ts, val};
    DevBuf *bufs[3] = {&stage_key, &stage_ts, &stage_val};
    dev_ranges.clear();   // (known_device: only this call's columns are trusted)
    const int64_t **dst[3] = {dk, dt, dv};
    for (int c = 0; c < 3; ++c) {
        if (!src[c]) {
            *dst[c] = nullptr;
            continue;
        }
        if (known_device(src[c], (size_t)n * 8)) {
            *dst[c] = (const int64_t *)src[c];
        } else {
            GWO_TRY(ensure_buf(*bufs[c], (size_t)n * 8));
            GWO_TRY(hipcheck(copy_in(bufs[c]->ptr, src[c], (size_t)n * 8, stream), "stage"));
            *dst[c] = (const int64_t *)bufs[c]->ptr;
        }
    }
    return GWO_OK;
}

// ---- geometry helpers ---------------------------------------------------------------------------
int64_t Handle::unit_start(long long u) const {  // start of window/pane u
    return (int64_t)((uint64_t)u * (uint64_t)geom.unit + (uint64_t)geom.unit_off_mod);
}

WindowGeom Handle::geom_now() const {
    WindowGeom g = geom;
    g.wm = wm;
    return g;
}

// ---- tumbling / pane insert -------------------------------------------------------------------------
// Rows of the batch's re-fire records in directory units [dir_base, dir_base + dir_len) (see
// refire_emit_kernel, gwo_kernels.hip): emitted before the batch's insert, which then adds them.
gwo_status Handle::refire_rows(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const WindowGeom &g,
                               long long dir_base, int dir_len, uint64_t mmax) {
    GWO_TRY(settle_out());   // out_rows is added to below
    std::vector<uint64_t> off(dir_len, 0);
    uint64_t tot = 0;
    for (int d = 0; d < dir_len; ++d) {
        off[d] = tot;
        if (h_dir[d].base) tot += h_dir[d].mask + 2;   // cap entries + the side slot
    }
    if (tot >= (1ull << 32))
        return poison(GWO_ERR_CAPACITY, "allowedLateness re-fire: the re-fired windows' tables exceed 2^32 entries");
    const uint64_t m8 = std::max<uint64_t>(mmax, 1);
    const uint64_t rs_blocks = (m8 + 4095) / 4096;
    // carve: blk[256] u32 | slot_off[dir_len] u64 | r_idx[m] i64 | r_u[m] i64 | before[m][MAX_WORDS] i64 |
    //        r_slot, k1, v1, k2, v2 [m] u32 | hist[256 * rs_blocks] u32
    size_t o_blk = 0, o_off = 1024, o_idx = o_off + (size_t)dir_len * 8;
    o_idx = (o_idx + 255) & ~(size_t)255;
    size_t o_u = o_idx + m8 * 8, o_before = o_u + m8 * 8, o_slot = o_before + m8 * GWO_MAX_WORDS * 8;
    size_t o_k1 = o_slot + m8 * 4, o_v1 = o_k1 + m8 * 4, o_k2 = o_v1 + m8 * 4, o_v2 = o_k2 + m8 * 4;
    size_t o_hist = (o_v2 + m8 * 4 + 255) & ~(size_t)255, total = o_hist + 256 * 4 * rs_blocks;
    GWO_TRY(ensure_buf(refire_buf, total));
    char *b = (char *)refire_buf.ptr;
    GWO_TRY(hipcheck(hipMemcpyAsync(b + o_off, off.data(), (size_t)dir_len * 8, hipMemcpyHostToDevice, stream), "refire"));
    launch_refire_collect(t, n, g, dir_base, dir_len, (uint32_t *)(b + o_blk), (int64_t *)(b + o_idx),
                          (long long *)(b + o_u), stream);
    GWO_TRY(launch_ok("refire collect"));
    std::vector<uint32_t> blk(256);
    GWO_TRY(hipcheck(hipMemcpyAsync(blk.data(), b + o_blk, 256 * 4, hipMemcpyDeviceToHost, stream), "refire count"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "refire count"));
    uint64_t m = 0;
    for (uint32_t c : blk) m += c;
    if (m == 0) return GWO_OK;
    if (m > mmax) return poison(GWO_ERR_HIP, "allowedLateness re-fire: more re-fire records than the scan counted");
    launch_refire_slots(k, (const int64_t *)(b + o_idx), (const long long *)(b + o_u), (int64_t)m, plan,
                        (const TableDesc *)dir_buf.ptr, dir_base, (const uint64_t *)(b + o_off), (uint32_t *)(b + o_slot),
                        (int64_t *)(b + o_before), stream);
    GWO_TRY(launch_ok("refire slots"));
    const int which = radix_sort_pairs((const uint32_t *)(b + o_slot), nullptr, (int64_t)m, 32, (uint32_t *)(b + o_k1),
                                       (uint32_t *)(b + o_v1), (uint32_t *)(b + o_k2), (uint32_t *)(b + o_v2),
                                       (uint32_t *)(b + o_hist), stream);
    GWO_TRY(launch_ok("refire sort"));
    GWO_TRY(ensure_output(m));
    const uint32_t *sk = (const uint32_t *)(b + (which ? o_k2 : o_k1));
    const uint32_t *sp = (const uint32_t *)(b + (which ? o_v2 : o_v1));
    launch_refire_emit(k, v, (const int64_t *)(b + o_idx), (const long long *)(b + o_u), (int64_t)m, sk, sp,
                       (const int64_t *)(b + o_before), plan, rplan, geom.unit, geom.unit_off_mod, geom.unit, out_cols(),
                       stream);
    GWO_TRY(launch_ok("refire emit"));
    out_rows += m;
    return GWO_OK;
}

// Combine path (gather + merge, gwo_kernels.hip): one pass over the batch classifies and pre-aggregates in
// LDS; after the host's checks the merge folds the workgroups' tables into the window tables.  *done = false
// leaves the batch untouched for the two-pass path (window range outside the histogram, side-output growth).
gwo_status Handle::insert_combined(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, bool *done) {
    *done = false;
    WindowGeom g = geom_now();
    g.refire_ok = 1;
    if (!cb_cus) GWO_TRY(hipcheck(hipDeviceGetAttribute(&cb_cus, hipDeviceAttributeMultiprocessorCount, cfg.device), "CUs"));
    const int NW = plan.nwords;
    const int64_t tile = gather_tile();
    if (!cb_max_wg) {
        cb_max_wg = 4 * cb_cus;
        if (const char *e = getenv("GWO_CB_WG")) cb_max_wg = std::max(1, atoi(e));
        if (const char *e = getenv("GWO_CB_OVERLAP")) cb_overlap = atoi(e) != 0;
    }
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>((n + tile - 1) / tile, (int64_t)cb_max_wg));
    int S = 2048;   // (4096-slot tables where one workgroup per CU leaves the LDS: no faster, the merge slower)
    while (S > 256 && gather_lds_bytes(S, NW) > 65536 + 512) S >>= 1;   // (tables + 64 spare words)
    // pipelined: a dump region per readback slot (the previous batch's merge may still read the other one)
    const bool pipe = combine_pipe_ok(k, t, v);
    const bool overlap = pipe && cb_overlap && use_combine_spec;
    const size_t key_region = ((size_t)G * 2 * S * 8 + (size_t)G * 4 + 255) & ~(size_t)255;
    const size_t acc_region = ((size_t)G * 2 * S * NW * 8 + 255) & ~(size_t)255;
    if (overlap && cb_side && (cb_dump_key.bytes < 2 * key_region || cb_dump_acc.bytes < 2 * acc_region)) {
        // (a reallocation frees the regions in-flight work may read)
        GWO_TRY(hipcheck(hipStreamSynchronize(cb_side), "gather sync"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "merge sync"));
    }
    GWO_TRY(ensure_buf(cb_dump_key, 2 * key_region));
    GWO_TRY(ensure_buf(cb_dump_acc, 2 * acc_region));
    GWO_TRY(ensure_buf(cb_ovf, (size_t)n * 4));
    if (!cb_ctr.ptr) {   // counters and statistics shards start reset; every gather leaves them reset
        GWO_TRY(ensure_buf(cb_ctr, 32));   // listed-record count, finished workgroups, speculation verdict
        GWO_TRY(hipcheck(hipMemsetAsync(cb_ctr.ptr, 0, 32, stream), "combine counters"));
        const int words = gather_stat_words();
        std::vector<unsigned long long> init((size_t)words, 0ull);
        for (int q = 0; q < words / 80; ++q) {
            init[(size_t)q * 80 + 7] = 0x7fffffffffffffffull;   // min / max words of each shard
            init[(size_t)q * 80 + 8] = 0x8000000000000000ull;
        }
        GWO_TRY(ensure_buf(cb_blk, (size_t)words * 8));
        GWO_TRY(hipcheck(hipMemcpy(cb_blk.ptr, init.data(), (size_t)words * 8, hipMemcpyHostToDevice), "shards"));
    }
    if (!cb_go.ptr) {   // per-slot verdicts [0..1] and per-slot {hint, incs} [2..9]
        GWO_TRY(ensure_buf(cb_go, 16 * 8));
        GWO_TRY(hipcheck(hipMemsetAsync(cb_go.ptr, 0, 16 * 8, stream), "verdicts"));
    }
    const int slot = cb_pend.active ? (cb_pend.slot ^ 1) : 0;
    CombineArgs a{};
    a.dump_key = (int64_t *)((char *)cb_dump_key.ptr + (size_t)slot * key_region);
    a.dump_acc = (int64_t *)((char *)cb_dump_acc.ptr + (size_t)slot * acc_region);
    a.dump_used = (uint32_t *)(a.dump_key + (size_t)G * 2 * S);
    a.ovf = (uint32_t *)cb_ovf.ptr;
    a.ovf_count = (unsigned long long *)cb_ctr.ptr;
    a.ovf_cap = (unsigned long long)n;
    a.blk = (unsigned long long *)cb_blk.ptr;
    if (!cb_arr.ptr) {
        GWO_TRY(ensure_buf(cb_arr, ARR_WORDS * 8));
        GWO_TRY(hipcheck(hipMemsetAsync(cb_arr.ptr, 0, ARR_WORDS * 8, stream), "arrival counters"));
    }
    a.done = (unsigned long long *)cb_arr.ptr;
    if (!cb_rb) {
        GWO_TRY(hipcheck(hipHostMalloc((void **)&cb_rb, 2 * CB_RB_WORDS * 8, hipHostMallocCoherent | hipHostMallocMapped),
                         "combine readback"));
        memset(cb_rb, 0, 2 * CB_RB_WORDS * 8);
        GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&cb_rb_dev, cb_rb, 0), "combine readback"));
        GWO_TRY(hipcheck(hipEventCreateWithFlags(&cb_ev, hipEventDisableTiming), "event"));
    }
    // pipelined: the previous batch's readback slot is still unread, so this batch takes the other one
    unsigned long long *const rb = cb_rb + (size_t)slot * CB_RB_WORDS;
    a.rb = cb_rb_dev + (size_t)slot * CB_RB_WORDS;
    a.seq = ++cb_seq;
    a.chain = cb_pend.active ? 1 : 0;
    a.side_enabled = side_enabled();
    // tumbling: the next window's table exists before its first records arrive (sized like the last retired one),
    // so the batch that crosses into it keeps the speculative merge (and a pipelined batch needs no redo)
    bool main_work = false;   // work queued on the handle's stream by this call that the gather must follow
    if (cfg.assigner == GWO_ASSIGNER_TUMBLING && use_combine_spec && !slide && tables.count(hist_hint) &&
        !tables.count(hist_hint + 1)) {
        const __int128 end1 = (__int128)(hist_hint + 2) * cfg.size + geom.unit_off_mod;   // window hint + 1's end
        if (end1 - 1 > (__int128)wm && end1 <= (__int128)(int64_t)0x7fffffffffffffffLL &&
            end1 - cfg.size >= (__int128)(int64_t)0x8000000000000000LL) {
            GWO_TRY(ensure_table(hist_hint + 1, 0));
            main_work = true;
        }
    }
    Table *hint_tab[2] = {nullptr, nullptr};
    for (int j = 0; j < 2; ++j) {
        auto it = tables.find(hist_hint + j);
        if (it != tables.end()) {
            hint_tab[j] = &it->second;
            a.occ[j] = ctr(it->second.counter);
        }
    }
    a.S = S;
    a.sbits = __builtin_ctz((unsigned)S);
    a.hint = hist_hint;
    a.full_range = cfg.key_group_start == 0 && cfg.key_group_end == cfg.max_parallelism - 1;
    if (cfg.assigner == GWO_ASSIGNER_TUMBLING) {   // windows hint .. hint + 3 (gwo_log.cpp log_thresholds)
        const __int128 size = cfg.size, s0 = (__int128)hist_hint * size + (__int128)geom.unit_off_mod;
        const __int128 lo = (__int128)(int64_t)0x8000000000000000LL, hi = (__int128)(int64_t)0x7fffffffffffffffLL;
        if (s0 > lo && s0 + 4 * size <= hi && s0 >= (__int128)geom.offset - size) {
            for (int j = 0; j <= 4; ++j) a.bound[j] = (int64_t)(s0 + (__int128)j * size);
            for (int j = 0; j < 4; ++j) {
                const int64_t max_ts = (int64_t)(s0 + (__int128)(j + 1) * size - 1);
                const uint32_t c = cleanup_time_host(max_ts) <= g.wm ? 1u : (max_ts <= g.wm ? 2u : 0u);
                a.cls |= c << (2 * j);
            }
            a.thr_ok = 1;
        }
    }
    a.side_cap = side_cap;
    // speculation (tumbling): the merge is queued behind the gather with the hint tables as its directory and
    // runs iff the gather's verdict says the batch needs nothing from the host
    const bool spec = use_combine_spec && cfg.assigner == GWO_ASSIGNER_TUMBLING;
    if (spec) {
        std::vector<TableDesc> sd(2, TableDesc{});
        for (int j = 0; j < 2; ++j)
            if (hint_tab[j]) {
                sd[j] = desc(*hint_tab[j]);
                a.cap[j] = hint_tab[j]->cap;
            }
        if (cb_spec_base != hist_hint || cb_spec_host.size() != 2 ||
            memcmp(cb_spec_host.data(), sd.data(), 2 * sizeof(TableDesc)) != 0) {
            GWO_TRY(ensure_buf(cb_spec_dir, 2 * sizeof(TableDesc)));
            GWO_TRY(hipcheck(hipMemcpyAsync(cb_spec_dir.ptr, sd.data(), 2 * sizeof(TableDesc), hipMemcpyHostToDevice,
                                            stream), "spec dir"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "spec dir"));
            cb_spec_host = sd;
            cb_spec_base = hist_hint;
        }
        a.go = (uint32_t *)((unsigned long long *)cb_ctr.ptr + 2);
        a.go_prev = a.go;
        if (pipe) {   // a verdict word per slot: the merge behind this gather reads this batch's
            a.go = (uint32_t *)((unsigned long long *)cb_go.ptr + slot);
            a.go_prev = (const uint32_t *)((unsigned long long *)cb_go.ptr + (slot ^ 1));
        }
        if (overlap) {
            a.inc_out = (unsigned long long *)cb_go.ptr + 2 + 4 * slot;
            if (cb_pend.active) a.inc_prev = (const unsigned long long *)cb_go.ptr + 2 + 4 * (slot ^ 1);
        }
    }
    static const int cb_trace = getenv("GWO_CB_TRACE") ? atoi(getenv("GWO_CB_TRACE")) : 0;
    std::vector<unsigned long long> h_dbg;
    if (cb_trace && !pipe) {   // phase times of this gather on the device wall clock (debugging aid)
        GWO_TRY(ensure_buf(cb_dbg, (size_t)G * 64));
        GWO_TRY(hipcheck(hipMemset(cb_dbg.ptr, 0, (size_t)G * 64), "trace"));
        a.dbg = (unsigned long long *)cb_dbg.ptr;
    }
    hipStream_t gs = stream;
    if (overlap) {
        if (!cb_side) {
            GWO_TRY(hipcheck(hipStreamCreateWithFlags(&cb_side, hipStreamNonBlocking), "gather stream"));
            for (hipEvent_t *e : {&cb_ev_main, &cb_ev_gather, &cb_ev_merge[0], &cb_ev_merge[1]})
                GWO_TRY(hipcheck(hipEventCreateWithFlags(e, hipEventDisableTiming), "event"));
            // a producer stream named to gwo_wait_stream before this point is covered by the join below
        }
        if (!cb_pend.active || main_work) {   // a chain starts (or a table was made): behind the handle's stream
            GWO_TRY(hipcheck(hipEventRecord(cb_ev_main, stream), "event"));
            GWO_TRY(hipcheck(hipStreamWaitEvent(cb_side, cb_ev_main, 0), "event wait"));
        }
        if (cb_merge_rec[slot])   // the merge that read this dump slot and verdict word
            GWO_TRY(hipcheck(hipStreamWaitEvent(cb_side, cb_ev_merge[slot], 0), "event wait"));
        gs = cb_side;
    }
    hp(16);
    prof_begin(GWO_KERNEL_SCAN, gs);
    launch_gather(k, t, v, n, g, plan, a, G, d_stats, (int64_t *)side_key.ptr, (int64_t *)side_ts.ptr,
                  (int64_t *)side_val.ptr, d_side_count, side_enabled() ? side_cap : 0, side_enabled(), gs);
    GWO_TRY(launch_ok("gather"));
    prof_end(GWO_KERNEL_SCAN, n, gs);
    if (spec) {
        if (overlap) {   // the merge follows its gather (and, on the handle's stream, every earlier merge)
            GWO_TRY(hipcheck(hipEventRecord(cb_ev_gather, gs), "event"));
            GWO_TRY(hipcheck(hipStreamWaitEvent(stream, cb_ev_gather, 0), "event wait"));
        }
        RingDesc none{};
        none.lo = 1;
        none.hi = 0;
        prof_begin(GWO_KERNEL_INSERT);
        launch_merge(k, t, v, g, plan, a, G, 0, (const TableDesc *)cb_spec_dir.ptr, hist_hint, 2, none, a.go, stream);
        GWO_TRY(launch_ok("merge"));
        prof_end(GWO_KERNEL_INSERT, n);
        hp(17);
        if (overlap) {
            GWO_TRY(hipcheck(hipEventRecord(cb_ev_merge[slot], stream), "event"));
            cb_merge_rec[slot] = true;
        }
    }
    if (pipe) {
        CbPend Q;
        Q.active = true;
        Q.k = k;
        Q.t = t;
        Q.v = v;
        Q.n = n;
        Q.slot = slot;
        Q.seq = a.seq;
        Q.hint = hist_hint;
        Q.wm = g.wm;
        Q.side = overlap;
        *done = true;
        if (!cb_pend.active) {   // nothing to complete: return with this batch in flight
            cb_pend = Q;
            return GWO_OK;
        }
        bool go = false;
        GWO_TRY(combine_resolve_pending(&go));   // the previous batch (usually finished by now)
        hp(18);
        if (go) {
            cb_pend = Q;
            return GWO_OK;
        }
        // the previous batch's verdict was no, so this one's is too (chained) and neither merge ran: once this
        // gather is done, both go through the regular path, in order
        GWO_TRY(spin_seq(rb + CB_RB_SEQ, Q.seq, "gather", gs));
        const CbPend P = cb_pend;   // (a turned-down batch stays in cb_pend)
        cb_pend.active = false;
        cb_redo = true;
        gwo_status s = insert_windowed(P.k, P.t, P.v, P.n);
        if (s == GWO_OK) s = insert_windowed(k, t, v, n);
        cb_redo = false;
        return s;
    }
    // the gather's last workgroup writes the readback block, sequence word last: spin on it (the stream is polled
    // now and then so that a failed launch cannot spin forever)
    GWO_TRY(spin_seq(rb + CB_RB_SEQ, a.seq, "gather"));
    if (cb_trace) {   // per phase: the latest workgroup end (from the first start) and the longest in-workgroup time
        h_dbg.resize((size_t)G * 8);
        GWO_TRY(hipcheck(hipMemcpy(h_dbg.data(), cb_dbg.ptr, (size_t)G * 64, hipMemcpyDeviceToHost), "trace"));
        unsigned long long t0 = ~0ull, last_start = 0, abs_[8] = {}, rel[8] = {};
        for (int w = 0; w < G; ++w) {
            const unsigned long long *d = &h_dbg[(size_t)w * 8];
            t0 = std::min(t0, d[0]);
            last_start = std::max(last_start, d[0]);
        }
        for (int w = 0; w < G; ++w) {
            const unsigned long long *d = &h_dbg[(size_t)w * 8];
            for (int q = 1; q < 8; ++q)
                if (d[q]) {
                    abs_[q] = std::max(abs_[q], d[q] - t0);
                    rel[q] = std::max(rel[q], d[q] - d[0]);
                }
        }
        fprintf(stderr, "[cb] G=%d: loads %.2f/%.2f classified %.2f/%.2f lds %.2f/%.2f counted %.2f/%.2f arrived "
                "%.2f/%.2f tail %.2f (us from the first start / within a workgroup); last start %.2f\n", G,
                abs_[6] / 100.0, rel[6] / 100.0, abs_[1] / 100.0, rel[1] / 100.0, abs_[2] / 100.0, rel[2] / 100.0,
                abs_[3] / 100.0, rel[3] / 100.0, abs_[4] / 100.0, rel[4] / 100.0, abs_[5] / 100.0,
                (last_start - t0) / 100.0);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    BatchStats &hs = *h_stats;
    memcpy(h_stats, rb, sizeof(BatchStats));
    *h_scalar = rb[CB_RB_SIDE];
    for (int j = 0; j < 2; ++j)
        if (hint_tab[j]) hint_tab[j]->occ = rb[CB_RB_OCC + j];   // exact: the previous merges are done
    if (spec && rb[CB_RB_GO]) {   // the speculative merge ran: only the bookkeeping is left
        if (side_enabled()) side_rows = side_rows_committed = *h_scalar;
        else late_dropped += hs.late;
        for (int j = 0; j < 2; ++j)   // upper bound until the next readback
            if (hint_tab[j] && hs.hist[j]) hint_tab[j]->occ += std::min<uint64_t>(hs.hist[j], hs.distinct[j]);
        adapt_preagg(hs.accepted, hs.distinct[0] + hs.distinct[1] + hs.overflow);
        hist_hint = hs.min_idx;
        for (auto &kv : tables) kv.second.dirty = true;
        *done = true;
        return GWO_OK;
    }
    if (hs.bad_ts) return poison(GWO_ERR_NO_TIMESTAMP,
                                 "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time "
                                 "characteristic set to 'ProcessingTime', or did you forget to call "
                                 "'DataStream.assignTimestampsAndWatermarks(...)'?");
    if (hs.bad_range) return poison(GWO_ERR_UNSUPPORTED, "sliding windows: timestamp < offset - slide (Java '%' quirk "
                                                         "range) is outside the pane restatement");
    if (hs.bad_kg)
        return poison(GWO_ERR_KEY_GROUP, ("Key group of key " + std::to_string(hs.bad_kg_key) +
                                          " is not in KeyGroupRange{startKeyGroup=" + std::to_string(cfg.key_group_start) +
                                          ", endKeyGroup=" + std::to_string(cfg.key_group_end) + "}.").c_str());
    auto give_back = [&]() -> gwo_status {   // nothing of the batch stays: the two-pass path takes it
        if (!side_enabled()) return GWO_OK;
        *h_scalar = side_rows_committed;
        GWO_TRY(hipcheck(hipMemcpyAsync(d_side_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "side reset"));
        return hipcheck(hipStreamSynchronize(stream), "side reset");
    };
    const uint64_t side_now = side_enabled() ? *h_scalar : 0;
    if (side_enabled() && (long long)side_now > side_cap) return give_back();
    const long long lo = hs.min_idx, hi = hs.max_idx;
    if (hs.accepted > 0 && (lo < hist_hint || hi >= hist_hint + GWO_HIST_BINS || hs.hist_out)) {
        hist_hint = lo;
        return give_back();
    }
    if (side_enabled()) side_rows = side_rows_committed = side_now;
    else late_dropped += hs.late;
    *done = true;
    if (hs.accepted == 0) return GWO_OK;
    const int dir_len = (int)(hi - lo + 1);
    for (int d = 0; d < dir_len; ++d) {   // a table outside the readback's two: refresh every occupancy
        auto it = tables.find(lo + d);
        if (it != tables.end() && &it->second != hint_tab[0] && &it->second != hint_tab[1]) {
            GWO_TRY(read_occupancy());
            break;
        }
    }
    h_dir.assign(dir_len, TableDesc{});
    for (int d = 0; d < dir_len; ++d) {
        const long long r = lo + d - hist_hint;
        uint64_t cnt = hs.hist[r];
        if (!cnt) continue;
        if (r < 2) cnt = std::min<uint64_t>(cnt, hs.distinct[r] + hs.overflow);   // keys, not records
        GWO_TRY(ensure_table(lo + d, cnt));
    }
    for (int d = 0; d < dir_len; ++d) {
        auto it = tables.find(lo + d);
        if (it != tables.end()) h_dir[d] = desc(it->second);
    }
    if (slide) GWO_TRY(slide_prepare_insert(lo, dir_len, hs.hist + (lo - hist_hint)));
    // the directory lives in its own buffer and is uploaded only when it changed (usually once per window)
    if (cb_dir_base != lo || cb_dir_host.size() != (size_t)dir_len ||
        memcmp(cb_dir_host.data(), h_dir.data(), dir_len * sizeof(TableDesc)) != 0) {
        GWO_TRY(ensure_buf(cb_dir, dir_len * sizeof(TableDesc)));
        GWO_TRY(hipcheck(hipMemcpyAsync(cb_dir.ptr, h_dir.data(), dir_len * sizeof(TableDesc), hipMemcpyHostToDevice,
                                        stream), "dir"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "dir"));   // h_dir is reused
        cb_dir_host = h_dir;
        cb_dir_base = lo;
    }
    if (hs.refire) {   // rows read the windows' state before the batch: before the merge
        GWO_TRY(ensure_buf(dir_buf, dir_len * sizeof(TableDesc)));
        GWO_TRY(hipcheck(hipMemcpyAsync(dir_buf.ptr, h_dir.data(), dir_len * sizeof(TableDesc), hipMemcpyHostToDevice,
                                        stream), "dir"));
        if (slide) GWO_TRY(slide_refire_rows(k, t, v, n, g, hs.refire));
        else GWO_TRY(refire_rows(k, t, v, n, g, lo, dir_len, hs.refire));
    }
    prof_begin(GWO_KERNEL_INSERT);
    launch_merge(k, t, v, g, plan, a, G, hs.overflow, (const TableDesc *)cb_dir.ptr, lo, dir_len, ring_desc(), nullptr,
                 stream);
    GWO_TRY(launch_ok("merge"));
    prof_end(GWO_KERNEL_INSERT, n);
    adapt_preagg(hs.accepted, hs.distinct[0] + hs.distinct[1] + hs.overflow);
    hist_hint = lo;
    for (auto &kv : tables) kv.second.dirty = true;
    return GWO_OK;
}


// The combine path may pipeline a batch (gwo_set_pipelined_submit): tumbling windows with the speculative merge,
// allowedLateness 0, no side output, one GPU, caller-owned device columns (staged host input is reused by the next
// batch), and not while a turned-down batch is being redone.
bool Handle::combine_pipe_ok(const int64_t *k, const int64_t *t, const int64_t *v) const {
    return pipe_submit && !cb_redo && use_combine_spec && cfg.assigner == GWO_ASSIGNER_TUMBLING && !slide && !sess &&
           !logst && cfg.allowed_lateness == 0 && !side_enabled() && !comm && !dict &&
           (const void *)k != stage_key.ptr && (const void *)t != stage_ts.ptr && (!v || (const void *)v != stage_val.ptr);
}

// Reads the pending batch's readback.  Yes: its speculative merge ran -- the bookkeeping insert_combined does after
// its own wait.  No: nothing of the batch was applied (cb_pend keeps it for the caller to redo).
gwo_status Handle::combine_resolve_pending(bool *go) {
    const CbPend &P = cb_pend;
    const unsigned long long *rb = cb_rb + (size_t)P.slot * CB_RB_WORDS;
    GWO_TRY(spin_seq(rb + CB_RB_SEQ, P.seq, "gather", P.side ? cb_side : nullptr));
    *go = rb[CB_RB_GO] != 0;
    if (!*go) return GWO_OK;
    memcpy(h_stats, rb, sizeof(BatchStats));
    const BatchStats &hs = *h_stats;
    for (int j = 0; j < 2; ++j) {
        auto it = tables.find(P.hint + j);
        if (it == tables.end()) continue;
        it->second.occ = rb[CB_RB_OCC + j];   // exact before the batch's merge, plus an upper bound of its keys
        if (hs.hist[j]) it->second.occ += std::min<uint64_t>(hs.hist[j], hs.distinct[j]);
    }
    late_dropped += hs.late;
    adapt_preagg(hs.accepted, hs.distinct[0] + hs.distinct[1] + hs.overflow);
    hist_hint = hs.min_idx;
    for (auto &kv : tables) kv.second.dirty = true;
    cb_pend.active = false;
    return GWO_OK;
}

gwo_status Handle::flush_pending() {
    GWO_TRY(combine_flush());
    return sess_resolve();
}

gwo_status Handle::combine_flush() {
    if (!cb_pend.active) return GWO_OK;
    bool go = false;
    GWO_TRY(combine_resolve_pending(&go));
    if (go) return GWO_OK;
    const CbPend P = cb_pend;
    cb_pend.active = false;
    cb_redo = true;
    const gwo_status s = insert_windowed(P.k, P.t, P.v, P.n);
    cb_redo = false;
    return s;
}

// Spins on a host-mapped readback block's sequence word (written last by a kernel's final workgroup).  After
// GWO_SPIN_QUERY_US (default 500 us) of spinning, and as often again, the producing stream is queried, so that a
// failed launch cannot spin forever: an idle stream whose word never arrived is an error.  (A query every 1024
// pauses -- ~30 us -- put a marker into the stream behind the queued kernels: the next batch's first kernel then
// started ~6 us after the one before it, C2's gather; profiles/r06_experiments.txt.)  Ends with an acquire fence:
// the block's other words are visible.
gwo_status Handle::spin_seq(const unsigned long long *word, unsigned long long seq, const char *what,
                            hipStream_t producer) {
    volatile const unsigned long long *w = word;
    if (*w == seq) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        return GWO_OK;
    }
    static const long long query_ns = 1000ll * (getenv("GWO_SPIN_QUERY_US") ? atoll(getenv("GWO_SPIN_QUERY_US")) : 500);
    auto now_ns = [] {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count();
    };
    long long next = now_ns() + query_ns;
    for (unsigned it = 1; *w != seq; ++it) {
        if ((it & 255) == 0 && now_ns() >= next) {
            hipError_t e = hipStreamQuery(producer ? producer : stream);
            if (e != hipSuccess && e != hipErrorNotReady) return hipcheck(e, what);
            if (e == hipSuccess && *w != seq) return poison(GWO_ERR_HIP, "readback sequence word not visible after completion");
            next = now_ns() + query_ns;
        }
        __builtin_ia32_pause();
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return GWO_OK;
}

// Speculative two-pass insert (tumbling tables without pre-aggregation, e.g. C1's 10K-record batches over 10K
// keys): the scan and the direct insert are queued together; the scan's last workgroup checks what the host
// would check after reading the statistics (errors, re-fires, units outside the hint tables, table load) and
// the insert runs only on its verdict.  The host spins on the scan's host-mapped readback block -- no stream
// synchronisation, no statistics copies, no directory upload while the hint tables stay the same.  *done =
// false: the verdict was no and nothing changed (the side-output count is restored); the caller's path runs.
gwo_status Handle::insert_speculative(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, bool *done) {
    *done = false;
    WindowGeom g = geom_now();
    g.refire_ok = 1;
    // the next window's table exists before its first records arrive (sized like the last retired one), so the
    // batch that crosses into it stays on this path; an empty table fires no rows
    if (tables.count(hist_hint) && !tables.count(hist_hint + 1)) {
        const __int128 end1 = (__int128)(hist_hint + 2) * cfg.size + geom.unit_off_mod;   // window hint + 1's end
        if (end1 - 1 > (__int128)wm && end1 <= (__int128)(int64_t)0x7fffffffffffffffLL &&
            end1 - cfg.size >= (__int128)(int64_t)0x8000000000000000LL)
            GWO_TRY(ensure_table(hist_hint + 1, 0));
    }
    Table *hint_tab[2] = {nullptr, nullptr};
    std::vector<TableDesc> sd(2, TableDesc{});
    ScanSpec sp{};
    for (int j = 0; j < 2; ++j) {
        auto it = tables.find(hist_hint + j);
        if (it == tables.end()) continue;
        hint_tab[j] = &it->second;
        sd[j] = desc(it->second);
        sp.occ[j] = ctr(it->second.counter);
        sp.cap[j] = it->second.cap;
    }
    if (!hint_tab[0] && !hint_tab[1]) return GWO_OK;   // nothing to speculate into: the host sizes the tables
    if (!sp_rb) {
        GWO_TRY(hipcheck(hipHostMalloc((void **)&sp_rb, CB_RB_WORDS * 8, hipHostMallocCoherent | hipHostMallocMapped),
                         "scan readback"));
        memset(sp_rb, 0, CB_RB_WORDS * 8);
        GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&sp_rb_dev, sp_rb, 0), "scan readback"));
        GWO_TRY(hipcheck(hipEventCreateWithFlags(&sp_ev, hipEventDisableTiming), "event"));
        GWO_TRY(ensure_buf(sp_go, 16));
    }
    if (sp_dir_base != hist_hint || sp_dir_host.size() != 2 ||
        memcmp(sp_dir_host.data(), sd.data(), 2 * sizeof(TableDesc)) != 0) {
        GWO_TRY(ensure_buf(sp_dir, 2 * sizeof(TableDesc)));
        GWO_TRY(hipcheck(hipMemcpyAsync(sp_dir.ptr, sd.data(), 2 * sizeof(TableDesc), hipMemcpyHostToDevice, stream),
                         "spec dir"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "spec dir"));   // sd is a local
        sp_dir_host = sd;
        sp_dir_base = hist_hint;
    }
    sp.rb = sp_rb_dev;
    sp.seq = ++sp_seq;
    sp.go = (uint32_t *)sp_go.ptr;
    sp.hint = hist_hint;
    sp.check_kg = !(cfg.key_group_start == 0 && cfg.key_group_end == cfg.max_parallelism - 1);
    // (no init_stats: the scan's last workgroup writes every statistic the verdict reads; the regular path resets
    // the rest before it runs)
    hp(20);
    prof_begin(GWO_KERNEL_SCAN);
    launch_scan(k, t, n, g, hist_hint, d_stats, (int64_t *)side_key.ptr, (int64_t *)side_ts.ptr, (int64_t *)side_val.ptr,
                v, d_side_count, side_enabled() ? side_cap : 0, side_enabled(), d_scan_sh, stream, &sp);
    GWO_TRY(launch_ok("scan"));
    prof_end(GWO_KERNEL_SCAN, n);
    prof_begin(GWO_KERNEL_INSERT);
    launch_insert(k, t, v, n, g, plan, (const TableDesc *)sp_dir.ptr, hist_hint, 2, 0, d_stats, ring_desc(), stream,
                  sp.go);
    GWO_TRY(launch_ok("insert"));
    prof_end(GWO_KERNEL_INSERT, n);
    hp(21);
    GWO_TRY(spin_seq(sp_rb + CB_RB_SEQ, sp.seq, "scan"));
    hp(22);
#define RBW(f) (int)(offsetof(BatchStats, f) / 8)
    const unsigned long long accepted = sp_rb[RBW(accepted)], late = sp_rb[RBW(late)];
    const long long lo = (long long)sp_rb[RBW(min_idx)];
    unsigned long long hist[2] = {sp_rb[RBW(hist)], sp_rb[RBW(hist) + 1]};
#undef RBW
    if (!sp_rb[CB_RB_GO]) {   // the insert exited: the caller's path takes the batch from the start
        if (side_enabled()) {
            *h_scalar = side_rows_committed;
            GWO_TRY(hipcheck(hipMemcpyAsync(d_side_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "side reset"));
            GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side reset"));
        }
        return GWO_OK;
    }
    if (side_enabled()) side_rows = side_rows_committed = sp_rb[CB_RB_SIDE];
    else late_dropped += late;
    for (int j = 0; j < 2; ++j)   // exact before the insert, plus an upper bound of the keys it added
        if (hint_tab[j]) hint_tab[j]->occ = sp_rb[CB_RB_OCC + j] + hist[j];
    adapt_preagg(accepted, 0);
    hist_hint = lo;
    for (auto &kv : tables) kv.second.dirty = true;
    *done = true;
    return GWO_OK;
}

gwo_status Handle::insert_windowed(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n,
                                   const WindowGeom *at) {
    if (cb_pend.active && (at || !use_preagg || !use_combine || n >= (1LL << 31) || !combine_pipe_ok(k, t, v)))
        GWO_TRY(combine_flush());   // a pipelined batch completes before a batch that takes another path
    if (!at && use_preagg && use_combine && n < (1LL << 31)) {
        bool done = false;
        GWO_TRY(insert_combined(k, t, v, n, &done));
        if (done) return GWO_OK;
    }
    if (!at && !use_preagg && use_scan_spec && cfg.assigner == GWO_ASSIGNER_TUMBLING && !slide && !sess) {
        bool done = false;
        GWO_TRY(insert_speculative(k, t, v, n, &done));
        if (done) return GWO_OK;
    }
    WindowGeom g = at ? *at : geom_now();
    const bool count_late = !g.refire_only;   // a refire_only pass: the log's K1 did the late accounting
    // re-fire records (allowedLateness > 0) are emitted per element and inserted
    g.refire_ok = 1;
    uint64_t refire_total = 0;
    bool slide_refired = false;
    long long hist_base = hist_hint;
    bool first_pass = true;
    BatchStats &hs = *h_stats;
    // one scan pass per 64-unit chunk of the batch's unit range (normally exactly one)
    long long lo = 0, hi = -1;
    while (true) {
        init_stats(hist_base);
        prof_begin(GWO_KERNEL_SCAN);
        launch_scan(k, t, n, g, hist_base, d_stats, (int64_t *)side_key.ptr, (int64_t *)side_ts.ptr,
                    (int64_t *)side_val.ptr, v, d_side_count, first_pass && count_late && side_enabled() ? side_cap : 0,
                    first_pass && count_late && side_enabled(), d_scan_sh, stream);
        GWO_TRY(launch_ok("scan"));
        prof_end(GWO_KERNEL_SCAN, n);
        GWO_TRY(hipcheck(hipMemcpyAsync(h_stats, d_stats, sizeof(BatchStats), hipMemcpyDeviceToHost, stream), "stats"));
        GWO_TRY(read_occupancy());  // syncs
        if (debug)
            fprintf(stderr, "[gwo] scan n=%lld base=%lld acc=%llu late=%llu refire=%llu badts=%llu range=%llu min=%lld max=%lld "
                    "hout=%llu h0=%llu h1=%llu wm=%lld\n", (long long)n, hist_base, hs.accepted, hs.late, hs.refire, hs.bad_ts,
                    hs.bad_range, hs.min_idx, hs.max_idx, hs.hist_out, hs.hist[0], hs.hist[1], (long long)g.wm);
        if (first_pass) {
            if (hs.bad_ts) return poison(GWO_ERR_NO_TIMESTAMP,
                                         "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time "
                                         "characteristic set to 'ProcessingTime', or did you forget to call "
                                         "'DataStream.assignTimestampsAndWatermarks(...)'?");
            if (hs.bad_range) return poison(GWO_ERR_UNSUPPORTED,
                                            "sliding windows: timestamp < offset - slide (Java '%' quirk range) is "
                                            "outside the pane restatement");
            refire_total = hs.refire;
            if (!count_late) {
                // late records were counted (or side-output) by the log's K1
            } else if (side_enabled()) {
                GWO_TRY(hipcheck(hipMemcpyAsync(h_scalar, d_side_count, 8, hipMemcpyDeviceToHost, stream), "side count"));
                GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side count sync"));
                side_rows = *h_scalar;
                if ((long long)side_rows > side_cap) {
                    // grow and re-collect this batch's side output (first pass only)
                    side_rows = side_rows_committed;
                    GWO_TRY(grow_side((long long)hs.late + (long long)side_rows_committed));
                    *h_scalar = side_rows;
                    GWO_TRY(hipcheck(hipMemcpyAsync(d_side_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "side reset"));
                    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side reset sync"));
                    continue;
                }
                side_rows_committed = side_rows;
            } else {
                late_dropped += hs.late;
            }
            if (hs.accepted == 0) return GWO_OK;
            lo = hs.min_idx;
            hi = hs.max_idx;
            first_pass = false;
            if (hist_base > lo || hist_base + GWO_HIST_BINS <= lo) {
                hist_base = lo;  // histogram missed the range: rescan this chunk
                continue;
            }
        }
        // process units [hist_base, min(hi, hist_base+63)] with exact per-unit counts
        long long chunk_hi = std::min<long long>(hi, hist_base + GWO_HIST_BINS - 1);
        int dir_len = (int)(chunk_hi - hist_base + 1);
        h_dir.assign(dir_len, TableDesc{});
        for (int d = 0; d < dir_len; ++d) {
            uint64_t cnt = hs.hist[d];
            if (!cnt) continue;
            GWO_TRY(ensure_table(hist_base + d, cnt));
        }
        for (int d = 0; d < dir_len; ++d) {
            auto it = tables.find(hist_base + d);
            if (it != tables.end()) h_dir[d] = desc(it->second);
        }
        if (slide) GWO_TRY(slide_prepare_insert(hist_base, dir_len, hs.hist));
        GWO_TRY(ensure_buf(dir_buf, dir_len * sizeof(TableDesc)));
        GWO_TRY(hipcheck(hipMemcpyAsync(dir_buf.ptr, h_dir.data(), dir_len * sizeof(TableDesc), hipMemcpyHostToDevice,
                                        stream), "dir"));
        if (refire_total && !slide) GWO_TRY(refire_rows(k, t, v, n, g, hist_base, dir_len, refire_total));
        if (refire_total && slide && !slide_refired) {   // whole batch, before its first insert
            GWO_TRY(slide_refire_rows(k, t, v, n, g, refire_total));
            slide_refired = true;
        }
        prof_begin(GWO_KERNEL_INSERT);
        launch_insert(k, t, v, n, g, plan, (const TableDesc *)dir_buf.ptr, hist_base, dir_len, use_preagg, d_stats,
                      ring_desc(), stream);
        GWO_TRY(launch_ok("insert"));
        prof_end(GWO_KERNEL_INSERT, n);
        // key-group violations surface at the next sync (Flink fails the task at that record)
        GWO_TRY(hipcheck(hipMemcpyAsync(&h_stats->bad_kg, &d_stats->bad_kg, 16, hipMemcpyDeviceToHost, stream), "kg"));
        GWO_TRY(hipcheck(hipMemcpyAsync(&h_stats->partials, &d_stats->partials, 8, hipMemcpyDeviceToHost, stream), "p"));
        GWO_TRY(hipcheck(hipStreamSynchronize(stream), "insert"));
        if (hs.bad_kg) {
            long long kg = -1;
            (void)kg;
            return poison(GWO_ERR_KEY_GROUP, ("Key group of key " + std::to_string(hs.bad_kg_key) +
                                              " is not in KeyGroupRange{startKeyGroup=" + std::to_string(cfg.key_group_start) +
                                              ", endKeyGroup=" + std::to_string(cfg.key_group_end) + "}.").c_str());
        }
        adapt_preagg(hs.accepted, hs.partials);
        if (chunk_hi >= hi) break;
        hist_base = chunk_hi + 1;
        // next chunk: skip empty unit ranges by rescanning from the next populated unit
    }
    hist_hint = lo;
    for (auto &kv : tables) kv.second.dirty = true;
    return GWO_OK;
}

void Handle::adapt_preagg(uint64_t accepted, uint64_t partials) {
    // Pre-aggregation pays when a tile folds several records per (key, window); measured by the
    // partials it flushed.  Off: re-probe after 32 batches, backing off (x2 up to 1024 batches) while the probes
    // keep finding no duplicates, so a stream without them stops paying for the probe.
    batches++;
    if (use_preagg) {
        if (accepted > 0 && (double)partials > 0.5 * (double)accepted) {
            use_preagg = 0;
            if (preagg_probing) preagg_probe_every = std::min<uint64_t>(2 * preagg_probe_every, 1024);
            preagg_probe_at = batches + preagg_probe_every;
        } else if (preagg_probing) {
            preagg_probe_every = 32;   // the probe paid: back to the short schedule when it stops paying
        }
        preagg_probing = false;
    } else if (batches >= preagg_probe_at) {
        use_preagg = 1;
        preagg_probing = true;
    }
    if (cfg_preagg >= 0) use_preagg = cfg_preagg;
}

void Handle::init_stats(long long hist_base) {
    BatchStats s;
    memset(&s, 0, sizeof s);
    s.min_idx = 0x7fffffffffffffffLL;
    s.max_idx = (long long)0x8000000000000000LL;
    (void)hist_base;
    *h_stats_init = s;   // pinned; the previous batch's copy has completed (every batch ends in a sync)
    (void)hipMemcpyAsync(d_stats, h_stats_init, sizeof(BatchStats), hipMemcpyHostToDevice, stream);
}

gwo_status Handle::grow_side(long long need) {
    long long ncap = std::max<long long>(need, side_cap * 2);
    ncap = std::max<long long>(ncap, 1024);
    DevBuf nk, nt, nv;
    GWO_TRY(ensure_buf(nk, ncap * 8));
    GWO_TRY(ensure_buf(nt, ncap * 8));
    GWO_TRY(ensure_buf(nv, ncap * 8));
    if (side_rows_committed) {
        GWO_TRY(hipcheck(hipMemcpyAsync(nk.ptr, side_key.ptr, side_rows_committed * 8, hipMemcpyDeviceToDevice, stream), "s"));
        GWO_TRY(hipcheck(hipMemcpyAsync(nt.ptr, side_ts.ptr, side_rows_committed * 8, hipMemcpyDeviceToDevice, stream), "s"));
        GWO_TRY(hipcheck(hipMemcpyAsync(nv.ptr, side_val.ptr, side_rows_committed * 8, hipMemcpyDeviceToDevice, stream), "s"));
    }
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "side grow"));
    side_key.release();
    side_ts.release();
    side_val.release();
    side_key = nk;
    side_ts = nt;
    side_val = nv;
    nk.ptr = nt.ptr = nv.ptr = nullptr;
    side_cap = ncap;
    return GWO_OK;
}

// ---- watermark: tumbling windows ---------------------------------------------------------------
// The exact row count of the last table-layout fire (fire_tumbling): waits for the copy queued behind it.
gwo_status Handle::settle_out() {
    if (!out_stale) return GWO_OK;
    out_stale = false;
    GWO_TRY(spin_event(ev_out, "row count"));
    const uint64_t v = *h_out_cnt;
    if (v > (uint64_t)out.cap) return poison(GWO_ERR_CAPACITY, "fire: more rows than output slots");
    if (discard_stale) {   // discarded while the count was in flight: the rows are gone
        rows_gone += v;
        discard_stale = false;
    } else {
        out_rows = v;
    }
    return GWO_OK;
}

gwo_status Handle::fire_tumbling(int64_t new_wm) {
    // restored emitted entries (rdone) of a window that got no new records by its maxTs: the window stays emitted as
    // restored (re-fires, cleanup)
    for (auto it = rdone.begin(); it != rdone.end();) {
        const int64_t max_ts = (int64_t)((uint64_t)unit_start(it->first) + (uint64_t)cfg.size - 1);
        if (max_ts <= new_wm && !tables.count(it->first)) {
            tables.emplace(it->first, it->second);   // (fired)
            it = rdone.erase(it);
        } else {
            ++it;
        }
    }
    // timers in timestamp order; each window has its maxTs (fire) and cleanup timers
    std::vector<long long> emit, clear;
    for (auto &kv : tables) {
        int64_t start = unit_start(kv.first);
        int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
        int64_t max_ts = (int64_t)((uint64_t)end - 1);
        int64_t cu = cleanup_time_host(max_ts);
        bool do_emit = !kv.second.fired && max_ts <= new_wm;
        bool do_clear = cu <= new_wm;
        if (do_emit) emit.push_back(kv.first);
        if (do_clear) clear.push_back(kv.first);
    }
    if (emit.empty() && clear.empty()) return GWO_OK;
    // the table layout alone (not the log layout's fired-window tables, whose fire counts rows right after):
    // no occupancy read -- output room for every slot of the emitted tables, the row count read back behind the
    // fire kernels (settle_out)
    bool any_rdone = false;
    for (long long u : emit) any_rdone |= rdone.count(u) != 0;
    const bool lazy = !logst && !any_rdone;
    GWO_TRY(settle_out());
    if (!lazy) GWO_TRY(read_occupancy());
    for (long long u : emit)   // room for the restored emitted entries that join the window after its emission
        if (rdone.count(u)) GWO_TRY(ensure_table(u, rdone[u].occ));
    uint64_t extra = 0;
    for (long long u : emit) extra += lazy ? tables[u].cap : tables[u].occ;
    GWO_TRY(ensure_output(extra));
    OutCols o = out;
    o.count = d_out_count;
    for (long long u : emit) {
        Table &t = tables[u];
        bool also_clear = std::find(clear.begin(), clear.end(), u) != clear.end();
        int64_t start = unit_start(u);
        int64_t end = (int64_t)((uint64_t)start + (uint64_t)cfg.size);
        auto rd = rdone.find(u);
        // keys with new records since the restore fire with their restored emitted entries too (existing keys only)
        if (rd != rdone.end()) launch_fold(desc(rd->second), rd->second.cap, desc(t), plan, +1, -1, nullptr, stream, 1);
        prof_begin(GWO_KERNEL_FIRE);
        launch_fire(desc(t), t.cap, plan, rplan, start, end, o, also_clear ? 1 : 0, -1, stream);
        GWO_TRY(launch_ok("fire"));
        prof_end(GWO_KERNEL_FIRE, (int64_t)t.cap);
        if (!lazy) out_rows += t.occ;
        t.fired = true;
        if (rd != rdone.end()) {   // the other restored entries join the (now emitted) window: re-fires, cleanup
            if (!also_clear) launch_fold(desc(rd->second), rd->second.cap, desc(t), plan, +1, -1, nullptr, stream, 2);
            OutCols none = o;
            none.cap = 0;
            GWO_TRY(hipcheck(hipMemsetAsync(d_scratch_count, 0, 8, stream), "z"));
            none.count = d_scratch_count;
            launch_fire(desc(rd->second), rd->second.cap, plan, rplan, 0, 0, none, 1, -1, stream);   // (reset)
            GWO_TRY(launch_ok("restored entries"));
            release_table(rd->second);
            rdone.erase(rd);
            t.dirty = true;
        }
    }
    if (lazy && !emit.empty()) {
        if (!h_out_cnt) {
            GWO_TRY(hipcheck(hipHostMalloc((void **)&h_out_cnt, 8, hipHostMallocDefault), "row count"));
            GWO_TRY(hipcheck(hipEventCreateWithFlags(&ev_out, hipEventDisableTiming), "event"));
        }
        GWO_TRY(hipcheck(hipMemcpyAsync(h_out_cnt, d_out_count, 8, hipMemcpyDeviceToHost, stream), "row count"));
        GWO_TRY(hipcheck(hipEventRecord(ev_out, stream), "row count"));
        out_rows += extra;   // an upper bound until settled
        out_stale = true;
    }
    for (long long u : clear) {
        Table &t = tables[u];
        if (std::find(emit.begin(), emit.end(), u) == emit.end()) {
            // state cleared without emission (already fired at maxTs): reset by a no-output sweep
            OutCols none = o;
            none.cap = 0;
            GWO_TRY(hipcheck(hipMemsetAsync(d_scratch_count, 0, 8, stream), "z"));
            none.count = d_scratch_count;
            launch_fire(desc(t), t.cap, plan, rplan, 0, 0, none, 1, -1, stream);
        }
        recent_cap = t.cap;
        release_table(t);
        tables.erase(u);
    }
    return GWO_OK;
}

int64_t Handle::cleanup_time_host(int64_t max_ts) const {
    int64_t c = (int64_t)((uint64_t)max_ts + (uint64_t)cfg.allowed_lateness);
    return c >= max_ts ? c : (int64_t)0x7fffffffffffffffLL;
}

}  // namespace gwo

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

void gwo_config_init(gwo_config *cfg) {
    memset(cfg, 0, sizeof *cfg);
    cfg->abi_version = GWO_ABI_VERSION;
    cfg->assigner = GWO_ASSIGNER_TUMBLING;
    cfg->num_aggs = 1;
    cfg->aggs[0] = GWO_AGG_SUM;
    cfg->max_parallelism = 128;
    cfg->key_group_start = 0;
    cfg->key_group_end = 127;
}

const char *gwo_status_string(gwo_status s) { return status_str(s); }

gwo_status gwo_create(const gwo_config *cfg, gwo_handle **out) {
    if (!cfg || !out) return GWO_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    Handle *h = new Handle();
    gwo_status s = h->init(*cfg);
    if (s != GWO_OK) {
        // keep the message reachable: hand back the half-built handle only on success
        fprintf(stderr, "gwo_create: %s\n", h->err.c_str());
        delete h;
        return s;
    }
    *out = reinterpret_cast<gwo_handle *>(h);
    return GWO_OK;
}

gwo_status gwo_destroy(gwo_handle *hh) {
    if (!hh) return GWO_ERR_INVALID_ARGUMENT;
    delete reinterpret_cast<Handle *>(hh);
    return GWO_OK;
}

#define H_OR_FAIL                                                            \
    Handle *h = reinterpret_cast<Handle *>(hh);                              \
    if (!h) return GWO_ERR_INVALID_ARGUMENT;                                 \
    if (h->poisoned) return h->poison_status;                                \
    DeviceGuard guard_(h->cfg.device);

gwo_status gwo_submit(gwo_handle *hh, const int64_t *key, const int64_t *ts, const void *value, int64_t n) {
    H_OR_FAIL;
    if (n < 0) return h->fail(GWO_ERR_INVALID_ARGUMENT, "negative record count");
    if (n > 0 && (!key || !ts)) return h->fail(GWO_ERR_INVALID_ARGUMENT, "key/ts columns are required");
    if (n > 0 && !value && h->needs_value) return h->fail(GWO_ERR_INVALID_ARGUMENT, "value column required");
    return h->submit(key, ts, value, n);
}

gwo_status gwo_submit_utf16(gwo_handle *hh, const uint16_t *chars, const int64_t *offsets, const int64_t *ts,
                            const void *value, int64_t n) {
    H_OR_FAIL;
    if (n < 0) return h->fail(GWO_ERR_INVALID_ARGUMENT, "negative record count");
    if (n == 0) return GWO_OK;
    if (!offsets || !ts) return h->fail(GWO_ERR_INVALID_ARGUMENT, "offsets/ts columns are required");
    if (!value && h->needs_value) return h->fail(GWO_ERR_INVALID_ARGUMENT, "value column required");
    const int64_t *ids = nullptr;
    GWO_TRY(h->intern_utf16(chars, offsets, n, &ids));
    return h->submit(ids, ts, value, n);
}

gwo_status gwo_intern_utf16(gwo_handle *hh, const uint16_t *chars, const int64_t *offsets, int64_t n,
                            int64_t *ids_out) {
    H_OR_FAIL;
    if (n < 0 || (n > 0 && (!offsets || !ids_out))) return h->fail(GWO_ERR_INVALID_ARGUMENT, "intern arguments");
    if (n == 0) return GWO_OK;
    const int64_t *ids = nullptr;
    GWO_TRY(h->intern_utf16(chars, offsets, n, &ids));
    return h->hipcheck(copy_out(ids_out, ids, (size_t)n * 8, h->stream), "intern ids");
}

gwo_status gwo_key_strings(gwo_handle *hh, const int64_t *ids, int64_t n, int64_t *offsets_out, uint16_t *chars_out,
                           int64_t chars_cap, int64_t *chars_needed) {
    H_OR_FAIL;
    if (n < 0 || !offsets_out || (n > 0 && !ids)) return h->fail(GWO_ERR_INVALID_ARGUMENT, "key_strings arguments");
    return h->key_strings(ids, n, offsets_out, chars_out, chars_cap, chars_needed);
}

gwo_status gwo_advance_watermark(gwo_handle *hh, int64_t wm) {
    H_OR_FAIL;
    return h->advance_watermark(wm);
}

gwo_status gwo_end_input(gwo_handle *hh) { return gwo_advance_watermark(hh, (int64_t)0x7fffffffffffffffLL); }

gwo_status gwo_output_count(gwo_handle *hh, int64_t *n) {
    H_OR_FAIL;
    if (!n) return GWO_ERR_INVALID_ARGUMENT;
    GWO_TRY(h->poll_fire());   // non-blocking: a fire still running contributes when it completes
    *n = (int64_t)h->out_rows;
    return GWO_OK;
}

gwo_status gwo_rows_emitted(gwo_handle *hh, int64_t *n) {
    H_OR_FAIL;
    if (!n) return GWO_ERR_INVALID_ARGUMENT;
    GWO_TRY(h->finish_fire());
    *n = (int64_t)(h->rows_gone + h->out_rows);
    return GWO_OK;
}

gwo_status gwo_output_view(gwo_handle *hh, gwo_out *cols, int64_t *n) {
    H_OR_FAIL;
    if (!cols || !n) return GWO_ERR_INVALID_ARGUMENT;
    GWO_TRY(h->finish_fire());
    GWO_TRY(h->hipcheck(hipStreamSynchronize(h->stream), "view"));
    cols->key = h->out.key;
    cols->start = h->out.start;
    cols->end = h->out.end;
    for (int a = 0; a < GWO_MAX_AGGS; ++a) cols->result[a] = h->out.res[a];
    *n = (int64_t)h->out_rows;
    return GWO_OK;
}

gwo_status gwo_discard_output(gwo_handle *hh) {
    H_OR_FAIL;
    if (h->out_stale) {   // the rows of a fire still being counted: accounted when the count arrives
        h->discard_stale = true;
        h->out_rows = 0;
        h->out_count_dirty = true;
        return GWO_OK;
    }
    GWO_TRY(h->poll_fire());
    if (h->fire_pending) h->discard_after_fire = true;   // the running fire's rows are dropped when it completes
    h->rows_gone += h->out_rows;
    h->out_rows = 0;
    h->out_count_dirty = true;   // the device row counter is reset before the next fire (ensure_output)
    return GWO_OK;
}

gwo_status gwo_drain(gwo_handle *hh, const gwo_out *cols, int64_t cap, int64_t *n_out) {
    H_OR_FAIL;
    if (!cols || !n_out || cap < 0) return GWO_ERR_INVALID_ARGUMENT;
    return h->drain(cols, cap, n_out);
}

gwo_status gwo_result_dtype(const gwo_handle *hh, int32_t agg, int32_t *dtype) {
    const Handle *h = reinterpret_cast<const Handle *>(hh);
    if (!h || !dtype || agg < 0 || agg >= h->rplan.naggs) return GWO_ERR_INVALID_ARGUMENT;
    int k = h->rplan.kind[agg];
    *dtype = (k == GWO_AGG_AVG || (k != GWO_AGG_COUNT && h->rplan.value_is_f64)) ? GWO_DTYPE_FLOAT64 : GWO_DTYPE_INT64;
    return GWO_OK;
}

gwo_status gwo_late_dropped(gwo_handle *hh, int64_t *count) {
    H_OR_FAIL;
    if (!count) return GWO_ERR_INVALID_ARGUMENT;
    GWO_TRY(h->flush_pending());
    GWO_TRY(h->log_flush());
    *count = (int64_t)h->late_dropped;
    return GWO_OK;
}

gwo_status gwo_side_output_count(gwo_handle *hh, int64_t *n) {
    H_OR_FAIL;
    if (!n) return GWO_ERR_INVALID_ARGUMENT;
    GWO_TRY(h->log_flush());
    *n = (int64_t)h->side_rows_committed;
    return GWO_OK;
}

gwo_status gwo_drain_side_output(gwo_handle *hh, const gwo_side_out *cols, int64_t cap, int64_t *n_out) {
    H_OR_FAIL;
    if (!cols || !n_out || cap < 0) return GWO_ERR_INVALID_ARGUMENT;
    GWO_TRY(h->log_flush());
    return h->drain_side(cols, cap, n_out);
}

gwo_status gwo_current_watermark(gwo_handle *hh, int64_t *wm) {
    H_OR_FAIL;
    if (!wm) return GWO_ERR_INVALID_ARGUMENT;
    *wm = h->wm;
    return GWO_OK;
}

gwo_status gwo_get_config(const gwo_handle *hh, gwo_config *out) {
    const Handle *h = reinterpret_cast<const Handle *>(hh);
    if (!h || !out) return GWO_ERR_INVALID_ARGUMENT;
    *out = h->cfg;
    return GWO_OK;
}

gwo_status gwo_state_size(gwo_handle *hh, int64_t *entries) {
    H_OR_FAIL;
    if (!entries) return GWO_ERR_INVALID_ARGUMENT;
    return h->state_size(entries);
}

gwo_status gwo_snapshot_rows(gwo_handle *hh, int64_t *n_rows, int32_t *n_words) {
    H_OR_FAIL;
    if (!n_rows || !n_words) return GWO_ERR_INVALID_ARGUMENT;
    *n_words = h->plan.nwords;
    if (h->slide_has_restored())
        return h->fail(GWO_ERR_UNSUPPORTED, "snapshot: sliding windows restored from a per-window savepoint are "
                                            "checkpointed in the heap layout (gwo_export_heap_state) until they retire");
    return h->snapshot_rows(n_rows);
}

gwo_status gwo_snapshot(gwo_handle *hh, const gwo_state_rows *rows, int64_t cap, int64_t *n_out, int64_t *watermark) {
    H_OR_FAIL;
    if (!rows || !n_out || !watermark || cap < 0 ||
        (cap > 0 && (!rows->key || !rows->window_start || !rows->window_end || !rows->words)))
        return GWO_ERR_INVALID_ARGUMENT;
    *watermark = h->wm;
    if (h->slide_has_restored())
        return h->fail(GWO_ERR_UNSUPPORTED, "snapshot: sliding windows restored from a per-window savepoint are "
                                            "checkpointed in the heap layout (gwo_export_heap_state) until they retire");
    return h->snapshot(rows, cap, n_out);
}

gwo_status gwo_restore(gwo_handle *hh, const gwo_state_rows *rows, int32_t n_words, int64_t n, int64_t watermark) {
    H_OR_FAIL;
    if (n < 0 || (n > 0 && (!rows || !rows->key || !rows->window_start || !rows->window_end || !rows->words)))
        return GWO_ERR_INVALID_ARGUMENT;
    return h->restore(rows, n_words, n, watermark);
}

gwo_status gwo_sync(gwo_handle *hh) {
    H_OR_FAIL;
    GWO_TRY(h->flush_pending());
    if (h->logst) GWO_TRY(h->log_flush());
    if (h->logst) GWO_TRY(h->log_resolve_split());
    GWO_TRY(h->finish_fire());
    return h->hipcheck(hipStreamSynchronize(h->stream), "sync");
}

gwo_status gwo_wait_fires(gwo_handle *hh) {
    H_OR_FAIL;
    return h->finish_fire();
}

gwo_status gwo_host_register(void *ptr, int64_t bytes) {
    if (!ptr || bytes <= 0) return GWO_ERR_INVALID_ARGUMENT;
    const hipError_t e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterPortable);
    if (e == hipErrorHostMemoryAlreadyRegistered) {
        (void)hipGetLastError();
        return GWO_OK;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return GWO_ERR_HIP;
    }
    return GWO_OK;
}

gwo_status gwo_host_unregister(void *ptr) {
    if (!ptr) return GWO_ERR_INVALID_ARGUMENT;
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return e == hipErrorHostMemoryNotRegistered ? GWO_ERR_INVALID_ARGUMENT : GWO_ERR_HIP;
    }
    return GWO_OK;
}

// Device input produced on another stream: the handle's stream waits (on the device) for the work queued there so
// far.  Without it a producer on a different stream races K1, whose stream is non-blocking (gwo.h "Buffers").
gwo_status gwo_wait_stream(gwo_handle *hh, void *producer) {
    H_OR_FAIL;
    if ((hipStream_t)producer == h->stream) return GWO_OK;
    if (!h->ev_input) GWO_TRY(h->hipcheck(hipEventCreateWithFlags(&h->ev_input, hipEventDisableTiming), "event"));
    GWO_TRY(h->hipcheck(hipEventRecord(h->ev_input, (hipStream_t)producer), "wait_stream record"));
    if (h->cb_side)   // the pipelined combine path's gathers run there (gwo_set_pipelined_submit)
        GWO_TRY(h->hipcheck(hipStreamWaitEvent(h->cb_side, h->ev_input, 0), "wait_stream"));
    return h->hipcheck(hipStreamWaitEvent(h->stream, h->ev_input, 0), "wait_stream");
}

gwo_status gwo_get_stream(gwo_handle *hh, void **stream) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h || !stream) return GWO_ERR_INVALID_ARGUMENT;
    *stream = (void *)h->stream;
    return GWO_OK;
}

const char *gwo_last_error(const gwo_handle *hh) {
    const Handle *h = reinterpret_cast<const Handle *>(hh);
    return h ? h->err.c_str() : "null handle";
}

gwo_status gwo_set_pipelined_submit(gwo_handle *hh, int32_t enabled) {
    H_OR_FAIL;
    return h->set_pipelined(enabled != 0);
}

gwo_status gwo_set_profiling(gwo_handle *hh, int32_t enabled) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h) return GWO_ERR_INVALID_ARGUMENT;
    h->profiling = enabled != 0;
    h->prof_mask = ~0u;
    return GWO_OK;
}

gwo_status gwo_set_profiling_mask(gwo_handle *hh, uint32_t mask) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h) return GWO_ERR_INVALID_ARGUMENT;
    h->profiling = mask != 0;
    h->prof_mask = mask;
    return GWO_OK;
}

gwo_status gwo_kernel_stats(gwo_handle *hh, int32_t kernel, int64_t *launches, double *total_ms, int64_t *items) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h || kernel < 0 || kernel >= GWO_KERNEL_COUNT_) return GWO_ERR_INVALID_ARGUMENT;
    DeviceGuard guard_(h->cfg.device);
    GWO_TRY(h->prof_collect());
    if (launches) *launches = h->kstats[kernel].launches;
    if (total_ms) *total_ms = h->kstats[kernel].ms;
    if (items) *items = h->kstats[kernel].items;
    return GWO_OK;
}

gwo_status gwo_reset_stats(gwo_handle *hh) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h) return GWO_ERR_INVALID_ARGUMENT;
    DeviceGuard guard_(h->cfg.device);
    GWO_TRY(h->prof_collect());
    for (auto &k : h->kstats) k = KStat{};
    return GWO_OK;
}

// ---- stateless helpers --------------------------------------------------------------------------
static gwo_status stateless_run(int32_t device, size_t n, const void *in, size_t out_words, void **outs, int nouts,
                                void (*body)(const int64_t *, void **, hipStream_t, void *), void *ctx) {
    DeviceGuard guard_(device);
    hipStream_t s;
    // a blocking stream: ordered behind the null stream's work (a producer there needs no host sync, gwo.h)
    if (hipStreamCreate(&s) != hipSuccess) return GWO_ERR_HIP;
    gwo_status st = GWO_OK;
    const int64_t *din = (const int64_t *)in;
    void *tmp_in = nullptr;
    void *tmp_out[2] = {nullptr, nullptr};
    void *douts[2] = {nullptr, nullptr};
    if (!is_device_ptr(in)) {
        if (hipMalloc(&tmp_in, n * 8 + 8) != hipSuccess) st = GWO_ERR_OUT_OF_MEMORY;
        else if (copy_in(tmp_in, in, n * 8, s) != hipSuccess) st = GWO_ERR_HIP;
        din = (const int64_t *)tmp_in;
    }
    for (int i = 0; i < nouts && st == GWO_OK; ++i) {
        if (!outs[i]) continue;
        if (is_device_ptr(outs[i])) {
            douts[i] = outs[i];
        } else {
            if (hipMalloc(&tmp_out[i], n * out_words + 8) != hipSuccess) st = GWO_ERR_OUT_OF_MEMORY;
            douts[i] = tmp_out[i];
        }
    }
    if (st == GWO_OK) {
        body(din, douts, s, ctx);
        for (int i = 0; i < nouts; ++i)
            if (tmp_out[i] && copy_out(outs[i], tmp_out[i], n * out_words, s) != hipSuccess) st = GWO_ERR_HIP;
        if (hipStreamSynchronize(s) != hipSuccess) st = GWO_ERR_HIP;
    }
    if (tmp_in) (void)hipFree(tmp_in);
    for (int i = 0; i < 2; ++i)
        if (tmp_out[i]) (void)hipFree(tmp_out[i]);
    (void)hipStreamDestroy(s);
    return st;
}

struct KgCtx {
    int64_t n;
    int32_t kind, maxp, par;
};
static void kg_body(const int64_t *in, void **outs, hipStream_t s, void *c) {
    KgCtx *k = (KgCtx *)c;
    launch_key_groups(in, k->n, k->kind, k->maxp, k->par, (int32_t *)outs[0], (int32_t *)outs[1], s);
}

gwo_status gwo_assign_key_groups(const int64_t *keys, int64_t n, int32_t key_kind, int32_t max_parallelism,
                                 int32_t parallelism, int32_t *kg_out, int32_t *op_out, int32_t device) {
    if (n < 0 || !keys || max_parallelism <= 0 || max_parallelism > 32768 || parallelism <= 0 ||
        parallelism > max_parallelism)
        return GWO_ERR_INVALID_ARGUMENT;
    if (n == 0) return GWO_OK;
    KgCtx c{n, key_kind, max_parallelism, parallelism};
    void *outs[2] = {kg_out, op_out};
    return stateless_run(device, (size_t)n, keys, 4, outs, 2, kg_body, &c);
}

gwo_status gwo_assign_key_groups_utf16(const uint16_t *chars, const int64_t *offsets, int64_t n,
                                       int32_t max_parallelism, int32_t parallelism, int32_t *hash_out, int32_t *kg_out,
                                       int32_t *op_out, int32_t device) {
    if (n < 0 || !offsets || max_parallelism <= 0 || max_parallelism > 32768 || parallelism <= 0 ||
        parallelism > max_parallelism)
        return GWO_ERR_INVALID_ARGUMENT;
    if (n == 0) return GWO_OK;
    DeviceGuard guard_(device);
    hipStream_t s;
    // a blocking stream: ordered behind the null stream's work (a producer there needs no host sync, gwo.h)
    if (hipStreamCreate(&s) != hipSuccess) return GWO_ERR_HIP;
    gwo_status st = GWO_OK;
    std::vector<void *> owned;
    auto dev_alloc = [&](size_t bytes) -> void * {
        void *p = nullptr;
        if (hipMalloc(&p, bytes + 8) != hipSuccess) {
            st = GWO_ERR_OUT_OF_MEMORY;
            return nullptr;
        }
        owned.push_back(p);
        return p;
    };
    // offsets (n + 1) and the total code-unit count
    const int64_t *d_off = offsets;
    int64_t nchars = 0;
    if (is_device_ptr(offsets)) {
        if (hipMemcpy(&nchars, offsets + n, 8, hipMemcpyDeviceToHost) != hipSuccess) st = GWO_ERR_HIP;
    } else {
        nchars = offsets[n];
        int64_t *p = (int64_t *)dev_alloc((size_t)(n + 1) * 8);
        if (p && copy_in(p, offsets, (size_t)(n + 1) * 8, s) != hipSuccess) st = GWO_ERR_HIP;
        d_off = p;
    }
    if (st == GWO_OK && (nchars < 0 || (nchars > 0 && !chars))) st = GWO_ERR_INVALID_ARGUMENT;
    const uint16_t *d_chars = chars;
    if (st == GWO_OK && nchars > 0 && !is_device_ptr(chars)) {
        uint16_t *p = (uint16_t *)dev_alloc((size_t)nchars * 2);
        if (p && copy_in(p, chars, (size_t)nchars * 2, s) != hipSuccess) st = GWO_ERR_HIP;
        d_chars = p;
    }
    int32_t *outs[3] = {hash_out, kg_out, op_out}, *douts[3] = {nullptr, nullptr, nullptr};
    for (int i = 0; i < 3 && st == GWO_OK; ++i) {
        if (!outs[i]) continue;
        douts[i] = is_device_ptr(outs[i]) ? outs[i] : (int32_t *)dev_alloc((size_t)n * 4);
    }
    if (st == GWO_OK) {
        launch_key_groups_utf16(d_chars, d_off, n, max_parallelism, parallelism, douts[0], douts[1], douts[2], s);
        if (hipGetLastError() != hipSuccess) st = GWO_ERR_HIP;
        for (int i = 0; i < 3 && st == GWO_OK; ++i)
            if (outs[i] && douts[i] != outs[i] && copy_out(outs[i], douts[i], (size_t)n * 4, s) != hipSuccess)
                st = GWO_ERR_HIP;
    }
    if (hipStreamSynchronize(s) != hipSuccess && st == GWO_OK) st = GWO_ERR_HIP;
    for (void *p : owned) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return st;
}

struct WsCtx {
    int64_t n, off, size;
};
static void ws_body(const int64_t *in, void **outs, hipStream_t s, void *c) {
    WsCtx *w = (WsCtx *)c;
    launch_window_starts(in, w->n, w->off, w->size, (int64_t *)outs[0], s);
}

gwo_status gwo_window_starts(const int64_t *ts, int64_t n, int64_t offset, int64_t size, int64_t *start_out,
                             int32_t device) {
    if (n < 0 || !ts || !start_out || size <= 0) return GWO_ERR_INVALID_ARGUMENT;
    if (n == 0) return GWO_OK;
    WsCtx c{n, offset, size};
    void *outs[2] = {start_out, nullptr};
    return stateless_run(device, (size_t)n, ts, 8, outs, 1, ws_body, &c);
}

gwo_status gwo_generate(const gwo_gen_spec *sp, int64_t n, int64_t *key, int64_t *ts, void *value, void *stream,
                        int32_t device) {
    if (!sp || n < 0 || !key || !ts || sp->num_keys <= 0 || sp->total_records <= 0 || sp->span_ms < 0 ||
        sp->disorder_ms < 0 || (value && sp->value_range <= 0))
        return GWO_ERR_INVALID_ARGUMENT;
    if (n == 0) return GWO_OK;
    if (!is_device_ptr(key) || !is_device_ptr(ts) || (value && !is_device_ptr(value))) return GWO_ERR_INVALID_ARGUMENT;
    DeviceGuard guard_(device);
    launch_generate(sp->seed, sp->first_index, sp->total_records, sp->num_keys, sp->span_ms, sp->disorder_ms, sp->t0,
                    sp->value_range, sp->value_dtype == GWO_DTYPE_FLOAT64, sp->key_mode, n, key, ts, value,
                    (hipStream_t)stream);
    if (!stream && hipDeviceSynchronize() != hipSuccess) return GWO_ERR_HIP;
    return hipGetLastError() == hipSuccess ? GWO_OK : GWO_ERR_HIP;
}

}  // extern "C"
