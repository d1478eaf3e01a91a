// gwo_snapshot.hip -- checkpoint rows of the keyed window state (kernels; host side: gwo_snapshot.cpp).
//
// The reference snapshots its heap keyed state per key group as (namespace, key, state) entries
// (CopyOnWriteStateMapSnapshot.java:127-129, HeapSnapshotStrategy.java:97-222) next to the per-key-group
// timers of the "window-timers" service (InternalTimeServiceManager.java:160-198).  Here a checkpoint row is
// (key, TimeWindow{start, end}, raw accumulator words, fire-timer flag), and rows are ordered by key group.
// Collection writes SoA scratch columns (SnapCols) with one block reservation per workgroup chunk.
#include "gwo_device.h"

namespace gwo {

__device__ __forceinline__ const int64_t *snap_entry(const TableDesc &t, uint64_t cap, int stride, uint64_t i) {
    return i < cap ? t.base + i * (uint64_t)stride : t.side;
}

// Every occupied entry of one window's (or pane's) hash table: the table layout's per-(key, window) state.
__global__ __launch_bounds__(256) void snap_table_kernel(TableDesc t, uint64_t cap, AccPlan p, int64_t start,
                                                         int64_t end, int32_t timer, SnapCols c) {
    for (uint64_t b0 = (uint64_t)blockIdx.x * 256; b0 < cap + 1; b0 += (uint64_t)gridDim.x * 256) {
        const uint64_t i = b0 + threadIdx.x;
        const int64_t *e = i <= cap ? snap_entry(t, cap, p.stride, i) : nullptr;
        const bool occ = e && (i < cap ? e[0] != GWO_EMPTY_KEY : e[0] != 0);
        const unsigned long long pos = block_reserve(occ ? 1u : 0u, c.count);
        if (occ && (long long)pos < c.cap) {
            c.key[pos] = i < cap ? e[0] : GWO_EMPTY_KEY;
            c.start[pos] = start;
            c.end[pos] = end;
            c.timer[pos] = timer;
            for (int w = 0; w < p.nwords; ++w) c.w[w][pos] = e[1 + w];
        }
    }
}

// Every in-flight session of every key (gwo_session.hip entry layout: key | count | [start, end, flags,
// words...] per session): the reference's session state windows (MergingWindowSet.java:81-109 persists the
// in-flight window -> state window mapping; here the merged window is its own namespace).
__global__ __launch_bounds__(256) void snap_session_kernel(TableDesc t, uint64_t cap, int stride, AccPlan p,
                                                           const int64_t *pool, SnapCols c) {
    const int sw = 3 + p.nwords;
    for (uint64_t b0 = (uint64_t)blockIdx.x * 256; b0 < cap + 1; b0 += (uint64_t)gridDim.x * 256) {
        const uint64_t i = b0 + threadIdx.x;
        const int64_t *e = nullptr;
        int64_t k = 0;
        unsigned ns = 0;
        if (i < cap) {
            e = t.base + i * (uint64_t)stride;
            k = e[0];
            if (k == GWO_EMPTY_KEY) e = nullptr;
        } else if (i == cap && t.side[0] != 0) {
            e = t.side;
            k = GWO_EMPTY_KEY;
        }
        const int64_t *list = nullptr;
        if (e) {   // inline sessions, or a spilled list in the pool
            ns = e[1] < 0 ? (unsigned)e[4] : (unsigned)e[1];
            list = e[1] < 0 ? pool + (uint64_t)e[2] * sw : e + 2;
        }
        unsigned long long pos = block_reserve(ns, c.count);
        for (unsigned s = 0; s < ns; ++s, ++pos) {
            if ((long long)pos >= c.cap) break;
            const int64_t *S = list + (uint64_t)s * sw;
            c.key[pos] = k;
            c.start[pos] = S[0];
            c.end[pos] = S[1];
            c.timer[pos] = (int32_t)(S[2] & 1);
            for (int w = 0; w < p.nwords; ++w) c.w[w][pos] = S[3 + w];
        }
    }
}

// Row j of the output = scratch row perm[j] (perm: the stable key-group order), words row-major.
__global__ __launch_bounds__(256) void snap_gather_kernel(SnapCols c, const uint32_t *__restrict__ perm,
                                                          const uint32_t *__restrict__ kg_sorted, int64_t n, int nw,
                                                          int64_t *key, int64_t *start, int64_t *end, int64_t *words,
                                                          int32_t *kg, int32_t *timer) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) {
        const uint32_t s = perm[j];
        key[j] = c.key[s];
        start[j] = c.start[s];
        end[j] = c.end[s];
        for (int w = 0; w < nw; ++w) words[j * nw + w] = c.w[w][s];
        kg[j] = (int32_t)kg_sorted[j];
        timer[j] = c.timer[s];
    }
}

__global__ void snap_fill_i32_kernel(int32_t *p, int64_t n, int32_t v) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) p[j] = v;
}

// Session restore: every row whose key group is this subtask's claims its key's entry and appends its session
// (order inside an entry is irrelevant: every operation scans all of a key's in-flight sessions).  A key with
// more restored sessions than its entry holds counts in err->capacity.
__global__ __launch_bounds__(256) void sess_restore_kernel(const int64_t *key, const int64_t *start, const int64_t *end,
                                                           const int32_t *timer, const int64_t *words, int64_t n,
                                                           TableDesc t, uint64_t cap, int stride, AccPlan p,
                                                           SessGeom g, SessErr *err) {
    const int sw = 3 + p.nwords;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x; j0 < n; j0 += step) {
        const int64_t j = j0 + threadIdx.x;
        bool claimed = false, added = false;
        if (j < n) {
            const int64_t k = key[j];
            const int32_t kg = key_group(k, g.key_kind, g.max_par);
            if (kg >= g.kg_lo && kg <= g.kg_hi) {
                int64_t *e = find_or_insert(t, stride, k, claimed) - 1;
                const unsigned long long idx = atomicAdd((unsigned long long *)&e[1], 1ull);
                if (idx >= (unsigned long long)g.smax) {
                    atomicAdd(&err->capacity, 1ull);
                } else {
                    int64_t *S = e + 2 + idx * sw;
                    S[0] = start[j];
                    S[1] = end[j];
                    S[2] = timer ? (timer[j] != 0 ? 1 : 0) : (jsub(end[j], 1) > g.wm ? 1 : 0);
                    for (int w = 0; w < p.nwords; ++w) S[3 + w] = words[j * p.nwords + w];
                    added = true;
                }
            }
        }
        count_claims(t.occ, claimed);
        wave_atomic_add(&err->live_delta, added ? 1ull : 0ull);
    }
}

// Keys restored with more sessions than an entry holds: their lists were uploaded into the spill pool by the
// host; each key's entry points at its list (word 1 = -1, pool record, capacity, count).
__global__ __launch_bounds__(256) void sess_restore_wide_kernel(const int64_t *key, const int64_t *off,
                                                                const int64_t *lcap, const int64_t *count, int64_t m,
                                                                TableDesc t, int stride) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x; j0 < m; j0 += step) {
        const int64_t j = j0 + threadIdx.x;
        bool claimed = false;
        if (j < m) {
            int64_t *e = find_or_insert(t, stride, key[j], claimed) - 1;
            e[1] = -1;
            e[2] = off[j];
            e[3] = lcap[j];
            e[4] = count[j];
        }
        count_claims(t.occ, claimed);
    }
}

// Rows (SoA, one per key) folded into a window's hash table: the log layout hands a fired window that must
// stay until its cleanup time (allowedLateness > 0) to the table path this way.
__global__ __launch_bounds__(256) void table_load_kernel(SnapCols c, int64_t n, TableDesc t, AccPlan p) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x; j0 < n; j0 += step) {
        const int64_t j = j0 + threadIdx.x;
        bool claimed = false;
        if (j < n) {
            int64_t *acc = find_or_insert(t, p.stride, c.key[j], claimed);
            for (int w = 0; w < p.nwords; ++w) atomic_combine(acc + w, p.op[w], c.w[w][j]);
        }
        count_claims(t.occ, claimed);
    }
}

static inline int snap_grid(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

void launch_snap_table(const TableDesc &t, uint64_t cap, const AccPlan &p, int64_t start, int64_t end, int32_t timer,
                       const SnapCols &c, hipStream_t s) {
    hipLaunchKernelGGL(snap_table_kernel, dim3(snap_grid((int64_t)cap + 1)), dim3(256), 0, s, t, cap, p, start, end,
                       timer, c);
}

void launch_snap_session(const TableDesc &t, uint64_t cap, int stride, const AccPlan &p, const int64_t *pool,
                         const SnapCols &c, hipStream_t s) {
    hipLaunchKernelGGL(snap_session_kernel, dim3(snap_grid((int64_t)cap + 1)), dim3(256), 0, s, t, cap, stride, p, pool,
                       c);
}

void launch_sess_restore_wide(const int64_t *key, const int64_t *off, const int64_t *lcap, const int64_t *count,
                              int64_t m, const TableDesc &t, int stride, hipStream_t s) {
    hipLaunchKernelGGL(sess_restore_wide_kernel, dim3(snap_grid(m)), dim3(256), 0, s, key, off, lcap, count, m, t,
                       stride);
}

void launch_snap_gather(const SnapCols &c, const uint32_t *perm, const uint32_t *kg_sorted, int64_t n, int nw,
                        int64_t *key, int64_t *start, int64_t *end, int64_t *words, int32_t *kg, int32_t *timer,
                        hipStream_t s) {
    hipLaunchKernelGGL(snap_gather_kernel, dim3(snap_grid(n)), dim3(256), 0, s, c, perm, kg_sorted, n, nw, key, start,
                       end, words, kg, timer);
}

void launch_table_load(const SnapCols &c, int64_t n, const TableDesc &t, const AccPlan &p, hipStream_t s) {
    hipLaunchKernelGGL(table_load_kernel, dim3(snap_grid(n)), dim3(256), 0, s, c, n, t, p);
}

void launch_snap_fill_i32(int32_t *p, int64_t n, int32_t v, hipStream_t s) {
    hipLaunchKernelGGL(snap_fill_i32_kernel, dim3(snap_grid(n)), dim3(256), 0, s, p, n, v);
}

void launch_sess_restore(const int64_t *key, const int64_t *start, const int64_t *end, const int32_t *timer,
                         const int64_t *words, int64_t n, const TableDesc &t, uint64_t cap, int stride,
                         const AccPlan &p, const SessGeom &g, SessErr *err, hipStream_t s) {
    hipLaunchKernelGGL(sess_restore_kernel, dim3(snap_grid(n)), dim3(256), 0, s, key, start, end, timer, words, n, t,
                       cap, stride, p, g, err);
}

}  // namespace gwo
