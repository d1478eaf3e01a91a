// gwo_comm.cpp -- multi-GPU keyBy shuffle and watermark agreement over RCCL (xGMI).
//
// One process (one gwo_handle) per GPU; the handle owns key groups
// computeKeyGroupRangeForOperatorIndex(maxP, nranks, rank) (KeyGroupRangeAssignment.java:88-101).
// gwo_submit on every rank: destination = computeOperatorIndexForKeyGroup(kg) per record, stable
// grouping by destination, counts exchanged, then one ncclSend/ncclRecv pair per peer inside a
// group (xGMI is point-to-point: each peer pair has its own link, so per-peer sends are the
// natural all-to-all).  The watermark is the min over ranks (StatusWatermarkValve.java:163-181).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "gwo_handle.h"

namespace gwo {

void launch_dest(const int64_t *key, int64_t n, int kind, int max_par, int nranks, uint32_t *dest, hipStream_t s);
void launch_dest_count(const uint32_t *dest, int64_t n, unsigned long long *counts, hipStream_t s);
void launch_pack(const int64_t *key, const int64_t *ts, const int64_t *val, const uint32_t *perm, int64_t n,
                 int64_t *out, hipStream_t s);
void launch_unpack(const int64_t *in, int64_t n, int64_t *key, int64_t *ts, int64_t *val, hipStream_t s);
int radix_sort_pairs(const uint32_t *keys, const uint32_t *vals, int64_t n, int key_bits, uint32_t *k1, uint32_t *v1,
                     uint32_t *k2, uint32_t *v2, uint32_t *hist, hipStream_t s);

struct Comm {
    ncclComm_t nc = nullptr;
    int nranks = 1, rank = 0;
    DevBuf dest, k1, v1, hist, sendbuf, recvbuf, rk, rt, rv, counts;
    unsigned long long *h_counts = nullptr;   // pinned: [send counts | recv counts]
    int64_t *h_wm = nullptr;                  // pinned
};

void Handle::comm_free() {
    if (!comm) return;
    if (comm->nc) ncclCommDestroy(comm->nc);
    for (DevBuf *b : {&comm->dest, &comm->k1, &comm->v1, &comm->hist, &comm->sendbuf, &comm->recvbuf, &comm->rk,
                      &comm->rt, &comm->rv, &comm->counts})
        b->release();
    if (comm->h_counts) (void)hipHostFree(comm->h_counts);
    if (comm->h_wm) (void)hipHostFree(comm->h_wm);
    delete comm;
    comm = nullptr;
}

static gwo_status nccl_ok(Handle *h, ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return GWO_OK;
    return h->poison(GWO_ERR_COMM, (std::string(what) + ": " + ncclGetErrorString(r)).c_str());
}

gwo_status Handle::comm_exchange(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const int64_t **rk,
                                 const int64_t **rt, const int64_t **rv, int64_t *rn) {
    Comm &C = *comm;
    const int P = C.nranks;
    GWO_TRY(ensure_buf(C.counts, (size_t)2 * P * 8));
    unsigned long long *d_send = (unsigned long long *)C.counts.ptr, *d_recv = d_send + P;
    GWO_TRY(hipcheck(hipMemsetAsync(d_send, 0, (size_t)2 * P * 8, stream), "counts"));
    const int64_t *perm_src = nullptr;
    prof_begin(GWO_KERNEL_PARTITION);
    if (n > 0) {
        GWO_TRY(ensure_buf(C.dest, n * 4));
        GWO_TRY(ensure_buf(C.k1, n * 4));
        GWO_TRY(ensure_buf(C.v1, n * 4));
        GWO_TRY(ensure_buf(C.hist, (size_t)256 * ((n + 4095) / 4096) * 4 + 16));
        GWO_TRY(ensure_buf(C.sendbuf, n * 24));
        launch_dest(k, n, cfg.key_kind, cfg.max_parallelism, P, (uint32_t *)C.dest.ptr, stream);
        launch_dest_count((const uint32_t *)C.dest.ptr, n, d_send, stream);
        // one stable 8-bit pass: destinations < 256; payload = record index (arrival order kept)
        radix_sort_pairs((const uint32_t *)C.dest.ptr, nullptr, n, 8, (uint32_t *)C.k1.ptr, (uint32_t *)C.v1.ptr,
                         nullptr, nullptr, (uint32_t *)C.hist.ptr, stream);
        launch_pack(k, t, v, (const uint32_t *)C.v1.ptr, n, (int64_t *)C.sendbuf.ptr, stream);
        GWO_TRY(launch_ok("partition"));
        perm_src = (const int64_t *)C.sendbuf.ptr;
    }
    prof_end(GWO_KERNEL_PARTITION, n);
    // exchange counts
    GWO_TRY(nccl_ok(this, ncclGroupStart(), "group"));
    for (int p = 0; p < P; ++p) {
        GWO_TRY(nccl_ok(this, ncclSend(d_send + p, 1, ncclUint64, p, C.nc, stream), "send count"));
        GWO_TRY(nccl_ok(this, ncclRecv(d_recv + p, 1, ncclUint64, p, C.nc, stream), "recv count"));
    }
    GWO_TRY(nccl_ok(this, ncclGroupEnd(), "group end"));
    GWO_TRY(hipcheck(hipMemcpyAsync(C.h_counts, d_send, (size_t)2 * P * 8, hipMemcpyDeviceToHost, stream), "counts"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "counts sync"));
    std::vector<uint64_t> soff(P + 1, 0), roff(P + 1, 0);
    for (int p = 0; p < P; ++p) {
        soff[p + 1] = soff[p] + C.h_counts[p];
        roff[p + 1] = roff[p] + C.h_counts[P + p];
    }
    const int64_t R = (int64_t)roff[P];
    GWO_TRY(ensure_buf(C.recvbuf, R * 24 + 24));
    prof_begin(GWO_KERNEL_EXCHANGE);
    GWO_TRY(nccl_ok(this, ncclGroupStart(), "group"));
    for (int p = 0; p < P; ++p) {
        uint64_t sc = C.h_counts[p], rc = C.h_counts[P + p];
        if (sc)
            GWO_TRY(nccl_ok(this, ncclSend(perm_src + 3 * soff[p], 3 * sc, ncclInt64, p, C.nc, stream), "send"));
        if (rc)
            GWO_TRY(nccl_ok(this, ncclRecv((int64_t *)C.recvbuf.ptr + 3 * roff[p], 3 * rc, ncclInt64, p, C.nc, stream),
                            "recv"));
    }
    GWO_TRY(nccl_ok(this, ncclGroupEnd(), "group end"));
    prof_end(GWO_KERNEL_EXCHANGE, R);
    GWO_TRY(ensure_buf(C.rk, R * 8 + 8));
    GWO_TRY(ensure_buf(C.rt, R * 8 + 8));
    GWO_TRY(ensure_buf(C.rv, R * 8 + 8));
    if (R > 0) {
        launch_unpack((const int64_t *)C.recvbuf.ptr, R, (int64_t *)C.rk.ptr, (int64_t *)C.rt.ptr, (int64_t *)C.rv.ptr,
                      stream);
        GWO_TRY(launch_ok("unpack"));
    }
    *rk = (const int64_t *)C.rk.ptr;
    *rt = (const int64_t *)C.rt.ptr;
    *rv = needs_value ? (const int64_t *)C.rv.ptr : nullptr;
    *rn = R;
    return GWO_OK;
}

gwo_status Handle::comm_min_watermark(int64_t wm_in, int64_t *out) {
    Comm &C = *comm;
    GWO_TRY(ensure_buf(C.counts, (size_t)2 * C.nranks * 8 + 16));
    int64_t *d = (int64_t *)C.counts.ptr;
    *C.h_wm = wm_in;
    GWO_TRY(hipcheck(hipMemcpyAsync(d, C.h_wm, 8, hipMemcpyHostToDevice, stream), "wm"));
    GWO_TRY(nccl_ok(this, ncclAllReduce(d, d, 1, ncclInt64, ncclMin, C.nc, stream), "allreduce wm"));
    GWO_TRY(hipcheck(hipMemcpyAsync(C.h_wm, d, 8, hipMemcpyDeviceToHost, stream), "wm"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "wm sync"));
    *out = *C.h_wm;
    return GWO_OK;
}

}  // namespace gwo

using namespace gwo;

extern "C" gwo_status gwo_comm_unique_id(uint8_t *id) {
    if (!id) return GWO_ERR_INVALID_ARGUMENT;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return GWO_ERR_COMM;
    static_assert(sizeof(u) == GWO_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, GWO_COMM_ID_BYTES);
    return GWO_OK;
}

extern "C" gwo_status gwo_comm_init(gwo_handle *hh, const uint8_t *id, int32_t nranks, int32_t rank) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h || !id || nranks < 1 || nranks > 256 || rank < 0 || rank >= nranks) return GWO_ERR_INVALID_ARGUMENT;
    if (h->poisoned) return h->poison_status;
    if (h->comm) return h->fail(GWO_ERR_STATE, "communicator already initialised");
    DeviceGuard guard_(h->cfg.device);
    const int maxp = h->cfg.max_parallelism;
    if (nranks > maxp) return h->fail(GWO_ERR_INVALID_ARGUMENT, "Maximum parallelism must not be smaller than parallelism.");
    const int lo = (rank * maxp + nranks - 1) / nranks, hi = ((rank + 1) * maxp - 1) / nranks;
    if (h->cfg.key_group_start != lo || h->cfg.key_group_end != hi)
        return h->fail(GWO_ERR_INVALID_ARGUMENT, "handle KeyGroupRange [%d, %d] != operator %d of %d: [%d, %d]",
                       h->cfg.key_group_start, h->cfg.key_group_end, rank, nranks, lo, hi);
    Comm *C = new Comm();
    C->nranks = nranks;
    C->rank = rank;
    if (hipHostMalloc((void **)&C->h_counts, (size_t)2 * nranks * 8 + 16, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&C->h_wm, 16, hipHostMallocDefault) != hipSuccess) {
        delete C;
        return GWO_ERR_OUT_OF_MEMORY;
    }
    ncclUniqueId u;
    memcpy(&u, id, GWO_COMM_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&C->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        (void)hipHostFree(C->h_counts);
        (void)hipHostFree(C->h_wm);
        delete C;
        return h->fail(GWO_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    h->comm = C;
    return GWO_OK;
}
