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
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <deque>
#include <vector>

#include "gwo_handle.h"
#include "gwo_log.h"

namespace gwo {

void launch_dest(const int64_t *key, int64_t n, int kind, int max_par, int nranks, uint32_t *dest, hipStream_t s);
void launch_dest_count(const uint32_t *dest, int64_t n, unsigned long long *counts, hipStream_t s);
void launch_pack(const int64_t *key, const int64_t *ts, const int64_t *val, const uint32_t *perm, int64_t n,
                 int64_t *out, hipStream_t s);
void launch_unpack(const int64_t *in, int64_t n, int64_t *key, int64_t *ts, int64_t *val, hipStream_t s);
void launch_route(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, int kind, int max_par,
                  int nranks, unsigned long long *cursor, uint64_t cap, int64_t *send, hipStream_t s);
void launch_route_collect(unsigned long long *cursor, int nranks, unsigned long long *counts, hipStream_t s);
size_t route_cursor_bytes();

struct Comm {
    ncclComm_t nc = nullptr;
    int nranks = 1, rank = 0;
    DevBuf dest, k1, v1, hist, sendbuf, recvbuf, rk, rt, rv, counts, cursor;
    unsigned long long *h_counts = nullptr;   // pinned: [send counts | recv counts]
    int64_t *h_wm = nullptr;                  // pinned
    // the records' exchange runs on its own stream, so the K1 of the records a rank keeps overlaps it
    hipStream_t cs = nullptr;
    hipEvent_t ev_routed = nullptr, ev_recv = nullptr;
    // Virtual ranks (GWO_COMM_VIRTUAL=P on a 1-rank communicator, log layout): K1 routes as if P GPUs shared the
    // key groups and this were GPU 0; the other "GPUs'" records go through RCCL to this rank itself and come back
    // as received records -- a rank's whole data path at P GPUs on one GPU (outputs unchanged: it owns every key).
    int vranks = 0;
    uint64_t rcap = 0, wcap = 0;  // narrow / wide send region capacities of the routed K1 (records)
    int64_t tbase = 0;            // the routed batch's timestamp base (20-B wire records carry int32 ts - tbase)
    // the min over ranks of their watermarks, as of comm_init or the last gwo_advance_watermark (collective calls):
    // every rank holds the same value, so sender and receiver derive the same tbase from it even when restored
    // subtasks hold different watermarks
    int64_t agreed_wm = (int64_t)0x8000000000000000LL;
    // Routed exchanges of the log layout rotate over NS send/receive buffer slots.  Batch i's routed K1
    // fills send slot i % NS and its per-destination counts; the counts are exchanged on the count communicator right
    // behind K1 and published to host-mapped memory, and batch i's record exchange is posted one batch later: at
    // batch i+1's gwo_submit right behind its K1 when the counts are there, else after that K1's readback, else at the
    // next batch (the counts follow batch i's K1 on a high-priority stream) -- no routed batch waits for them; only a
    // flush, or a slot coming round with its batch's counts still missing, would.
    // Its received records are inserted at batch i+2 (or at any earlier flush: a fire they may fall into, a snapshot,
    // gwo_sync, a state query).  Slot reuse is ordered on the device: a routed K1 waits for the exchange that last
    // sent from its slot, an exchange waits for the K1 that last read its receive slot.
    static constexpr int NS = 3;
    DevBuf rsend[NS], rrecv[NS], rcnt[NS];         // send regions; receive buffer; (narrow, wide) counts, 4P words
    hipEvent_t ev_rrecv[NS] = {};                  // the slot's record exchange finished (cs)
    hipEvent_t ev_rout[NS] = {};                   // the slot's routed K1 (and re-route) finished (main stream)
    hipEvent_t ev_read[NS] = {};                   // the slot's received records were read (main stream)
    hipEvent_t ev_cnt[NS] = {};                    // the slot's count exchange was published (count stream)
    bool used_send[NS] = {}, used_read[NS] = {};
    unsigned long long *hcnt[NS] = {}, *hcnt_dev[NS] = {};   // host-mapped: 4P count words + sequence word
    unsigned long long cnt_seq = 0;
    int rslot = 0;
    // Counts and watermark agreement run on a second communicator (ncclCommSplit of nc) and stream: RCCL orders the
    // operations of one communicator, so on nc they would queue behind the previous batch's record exchange.
    ncclComm_t nc2 = nullptr;
    hipStream_t cs2 = nullptr;
    struct Post {                  // a routed batch whose record exchange is not posted yet
        int slot = 0;
        unsigned long long seq = 0;
        uint64_t rcap = 0, wcap = 0;
        int64_t tbase = 0;
        WindowGeom g{};
    };
    std::deque<Post> posts;        // (oldest first; at most 2: the current batch's and the previous one's)
    struct Recv {
        int slot = 0;
        int64_t n = 0, w = 0;      // narrow / wide records received
        int64_t off_w = 0;         // word offset of the wide records in the slot's receive buffer
        int64_t tbase = 0;
        WindowGeom g{};            // the geometry (watermark) of the batch they belong to
    };
    std::deque<Recv> recvq;        // posted exchanges whose records are not inserted yet (oldest first)
    // host round trips of the routed exchange: batches routed, waits for a batch's counts (only a flush waits: a fire
    // its records may fall into, a snapshot, gwo_sync), synchronous watermark agreements
    int64_t routed = 0, count_waits = 0, wm_waits = 0;
    // waits while the device was still running the newest routed batches (the host ran ahead by more than the slot
    // ring holds: flow control, not a protocol round trip) -- kept apart from count_waits / wm_waits
    int64_t bp_count_waits = 0, bp_wm_waits = 0;
    int64_t count_wait_ns = 0, wm_wait_ns = 0;   // host time spent in those waits
    int64_t flow_wait_ns = 0;                     // host time spent in flow-control waits
    int wm_after_slot = -1;        // the count exchange the queued asynchronous agreement follows on the count stream
    // asynchronous watermark agreement (gwo_comm_set_async_watermark): two host-mapped result blocks, alternating
    bool async_wm = false, wm_pending = false;
    unsigned long long *hwm[2] = {}, *hwm_dev[2] = {};
    unsigned long long wm_seq = 0;
    bool defer = true;             // GWO_COMM_DEFER=0: insert every batch's received records inside its gwo_submit
    int hold = 0;                  // GWO_COMM_HOLD_COUNTS (diagnostics, counts_arrived)
};

static int route_ranks(const Comm &C) { return C.vranks > 1 ? C.vranks : C.nranks; }

// A wait is flow control, not a round trip of the protocol, when the device has not even run what the awaited result
// is queued behind: a batch's counts behind its routed K1, a watermark agreement behind the previous batch's count
// exchange.  (The host then runs ahead of the device by more than the slot ring holds.)
static bool not_done(hipEvent_t e) { return hipEventQuery(e) == hipErrorNotReady; }

static bool comm_events(Comm *C) {
    for (int q = 0; q < Comm::NS; ++q)
        for (hipEvent_t *e : {&C->ev_rrecv[q], &C->ev_rout[q], &C->ev_read[q], &C->ev_cnt[q]})
            if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return false;
    return true;
}

void Handle::comm_free() {
    if (!comm) return;
    if (comm->cs) (void)hipStreamSynchronize(comm->cs);
    if (comm->cs2) (void)hipStreamSynchronize(comm->cs2);
    if (comm->nc2) ncclCommDestroy(comm->nc2);
    if (comm->nc) ncclCommDestroy(comm->nc);
    for (DevBuf *b : {&comm->dest, &comm->k1, &comm->v1, &comm->hist, &comm->sendbuf, &comm->recvbuf, &comm->rk,
                      &comm->rt, &comm->rv, &comm->counts, &comm->cursor})
        b->release();
    for (int q = 0; q < Comm::NS; ++q) {
        comm->rsend[q].release();
        comm->rrecv[q].release();
        comm->rcnt[q].release();
        for (hipEvent_t e : {comm->ev_rrecv[q], comm->ev_rout[q], comm->ev_read[q], comm->ev_cnt[q]})
            if (e) (void)hipEventDestroy(e);
        if (comm->hcnt[q]) (void)hipHostFree(comm->hcnt[q]);
    }
    for (unsigned long long *p : comm->hwm)
        if (p) (void)hipHostFree(p);
    if (comm->cs) (void)hipStreamDestroy(comm->cs);
    if (comm->cs2) (void)hipStreamDestroy(comm->cs2);
    if (comm->ev_routed) (void)hipEventDestroy(comm->ev_routed);
    if (comm->ev_recv) (void)hipEventDestroy(comm->ev_recv);
    if (comm->h_counts) (void)hipHostFree(comm->h_counts);
    if (comm->h_wm) (void)hipHostFree(comm->h_wm);
    delete comm;
    comm = nullptr;
}

static gwo_status nccl_ok(Handle *h, ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return GWO_OK;
    return h->poison(GWO_ERR_COMM, (std::string(what) + ": " + ncclGetErrorString(r)).c_str());
}

// keyBy shuffle of one batch: every record goes to the GPU owning its key group.  Returns the records this
// rank keeps (its own region of the send buffer: they never touch the wire) and the records it receives from
// the other ranks, both as 24-B {key, ts, value} records (AoS).  Order-insensitive state (tumbling/sliding)
// uses the fused route kernel; sessions need each source's arrival order per key, so they group by
// destination with a stable radix pass instead.  One host round trip per batch: the per-destination counts
// are exchanged on the device right behind the route, and one copy brings both directions' counts back (a
// region overflow re-routes locally -- the exchanged counts are exact either way).
gwo_status Handle::comm_exchange(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, const int64_t **aos,
                                 int64_t *rn, const int64_t **local, int64_t *ln) {
    Comm &C = *comm;
    const int P = C.nranks, me = C.rank;
    const bool stable = cfg.assigner == GWO_ASSIGNER_SESSION;
    GWO_TRY(ensure_buf(C.counts, (size_t)2 * P * 8));
    unsigned long long *d_send = (unsigned long long *)C.counts.ptr, *d_recv = d_send + P;
    std::vector<uint64_t> soff(P + 1, 0), roff(P + 1, 0);
    uint64_t cap = 0;
    auto route = [&]() -> gwo_status {
        GWO_TRY(ensure_buf(C.sendbuf, (size_t)P * cap * 24 + 24));
        if (n > 0)
            launch_route(k, t, v, n, cfg.key_kind, cfg.max_parallelism, P, (unsigned long long *)C.cursor.ptr, cap,
                         (int64_t *)C.sendbuf.ptr, stream);
        launch_route_collect((unsigned long long *)C.cursor.ptr, P, d_send, stream);
        return launch_ok("route");
    };
    prof_begin(GWO_KERNEL_PARTITION);
    if (!stable) {
        if (!C.cursor.ptr) {
            GWO_TRY(ensure_buf(C.cursor, route_cursor_bytes()));
            GWO_TRY(hipcheck(hipMemsetAsync(C.cursor.ptr, 0, route_cursor_bytes(), stream), "route cursors"));
        }
        const double mean = (double)n / P;
        cap = (uint64_t)(mean + 6.0 * std::sqrt(mean) + 64.0);
        GWO_TRY(route());
    } else {
        GWO_TRY(hipcheck(hipMemsetAsync(d_send, 0, (size_t)2 * P * 8, stream), "counts"));
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
        }
    }
    prof_end(GWO_KERNEL_PARTITION, n);
    // counts, on the device right behind the route (xGMI is point-to-point: one send/recv pair per peer)
    if (P > 1) {
        GWO_TRY(nccl_ok(this, ncclGroupStart(), "group"));
        for (int p = 0; p < P; ++p) {
            if (p == me) continue;
            GWO_TRY(nccl_ok(this, ncclSend(d_send + p, 1, ncclUint64, p, C.nc, stream), "send count"));
            GWO_TRY(nccl_ok(this, ncclRecv(d_recv + p, 1, ncclUint64, p, C.nc, stream), "recv count"));
        }
        GWO_TRY(nccl_ok(this, ncclGroupEnd(), "group end"));
    }
    GWO_TRY(hipcheck(hipMemcpyAsync(C.h_counts, d_send, (size_t)2 * P * 8, hipMemcpyDeviceToHost, stream), "counts"));
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "counts sync"));
    C.h_counts[P + me] = 0;   // our own records stay here
    if (!stable) {
        uint64_t mx = 0;
        for (int p = 0; p < P; ++p) mx = std::max<uint64_t>(mx, C.h_counts[p]);
        if (mx > cap) {   // skewed keys: a destination overflowed its region -- re-route with the exact size
            cap = mx;
            GWO_TRY(route());
        }
        for (int p = 0; p < P; ++p) soff[p] = (uint64_t)p * cap;   // region starts (records)
    } else {
        for (int p = 0; p < P; ++p) soff[p + 1] = soff[p] + C.h_counts[p];
    }
    for (int p = 0; p < P; ++p) roff[p + 1] = roff[p] + C.h_counts[P + p];
    const int64_t R = (int64_t)roff[P];
    GWO_TRY(ensure_buf(C.recvbuf, R * 24 + 24));
    const int64_t *sb = (const int64_t *)C.sendbuf.ptr;
    if (P > 1) {
        // on the comm stream, behind the route (and so behind everything earlier batches did with the buffers);
        // comm_wait_received puts the main stream behind it before the received records are read
        GWO_TRY(hipcheck(hipEventRecord(C.ev_routed, stream), "event"));
        GWO_TRY(hipcheck(hipStreamWaitEvent(C.cs, C.ev_routed, 0), "event wait"));
        prof_begin(GWO_KERNEL_EXCHANGE, C.cs);
        GWO_TRY(nccl_ok(this, ncclGroupStart(), "group"));
        for (int p = 0; p < P; ++p) {
            if (p == me) continue;
            const uint64_t sc = C.h_counts[p], rc = C.h_counts[P + p];
            if (sc) GWO_TRY(nccl_ok(this, ncclSend(sb + 3 * soff[p], 3 * sc, ncclInt64, p, C.nc, C.cs), "send"));
            if (rc)
                GWO_TRY(nccl_ok(this, ncclRecv((int64_t *)C.recvbuf.ptr + 3 * roff[p], 3 * rc, ncclInt64, p, C.nc,
                                               C.cs), "recv"));
        }
        GWO_TRY(nccl_ok(this, ncclGroupEnd(), "group end"));
        prof_end(GWO_KERNEL_EXCHANGE, R, C.cs);
        GWO_TRY(hipcheck(hipEventRecord(C.ev_recv, C.cs), "event"));
    }
    *local = sb + 3 * soff[me];
    *ln = (int64_t)C.h_counts[me];
    *aos = (const int64_t *)C.recvbuf.ptr;
    *rn = R;
    return GWO_OK;
}

// Routing fused into the log layout's first K1 of a batch (gwo_log.hip log_part_kernel<.., true>): K1 appends
// the records of other GPUs to per-destination regions of the send buffer while it partitions its own, so a
// batch is read once -- the route kernel of comm_exchange (24 B read + 24 B written per record, then K1 reads
// the kept records again) is gone from the log path.  Regions hold mean + 6 sigma + 64 records; a skewed batch
// that overflows one is re-routed with exact capacities (comm_check_route, from K1's readback).
gwo_status Handle::comm_route_args(int64_t n, LogRoute *rt, bool *on) {
    Comm &C = *comm;
    const int P = route_ranks(C);
    *on = P > 1;
    if (!*on) return GWO_OK;
    const int slot = C.rslot;
    GWO_TRY(ensure_buf(C.rcnt[slot], (size_t)4 * P * 8 + 16));
    if (!C.cursor.ptr) {
        GWO_TRY(ensure_buf(C.cursor, std::max(route_cursor_bytes(), (size_t)2 * LOG_RT_MAX * LOG_CUR_STRIDE * 8)));
        GWO_TRY(hipcheck(hipMemsetAsync(C.cursor.ptr, 0, C.cursor.bytes, stream), "route cursors"));
    }
    if (!C.hcnt[slot]) {
        GWO_TRY(hipcheck(hipHostMalloc((void **)&C.hcnt[slot], (size_t)4 * P * 8 + 16,
                                       hipHostMallocCoherent | hipHostMallocMapped), "count readback"));
        GWO_TRY(hipcheck(hipHostGetDevicePointer((void **)&C.hcnt_dev[slot], C.hcnt[slot], 0), "count readback"));
    }
    const double mean = (double)n / P;
    C.rcap = ((uint64_t)(mean + 6.0 * std::sqrt(mean) + 64.0) + 1) & ~1ull;   // even: regions stay 8-B aligned
    C.wcap = 256 + (uint64_t)n / 1024;
    C.tbase = log_rt_tbase(C.agreed_wm);   // the same on every rank (min over ranks)
    // the batch NS ago used this slot: its exchange is posted by now (in the rare case that its counts were still
    // missing at every earlier chance, this waits for them)
    while (!C.posts.empty() && std::any_of(C.posts.begin(), C.posts.end(), [&](const Comm::Post &Q) { return Q.slot == slot; }))
        GWO_TRY(comm_post());
    DevBuf &sb = C.rsend[slot];
    // the slot's last exchange (NS batches ago) sent from this buffer: K1 overwrites it only behind that (device-side)
    if (C.used_send[slot]) GWO_TRY(hipcheck(hipStreamWaitEvent(stream, C.ev_rrecv[slot], 0), "send slot"));
    const size_t need = (size_t)P * (C.rcap * 20 + C.wcap * 24) + 24;
    if (sb.bytes < need) {
        if (C.used_send[slot]) GWO_TRY(hipcheck(hipEventSynchronize(C.ev_rrecv[slot]), "send slot"));   // (growth only)
        GWO_TRY(ensure_buf(sb, need));
    }
    *rt = LogRoute{};
    rt->mode = 1;
    rt->nranks = P;
    rt->me = C.rank;
    rt->send = (int64_t *)sb.ptr;
    rt->rcap = C.rcap;
    rt->wcap = C.wcap;
    rt->tbase = C.tbase;
    rt->cursor = (unsigned long long *)C.cursor.ptr;
    rt->count = (unsigned long long *)C.rcnt[slot].ptr;
    if (n == 0) GWO_TRY(hipcheck(hipMemsetAsync(C.rcnt[slot].ptr, 0, (size_t)2 * P * 8, stream), "counts"));
    return GWO_OK;
}

// Right behind the routed K1 (main stream): the slot's exchange may start once K1 has finished.
gwo_status Handle::comm_mark_routed() {
    return hipcheck(hipEventRecord(comm->ev_rout[comm->rslot], stream), "event");
}

// After the routed K1 of batch i is queued: its per-destination (narrow, wide) counts are exchanged on the count
// communicator and stream right behind K1 (the counts never queue behind records on the wire) and published, with
// the counts received, to host-mapped memory by a one-wave kernel (sequence word last).  Then batch i-1's record
// exchange is posted: its counts arrived while batch i's K1 ran, so the host reads them without waiting.
gwo_status Handle::comm_after_route(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n) {
    (void)k;
    (void)t;
    (void)v;
    Comm &C = *comm;
    const int P = route_ranks(C), me = C.rank;
    const bool virt = C.vranks > 1;
    const int slot = C.rslot;
    unsigned long long *d_send = (unsigned long long *)C.rcnt[slot].ptr, *d_recv = d_send + 2 * P;
    if (n == 0) GWO_TRY(comm_mark_routed());   // (no K1 ran: the counts were zeroed on the main stream)
    GWO_TRY(hipcheck(hipStreamWaitEvent(C.cs2, C.ev_rout[slot], 0), "event wait"));
    // one send/recv pair per peer; virtual ranks send to this rank itself, so what it routes to virtual GPU p
    // comes back "from p" through the same RCCL calls a real rank makes
    GWO_TRY(nccl_ok(this, ncclGroupStart(), "group"));
    for (int p = 0; p < P; ++p) {
        if (p == me) continue;
        const int peer = virt ? me : p;
        GWO_TRY(nccl_ok(this, ncclSend(d_send + 2 * p, 2, ncclUint64, peer, C.nc2, C.cs2), "send count"));
        GWO_TRY(nccl_ok(this, ncclRecv(d_recv + 2 * p, 2, ncclUint64, peer, C.nc2, C.cs2), "recv count"));
    }
    GWO_TRY(nccl_ok(this, ncclGroupEnd(), "group end"));
    launch_publish_words(d_send, 4 * P, C.hcnt_dev[slot], ++C.cnt_seq, C.cs2);
    GWO_TRY(launch_ok("count readback"));
    GWO_TRY(hipcheck(hipEventRecord(C.ev_cnt[slot], C.cs2), "event"));
    C.routed++;
    C.posts.emplace_back();
    Comm::Post &Q = C.posts.back();
    Q.slot = slot;
    Q.seq = C.cnt_seq;
    Q.rcap = C.rcap;
    Q.wcap = C.wcap;
    Q.tbase = C.tbase;
    Q.g = log_geom_now();
    C.used_send[slot] = true;
    C.rslot = (slot + 1) % Comm::NS;
    // batch i-1's exchange now, behind this K1, if its counts are there (no wait); else after this batch's readback,
    // or at the latest when its slot comes round again.  (Inside this batch's insert: no received records may be
    // inserted here, so a post whose receive slot still holds some waits for gwo_submit's own call.)
    return comm_post_older(false, false);
}

// Counts of a routed batch are on the host (GWO_COMM_HOLD_COUNTS=n, diagnostics: every 4th batch's counts count as
// missing until n more batches were routed -- the late-count interleavings of a loaded node, on one GPU).
static bool counts_arrived(const Comm &C, const Comm::Post &Q, int P) {
    if (C.hold > 0 && Q.seq % 4 == 1 && C.cnt_seq < Q.seq + (unsigned long long)C.hold) return false;
    return *(volatile const unsigned long long *)(C.hcnt[Q.slot] + 4 * P) == Q.seq;
}

// Posts the record exchanges of the routed batches before the newest, oldest first: all of them (wait: missing counts
// are waited for, counted in count_waits), or (!wait) as long as their counts have arrived.  may_insert: the caller is
// between batches, so received records still in a post's receive slot may be inserted first (comm_post); else such a
// post stops the loop.
gwo_status Handle::comm_post_older(bool wait, bool may_insert) {
    Comm &C = *comm;
    const int P = route_ranks(C);
    while (C.posts.size() > 1) {
        const Comm::Post &Q = C.posts.front();
        if (!wait && !counts_arrived(C, Q, P)) break;
        if (!may_insert && std::any_of(C.recvq.begin(), C.recvq.end(), [&](const Comm::Recv &R) { return R.slot == Q.slot; }))
            break;
        GWO_TRY(comm_post());
    }
    return GWO_OK;
}

// K1's readback of a routed batch (its largest destination counts): a region that overflowed its capacity (skewed
// keys) is routed again with exact capacities, inside the batch's gwo_submit -- the batch's columns are still the
// caller's.  This GPU's records were partitioned by the first K1 (route-only mode skips them); the counts already
// exchanged are exact either way.
gwo_status Handle::comm_check_route(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n, uint64_t maxn,
                                    uint64_t maxw) {
    Comm &C = *comm;
    if (C.posts.empty()) return GWO_OK;
    Comm::Post &Q = C.posts.back();   // the batch being resolved (the newest routed one: no pipelining with a comm)
    if (maxn <= Q.rcap && maxw <= Q.wcap) return GWO_OK;
    const int P = route_ranks(C);
    const uint64_t rcap = (std::max<uint64_t>(Q.rcap, maxn) + 1) & ~1ull, wcap = std::max<uint64_t>(Q.wcap, maxw);
    DevBuf &sbuf = C.rsend[Q.slot];
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "re-route"));   // the send buffer may move (rare: skewed keys)
    GWO_TRY(ensure_buf(sbuf, (size_t)P * (rcap * 20 + wcap * 24) + 24));
    LogRoute rt{};
    rt.mode = 3;   // route only: this GPU's records were partitioned by the first K1
    rt.nranks = P;
    rt.me = C.rank;
    rt.send = (int64_t *)sbuf.ptr;
    rt.rcap = rcap;
    rt.wcap = wcap;
    rt.tbase = Q.tbase;
    rt.cursor = (unsigned long long *)C.cursor.ptr;
    GWO_TRY(ensure_buf(C.counts, (size_t)6 * P * 8 + 16));
    rt.count = (unsigned long long *)C.counts.ptr + 4 * P;   // (scratch: the counts are known)
    GWO_TRY(log_route_only(k, t, v, n, rt));
    GWO_TRY(hipcheck(hipEventRecord(C.ev_rout[Q.slot], stream), "event"));
    Q.rcap = rcap;
    Q.wcap = wcap;
    return GWO_OK;
}

// Posts the record exchange of the oldest routed batch not posted yet: its counts from the host-mapped block (already
// there unless a flush forces the current batch's exchange), then per peer the narrow records as three arrays (keys,
// values, int32 timestamps: 20 B a record) and the wide ones, on the record stream behind the batch's routed K1.
gwo_status Handle::comm_post() {
    Comm &C = *comm;
    const Comm::Post Q = C.posts.front();
    C.posts.pop_front();
    const int P = route_ranks(C), me = C.rank;
    const bool virt = C.vranks > 1;
    constexpr int NSLOT = Comm::NS;
    (void)NSLOT;
    volatile const unsigned long long *seqw = C.hcnt[Q.slot] + 4 * P;
    if (*seqw != Q.seq) {   // the counts are not there yet: this post waits for them
        const bool flow = not_done(C.ev_rout[Q.slot]);   // (their K1 has not even finished: flow control)
        (flow ? C.bp_count_waits : C.count_waits)++;
        static const bool trace = getenv("GWO_COMM_TRACE") != nullptr;   // (diagnostics)
        const hipError_t q2 = trace ? hipStreamQuery(C.cs2) : hipSuccess, q1 = trace ? hipStreamQuery(C.cs) : hipSuccess,
                         q0 = trace ? hipStreamQuery(stream) : hipSuccess;
        const unsigned long long seen = *seqw;
        const auto t0 = std::chrono::steady_clock::now();
        GWO_TRY(spin_seq((const unsigned long long *)seqw, Q.seq, "count exchange", C.cs2));
        const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        (flow ? C.flow_wait_ns : C.count_wait_ns) += ns;
        if (trace)
            fprintf(stderr, "[comm] post seq %llu (latest %llu) saw %llu: waited %.1f us; cs2 %s cs %s main %s\n", Q.seq,
                    C.cnt_seq, seen, ns / 1e3, q2 == hipSuccess ? "idle" : "busy", q1 == hipSuccess ? "idle" : "busy",
                    q0 == hipSuccess ? "idle" : "busy");
    }
    unsigned long long hs[2 * LOG_RT_MAX], hr[2 * LOG_RT_MAX];
    memcpy(hs, C.hcnt[Q.slot], (size_t)2 * P * 8);
    memcpy(hr, C.hcnt[Q.slot] + 2 * P, (size_t)2 * P * 8);
    hs[2 * me] = hs[2 * me + 1] = 0;   // (K1 never routes a record to its own GPU)
    hr[2 * me] = hr[2 * me + 1] = 0;
    std::vector<uint64_t> rn(P + 1, 0), rw(P + 1, 0);
    for (int p = 0; p < P; ++p) {
        rn[p + 1] = rn[p] + hr[2 * p];
        rw[p + 1] = rw[p] + hr[2 * p + 1];
    }
    const int64_t RN = (int64_t)rn[P], RW = (int64_t)rw[P];
    // receive buffer: keys[RN], values[RN], int32 ts[RN] (padded to a word), then the wide records
    const int64_t ts_words = (RN + 1) / 2;
    Comm::Recv R;
    R.slot = Q.slot;
    R.n = RN;
    R.w = RW;
    R.off_w = 2 * RN + ts_words;
    R.tbase = Q.tbase;
    R.g = Q.g;
    // Received records still waiting in this receive slot (an older batch's, kept back while a later batch's counts
    // were late) are inserted first, oldest first, so ev_read below covers them: otherwise this exchange would
    // overwrite them (or the growth path free their buffer) before their K1 read them.  (Callers inside a batch's
    // insert never get here with such records: comm_post_older(.., false) leaves the post for later.)
    for (size_t i = C.recvq.size(); i-- > 0;)
        if (C.recvq[i].slot == Q.slot) {
            GWO_TRY(comm_insert_received(C.recvq.size() - (i + 1)));
            break;
        }
    // the exchange follows the batch's routed K1 and the K1 that last read this receive slot (device-side order)
    GWO_TRY(hipcheck(hipStreamWaitEvent(C.cs, C.ev_rout[Q.slot], 0), "event wait"));
    if (C.used_read[Q.slot]) GWO_TRY(hipcheck(hipStreamWaitEvent(C.cs, C.ev_read[Q.slot], 0), "event wait"));
    DevBuf &rbuf = C.rrecv[Q.slot];
    const size_t need = (size_t)(R.off_w + 3 * RW) * 8 + 24;
    if (rbuf.bytes < need) {
        if (C.used_read[Q.slot]) GWO_TRY(hipcheck(hipEventSynchronize(C.ev_read[Q.slot]), "receive slot"));   // (growth)
        GWO_TRY(ensure_buf(rbuf, need));
    }
    int64_t *rb = (int64_t *)rbuf.ptr;
    int64_t *sb = (int64_t *)C.rsend[Q.slot].ptr;
    prof_begin(GWO_KERNEL_EXCHANGE, C.cs);
    GWO_TRY(nccl_ok(this, ncclGroupStart(), "group"));
    for (int p = 0; p < P; ++p) {
        if (p == me) continue;
        const int peer = virt ? me : p;
        const uint64_t sn = hs[2 * p], sw = hs[2 * p + 1], qn = hr[2 * p], qw = hr[2 * p + 1];
        if (sn) {
            GWO_TRY(nccl_ok(this, ncclSend(log_rt_keys(sb, Q.rcap, p), sn, ncclInt64, peer, C.nc, C.cs), "send keys"));
            GWO_TRY(nccl_ok(this, ncclSend(log_rt_vals(sb, Q.rcap, p), sn, ncclInt64, peer, C.nc, C.cs), "send values"));
            GWO_TRY(nccl_ok(this, ncclSend(log_rt_ts32(sb, Q.rcap, p), sn, ncclInt32, peer, C.nc, C.cs), "send ts"));
        }
        if (sw)
            GWO_TRY(nccl_ok(this, ncclSend(log_rt_wide(sb, Q.rcap, P, Q.wcap, p), 3 * sw, ncclInt64, peer, C.nc, C.cs),
                            "send wide"));
        if (qn) {
            GWO_TRY(nccl_ok(this, ncclRecv(rb + rn[p], qn, ncclInt64, peer, C.nc, C.cs), "recv keys"));
            GWO_TRY(nccl_ok(this, ncclRecv(rb + RN + rn[p], qn, ncclInt64, peer, C.nc, C.cs), "recv values"));
            GWO_TRY(nccl_ok(this, ncclRecv((int32_t *)(rb + 2 * RN) + rn[p], qn, ncclInt32, peer, C.nc, C.cs),
                            "recv ts"));
        }
        if (qw)
            GWO_TRY(nccl_ok(this, ncclRecv(rb + R.off_w + 3 * rw[p], 3 * qw, ncclInt64, peer, C.nc, C.cs),
                            "recv wide"));
    }
    GWO_TRY(nccl_ok(this, ncclGroupEnd(), "group end"));
    prof_end(GWO_KERNEL_EXCHANGE, RN + RW, C.cs);
    GWO_TRY(hipcheck(hipEventRecord(C.ev_rrecv[Q.slot], C.cs), "event"));
    C.recvq.push_back(R);
    return GWO_OK;
}

// The main stream waits for the non-log exchange's receives (comm_exchange, comm stream) before reading them.
gwo_status Handle::comm_wait_received() {
    if (route_ranks(*comm) == 1) return GWO_OK;
    return hipcheck(hipStreamWaitEvent(stream, comm->ev_recv, 0), "exchange wait");
}

// Deferred receives (tumbling log layout, allowedLateness 0, no side output): a routed batch's exchange is posted at
// the next routed batch and its received records are inserted at the one after -- or at any earlier point that
// observes state or fires a window they may fall into (log_flush).  They are classified at their own batch's
// watermark (the geometry kept with them), exactly as if inserted at once: a fire that could take them flushes them
// first (log_pending_may_fire).
bool Handle::comm_defers() const {
    return comm && logst && !slog && cfg.allowed_lateness == 0 && !side_enabled() && route_ranks(*comm) > 1 &&
           comm->defer;
}

// Inserts received records: every posted exchange but the `keep` newest (whose records may still be on the wire).
gwo_status Handle::comm_insert_received(size_t keep) {
    Comm &C = *comm;
    while (C.recvq.size() > keep) {
        const Comm::Recv R = C.recvq.front();
        C.recvq.pop_front();
        GWO_TRY(hipcheck(hipStreamWaitEvent(stream, C.ev_rrecv[R.slot], 0), "exchange wait"));
        const int64_t *rb = (const int64_t *)C.rrecv[R.slot].ptr;
        if (R.n) GWO_TRY(insert_log(rb, (const int64_t *)(rb + 2 * R.n), rb + R.n, R.n, 1, nullptr, true, R.tbase, &R.g));
        if (R.w) GWO_TRY(insert_log(rb + R.off_w, rb + R.off_w + 1, rb + R.off_w + 2, R.w, 3, nullptr, false, 0, &R.g));
        GWO_TRY(hipcheck(hipEventRecord(C.ev_read[R.slot], stream), "event"));
        C.used_read[R.slot] = true;
    }
    return GWO_OK;
}

// Every routed batch's records inserted: the pending exchange posted (this waits for its counts), all receives read.
gwo_status Handle::comm_flush_received() {
    if (!comm) return GWO_OK;
    while (!comm->posts.empty()) GWO_TRY(comm_post());
    return comm_insert_received(0);
}

// The oldest watermark any routed batch not yet inserted was classified at.
bool Handle::comm_pending_wm(int64_t *wm) const {
    if (!comm) return false;
    bool any = false;
    int64_t m = 0;
    for (const Comm::Post &Q : comm->posts) {
        m = any ? std::min(m, Q.g.wm) : Q.g.wm;
        any = true;
    }
    for (const Comm::Recv &R : comm->recvq) {
        m = any ? std::min(m, R.g.wm) : R.g.wm;
        any = true;
    }
    if (any) *wm = m;
    return any;
}

// AoS {key, ts, value} records -> the handle's column scratch (table, sliding and session layouts)
gwo_status Handle::comm_unpack(const int64_t *aos, int64_t n, const int64_t **rk, const int64_t **rt,
                               const int64_t **rv) {
    Comm &C = *comm;
    GWO_TRY(ensure_buf(C.rk, n * 8 + 8));
    GWO_TRY(ensure_buf(C.rt, n * 8 + 8));
    GWO_TRY(ensure_buf(C.rv, n * 8 + 8));
    if (n > 0) {
        launch_unpack(aos, n, (int64_t *)C.rk.ptr, (int64_t *)C.rt.ptr, (int64_t *)C.rv.ptr, stream);
        GWO_TRY(launch_ok("unpack"));
    }
    *rk = (const int64_t *)C.rk.ptr;
    *rt = (const int64_t *)C.rt.ptr;
    *rv = needs_value ? (const int64_t *)C.rv.ptr : nullptr;
    return GWO_OK;
}

// The min over ranks of the channel watermarks (StatusWatermarkValve.java:163-181): an RCCL all-reduce on the main
// stream.  It also runs on a 1-rank communicator that rehearses P virtual ranks, so that call executes on one GPU too.
static gwo_status allreduce_min(Handle *h, int64_t v, int64_t *out) {
    Comm &C = *h->comm;
    int64_t *d = (int64_t *)C.counts.ptr + 6 * std::max(C.nranks, C.vranks);   // past the count words and scratch
    *C.h_wm = v;
    // on the count communicator's stream: it does not wait for a record exchange still on the wire
    GWO_TRY(h->hipcheck(hipMemcpyAsync(d, C.h_wm, 8, hipMemcpyHostToDevice, C.cs2), "wm"));
    GWO_TRY(nccl_ok(h, ncclAllReduce(d, d, 1, ncclInt64, ncclMin, C.nc2, C.cs2), "allreduce wm"));
    GWO_TRY(h->hipcheck(hipMemcpyAsync(C.h_wm, d, 8, hipMemcpyDeviceToHost, C.cs2), "wm"));
    GWO_TRY(h->hipcheck(hipStreamSynchronize(C.cs2), "wm sync"));
    *out = *C.h_wm;
    return GWO_OK;
}

// Asynchronous agreement (gwo_comm_set_async_watermark): this call's all-reduce is queued with its result published to
// host-mapped memory, and the min the previous call queued -- long complete -- is applied.  Every rank applies the
// same agreed values, one call later than the synchronous mode (as if one channel's watermark arrived one step
// later: a valid StatusWatermarkValve history, monotone because each rank's input is).  The end of input
// (Long.MAX_VALUE) and a single real rank (virtual ranks: the min is its own) agree synchronously.
static gwo_status allreduce_min_async(Handle *h, int64_t v, int64_t *applied) {
    Comm &C = *h->comm;
    int64_t *d = (int64_t *)C.counts.ptr + 6 * std::max(C.nranks, C.vranks) + 2;   // (past the synchronous word)
    const int q = (int)(C.wm_seq & 1);
    if (!C.hwm[q]) {
        // [0] the published min, [1] its sequence word
        GWO_TRY(h->hipcheck(hipHostMalloc((void **)&C.hwm[q], 32, hipHostMallocCoherent | hipHostMallocMapped), "wm"));
        GWO_TRY(h->hipcheck(hipHostGetDevicePointer((void **)&C.hwm_dev[q], C.hwm[q], 0), "wm"));
    }
    if (C.wm_pending) {   // the previous call's min
        volatile const unsigned long long *seqw = C.hwm[q ^ 1] + 1;
        if (*seqw != C.wm_seq) {   // (queued behind the previous batch's count exchange, itself behind its K1)
            // (the agreement was queued right behind the then newest routed batch's count exchange)
            const bool flow = C.wm_after_slot >= 0 && not_done(C.ev_cnt[C.wm_after_slot]);
            (flow ? C.bp_wm_waits : C.wm_waits)++;
            const auto t0 = std::chrono::steady_clock::now();
            GWO_TRY(h->spin_seq((const unsigned long long *)seqw, C.wm_seq, "watermark agreement", C.cs2));
            (flow ? C.flow_wait_ns : C.wm_wait_ns) +=
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        }
        *applied = (int64_t)C.hwm[q ^ 1][0];
    } else {
        *applied = C.agreed_wm;
    }
    C.wm_after_slot = C.routed > 0 ? (C.rslot + Comm::NS - 1) % Comm::NS : -1;
    launch_put_word((unsigned long long *)d, (unsigned long long)v, C.cs2);   // (no copy from host memory)
    GWO_TRY(h->launch_ok("wm"));
    GWO_TRY(nccl_ok(h, ncclAllReduce(d, d, 1, ncclInt64, ncclMin, C.nc2, C.cs2), "allreduce wm"));
    launch_publish_words((const unsigned long long *)d, 1, C.hwm_dev[q], ++C.wm_seq, C.cs2);
    GWO_TRY(h->launch_ok("wm readback"));
    C.wm_pending = true;
    return GWO_OK;
}

gwo_status Handle::comm_min_watermark(int64_t wm_in, int64_t *out) {
    Comm &C = *comm;
    if (C.nranks == 1 && C.vranks <= 1) {   // nothing to agree on
        *out = C.agreed_wm = wm_in;
        return GWO_OK;
    }
    if (C.async_wm && wm_in != (int64_t)0x7fffffffffffffffLL) {
        int64_t applied = C.agreed_wm;
        GWO_TRY(allreduce_min_async(this, wm_in, &applied));
        if (C.nranks == 1) applied = wm_in;   // virtual ranks: the collective ran, the min over one rank is its input
        *out = C.agreed_wm = std::max(C.agreed_wm, applied);
        return GWO_OK;
    }
    if (C.wm_pending) {   // a queued asynchronous agreement completes first (RCCL orders the count communicator)
        const int q = (int)(C.wm_seq & 1) ^ 1;
        GWO_TRY(spin_seq(C.hwm[q] + 1, C.wm_seq, "watermark agreement", C.cs2));
        C.wm_pending = false;
    }
    C.wm_waits++;
    const auto t0 = std::chrono::steady_clock::now();
    GWO_TRY(allreduce_min(this, wm_in, out));
    C.wm_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    C.agreed_wm = *out;
    return GWO_OK;
}

}  // namespace gwo

using namespace gwo;

// RCCL connects peers lazily, at a communicator's first operation of a kind: one word to and from every peer on both
// communicators now, so the first routed batch and watermark do not pay for the connection setup (measured: the
// first asynchronous watermark agreements were still queued behind it when the next watermark came).
static gwo_status comm_warm(Handle *h) {
    Comm &C = *h->comm;
    const int P = route_ranks(C), me = C.rank;
    if (P <= 1) return GWO_OK;
    uint64_t *d = (uint64_t *)C.counts.ptr;   // word 0 is sent, words 1 + p receive (scratch: 6 * P words)
    for (int pass = 0; pass < 2; ++pass) {
        ncclComm_t nc = pass ? C.nc : C.nc2;
        hipStream_t s = pass ? C.cs : C.cs2;
        GWO_TRY(nccl_ok(h, ncclGroupStart(), "group"));
        for (int p = 0; p < P; ++p) {
            if (p == me) continue;
            const int peer = C.vranks > 1 ? me : p;
            GWO_TRY(nccl_ok(h, ncclSend(d, 1, ncclUint64, peer, nc, s), "warm send"));
            GWO_TRY(nccl_ok(h, ncclRecv(d + 1 + p, 1, ncclUint64, peer, nc, s), "warm recv"));
        }
        GWO_TRY(nccl_ok(h, ncclGroupEnd(), "group end"));
        GWO_TRY(h->hipcheck(hipStreamSynchronize(s), "comm warm-up"));
    }
    return GWO_OK;
}

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
    if (h->cfg.key_kind == GWO_KEY_STRING)   // ids are per handle: the exchange would have to ship the Strings
        return h->fail(GWO_ERR_UNSUPPORTED, "the multi-GPU exchange carries int64 keys; route String keys on the host "
                                            "(gwo_assign_key_groups_utf16) and submit per GPU");
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
    if (nranks == 1)
        if (const char *e = getenv("GWO_COMM_VIRTUAL")) {   // bench/test rehearsal of a rank's data path at P GPUs
            const int v = atoi(e);
            C->vranks = v > 1 && v <= LOG_RT_MAX ? v : 0;
        }
    const int cranks = std::max(nranks, C->vranks);
    if (hipHostMalloc((void **)&C->h_counts, (size_t)4 * cranks * 8 + 16, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&C->h_wm, 16, hipHostMallocDefault) != hipSuccess) {
        delete C;
        return GWO_ERR_OUT_OF_MEMORY;
    }
    if (const char *e = getenv("GWO_COMM_DEFER")) C->defer = atoi(e) != 0;
    if (const char *e = getenv("GWO_COMM_HOLD_COUNTS")) C->hold = atoi(e);
    // The count stream gets the greatest priority: HIP multiplexes streams onto a few hardware queues (4 per process
    // on this pool), and a default-priority count stream shared the record stream's queue (measured in the kernel
    // trace), so the watermark all-reduce waited behind the previous batch's records on the wire.
    int prio_least = 0, prio_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    if (hipStreamCreateWithFlags(&C->cs, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&C->cs2, hipStreamNonBlocking, prio_greatest) != hipSuccess ||
        hipEventCreateWithFlags(&C->ev_routed, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&C->ev_recv, hipEventDisableTiming) != hipSuccess || !comm_events(C)) {
        h->comm = C;   // comm_free releases what was created
        h->comm_free();
        return GWO_ERR_HIP;
    }
    ncclUniqueId u;
    memcpy(&u, id, GWO_COMM_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&C->nc, nranks, u, rank);
    // the count communicator: same ranks, its own RCCL ordering (a collective: every rank splits here)
    if (r == ncclSuccess) r = ncclCommSplit(C->nc, 0, rank, &C->nc2, nullptr);
    h->comm = C;
    if (r != ncclSuccess) {
        h->comm_free();
        return h->fail(GWO_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    // the ranks' watermarks may differ (subtasks restored from different checkpoints): agree on their min now, so
    // every rank's first routed batch encodes and decodes wire timestamps against the same base
    gwo_status st = h->ensure_buf(C->counts, (size_t)6 * cranks * 8 + 32);   // (never reallocated later)
    if (const char *e = getenv("GWO_COMM_ASYNC_WM")) C->async_wm = atoi(e) != 0;
    if (st == GWO_OK) st = allreduce_min(h, h->wm, &C->agreed_wm);
    if (st == GWO_OK) st = comm_warm(h);
    return st;
}

// Stateless batch form of KeyGroupStreamPartitioner.selectChannel (the route kernel the exchange
// uses), for hosts that run their own transport and for the tests.  Host or device pointers.
extern "C" gwo_status gwo_partition_by_operator(const int64_t *key, const int64_t *ts, const int64_t *value, int64_t n,
                                                int32_t key_kind, int32_t max_parallelism, int32_t parallelism,
                                                int64_t *out, int64_t cap, int64_t *counts, int32_t device) {
    if (n < 0 || cap < 0 || !out || !counts || (n > 0 && (!key || !ts))) return GWO_ERR_INVALID_ARGUMENT;
    if (max_parallelism < 1 || max_parallelism > 32768 || parallelism < 1 || parallelism > 256 ||
        parallelism > max_parallelism || (key_kind != GWO_KEY_LONG && key_kind != GWO_KEY_INT))
        return GWO_ERR_INVALID_ARGUMENT;
    DeviceGuard guard_(device);
    hipStream_t s;
    // a blocking stream: ordered behind the null stream's work (a producer there needs no host sync, gwo.h)
    if (hipStreamCreate(&s) != hipSuccess) return GWO_ERR_HIP;
    const size_t nb = (size_t)n * 8 + 8, ob = (size_t)parallelism * cap * 24 + 24;
    void *dk = nullptr, *dt = nullptr, *dv = nullptr, *dout = nullptr, *dcur = nullptr, *dcnt = nullptr;
    gwo_status st = GWO_OK;
    if (hipMalloc(&dk, nb) != hipSuccess || hipMalloc(&dt, nb) != hipSuccess || hipMalloc(&dv, nb) != hipSuccess ||
        hipMalloc(&dout, ob) != hipSuccess || hipMalloc(&dcur, route_cursor_bytes()) != hipSuccess ||
        hipMalloc(&dcnt, 256 * 8) != hipSuccess)
        st = GWO_ERR_OUT_OF_MEMORY;
    if (st == GWO_OK) {
        (void)hipMemsetAsync(dcur, 0, route_cursor_bytes(), s);
        (void)hipMemsetAsync(dv, 0, nb, s);
        if (n > 0) {
            if (copy_in(dk, key, n * 8, s) != hipSuccess || copy_in(dt, ts, n * 8, s) != hipSuccess ||
                (value && copy_in(dv, value, n * 8, s) != hipSuccess))
                st = GWO_ERR_HIP;
            launch_route((const int64_t *)dk, (const int64_t *)dt, (const int64_t *)dv, n, key_kind, max_parallelism,
                         parallelism, (unsigned long long *)dcur, (uint64_t)cap, (int64_t *)dout, s);
        }
        launch_route_collect((unsigned long long *)dcur, parallelism, (unsigned long long *)dcnt, s);
        if (copy_out(out, dout, (size_t)parallelism * cap * 24, s) != hipSuccess ||
            copy_out(counts, dcnt, (size_t)parallelism * 8, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            st = GWO_ERR_HIP;
    }
    for (void *p : {dk, dt, dv, dout, dcur, dcnt})
        if (p) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return st;
}

extern "C" gwo_status gwo_comm_set_async_watermark(gwo_handle *hh, int32_t enabled) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h) return GWO_ERR_INVALID_ARGUMENT;
    if (h->poisoned) return h->poison_status;
    if (!h->comm) return h->fail(GWO_ERR_STATE, "no communicator: gwo_comm_init first");
    h->comm->async_wm = enabled != 0;
    return GWO_OK;
}

extern "C" gwo_status gwo_comm_stats(gwo_handle *hh, int64_t *routed_batches, int64_t *count_waits, int64_t *wm_waits) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h || !routed_batches || !count_waits || !wm_waits) return GWO_ERR_INVALID_ARGUMENT;
    if (!h->comm) return h->fail(GWO_ERR_STATE, "no communicator");
    *routed_batches = h->comm->routed;
    *count_waits = h->comm->count_waits;
    *wm_waits = h->comm->wm_waits;
    return GWO_OK;
}

extern "C" gwo_status gwo_comm_wait_stats(gwo_handle *hh, gwo_comm_waits *out) {
    Handle *h = reinterpret_cast<Handle *>(hh);
    if (!h || !out) return GWO_ERR_INVALID_ARGUMENT;
    if (!h->comm) return h->fail(GWO_ERR_STATE, "no communicator");
    const Comm &C = *h->comm;
    out->routed_batches = C.routed;
    out->count_waits = C.count_waits;
    out->wm_waits = C.wm_waits;
    out->flow_count_waits = C.bp_count_waits;
    out->flow_wm_waits = C.bp_wm_waits;
    out->count_wait_ns = C.count_wait_ns;
    out->wm_wait_ns = C.wm_wait_ns;
    out->flow_wait_ns = C.flow_wait_ns;
    return GWO_OK;
}
