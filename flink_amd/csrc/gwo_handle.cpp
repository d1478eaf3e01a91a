// gwo_handle.cpp -- handle lifecycle, batch submit, watermark dispatch and output draining.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>

#include "gwo_handle.h"
#include "gwo_slide.h"
#include "gwo_log.h"

namespace gwo {

static int64_t floor_mod(int64_t a, int64_t b) {
    int64_t r = a % b;
    return r < 0 ? r + b : r;
}

// WindowOperator ctor + assigner ctors: argument checks mirror the reference exceptions.
gwo_status Handle::init(const gwo_config &c) {
    cfg = c;
    if (c.abi_version != GWO_ABI_VERSION) return fail(GWO_ERR_INVALID_ARGUMENT, "ABI version %d != %d", c.abi_version, GWO_ABI_VERSION);
    if (c.allowed_lateness < 0) return fail(GWO_ERR_INVALID_ARGUMENT, "The allowed lateness cannot be negative.");
    switch (c.assigner) {
        case GWO_ASSIGNER_TUMBLING:
            // TumblingEventTimeWindows.java:57-60
            if (c.size <= 0 || (c.offset < 0 ? -c.offset : c.offset) >= c.size)
                return fail(GWO_ERR_INVALID_ARGUMENT, "TumblingEventTimeWindows parameters must satisfy abs(offset) < size");
            break;
        case GWO_ASSIGNER_SLIDING:
            // SlidingEventTimeWindows.java:56-60
            if ((c.offset < 0 ? -c.offset : c.offset) >= c.slide || c.size <= 0)
                return fail(GWO_ERR_INVALID_ARGUMENT,
                            "SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0");
            break;
        case GWO_ASSIGNER_SESSION:
            // EventTimeSessionWindows.java:50-55
            if (c.gap <= 0) return fail(GWO_ERR_INVALID_ARGUMENT, "EventTimeSessionWindows parameters must satisfy 0 < size");
            break;
        default: return fail(GWO_ERR_UNSUPPORTED, "unknown assigner %d", c.assigner);
    }
    if (c.max_parallelism <= 0 || c.max_parallelism > 32768)
        return fail(GWO_ERR_INVALID_ARGUMENT, "maxParallelism must be in (0, 32768]");
    if (c.key_group_start < 0 || c.key_group_end >= c.max_parallelism || c.key_group_start > c.key_group_end)
        return fail(GWO_ERR_INVALID_ARGUMENT, "invalid KeyGroupRange [%d, %d]", c.key_group_start, c.key_group_end);
    if (c.key_kind != GWO_KEY_LONG && c.key_kind != GWO_KEY_INT && c.key_kind != GWO_KEY_STRING)
        return fail(GWO_ERR_UNSUPPORTED, "key kind %d", c.key_kind);
    if (c.value_dtype != GWO_DTYPE_INT64 && c.value_dtype != GWO_DTYPE_FLOAT64)
        return fail(GWO_ERR_UNSUPPORTED, "value dtype %d", c.value_dtype);
    if (c.num_aggs < 1 || c.num_aggs > GWO_MAX_AGGS) return fail(GWO_ERR_INVALID_ARGUMENT, "num_aggs must be 1..4");

    // ---- accumulator plan ----
    const bool f64 = c.value_dtype == GWO_DTYPE_FLOAT64;
    plan = AccPlan{};
    plan.value_is_f64 = f64;
    rplan = ResultPlan{};
    rplan.naggs = c.num_aggs;
    rplan.value_is_f64 = f64;
    needs_value = false;
    int w = 0;
    auto add_word = [&](int op, int src, int64_t ident) {
        plan.op[w] = op;
        plan.src[w] = src;
        plan.ident[w] = ident;
        ++w;
    };
    for (int a = 0; a < c.num_aggs; ++a) {
        rplan.kind[a] = c.aggs[a];
        rplan.word[a] = w;
        switch (c.aggs[a]) {
            case GWO_AGG_COUNT: add_word(ACC_ADD_I64, SRC_ONE, 0); break;
            case GWO_AGG_SUM:
                add_word(f64 ? ACC_ADD_F64 : ACC_ADD_I64, SRC_VALUE, 0);
                needs_value = true;
                break;
            case GWO_AGG_MIN:
                add_word(ACC_MIN_I64, f64 ? SRC_ORDER : SRC_VALUE, (int64_t)0x7fffffffffffffffLL);
                needs_value = true;
                break;
            case GWO_AGG_MAX:
                add_word(ACC_MAX_I64, f64 ? SRC_ORDER : SRC_VALUE, (int64_t)0x8000000000000000LL);
                needs_value = true;
                break;
            case GWO_AGG_AVG:
                add_word(f64 ? ACC_ADD_F64 : ACC_ADD_I64, SRC_VALUE, 0);
                add_word(ACC_ADD_I64, SRC_ONE, 0);
                needs_value = true;
                break;
            default: return fail(GWO_ERR_UNSUPPORTED, "aggregate kind %d", c.aggs[a]);
        }
    }
    plan.nwords = w;
    plan.stride = ((1 + w) + 1) & ~1;

    // ---- geometry ----
    geom = WindowGeom{};
    geom.size = c.size;
    geom.offset = c.offset;
    geom.lateness = c.allowed_lateness;
    geom.key_kind = c.key_kind;
    geom.max_par = c.max_parallelism;
    geom.kg_lo = c.key_group_start;
    geom.kg_hi = c.key_group_end;
    if (c.assigner == GWO_ASSIGNER_TUMBLING) {
        geom.sliding = 0;
        geom.unit = c.size;
        geom.slide = c.size;
        geom.unit_off = c.offset % c.size;  // (globalOffset + staggerOffset) % size, ALIGNED stagger
        geom.offset = geom.unit_off;
        geom.unit_off_mod = floor_mod(c.offset, c.size);
    } else if (c.assigner == GWO_ASSIGNER_SLIDING) {
        geom.sliding = 1;
        geom.slide = c.slide;
        geom.unit = std::gcd(c.size, c.slide);
        geom.unit_off = c.offset;
        geom.unit_off_mod = floor_mod(c.offset, geom.unit);
    }

    if (geom.size > 0) geom.inv_size = 1.0 / (double)geom.size;
    if (geom.slide > 0) geom.inv_slide = 1.0 / (double)geom.slide;
    if (geom.unit > 0) geom.inv_unit = 1.0 / (double)geom.unit;
    debug = getenv("GWO_DEBUG") != nullptr;
    ktrace = getenv("GWO_KTRACE") != nullptr;
    hprof = getenv("GWO_HOST_PROF") != nullptr && atoi(getenv("GWO_HOST_PROF")) != 0;
    if (ktrace) ktrace_enable(1);
    if (const char *e = getenv("GWO_ASYNC_FIRE")) async_fire = atoi(e) != 0;
    const char *pa = getenv("GWO_PREAGG");
    if (pa) cfg_preagg = atoi(pa) ? 1 : 0;
    if (cfg_preagg >= 0) use_preagg = cfg_preagg;
    if (const char *cb = getenv("GWO_COMBINE")) use_combine = atoi(cb) ? 1 : 0;
    if (const char *cs = getenv("GWO_COMBINE_SPEC")) use_combine_spec = atoi(cs) ? 1 : 0;
    if (const char *ss = getenv("GWO_SCAN_SPEC")) use_scan_spec = atoi(ss) ? 1 : 0;

    // ---- device resources ----
    if (hipSetDevice(c.device) != hipSuccess) return fail(GWO_ERR_HIP, "hipSetDevice(%d) failed", c.device);
    if (c.stream) {
        stream = (hipStream_t)c.stream;
    } else {
        GWO_TRY(hipcheck(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream"));
        own_stream = true;
    }
    GWO_TRY(dalloc((void **)&d_stats, sizeof(BatchStats)));
    {
        std::vector<unsigned long long> sh(SCAN_SHARD_WORDS, 0ull);
        for (int q = 0; q < SCAN_SHARDS; ++q) {
            sh[(size_t)q * SCAN_SW] = 0x7fffffffffffffffull;
            sh[(size_t)q * SCAN_SW + 1] = 0x8000000000000000ull;
        }
        GWO_TRY(dalloc((void **)&d_scan_sh, sh.size() * 8));
        GWO_TRY(hipcheck(hipMemcpy(d_scan_sh, sh.data(), sh.size() * 8, hipMemcpyHostToDevice), "scan shards"));
    }
    GWO_TRY(hipcheck(hipHostMalloc((void **)&h_stats, sizeof(BatchStats), hipHostMallocDefault), "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&h_stats_init, sizeof(BatchStats), hipHostMallocDefault), "pinned"));
    const int kCounters = 1 << 12;
    counter_used.assign(kCounters, 0);
    GWO_TRY(dalloc((void **)&d_counters, (size_t)kCounters * GWO_OCC_WORDS * 8));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&h_counters, (size_t)kCounters * GWO_OCC_WORDS * 8, hipHostMallocDefault),
                     "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&h_scalar, 64, hipHostMallocDefault), "pinned"));
    GWO_TRY(hipcheck(hipHostMalloc((void **)&h_ident_side, GWO_MAX_WORDS * 16 + 16, hipHostMallocDefault), "pinned"));
    GWO_TRY(dalloc((void **)&d_out_count, 8));
    GWO_TRY(dalloc((void **)&d_scratch_count, 8));
    GWO_TRY(dalloc((void **)&d_side_count, 8));
    GWO_TRY(hipcheck(hipMemsetAsync(d_out_count, 0, 8, stream), "memset"));
    GWO_TRY(hipcheck(hipMemsetAsync(d_side_count, 0, 8, stream), "memset"));
    GWO_TRY(hipcheck(hipMemsetAsync(d_counters, 0, (size_t)kCounters * GWO_OCC_WORDS * 8, stream), "memset"));
    if (side_enabled()) GWO_TRY(grow_side(4096));
    if (c.assigner == GWO_ASSIGNER_SLIDING) GWO_TRY(slide_init());   // may append a hidden count word
    if (c.assigner == GWO_ASSIGNER_SESSION) GWO_TRY(session_init());
    if (c.state_layout < GWO_STATE_AUTO || c.state_layout > GWO_STATE_LOG)
        return fail(GWO_ERR_INVALID_ARGUMENT, "state layout %d", c.state_layout);
    // sliding windows over logged panes: every aggregate word an int64 sum (the ring), allowedLateness 0, and
    // the slide divides the size (a pane is one slide)
    const bool slog_ok = c.assigner == GWO_ASSIGNER_SLIDING && slide && slide->ring && c.allowed_lateness == 0 &&
                         c.size % c.slide == 0 && getenv("GWO_SLIDE_TABLE") == nullptr;
    if (c.state_layout == GWO_STATE_LOG && c.assigner == GWO_ASSIGNER_SESSION)
        return fail(GWO_ERR_UNSUPPORTED, "the log-structured state layout serves tumbling and sliding windows only");
    if (c.state_layout == GWO_STATE_LOG && c.assigner == GWO_ASSIGNER_SLIDING && !slog_ok)
        return fail(GWO_ERR_UNSUPPORTED, "the log-structured sliding layout needs int64 count/sum/avg aggregates, "
                                         "allowedLateness 0 and a size that is a multiple of the slide");
    const bool big = c.state_layout == GWO_STATE_LOG ||
                     (c.state_layout == GWO_STATE_AUTO && c.expected_keys >= (1 << 20) && c.allowed_lateness == 0);
    if (c.assigner == GWO_ASSIGNER_TUMBLING && big) GWO_TRY(log_init());
    if (c.assigner == GWO_ASSIGNER_SLIDING && big && slog_ok) {
        GWO_TRY(slog_init());   // (before log_init: the log's lp choice and warm-up see the sliding log)
        GWO_TRY(log_init());
    }
    memset(h_ident_side, 0, GWO_MAX_WORDS * 16 + 16);
    for (int w = 0; w < plan.nwords; ++w) h_ident_side[1 + w] = plan.ident[w];
    return hipcheck(hipStreamSynchronize(stream), "init");
}

Handle::~Handle() {
    DeviceGuard g(cfg.device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (fire_stream) (void)hipStreamSynchronize(fire_stream);
    if (cb_side) (void)hipStreamSynchronize(cb_side);
    if (ktrace) ktrace_report();
    if (hprof) {
        fprintf(stderr, "host us per point:");
        for (int i = 0; i < 32; ++i)
            if (hp_cnt[i]) fprintf(stderr, " [%d] %.2f", i, hp_sum[i] / 1e3 / hp_cnt[i]);
        fprintf(stderr, "\n");
    }
    (void)prof_collect();
    for (hipEvent_t e : event_pool) (void)hipEventDestroy(e);
    comm_free();
    log_free();
    slog_free();
    session_free();
    slide_free();
    dict_free();
    for (auto &kv : tables) (void)hipFree(kv.second.base);
    for (auto &kv : rdone) (void)hipFree(kv.second.base);
    for (auto &t : aux_tables) (void)hipFree(t.base);
    trim_pool();
    if (d_stats) (void)hipFree(d_stats);
    if (d_scan_sh) (void)hipFree(d_scan_sh);
    if (h_stats) (void)hipHostFree(h_stats);
    if (h_stats_init) (void)hipHostFree(h_stats_init);
    if (d_counters) (void)hipFree(d_counters);
    if (h_counters) (void)hipHostFree(h_counters);
    if (h_scalar) (void)hipHostFree(h_scalar);
    if (h_ident_side) (void)hipHostFree(h_ident_side);
    dir_buf.release();
    refire_buf.release();
    for (DevBuf *b : {&cb_dump_key, &cb_dump_acc, &cb_ovf, &cb_blk, &cb_ctr, &cb_dir, &cb_arr, &cb_spec_dir, &sp_dir, &sp_go, &cb_dbg})
        b->release();
    if (cb_rb) (void)hipHostFree(cb_rb);
    if (cb_ev) (void)hipEventDestroy(cb_ev);
    for (hipEvent_t e : {cb_ev_main, cb_ev_gather, cb_ev_merge[0], cb_ev_merge[1]})
        if (e) (void)hipEventDestroy(e);
    if (cb_side) (void)hipStreamDestroy(cb_side);
    cb_go.release();
    if (sp_rb) (void)hipHostFree(sp_rb);
    if (sp_ev) (void)hipEventDestroy(sp_ev);
    stage_key.release();
    stage_ts.release();
    stage_val.release();
    side_key.release();
    side_ts.release();
    side_val.release();
    int64_t *cols[7] = {out.key, out.start, out.end, out.res[0], out.res[1], out.res[2], out.res[3]};
    for (auto *p : cols)
        if (p) (void)hipFree(p);
    if (d_out_count) (void)hipFree(d_out_count);
    if (d_scratch_count) (void)hipFree(d_scratch_count);
    if (d_side_count) (void)hipFree(d_side_count);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
    if (fire_stream) (void)hipStreamDestroy(fire_stream);
    if (ev_main) (void)hipEventDestroy(ev_main);
    if (ev_fire) (void)hipEventDestroy(ev_fire);
    if (ev_out) (void)hipEventDestroy(ev_out);
    if (ev_input) (void)hipEventDestroy(ev_input);
    if (h_out_cnt) (void)hipHostFree(h_out_cnt);
}

gwo_status Handle::submit(const int64_t *key, const int64_t *ts, const void *val, int64_t n) {
    const int64_t *dk = nullptr, *dt = nullptr, *dv = nullptr;
    if (!comm && n == 0) return GWO_OK;
    hp(12, true);
    if (n > 0) GWO_TRY(stage_inputs(key, ts, needs_value ? val : nullptr, n, &dk, &dt, &dv));
    hp(13);
    if (comm && logst) {
        // log layout: K1 routes other GPUs' records while it partitions this one's (comm_route_args)
        LogRoute rt{};
        bool routed = false;
        GWO_TRY(comm_route_args(n, &rt, &routed));
        if (!routed) return n ? insert_log(dk, dt, dv, n) : GWO_OK;   // one rank: nothing leaves this GPU
        if (n > 0) GWO_TRY(insert_log(dk, dt, dv, n, 1, &rt));
        else GWO_TRY(comm_after_route(dk, dt, dv, 0));
        // deferred: the previous batch's exchange is posted (behind this batch's K1 when its counts had arrived, else
        // now if they have, else later -- never waiting), the exchanges posted before the newest have landed and are
        // inserted now; otherwise this batch's exchange completes inside its submit
        if (!comm_defers()) return comm_flush_received();
        GWO_TRY(comm_post_older(false, true));
        return comm_insert_received(1);
    }
    if (comm) {
        const int64_t *aos = nullptr, *loc = nullptr;
        int64_t rn = 0, ln = 0;
        GWO_TRY(comm_exchange(dk, dt, dv, n, &aos, &rn, &loc, &ln));
        // the records this rank keeps (never on the wire), then the ones it received; the log layout's K1 reads
        // both in place (24-B records), the other layouts unpack them to columns
        const int64_t *parts[2] = {loc, aos};
        const int64_t counts[2] = {ln, rn};
        for (int q = 0; q < 2; ++q) {
            if (q == 1) GWO_TRY(comm_wait_received());   // the kept records' pass overlapped the exchange
            if (counts[q] == 0) continue;
            if (logst) {
                GWO_TRY(insert_log(parts[q], parts[q] + 1, parts[q] + 2, counts[q], 3));
                continue;
            }
            const int64_t *rk, *rt, *rv;
            GWO_TRY(comm_unpack(parts[q], counts[q], &rk, &rt, &rv));
            GWO_TRY(submit_local(rk, rt, rv, counts[q]));
        }
        return GWO_OK;
    }
    return submit_local(dk, dt, dv, n);
}

gwo_status Handle::submit_local(const int64_t *k, const int64_t *t, const int64_t *v, int64_t n) {
    if (n == 0) return GWO_OK;
    if (cfg.assigner == GWO_ASSIGNER_SESSION) return insert_session(k, t, v, n);
    if (logst) return insert_log(k, t, v, n);
    return insert_windowed(k, t, v, n);
}

// StatusWatermarkValve.inputWatermark (SJ/runtime/streamstatus/StatusWatermarkValve.java:86-101,163-181): a
// channel's watermark that does not increase is ignored, the operator watermark is the min over channels (ranks)
// and it is forwarded -- here: windows fire -- only when that min grows.  With a communicator every rank must call
// this (the min is a collective), including the calls that turn out to be no-ops.
gwo_status Handle::advance_watermark(int64_t new_wm) {
    if (new_wm > in_wm) in_wm = new_wm;
    new_wm = in_wm;
    if (comm) GWO_TRY(comm_min_watermark(in_wm, &new_wm));
    if (new_wm <= wm) return GWO_OK;
    // a pipelined combine batch whose windows this watermark may fire is resolved first
    if (cb_pend.active && log_may_fire_since(cb_pend.wm, new_wm)) GWO_TRY(combine_flush());
    gwo_status s = GWO_OK;
    switch (cfg.assigner) {
        case GWO_ASSIGNER_TUMBLING: s = logst ? fire_log(new_wm) : fire_tumbling(new_wm); break;
        case GWO_ASSIGNER_SLIDING: s = slog ? fire_slog(new_wm) : fire_sliding(new_wm); break;
        default: s = fire_session(new_wm); break;
    }
    wm = new_wm;
    return s;
}

gwo_status Handle::drain(const gwo_out *cols, int64_t cap, int64_t *n_out) {
    GWO_TRY(finish_fire());
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "drain"));
    uint64_t take = std::min<uint64_t>((uint64_t)cap, out_rows);
    *n_out = (int64_t)take;
    rows_gone += take;
    if (take == 0) return GWO_OK;
    int64_t *src[7] = {out.key, out.start, out.end, out.res[0], out.res[1], out.res[2], out.res[3]};
    void *dst[7] = {cols->key, cols->start, cols->end, cols->result[0], cols->result[1], cols->result[2], cols->result[3]};
    int ncols = 3 + rplan.naggs;
    for (int c = 0; c < ncols; ++c) {
        if (!dst[c]) continue;
        GWO_TRY(hipcheck(copy_out(dst[c], src[c], take * 8, stream), "drain copy"));
    }
    uint64_t rest = out_rows - take;
    for (uint64_t off = 0; off < rest; off += take) {
        uint64_t len = std::min<uint64_t>(take, rest - off);
        for (int c = 0; c < ncols; ++c)
            GWO_TRY(hipcheck(hipMemcpyAsync(src[c] + off, src[c] + take + off, len * 8, hipMemcpyDeviceToDevice, stream),
                             "drain shift"));
    }
    out_rows = rest;
    *h_scalar = rest;
    GWO_TRY(hipcheck(hipMemcpyAsync(d_out_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "drain count"));
    return hipcheck(hipStreamSynchronize(stream), "drain sync");
}

gwo_status Handle::drain_side(const gwo_side_out *cols, int64_t cap, int64_t *n_out) {
    GWO_TRY(hipcheck(hipStreamSynchronize(stream), "drain side"));
    uint64_t take = std::min<uint64_t>((uint64_t)cap, side_rows_committed);
    *n_out = (int64_t)take;
    if (take == 0) return GWO_OK;
    DevBuf *src[3] = {&side_key, &side_ts, &side_val};
    void *dst[3] = {cols->key, cols->ts, cols->value};
    for (int c = 0; c < 3; ++c)
        if (dst[c]) GWO_TRY(hipcheck(copy_out(dst[c], src[c]->ptr, take * 8, stream), "side copy"));
    uint64_t rest = side_rows_committed - take;
    for (uint64_t off = 0; off < rest; off += take) {
        uint64_t len = std::min<uint64_t>(take, rest - off);
        for (int c = 0; c < 3; ++c)
            GWO_TRY(hipcheck(hipMemcpyAsync((int64_t *)src[c]->ptr + off, (int64_t *)src[c]->ptr + take + off, len * 8,
                                            hipMemcpyDeviceToDevice, stream), "side shift"));
    }
    side_rows_committed = side_rows = rest;
    *h_scalar = rest;
    GWO_TRY(hipcheck(hipMemcpyAsync(d_side_count, h_scalar, 8, hipMemcpyHostToDevice, stream), "side count"));
    return hipcheck(hipStreamSynchronize(stream), "side sync");
}

// ---- asynchronous fire ---------------------------------------------------------------------------
gwo_status Handle::poll_fire() {
    GWO_TRY(settle_out());
    if (!fire_pending) return GWO_OK;
    const int sp = sess ? sess_fire_poll() : -1;
    if (sp == 0) return GWO_OK;
    if (sp < 0 && hipEventQuery(ev_fire) == hipErrorNotReady) return GWO_OK;
    return finish_fire();
}

gwo_status Handle::state_size(int64_t *entries) {
    GWO_TRY(flush_pending());
    if (cfg.assigner == GWO_ASSIGNER_SESSION) return session_state_size(entries);
    int64_t s = 0;   // sliding windows restored from a per-window savepoint: their entries
    if (slide) {
        for (auto &kv : slide->rwin) s += (int64_t)(kv.second.n_pend + kv.second.n_done);
        if (slog) s += (int64_t)slog_rwin_count();
    }
    if (logst) {
        GWO_TRY(log_state_size(entries));
        *entries += s;
        return GWO_OK;
    }
    if (!rdone.empty()) {   // restored emitted entries: a key with new records is one entry, not two (snapshot merges)
        int64_t bound = 0, got = 0;
        GWO_TRY(snapshot_rows(&bound));
        const size_t m = (size_t)std::max<int64_t>(bound, 1);
        std::vector<int64_t> k(m), st(m), en(m), w(m * (size_t)std::max(plan.nwords, 1));
        gwo_state_rows rows{k.data(), st.data(), en.data(), w.data(), nullptr, nullptr};
        GWO_TRY(snapshot(&rows, (int64_t)m, &got));
        *entries = s + got;
        return GWO_OK;
    }
    GWO_TRY(read_occupancy());
    for (auto &kv : tables) s += (int64_t)kv.second.occ;
    *entries = s;
    return GWO_OK;
}

}  // namespace gwo
