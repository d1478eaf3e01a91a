// gwo_log_state.h -- host-side bookkeeping of the log-structured state (gwo_log.cpp, gwo_slog.cpp).
#pragma once
#include <map>
#include <vector>

#include "gwo_handle.h"
#include "gwo_log.h"

namespace gwo {

struct LogChunk {
    char *base = nullptr;
    size_t size = 0;
    size_t used = 0;
};

struct LogWindow {
    int lp = 0;
    std::vector<LogSegDesc> segs;
    std::vector<LogChunk> chunks;
    uint64_t records = 0;
    LogSegDesc partial{};        // restored checkpoint accumulators (rec == nullptr: none), folded at the fire
    uint64_t partial_rows = 0;
};

// One K1 launch over a window range of a batch (re-launched with a new range or capacity as needed).
struct LogJob {
    bool active = false;
    const int64_t *k = nullptr, *t = nullptr, *v = nullptr;
    int64_t n = 0, stride = 1;
    WindowGeom g{};              // geometry + watermark at gwo_submit time (classification input)
    long long base = 0;          // first window of the range
    int nunits = 1;
    uint64_t cap = 0;            // records per (window, coarse digit, region group) region of the batch buffer
    int slot = 0;                // batch buffer / readback slot
    unsigned long long seq = 0;  // readback sequence number of the last K1 launch
    LogSegDesc desc[LOG_NU] = {}; // the range's new segments: counters/offsets carved at launch, records after
    // speculative pass 2 (queued right behind K1, no host round trip): each window's segment records were
    // carved at launch with an upper bound; the readback either commits them (trimmed to the device plan's
    // size) or the host un-carves them and takes the planned path
    bool spec = false;
    uint64_t seg_cap[LOG_NU] = {};
    char *carve_at[LOG_NU] = {};  // start of the carved segment records
    char *carve_end[LOG_NU] = {}; // end of the carve (the window's chunk cursor right after it)
    LogRoute rt{};               // multi-GPU: the first K1 routes other GPUs' records (mode 1), re-runs skip them (2)
    bool ts32 = false;           // t holds int32 timestamps - tbase (records received in the 20-B wire format)
    int64_t tbase = 0;
    bool timed = false;          // the last K1 launch carries its own device timestamps (profiling)
    bool only_refire = false;    // sliding log late pass: only records of panes already in the running total
};

struct LogState {
    std::map<long long, LogWindow> wins;
    std::multimap<size_t, char *> free_chunks;
    // batch buffers: one for the K1 in flight, one for the deferred pass 2, one for the next K1
    DevBuf tmp[LOG_SLOTS], firedesc;
    // the last pass-2 launch, checked for overflow at the next sync point (deferred so the next batch's
    // K1 queues right behind it); its segments are already in the windows
    struct {
        bool active = false;
        int tmpx = 0, nunits = 0;
        long long base = 0;
        unsigned long long after_seq = 0;   // a K1 readback with a higher sequence number follows it
        bool has_event = false;
        uint64_t cap = 0;
        std::vector<uint64_t> counts;
    } pend;
    hipEvent_t ev_split = nullptr;               // after the deferred pass 2 (pipelined mode only)
    // GWO_SPLIT_STREAM=1: pass 2 runs on its own stream behind an event after its K1, so the next batch's K1 (main
    // stream) overlaps it; its completion is its event (ev_p2[slot]), never inferred from a later readback
    bool split_mode = false;
    hipStream_t split_stream = nullptr;
    hipEvent_t ev_k1done[LOG_SLOTS] = {}, ev_p2[LOG_SLOTS] = {};
    unsigned long long seen_seq = 0;             // highest K1 readback sequence number observed complete
    uint32_t *d_slow = nullptr;                  // [LOG_SLOW_CAP] partitions the fire's fast instance left, then their count
    unsigned *h_split_flag = nullptr;            // pinned, device-written [LOG_SLOTS]: pass-2 overflow flags
    unsigned *d_split_flag = nullptr;            // device view of h_split_flag
    unsigned *d_go = nullptr;                    // [LOG_SLOTS] K1's verdict on the speculative pass 2
    unsigned long long *d_done = nullptr;        // K1 arrival counters (LOG_DONE_WORDS; reset by the last one)
    unsigned long long *d_k1sh = nullptr;        // K1 statistics shards (reset by the last one)
    // pipelined submission (gwo_set_pipelined_submit): the batch whose K1 is in flight, resolved by the
    // next call on the handle
    bool pipeline = false;
    LogJob job;
    // the fire in flight on fire_stream
    std::vector<long long> fire_units;
    uint64_t fire_rows0 = 0, fire_bound = 0;
    unsigned long long *h_fire_out = nullptr;    // pinned [3]: row counter, overflow, slow partitions
    unsigned long long *d_cursor = nullptr;      // [LOG_NU * LOG_ND * LOG_XG * LOG_CUR_STRIDE] region cursors of K1
    // K1 readback per slot (LOG_RB_* layout), written into pinned host memory by log_collect_kernel,
    // which also leaves the device plan of pass 2 in d_bk (per slot) and resets cursors and stats
    unsigned long long *h_rb = nullptr, *d_rbh = nullptr;   // host / device views
    LogBucket *d_bk = nullptr;                   // [LOG_SLOTS][LOG_NU * LOG_ND + 1]
    hipEvent_t ev_rb[LOG_SLOTS] = {};
    bool rb_event[LOG_SLOTS] = {};   // ev_rb[slot] was recorded behind the slot's last K1 (side output only)
    // host-planned pass 2 (exact re-run after an overflow): [nb + 1] buckets, one H2D copy
    LogBucket *d_plan = nullptr, *h_buckets = nullptr;
    std::vector<LogSegDesc> h_fire;
    unsigned long long *d_overflow = nullptr;
    uint64_t last_window_keys = 0;               // distinct keys of the last fired window
    uint64_t last_window_records = 0;            // records of the last fired window
    long long span_hint = 1;                     // windows the previous batch spanned
    int cap_log2 = 0;
    int max_groups = 0;                          // persistent fire workgroups (2 per CU)
    unsigned long long seq = 0;                  // last readback sequence number issued
    unsigned long long *d_t0 = nullptr;          // K1's start timestamp (profiling)
    int clock_khz = 0;                           // device wall-clock rate

    unsigned long long *rb(int slot) const { return h_rb + (size_t)slot * LOG_RB_WORDS; }
    unsigned long long *rb_dev(int slot) const { return d_rbh + (size_t)slot * LOG_RB_WORDS; }
    LogBucket *bk(int slot) const { return d_bk + (size_t)slot * (LOG_NU * LOG_ND + 1); }
    // a batch buffer neither the K1 in flight nor the deferred pass 2 holds
    int free_slot() const {
        for (int s = 0; s < LOG_SLOTS; ++s)
            if (!(job.active && job.slot == s) && !(pend.active && pend.tmpx == s)) return s;
        return 0;   // unreachable: LOG_SLOTS = 3 > 2 busy slots
    }
};

}  // namespace gwo
