// gwo_log.h -- log-structured tumbling-window state (gwo_log.hip kernels, gwo_log.cpp host).
#pragma once
#include <stdint.h>

#include "gwo_internal.h"

#define LOG_NU 4                 // windows one partition launch (K1) covers
#define LOG_SLOTS 3              // batch buffers: K1 in flight (pipelined), deferred pass 2, next K1
#ifndef LOG_K1_PER
#define LOG_K1_PER 16            // K1 tile: up to 256 threads x 16 records (64 KiB of 16-B records in LDS, two
#endif                           // workgroups per CU); a launch's tiles are sized so every workgroup loops over
#ifndef LOG_K1_THREADS
#define LOG_K1_THREADS 256       // the same number of them (log_k1_tile)
#endif
#define LOG_K1_TILE (LOG_K1_PER * LOG_K1_THREADS)
#ifndef LOG_K1_GRID
#define LOG_K1_GRID 512          // K1 workgroups: 2 per CU on MI355X's 256 CUs, all resident, each looping over
                                 // tiles with the next tile prefetched (measured: 0.223 ms vs 0.249 at 2048)
#endif
// K1's trash lines (after the region cursors in the same allocation): a write-phase lane with no record to write
// stores to its workgroup's line instead of skipping the store, so every tile issues exactly LOG_K1_PER stores per
// thread and the compiler's wait counting stays exact (a skippable store counts as none: the next tile's waits for
// its prefetched values became waits for everything in flight)
#define LOG_CURSOR_WORDS (LOG_NU * LOG_ND * LOG_XG * LOG_CUR_STRIDE)
#define LOG_K1_TRASH_WG (2 * LOG_K1_PER)           // words per workgroup (one 16-B record per store of a tile)
#define LOG_K1_TRASH_WORDS (LOG_K1_GRID * LOG_K1_TRASH_WG)
#define LOG_TILE_PER 7            // pass-2 chunk: 512 threads x 7 records
#define LOG_TILE_THREADS 512
#define LOG_TILE (LOG_TILE_PER * LOG_TILE_THREADS)   // 3584 records: 56 KiB of 16-B records in LDS
static_assert(LOG_K1_TILE <= 65536, "K1 ranks within a tile are 16-bit");
#ifndef LOG_DB
#define LOG_DB 8                 // coarse digit bits: K1 groups a window's records by the top LOG_DB bits
#endif
#define LOG_ND (1 << LOG_DB)     // coarse digits (K1 buckets) per window
#define LOG_MIN_LP 8             // a window has at least 256 partitions
#define LOG_MAX_LP (LOG_DB + 10 < 18 ? LOG_DB + 10 : 18)   // <= 1024 partitions per coarse digit (pass-2 LDS)
#define LOG_FIRE_THREADS 512
#define LOG_CUR_STRIDE 16        // K1 bucket cursors: one per 128-B line (memory-side atomics serialise per line)
#ifndef LOG_XG
#define LOG_XG 1                 // K1 region groups per bucket: workgroup w appends to group w % LOG_XG.  With 8
                                 // (workgroups w and w + 8 share an XCD) each group's runs merge in one L2: K1 alone
                                 // ran 13 % faster in isolation, but end to end K1 + pass 2 measured 221 + 100 us (1
                                 // group), 224 + 122 (4), 223 + 134 (8) per C4 batch -- so one group.  (r04: one run per
                                 // (bucket, workgroup), no reservation atomics, a count table read by pass 2 through a
                                 // binary search: K1 -5 us, pass 2 +13 us, writes 1.22x -> 1.17x -- reverted.)
#endif
#define FIRE_RPT 7                                   // records per thread in the fire's register prefetch
#define FIRE_RCAP (FIRE_RPT * LOG_FIRE_THREADS)      // 3584: records per partition of the fire's fast path
#ifndef FIRE_P3_BCAST
#define FIRE_P3_BCAST 1                              // P3: followers' unused election-table read at word 0
#endif
#ifndef FIRE_EMIT_V
#define FIRE_EMIT_V 4                                // values per row the direct emit reads unconditionally
#endif
static_assert(FIRE_EMIT_V <= 8, "the direct emit's unclamped reads stay inside the fire's LDS");
#define FIRE_OWN_LOG2 13
#define FIRE_OWN (1 << FIRE_OWN_LOG2)                // election table slots of the fire's fast path
#define FIRE_LDS (FIRE_RCAP * 8 * 2 + (FIRE_RCAP + 4) * 4)   // fast-path dynamic LDS: keys, values, counts (70 KiB)
#ifndef LOG_PART_FILL
#define LOG_PART_FILL 7          // a new window's partitions are sized for LOG_PART_FILL/8 of FIRE_RCAP records
#endif
#define LOG_SLOW_CAP (1 << LOG_MAX_LP)   // partitions of a window (the fire's slow-path list)
#define LOG_MAX_SEGS 512         // segments (batches) per window that one fire folds (= LOG_FIRE_THREADS)

// One segment = the records one batch appended to one window.  Partition p's records are
// rec[off[p] .. off[p] + cnt[p]) ((key, value) pairs, or keys only when no aggregate reads the value).
struct LogSegDesc {
    int64_t *rec;
    uint32_t *off;               // 2^lp start offsets (in records)
    uint32_t *cnt;               // 2^lp record counts (atomic cursors while pass 2 runs)
    int32_t lp;
    uint32_t nrec;               // records carved for the segment (every partition's run lies inside them)
};

// Pass-2 work description of one coarse bucket b (window w of the launch, coarse digit d).  The bucket's
// records sit in LOG_XG regions of the batch buffer: group x holds records [(b * LOG_XG + x) * cap, + count).
struct LogBucket {
    uint32_t n;                  // records in the bucket
    uint32_t pcap;               // capacity of each of the bucket's 2^(lp-8) partitions in the segment
    uint32_t seg_base;           // first record of the bucket's partitions in the segment
    uint32_t chunk0;             // first pass-2 workgroup of the bucket (prefix over buckets)
    uint32_t xoff[LOG_XG];       // exclusive prefix of the groups' record counts (the bucket read as one array)
};

// K1's classification by window bounds (tumbling): a record with bound[0] <= ts < bound[nunits] belongs to
// window base + j for the j with bound[j] <= ts < bound[j + 1] -- a few compares instead of the window
// arithmetic; valid only where getWindowStartWithOffset is monotone (ts >= offset - size).  Records outside
// take the full restatement.
struct LogThr {
    int64_t bound[LOG_NU + 1];   // window starts base .. base + nunits (unused entries: Long.MAX_VALUE)
    uint32_t cls;                // 2 bits per window: 0 accept, 1 window late (cleanup time passed), 2 re-fire
    int32_t ok;                  // 1: the bounds are valid
    int32_t full_range;          // 1: the subtask owns every key group (no key-group check needed)
    int32_t ts32;                // 1: `ts` holds int32 timestamps - tbase (records received in the 20-B wire format)
    int32_t only_refire;         // 1: the sliding-log late pass -- accept only records whose pane is already in the
                                 //    running total (class 2), skip every other record without counting it
    int64_t tbase;
};

// The segment descriptors of one pass-2 launch (kernel argument).
struct LogSegSet {
    LogSegDesc s[LOG_NU];
};

// K1 readback block (host-visible, written by K1's last workgroup): [LOG_NU * LOG_ND] bucket counts, the
// BatchStats words, [LOG_NU] segment sizes (records) of the device plan, its pass-2 workgroup count, the
// speculation verdict (1: the speculative pass 2 queued behind K1 runs the plan), and the sequence number.
static constexpr int LOG_RB_STATS = LOG_NU * LOG_ND;
static constexpr int LOG_RB_SEG = LOG_RB_STATS + (int)((sizeof(BatchStats) + 7) / 8);
static constexpr int LOG_RB_CHUNKS = LOG_RB_SEG + LOG_NU;
static constexpr int LOG_RB_GO = LOG_RB_CHUNKS + 1;
static constexpr int LOG_RB_MAXREG = LOG_RB_GO + 1;      // largest region count (> cap: K1 dropped records)
static constexpr int LOG_RB_NEXT = LOG_RB_MAXREG + 1;    // the first window after the launch's range holding accepted
                                                         // records (Long.MAX_VALUE: none) -- the next K1 range starts there
static constexpr int LOG_RB_RMAX = LOG_RB_NEXT + 1;      // routed K1: the largest narrow / wide destination count (above
static constexpr int LOG_RB_RWMAX = LOG_RB_RMAX + 1;     //   the region capacity: records were dropped, the host re-routes)
static constexpr int LOG_RB_T0 = LOG_RB_RWMAX + 1;       // device wall clock when workgroup 0 started (profiling)
static constexpr int LOG_RB_T1 = LOG_RB_T0 + 1;          // device wall clock when the tail finished its work
static constexpr int LOG_RB_SEQ = LOG_RB_T1 + 1;         // written last: the launch's sequence number
static constexpr int LOG_RB_WORDS = LOG_RB_SEQ + 1;

// What K1's last workgroup needs to plan pass 2 (the former collect step, fused into K1's tail).
struct CollectArgs {
    int nunits;
    int lp[LOG_NU];              // partition bits of each window of the launch
    uint32_t *cnt[LOG_NU];       // the windows' new segment counters (zeroed by every K1 workgroup first)
    uint64_t cap;                // region capacity of the batch buffer (records per bucket and region group)
    uint64_t seg_cap[LOG_NU];    // speculative pass 2: segment records carved per window (spec only)
    int spec;                    // 1: a pass 2 is queued behind K1 and runs iff the plan fits (rb[LOG_RB_GO])
    LogBucket *bk;               // out: [nunits * LOG_ND + 1] pass-2 plan (device)
    unsigned *go;                // out: 1 = the queued speculative pass 2 runs the plan, 0 = it exits
    unsigned long long *rb;      // out: readback block (pinned host memory)
    unsigned long long seq;      // written to rb[LOG_RB_SEQ] after every other readback word
    unsigned long long *done;    // K1 workgroups finished: shard counters [LOG_SHARDS * LOG_CUR_STRIDE], then the
                                 // count of finished shards at done[LOG_SHARDS * LOG_CUR_STRIDE] (the last plans)
    unsigned long long *shard;   // [LOG_SHARDS * LOG_CUR_STRIDE] K1 statistics shards (K1_SW words each, one line)
    unsigned long long *t0;      // device wall clock at workgroup 0's start (K1 timing without stream markers)
    unsigned long long *reset_rows;   // non-null: the output's row counter, zeroed by the tail (sliding window steps:
                                      // after a discard, instead of a memset ahead of the next step)
};

// K1's statistics: every workgroup reduces its counters in LDS and folds them into shard blockIdx % LOG_SHARDS
// (device-scope atomics on the same address serialise at ~12 ns each on MI355X: 4 per-wave atomics per
// workgroup on one word cost ~25 us at the end of a 512-workgroup launch); the tail folds the shards.
#define LOG_SHARDS 16
enum : int { K1S_MIN = 0, K1S_MAX, K1S_ACC, K1S_LATE, K1S_REFIRE, K1S_BADTS, K1S_BADKG, K1S_HOUT, K1S_BADR, K1S_NEXT,
             K1_SW };
static constexpr size_t LOG_DONE_WORDS = (LOG_SHARDS + 1) * LOG_CUR_STRIDE;

// Multi-GPU keyBy routing fused into K1 (the log layout's first K1 over a batch): a record whose key group
// belongs to another GPU -- computeOperatorIndexForKeyGroup(assignToKeyGroup(key)) != me,
// KeyGroupRangeAssignment.java:118-119 -- is not classified here (its owner does that) but appended to that
// destination's send region; one reservation per (tile, destination).  Wire format: 20-B records, SoA per
// destination region (keys, values, int32 timestamp - tbase); tbase = the watermark every rank shares (the
// watermark is the min over ranks), so a timestamp within +-24.8 days of it travels as 4 bytes.  A record outside
// that goes as a 24-B {key, ts, value} record to the destination's small "wide" region (one atomic each: rare).
#define LOG_RT_MAX 256           // destinations (ranks) K1 routes to
#define LOG_RT_B 1024            // K1 code of a routed record: bucket field LOG_RT_B + destination
struct LogRoute {
    int32_t mode;                // 0: no routing; 1: route remote records; 2: skip them (a re-run of a routed batch);
                                 // 3: route only, this GPU's records skipped (exact-capacity re-route after an overflow)
    int32_t nranks;              // destinations
    int32_t me;                  // this GPU's index: its records stay
    int32_t pad;
    int64_t *send;               // nranks narrow regions (log_rt_keys/vals/ts32), then nranks wide regions (log_rt_wide)
    uint64_t rcap;               // narrow region capacity (records, even: regions stay 8-B aligned)
    uint64_t wcap;               // wide region capacity (records)
    int64_t tbase;               // timestamps travel as int32 ts - tbase
    unsigned long long *cursor;  // [2 * LOG_RT_MAX * LOG_CUR_STRIDE]: narrow cursors, then wide cursors (the tail moves
                                 // them to count and zeroes them)
    unsigned long long *count;   // out: [2 * nranks] (narrow, wide) records per destination (above capacity: overflow)
};
// narrow region d: keys[rcap] (int64), values[rcap] (int64), ts[rcap] (int32); 20 B per record = 2.5 words
static inline __host__ __device__ int64_t *log_rt_keys(int64_t *send, uint64_t rcap, int d) {
    return send + (uint64_t)d * rcap * 5 / 2;
}
static inline __host__ __device__ int64_t *log_rt_vals(int64_t *send, uint64_t rcap, int d) {
    return log_rt_keys(send, rcap, d) + rcap;
}
static inline __host__ __device__ int32_t *log_rt_ts32(int64_t *send, uint64_t rcap, int d) {
    return (int32_t *)(log_rt_keys(send, rcap, d) + 2 * rcap);
}
static inline __host__ __device__ int64_t *log_rt_wide(int64_t *send, uint64_t rcap, int nranks, uint64_t wcap, int d) {
    return send + (uint64_t)nranks * rcap * 5 / 2 + (uint64_t)d * wcap * 3;
}
static inline __host__ __device__ bool log_rt_fits(int64_t t, int64_t tbase) {
    return t >= tbase ? (uint64_t)t - (uint64_t)tbase <= 0x7fffffffull : (uint64_t)tbase - (uint64_t)t <= 0x80000000ull;
}
static inline int64_t log_rt_tbase(int64_t wm) { return wm == (int64_t)0x8000000000000000LL ? 0 : wm; }

namespace gwo {
int log_k1_grid(int64_t n);                                    // K1 workgroups for n records
// K1: classify + key-group check + late accounting + (window, coarse digit) grouping of a batch; its last
// workgroup writes the readback block and the device plan of pass 2, and resets cursors and statistics.
// key/ts/val columns with `stride` int64 words between records (1: SoA columns; 3: {key, ts, value} records)
// (thr.ts32: `ts` points at int32 timestamps - thr.tbase, columns only)
void launch_log_part(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, int64_t stride,
                     const WindowGeom &g,
                     long long base, int nunits, int has_val, unsigned long long *cursor, uint64_t cap,
                     int64_t *tmp, BatchStats *st, int64_t *side_key, int64_t *side_ts, int64_t *side_val,
                     unsigned long long *side_count, long long side_cap, int side_enabled, const CollectArgs &ca,
                     const LogThr &thr, const LogRoute &rt, hipStream_t s);
// Pass 2: every coarse bucket -> its window's segment, grouped by partition.  `overflow` is a
// host-visible flag (set to 1 when a partition exceeds its capacity).  go != NULL: a speculative launch
// of `nchunks` (an upper bound) workgroups that exits unless *go (K1's verdict) is set.
void launch_log_split(const int64_t *tmp, uint64_t cap, int has_val, const LogBucket *buckets, int nb,
                      const LogSegSet &segs, unsigned *overflow, uint32_t nchunks, const unsigned *go, hipStream_t s);
int log_fire_cap_log2(int nwords);
// Loads the fire and pass-2 code objects with empty launches (HIP loads a kernel's code on its first launch:
// ~0.25 ms that would otherwise land on the first watermark that fires a window).
void warm_log_kernels(int nwords, int has_val, hipStream_t s);
// GWO_KTRACE=1: per-phase shader-clock sums of K1 and the fire, printed at handle destruction (diagnostics).
void ktrace_enable(int on);
void ktrace_report();
// Folds a window's segments (plus, when partial.rec is set, the restored accumulators of a checkpoint: records
// of 1 + nwords words grouped by partition like a segment) and emits one row per key.  slow_only: every
// partition takes the LDS hash-table path (a checkpoint fold with a raw-word result plan: up to 8 columns).
void launch_log_fire(const LogSegDesc *segs, int nseg, int lp, int has_val, const AccPlan &plan,
                     const ResultPlan &rp, int64_t start, int64_t end, OutCols out, unsigned long long *overflow,
                     int cus, int max_per_cu, int slow_only, const LogSegDesc &partial, uint32_t *slow_list,
                     uint32_t *slow_cnt, hipStream_t s);   // slow_list: [2^lp] partitions + slow_cnt, device scratch
}  // namespace gwo
