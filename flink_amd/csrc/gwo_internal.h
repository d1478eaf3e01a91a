// gwo_internal.h -- structures shared by the host runtime and the gfx950 kernels.
//
// State layout in HBM: every live (key, window) -- or (key, pane) for sliding
// windows -- is one entry of an open-addressed hash table.  There is one table per window (per
// pane), so a window's fire is a coalesced sweep of one contiguous allocation and the window start
// is implicit in the table, not stored per entry.  An entry is `stride` int64 words:
//   word 0           the key (EMPTY_KEY = Long.MIN_VALUE marks a free slot; a real key equal to
//                    Long.MIN_VALUE lives in the table's one-entry side slot, so no key is lost)
//   words 1..nwords  the accumulator words (sum / count / min / max ...), see AccPlan
// padded to a multiple of two words (16 B).
#pragma once
#include <stdint.h>

#define GWO_EMPTY_KEY ((int64_t)0x8000000000000000LL)
#define GWO_MAX_WORDS 8
#define GWO_HIST_BINS 64
#define GWO_OCC_SHARDS 8          // occupancy counter shards (gwo_device.h occ_add)
#define GWO_OCC_SHARD_STRIDE 8    // words between shards: one 64-B line each
#define GWO_OCC_WORDS (GWO_OCC_SHARDS * GWO_OCC_SHARD_STRIDE)
#define ARR_SHARDS 16             // grid_arrive_last (gwo_device.h): arrival counter shards, a 128-B line each
#define ARR_WORDS ((ARR_SHARDS + 1) * 16)
// scan_kernel statistics shards: SCAN_SHARDS x SCAN_SW words (min, max, 6 counters, the histogram), then
// SCAN_SHARDS + 1 arrival counters 16 words apart; min/max preset, every scan leaves them reset
#define SCAN_SHARDS 16
#define SCAN_CNT 9        // min, max, accepted, late, refire, bad_ts, bad_range, hist_out, bad_kg (speculative scan)
#define SCAN_SW 80
#define SCAN_SHARD_WORDS (SCAN_SHARDS * SCAN_SW + (SCAN_SHARDS + 1) * 16)

// Combine ops per accumulator word.  Every aggregate decomposes into word-wise commutative
// monoids, so inserting a record, merging two partials (sessions, pre-aggregation) and folding
// panes all use the same per-word combine.
enum AccOp : int32_t {
    ACC_ADD_I64 = 0,   // Java long +, wrap-around (SumFunction.java:63-68)
    ACC_ADD_F64 = 1,   // double +  (SumFunction.java:72-78)
    ACC_MIN_I64 = 2,   // signed min (int64 values, or Double.compareTo order keys)
    ACC_MAX_I64 = 3,
};
// How a record's value is lifted into a word.
enum AccSrc : int32_t {
    SRC_VALUE = 0,     // the int64 value, or the float64 value's bits for ACC_ADD_F64
    SRC_ONE = 1,       // constant 1 (count)
    SRC_ORDER = 2,     // Double.compareTo total-order key of the float64 value
};

struct AccPlan {
    int32_t nwords;
    int32_t stride;                    // words per entry incl. key, even
    int32_t value_is_f64;
    int32_t pad;
    int32_t op[GWO_MAX_WORDS];
    int32_t src[GWO_MAX_WORDS];
    int64_t ident[GWO_MAX_WORDS];      // identity of each word's monoid
};

// One hash table in HBM.
struct TableDesc {
    int64_t *base;                     // cap * stride words
    int64_t *side;                     // side slot for key == EMPTY_KEY: [flag, acc words...]
    unsigned long long *occ;           // occupied slots (incl. side slot): GWO_OCC_SHARDS sharded words
    uint64_t mask;                     // cap - 1 (cap is a power of two)
};

// Sliding windows, invertible aggregates: the running total of the next window to fire
// ("ring").  Records whose pane lies in [lo, hi] are also added to it; `live` counts entries whose
// hidden count word (`count_word`) is > 0, i.e. keys present in that window.
struct RingDesc {
    TableDesc t;
    long long lo, hi;                  // pane index range of the window (lo > hi: disabled)
    unsigned long long *live;
    int32_t count_word;
    int32_t pad;
};

// Result of the per-batch pre-pass (scan kernel), copied back to the host once per batch.
struct BatchStats {
    long long min_idx;                 // min/max window (pane) index over accepted records
    long long max_idx;
    unsigned long long accepted;       // records that reach at least one window
    unsigned long long late;           // dropped as late (or routed to the side output)
    unsigned long long refire;         // accepted into an already-fired window (allowedLateness > 0)
    unsigned long long bad_ts;         // Long.MIN_VALUE timestamps
    unsigned long long bad_kg;         // keys outside the KeyGroupRange
    long long bad_kg_key;
    unsigned long long bad_range;      // sliding: ts - offset + slide < 0 (Java '%' quirk region)
    unsigned long long partials;       // pre-aggregated partials flushed by the insert kernel
    unsigned long long hist_out;       // accepted records outside the histogram range
    unsigned long long hist[GWO_HIST_BINS];
    unsigned long long distinct[2];    // combine path: (key, unit) entries of units hint, hint + 1 summed over
                                       // workgroups (an upper bound of the keys the batch adds to each)
    unsigned long long overflow;       // combine path: records left to the merge one by one
};

// Window geometry of the handle, kernel-parameter sized.
struct WindowGeom {
    int64_t unit;                      // tumbling: size; sliding: pane = gcd(size, slide)
    int64_t unit_off;                  // offset passed to getWindowStartWithOffset for the unit
    int64_t unit_off_mod;              // floorMod(start, unit) of every unit start
    int64_t size;                      // window size
    int64_t slide;                     // sliding slide (== size for tumbling)
    int64_t offset;                    // assigner offset
    int64_t lateness;
    int64_t wm;                        // current watermark when the batch is processed
    double inv_size;                   // 1.0 / size, 1.0 / slide, 1.0 / unit: fast exact division
    double inv_slide;                  //   (gwo_device.h fdiv_floor)
    double inv_unit;
    int32_t sliding;
    int32_t key_kind;
    int32_t max_par;
    int32_t kg_lo;
    int32_t kg_hi;
    int32_t refire_ok;                 // table passes: re-fire records are emitted + inserted
    int32_t refire_only;               // table pass over the log layout's fired windows: re-fire records only
};

// Combine path buffers (gwo_kernels.hip gather / merge): per-workgroup LDS table dumps, the records left to
// the merge, per-workgroup statistics slots.
struct CombineArgs {
    int64_t *dump_key;                 // [G][2 * S]
    int64_t *dump_acc;                 // [G][2 * S][nwords] (occupied slots only)
    uint32_t *dump_used;               // [G]: bit u set when workgroup g dumped the table of unit hint + u
    uint32_t *ovf;                     // record indices left to the merge
    unsigned long long *ovf_count;     // reset by the gather's last workgroup
    unsigned long long ovf_cap;
    unsigned long long *blk;           // statistics shards (gather_stat_words(); min/max words preset)
    unsigned long long *done;          // arrival counters of the gather's workgroups (ARR_WORDS, left zero)
    int32_t S;                         // LDS slots per unit (power of two)
    int32_t sbits;                     // log2(S)
    long long hint;                    // units hint, hint + 1 fold in LDS; the histogram starts at hint
    // tumbling: windows hint .. hint + 3 by comparisons -- starts bound[0..4], 2-bit class per window
    // (0 accept, 1 every window late, 2 re-fire); thr_ok = 0: classify every record
    int64_t bound[5];
    uint32_t cls;
    int32_t thr_ok;
    int32_t full_range;                // the handle owns every key group: no per-record key-group check
    int32_t side_enabled;
    // readback (host-mapped): BatchStats words, side-output count, occupancy of the tables of units hint and
    // hint + 1 (occ[i] NULL: no table), then the sequence word, written last
    unsigned long long *rb;
    unsigned long long seq;
    unsigned long long *occ[2];
    // speculation: the merge queued right behind the gather runs iff the gather's verdict *go is 1 -- no error,
    // no re-fire, no listed record, every record in units hint / hint + 1 whose tables exist with room
    uint32_t *go;                      // NULL: no speculative merge
    // pipelined submission: *go still holds the previous batch's verdict, which the host has not read yet; a no
    // there is a no here too (the host redoes both batches in order)
    int32_t chain;
    // pipelined submission: the previous batch's verdict word (chain) -- each batch has its own word, so that a merge
    // queued behind its gather reads its own batch's verdict
    const uint32_t *go_prev;
    // overlapped pipelining (the gather on a side stream beside the previous batch's merge): the previous batch's
    // {hint, keys of unit hint, keys of unit hint + 1} (upper bounds of the entries its merge may still be claiming),
    // added to the occupancy this verdict reads; this batch's own go to inc_out for the next (NULL: not overlapped)
    const unsigned long long *inc_prev;
    unsigned long long *inc_out;
    uint64_t cap[2];                   // capacities of the hint tables
    long long side_cap;
    unsigned long long *dbg;           // GWO_CB_TRACE: phase times on the device wall clock (NULL: off)
};
#define CB_RB_STATS_WORDS ((int)((sizeof(BatchStats) + 7) / 8))
#define CB_RB_SIDE (CB_RB_STATS_WORDS)
#define CB_RB_OCC (CB_RB_STATS_WORDS + 1)
#define CB_RB_GO (CB_RB_STATS_WORDS + 3)
#define CB_RB_SEQ (CB_RB_STATS_WORDS + 4)
#define CB_RB_WORDS (CB_RB_STATS_WORDS + 5)

// Speculative two-pass insert (table layout, tumbling; gwo_runtime.cpp insert_speculative): the scan's last
// workgroup writes the batch statistics into the host-mapped readback block (CB_RB_* layout) and decides whether
// the insert queued behind it may run with the tables of units hint and hint + 1 as its directory -- no error,
// no re-fire, every accepted record in those units, whose tables exist with room.  rb == NULL: a plain scan.
struct ScanSpec {
    unsigned long long *rb;            // host-mapped readback block (device address), CB_RB_WORDS words
    unsigned long long seq;
    uint32_t *go;                      // the insert's verdict word
    unsigned long long *occ[2];        // occupancy counters of the hint tables (NULL: no table)
    uint64_t cap[2];                   // their capacities
    long long hint;                    // == the scan's hist_base
    int32_t check_kg;                  // the handle does not own every key group: check each accepted key
};

// Output columns (SoA) in HBM.
struct OutCols {
    int64_t *key;
    int64_t *start;
    int64_t *end;
    int64_t *res[GWO_MAX_WORDS];       // result columns (a checkpoint's raw accumulator words use up to 8)
    unsigned long long *count;         // device row counter
    long long cap;
};

struct ResultPlan {
    int32_t naggs;                     // result columns (<= 4 aggregates; a raw-word plan: nwords <= 8)
    int32_t kind[GWO_MAX_WORDS];       // gwo_agg_kind (COUNT = the word itself)
    int32_t word[GWO_MAX_WORDS];       // first accumulator word of each aggregate
    int32_t value_is_f64;
};

// Checkpoint rows being collected on the device (SoA): one per (key, window) -- per pane for sliding windows,
// per in-flight session for session windows -- with the raw accumulator words and the fire-timer flag.
struct SnapCols {
    int64_t *key, *start, *end;
    int32_t *timer;                    // 1: the window's event-time fire timer is still pending
    int64_t *w[GWO_MAX_WORDS];
    unsigned long long *count;         // rows written (block reservations)
    long long cap;
};

// Sessions (gwo_session.hip)
// A key entry holds up to smax in-flight sessions inline: word 1 = their count.  A key that needs more
// spills its session list into the pool (word 1 = -1, word 2 = first pool record, word 3 = capacity in
// sessions, word 4 = count); pool arrays double when full and are bump-allocated from *pool_top.
struct SessGeom {
    int64_t gap;
    int64_t lateness;
    int64_t wm;
    int32_t smax;                      // in-flight sessions per key held inline in its entry
    int32_t key_kind, max_par, kg_lo, kg_hi;
    int32_t side_enabled;
    int64_t *pool;                     // spilled session lists: (3 + nwords)-word session records
    unsigned long long *pool_top;      // next free pool record (device bump counter)
    uint64_t pool_cap;                 // pool capacity in session records
    int64_t *due;                      // [cap + 1] per slot (side slot = cap): the earliest watermark at which its
                                       // sessions fire or retire (SESS_NONE: none) -- the fire sweep skips the rest
};
#define SESS_NONE 0x7f7f7f7f7f7f7f7fLL   // a slot without sessions (a byte pattern: set with one memset)

struct SessErr {
    unsigned long long bad_ts, bad_kg, merge_late, capacity;
    long long bad_kg_key;
    unsigned long long late;
    unsigned long long emitted;
    unsigned long long live_delta;     // sessions created - removed (two's complement)
    unsigned long long pool_full;      // a spill found no pool room (the host sizes the pool so it cannot)
    unsigned long long long_slots;     // keys with more records in a batch than their bucket holds (SessLists)
};

// A batch's records grouped by key without a sort (gwo_session.hip): the slot pass appends each record's index to
// its slot's bucket -- word 0 the count, words 1..SESS_BKT_N the indices, in atomic order -- and marks the slot's
// first record (SESS_OWNER in its rec_slot word); the process pass's owner lanes order their buckets by index
// (arrival order) and reset the counts.  A slot with more records than its bucket holds is queued on `longs` and
// applied by sess_long_kernel from the records' slots in index order.
#define SESS_BKT 16
#define SESS_BKT_N (SESS_BKT - 1)
#define SESS_OWNER 0x80000000u
struct SessLists {
    uint32_t *bkt;                     // [(cap + 1) * SESS_BKT], counts zero between batches
    uint32_t *longs;                   // slots whose records overflowed their bucket
    uint32_t *ctl;                     // [1] long count, [2] workgroups done (sess_long_kernel), [3] workgroups
                                       // done (sess_fire_kernel)
    unsigned long long *shards;        // SESS_SHARDS x SESS_SHARD_STRIDE words: [0] live-session change (process
                                       // kernel), [1] sweep rows, [2] sweep live change; folded by the last workgroups
};
// Per-wave statistics adds spread over line-separated shards: ~1200 device-scope adds per batch on ONE address
// serialise where they meet (one per wave of the process kernel, measured as most of its time).
#define SESS_SHARDS 64
#define SESS_SHARD_STRIDE 16

// ---- host-side launchers (gwo_kernels.hip) -----------------------------------------------------
#include <hip/hip_runtime.h>

namespace gwo {

void launch_scan(const int64_t *key, const int64_t *ts, int64_t n, const WindowGeom &g, long long hist_base,
                 BatchStats *stats, int64_t *side_key, int64_t *side_ts, int64_t *side_val, const int64_t *val,
                 unsigned long long *side_count, long long side_cap, int side_enabled, unsigned long long *shards,
                 hipStream_t s, const ScanSpec *spec = nullptr);

void launch_put_word(unsigned long long *dst, unsigned long long v, hipStream_t s);
void launch_publish_words(const unsigned long long *src, int nw, unsigned long long *rb, unsigned long long seq,
                          hipStream_t s);

void launch_insert(const int64_t *key, const int64_t *ts, const void *val, int64_t n, const WindowGeom &g,
                   const AccPlan &plan, const TableDesc *dir, long long dir_base, int dir_len, int preagg,
                   BatchStats *stats, const RingDesc &ring, hipStream_t s, const uint32_t *go = nullptr);

void launch_restore(const int64_t *key, const int64_t *wstart, const int64_t *words, int64_t n, const AccPlan &p,
                    const WindowGeom &g, const TableDesc *dir, long long dir_base, int dir_len, hipStream_t s);
void launch_refire_collect(const int64_t *ts, int64_t n, const WindowGeom &g, long long dir_base, int dir_len,
                           uint32_t *blk, int64_t *r_idx, long long *r_u, hipStream_t s);
void launch_refire_slots(const int64_t *key, const int64_t *r_idx, const long long *r_u, int64_t m, const AccPlan &p,
                         const TableDesc *dir, long long dir_base, const uint64_t *slot_off, uint32_t *r_slot,
                         int64_t *before, hipStream_t s);
void launch_refire_emit(const int64_t *key, const int64_t *val, const int64_t *r_idx, const long long *r_u, int64_t m,
                        const uint32_t *skey, const uint32_t *spay, const int64_t *before, const AccPlan &p,
                        const ResultPlan &rp, int64_t unit, int64_t unit_off_mod, int64_t span, OutCols o,
                        hipStream_t s);
size_t gather_lds_bytes(int S, int nwords);
int gather_tile();         // records per gather workgroup tile
int gather_stat_words();   // statistics shard words (zeroed once; the gather leaves them reset)
void launch_gather(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const WindowGeom &g,
                   const AccPlan &p, const CombineArgs &a, int grid, BatchStats *st, int64_t *side_key, int64_t *side_ts,
                   int64_t *side_val, unsigned long long *side_count, long long side_cap, int side_enabled,
                   hipStream_t s);
void launch_merge(const int64_t *key, const int64_t *ts, const int64_t *val, const WindowGeom &g, const AccPlan &p,
                  const CombineArgs &a, int G, uint64_t novf, const TableDesc *dir, long long dir_base, int dir_len,
                  const RingDesc &ring, const uint32_t *go, hipStream_t s);
void launch_slide_refire_slots(const int64_t *key, const int64_t *r_idx, const long long *r_u, int64_t m,
                               const AccPlan &p, const WindowGeom &g, unsigned long long *keytab, uint64_t kmask,
                               long long j0, uint32_t nj, const TableDesc *pdir, long long pane_base,
                               long long pane_len, const TableDesc *wdir, uint32_t *r_slot, int64_t *before,
                               hipStream_t s);
// gwo_sort.hip: stable LSD radix sort of (uint32 key, uint32 payload; vals NULL = index); returns 0 when the
// result is in (k1, v1), 1 when in (k2, v2).  hist holds hist_cap words (at least 256 * ceil(n / 4096); more lets a
// small sort use smaller tiles)
int radix_sort_pairs(const uint32_t *keys, const uint32_t *vals, int64_t n, int key_bits, uint32_t *k1, uint32_t *v1,
                     uint32_t *k2, uint32_t *v2, uint32_t *hist, hipStream_t s, int digit_bits = 8,
                     int64_t hist_cap = 0);
void launch_key_groups_utf16(const uint16_t *chars, const int64_t *offsets, int64_t n, int max_par, int par,
                             int32_t *hash, int32_t *kg, int32_t *op, hipStream_t s);
void launch_table_load(const SnapCols &c, int64_t n, const TableDesc &t, const AccPlan &p, hipStream_t s);
// Emits every occupied entry (with live_word >= 0: every entry whose word live_word is > 0).
void launch_fire(const TableDesc &t, uint64_t cap, const AccPlan &plan, const ResultPlan &rp, int64_t start,
                 int64_t end, OutCols out, int reset, int live_word, hipStream_t s);

// dst += sign * src for every occupied entry of src (sign -1 only for all-ACC_ADD_I64 plans);
// live_word/live maintain dst's count of entries with a positive count word.  existing 1: only the keys dst already
// holds (live, with live_word >= 0) are combined; 2: only the keys it does not hold.
void launch_fold(const TableDesc &src, uint64_t src_cap, const TableDesc &dst, const AccPlan &plan, int sign,
                 int live_word, unsigned long long *live, hipStream_t s, int existing = 0);
// rows (key[i], words[i * nwords ...]) combined into table t
void launch_rows_insert(const int64_t *key, const int64_t *words, int64_t n, const TableDesc &t, const AccPlan &p,
                        hipStream_t s);

// rehash keeping only entries whose live_word is > 0 (live_word < 0: every occupied entry)
void launch_rehash_live(const TableDesc &src, uint64_t src_cap, const TableDesc &dst, const AccPlan &plan,
                        int live_word, hipStream_t s);

void launch_fill(int64_t *base, uint64_t cap, const AccPlan &plan, hipStream_t s);

void launch_rehash(const TableDesc &src, uint64_t src_cap, const TableDesc &dst, const AccPlan &plan,
                   hipStream_t s);

void launch_key_groups(const int64_t *keys, int64_t n, int key_kind, int max_par, int par, int32_t *kg,
                       int32_t *op, hipStream_t s);

void launch_window_starts(const int64_t *ts, int64_t n, int64_t offset, int64_t size, int64_t *out,
                          hipStream_t s);

void launch_generate(uint64_t seed, int64_t first, int64_t total, int64_t nkeys, int64_t span, int64_t disorder,
                     int64_t t0, int64_t vrange, int vf64, int key_mode, int64_t n, int64_t *key, int64_t *ts,
                     void *val, hipStream_t s);

}  // namespace gwo
