// gwo_slog.h -- sliding windows over logged panes with a partitioned running total.
//
// The reference adds every record to ceil(size/slide) windows (SlidingEventTimeWindows.java:68-82) and
// keeps one heap entry plus one timer per (key, window) (WindowOperator.java:294-427).  Here a record is
// logged once into its pane (a tumbling window of `slide`, through the log layout's K1 + pass 2), and
// the running total R of the last fired window is kept partitioned exactly like the pane logs (top lp
// bits of digit_hash).  Firing window J is one pass over the partitions: R_p (from HBM) + the entering
// pane's records of partition p - the leaving pane's records of partition p, folded in an LDS hash
// table; every key whose window count is positive emits its row and goes back to HBM as R'_p.  Every
// aggregate word is a wrap-around int64 sum (COUNT, SUM/AVG over int64): subtraction is exact.
#pragma once
#include <stdint.h>

#include "gwo_internal.h"

#ifndef SLOG_THREADS
#define SLOG_THREADS 256         // a small workgroup: ~5 per CU keep that many partitions' HBM round trips in flight
#endif
#define SLOG_MAX_SEGS 63          // signed inputs of one window step (pane segments, restored partials): wave 0
                                  // scans R_p and the segments, one lane each
#define SLOG_SHARDS 16            // statistics shards (one 128-B line each)
#define SLOG_STAT_STRIDE 16

// One signed input of a window step: a pane segment (records (key, value), or keys only) or a restored
// pane's partial accumulators (key + nwords raw words), grouped by the top `lp` bits of digit_hash.
struct SlogSeg {
    const int64_t *rec;
    const uint32_t *off;          // [2^lp] first record of each partition
    const uint32_t *cnt;          // [2^lp] records of each partition
    int32_t lp;
    int32_t sign;                 // +1: the pane enters the window, -1: it leaves
    int32_t fmt;                  // 0: value records (has_val: key, value; else key), 1: key + nwords raw words
    uint32_t nrec;                // records carved for the segment (0: unknown): a partition's run is clamped to it,
                                  // so a step queued speculatively behind a pass 2 whose partition overflowed (its
                                  // count is then the uncapped cursor; the step is redone) never reads past the carve
};

// The running total: partition q holds cnt[q] entries in the region rec[q * rcap * (1 + nwords)] as SoA columns
// (keys[rcap], then each word's [rcap]), in the order of the window step's LDS table buckets (8 slots each, bucket of a
// key = slog_bucket_hash); bkt[q * nb + b] = the entries of bucket b (bits 0-3) | bucket b overflowed (bit 4: a
// key was displaced past it, so a search may not stop there).  The next window step places every entry straight
// into its bucket -- no hashing, probing or atomics for the running total, only for the panes' records.  cnt[q]
// bit 31: the partition is unstructured (written by the range rounds): its entries are probed like records.
struct SlogRing {
    int64_t *rec;
    uint32_t *cnt;
    uint8_t *bkt;
    uint64_t rcap;
    int32_t lp;
    int32_t pad;
    uint16_t *slot;               // GWO_SLOG_SLOTS: slot[q * rcap + i] = entry i's table slot (0xffff: the side entry)
};
#define SLOG_UNSTRUCT 0x80000000u
#define SLOG_MAX_NB 256           // buckets of the LDS table at most (2048 slots)

// Statistics words per shard: live entries written, largest partition, R' capacity overflow, a negative
// count (an inconsistent leave), LDS table overflow, partitions that took the range rounds.
enum : int { SLS_LIVE = 0, SLS_MAXP, SLS_ROVF, SLS_NEG, SLS_LDS, SLS_SLOW, SLS_WORDS };

#ifndef GWO_SLOG_CHECK
#define GWO_SLOG_CHECK 0          // 1: a diagnostic build -- every HBM access of the window step is checked against
                                  // the host's allocation sizes; a violation is recorded (and skipped), not made
#endif
#if GWO_SLOG_CHECK
// Allocation sizes (int64 / uint16 elements) and the first violation: viol[0] = count, viol[1..7] = what, partition,
// index, bound, round width, in lp, out lp.
struct SlogCheck {
    uint64_t in_rec, in_slot, out_rec, out_slot;
    unsigned long long *viol;
};
enum : int { SLC_IN_REC = 1, SLC_IN_SLOT, SLC_SLOT_RANGE, SLC_SEG_CNT, SLC_SEG_REC, SLC_OUT_REC, SLC_OUT_SLOT, SLC_PART };
#endif

struct SlogArgs {
    SlogRing in, out;             // out.lp == in.lp (same partitions) or in.lp + 1 (each partition splits in two)
    const SlogSeg *segs;
    int32_t nseg;
    int32_t has_val;
    int32_t count_word;           // the word whose value > 0 marks a key present in the window
    int32_t cap_log2;             // LDS table slots
    int64_t start, end;           // the window being emitted
    AccPlan p;
    ResultPlan rp;
    OutCols o;
    unsigned long long *stat;     // [SLOG_SHARDS * SLOG_STAT_STRIDE]
    unsigned long long *dbg;      // optional (GWO_SLOG_TRACE): phase timestamps of workgroup 0, then each workgroup's
                                  // start and end
#define SLOG_DBG_PHASES 256       // 32 partitions x 8 phase stamps
#define SLOG_DBG_BLOCKS 4096
    int32_t mode;                 // diagnostics only (GWO_SLOG_MODE, results invalid): 4 no row reservation,
                                  // 8 no R' stores, 16 no row stores
    int32_t emit;                 // 0: an intermediate step of a chunked window step (R' only, no rows)
    // the step's segment descriptors travel in the kernel arguments (read through the kernarg segment pointer): no
    // copy from pageable host memory ahead of every window step
    SlogSeg seg[SLOG_MAX_SEGS];
#if GWO_SLOG_CHECK
    SlogCheck chk;
#endif
};
static_assert(sizeof(SlogArgs) <= 4096, "kernel arguments are limited to 4 KiB");

#ifndef GWO_SLOG_TABLE_KB
#define GWO_SLOG_TABLE_KB 32
#endif
#ifndef GWO_SLOG_BIG
#define GWO_SLOG_BIG 0            // 1: 2048-slot tables up to 64 KiB run by 512-thread workgroups (r05 experiment, off)
#endif
// log2 of the window step's LDS table slots for nwords accumulator words: the largest of 2^9..2^11 whose table fits
// GWO_SLOG_TABLE_KB KiB (32: about five workgroups share a CU and overlap their partitions' HBM round trips)
constexpr int slog_cap_log2_for(int nwords) {
    if (GWO_SLOG_BIG && 2048LL * (1 + nwords) * 8 <= 64 * 1024) return 11;
    int c = 11;
    while (c > 9 && ((long long)1 << c) * (long long)(1 + nwords) * 8 > GWO_SLOG_TABLE_KB * 1024) c--;
    return c;
}
// threads of the window step's workgroup: 512 for a table above GWO_SLOG_TABLE_KB (GWO_SLOG_BIG), else SLOG_THREADS
constexpr int slog_threads_for(int nwords) {
    return ((1LL << slog_cap_log2_for(nwords)) * (1 + nwords) * 8 > GWO_SLOG_TABLE_KB * 1024) ? 512 : SLOG_THREADS;
}

namespace gwo {
// Dynamic LDS bytes of the fire kernel for a table of 2^cap_log2 slots.
size_t slog_lds_bytes(int cap_log2, int nwords);
// log2 of the table slots the kernel instance for nwords is built for (slog_cap_log2_for, in the kernels' unit)
int slog_table_log2(int nwords);
// One window step over every partition of a.in (persistent grid: every workgroup resident on the `cus` CUs).
void launch_slog_fire(const SlogArgs &a, int cus, hipStream_t s);
void launch_slog_stat_publish(unsigned long long *stat, unsigned long long *rb, unsigned long long seq, hipStream_t s);
}  // namespace gwo
