// gwo_log.h -- log-structured tumbling-window state (gwo_log.hip kernels, gwo_log.cpp host).
#pragma once
#include <stdint.h>

#include "gwo_internal.h"

#define LOG_UNITS 16            // windows covered by one scan/scatter chunk
#define LOG_FIRE_THREADS 512
#define LOG_MAX_LP 18           // at most 2^18 partitions per window
#define LOG_MAX_SEGS 512        // segments (batches) per window that one fire folds (= LOG_FIRE_THREADS)

// One segment = the records one batch appended to one window, grouped by partition:
// partition p's records are key[off[p] .. off[p+1]) (and val[...] unless the aggregates need no value).
struct LogSegDesc {
    int64_t *key;
    int64_t *val;
    uint32_t *off;              // 2^lp + 1 entries
    int32_t lp;
    int32_t pad;
};

namespace gwo {
void launch_log_scan(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const WindowGeom &g,
                     long long base, BatchStats *st, unsigned *chist, int64_t *side_key, int64_t *side_ts,
                     int64_t *side_val, unsigned long long *side_count, long long side_cap, int side_enabled,
                     hipStream_t s);
void launch_log_pass1(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const WindowGeom &g,
                      long long base, int nunits, unsigned long long *cursor, int64_t *tkey, int64_t *tval,
                      hipStream_t s);
void launch_log_pass2(const int64_t *tkey, const int64_t *tval, const unsigned long long *cbase, int nunits,
                      const LogSegDesc *segs, hipStream_t s);
int log_fire_cap_log2(int nwords);
void launch_log_fire(const LogSegDesc *segs, int nseg, int lp, const AccPlan &plan, const ResultPlan &rp,
                     int64_t start, int64_t end, OutCols out, unsigned long long *overflow, hipStream_t s);
}  // namespace gwo
