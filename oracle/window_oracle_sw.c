/*
 * window_oracle_sw.c -- C restatement of Flink's WindowOperator for event-time SLIDING and SESSION windows with
 * EventTimeTrigger and an AggregatingState of count/sum/min/max/avg over int64 values -- TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ for parity at the full sizes of configs C3 (sliding 60 s / 1 s, 10M keys) and C5 (sessions,
 * 100K keys, 10M records), where the record-at-a-time Python oracle (oracle/flink_oracle.py) cannot run.  It is
 * pinned against that oracle on random streams in tests/test_oracle_c.py.  Never linked into or called by the
 * product library.
 *
 * Structure: records are routed to subtasks (threads) by key group (KeyGroupRangeAssignment.java:60-73,118-119);
 * inside a subtask the keys are independent -- window state, timers and merging sets are all per key
 * (HeapKeyedStateBackend keys every state by (key, namespace)) and a timer only touches its own key's state --
 * so each key's records are replayed in arrival order against the watermark sequence:
 *   - the watermark in force for a record of batch b is the (running max of the) watermark after batch b - 1;
 *   - a timer at time t fires in the first batch s whose watermark is >= t (InternalTimerServiceImpl.java:268-278),
 *     so a pending fire is emitted with step s, lazily, before the key's next record after s (or at its end);
 *     a row emitted by EventTimeTrigger.onElement (allowedLateness re-fire) carries the record's batch b.
 * Sliding: WindowOperator.java:386-427 for every window of SlidingEventTimeWindows.assignWindows
 *   (SlidingEventTimeWindows.java:68-83): isWindowLate (:578-580) per window, onElement FIRE (EventTimeTrigger.java:
 *   37-45), registerCleanupTimer (:598-610), onEventTime (:430-473), isSkippedElement + isElementLate (:420-426).
 * Sessions: WindowOperator.java:294-383 with MergingWindowSet.addWindow (MergingWindowSet.java:156-225) over
 *   TimeWindow.mergeWindows (TimeWindow.java:217-261: sort by start, merge while intersects(), cover()), the merge
 *   function (WindowOperator.java:309-349: late merge -> UnsupportedOperationException, EventTimeTrigger.onMerge
 *   :72-81, deleting the merged windows' timers, AbstractHeapMergingState.mergeNamespaces), retireWindow of a late
 *   window (:358-362) and the cleanup timer (:639-653).
 *
 * Output: per watermark step the row count and an order-independent checksum (wrapping sum of an FNV-1a hash of
 * the row's words key, start, end, result[0..naggs)); optionally the rows of selected steps.  Results are
 * int64, except AVG (gwo_agg_kind 4): the bits of (double)sum / count.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "jsem.h"

enum { AGG_COUNT = 0, AGG_SUM = 1, AGG_MIN = 2, AGG_MAX = 3, AGG_AVG = 4 };
enum { ERR_NONE = 0, ERR_MERGE_LATE = 7 };

typedef struct {
    int64_t sum, min, max, count;
} Acc;

static inline void acc_init(Acc *a) {
    a->sum = 0;
    a->min = LMAX;
    a->max = LMIN;
    a->count = 0;
}
static inline void acc_add(Acc *a, int64_t v) {
    a->sum = jadd(a->sum, v);
    if (v < a->min) a->min = v;
    if (v > a->max) a->max = v;
    a->count++;
}
static inline void acc_merge(Acc *a, const Acc *b) {   /* AggregateFunction.merge of the state namespaces */
    a->sum = jadd(a->sum, b->sum);
    if (b->min < a->min) a->min = b->min;
    if (b->max > a->max) a->max = b->max;
    a->count += b->count;
}

/* ---- shared run context --------------------------------------------------------------------------------------- */
typedef struct {
    const int64_t *key, *ts, *val;
    const int64_t *bend;     /* batch b = records [bend[b-1], bend[b]) then watermark bwm[b] */
    int64_t *wmax;           /* running max of bwm (the watermark in force after batch b) */
    int nb;
    int naggs;
    const int32_t *aggs;
    const uint8_t *keep;     /* nb + 1 flags: keep the rows of these steps (NULL: none) */
    int64_t size, slide, offset, gap, lateness;
    int sessions;
} Ctx;

typedef struct {
    const Ctx *cx;
    const int64_t *idx;      /* this subtask's record indices, grouped by key, arrival order within a key */
    int64_t nidx;
    int64_t *step_rows;      /* nb + 1 */
    uint64_t *step_cs;
    int64_t *rows;           /* kept rows: (3 + naggs + 1) words each, the last one the step */
    int64_t nrows, caprows;
    int64_t late;
    int err;
    /* per-key scratch */
    void *scratch, *scratch2;
    int64_t scap, scap2;
} Sub;

static int64_t batch_of(const Ctx *c, int64_t i) {   /* first b with i < bend[b] (nb: after the last batch) */
    int lo = 0, hi = c->nb;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (i < c->bend[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}
static inline int64_t wm_before(const Ctx *c, int64_t b) { return b == 0 ? LMIN : c->wmax[b - 1]; }
/* the first step whose watermark reaches t (a timer at t fires there); nb: never */
static int64_t fire_step(const Ctx *c, int64_t t) {
    int lo = 0, hi = c->nb;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (c->wmax[mid] >= t) hi = mid; else lo = mid + 1;
    }
    return lo;
}

static void emit(Sub *s, int64_t key, int64_t start, int64_t end, const Acc *a, int64_t step) {
    const Ctx *c = s->cx;
    int64_t row[3 + 4 + 1];
    row[0] = key;
    row[1] = start;
    row[2] = end;
    for (int q = 0; q < c->naggs; ++q) {
        int64_t r;
        switch (c->aggs[q]) {
            case AGG_COUNT: r = a->count; break;
            case AGG_MIN: r = a->min; break;
            case AGG_MAX: r = a->max; break;
            case AGG_AVG: {
                double d = (double)a->sum / (double)a->count;
                memcpy(&r, &d, 8);
                break;
            }
            default: r = a->sum; break;
        }
        row[3 + q] = r;
    }
    const int nw = 3 + c->naggs;
    uint64_t h = 1469598103934665603ull;
    for (int q = 0; q < nw; ++q) h = (h ^ (uint64_t)row[q]) * 1099511628211ull;
    s->step_rows[step]++;
    s->step_cs[step] += h;
    if (c->keep && c->keep[step]) {
        if (s->nrows == s->caprows) {
            s->caprows = s->caprows ? s->caprows * 2 : 4096;
            s->rows = (int64_t *)realloc(s->rows, (size_t)s->caprows * (nw + 1) * sizeof(int64_t));
        }
        row[nw] = step;
        memcpy(s->rows + s->nrows * (nw + 1), row, (size_t)(nw + 1) * sizeof(int64_t));
        s->nrows++;
    }
}

/* ---- sliding: one key ------------------------------------------------------------------------------------------ */
typedef struct {
    int64_t start;
    Acc acc;
    int64_t fire;         /* step in which the window's maxTs timer fires */
    int32_t used, timer, fired;   /* timer: registered (an element arrived while maxTs > watermark) */
} SW;

static void slide_key(Sub *s, const int64_t *ix, int64_t m) {
    const Ctx *c = s->cx;
    const int64_t k = c->key[ix[0]];
    /* open-addressed hash of the key's windows by start: capacity >= 2 x (records x windows per record), a power
     * of two; only the slots this key used are cleared afterwards (the list after the table) */
    const int64_t per = c->size / c->slide + 2;
    uint64_t cap = 64;
    while (cap < (uint64_t)(2 * m * per) && cap < (1ull << 26)) cap <<= 1;
    if ((int64_t)(cap * sizeof(SW)) > s->scap) {   /* (a table only ever holds cleared slots between keys) */
        free(s->scratch);
        s->scratch = calloc(cap, sizeof(SW));
        s->scap = (int64_t)(cap * sizeof(SW));
    }
    if ((int64_t)(cap * sizeof(uint32_t)) > s->scap2) {
        free(s->scratch2);
        s->scratch2 = malloc(cap * sizeof(uint32_t));
        s->scap2 = (int64_t)(cap * sizeof(uint32_t));
    }
    SW *t = (SW *)s->scratch;
    uint32_t *list = (uint32_t *)s->scratch2;
    uint64_t used = 0;
    for (int64_t r = 0; r < m && !s->err; ++r) {
        const int64_t i = ix[r];
        const int64_t ts = c->ts[i], v = c->val ? c->val[i] : 0;
        const int64_t b = batch_of(c, i);
        const int64_t wm = wm_before(c, b);
        int skipped = 1;
        const int64_t last = window_start(ts, c->offset, c->slide);
        for (int64_t st = last; st > jsub(ts, c->size); st = jsub(st, c->slide)) {
            const int64_t end = jadd(st, c->size), max_ts = jsub(end, 1);
            const uint64_t hsh = ((uint64_t)st * 0x9E3779B97F4A7C15ull) >> 20;
            SW *e = NULL;
            for (uint64_t p = hsh & (cap - 1);; p = (p + 1) & (cap - 1)) {
                if (!t[p].used) {
                    e = &t[p];
                    e->used = 1;
                    e->start = st;
                    acc_init(&e->acc);
                    e->fire = fire_step(c, max_ts);
                    list[used++] = (uint32_t)p;
                    break;
                }
                if (t[p].start == st) {
                    e = &t[p];
                    break;
                }
            }
            if (used * 2 > cap) {   /* only a key spanning more than 2^25 windows gets here */
                s->err = -1;
                break;
            }
            /* the window's timer fired at step e->fire < b: its row precedes this record's update of the window */
            if (e->timer && !e->fired && e->fire < b) {
                emit(s, k, st, end, &e->acc, e->fire);
                e->fired = 1;
            }
            if (cleanup_time(max_ts, c->lateness) <= wm) continue;   /* isWindowLate */
            skipped = 0;
            acc_add(&e->acc, v);
            if (max_ts <= wm) emit(s, k, st, end, &e->acc, b);      /* onElement FIRE (re-fire) */
            else e->timer = 1;   /* registerEventTimeTimer(maxTs), deduplicated; it fires at step e->fire */
        }
        if (skipped && jadd(ts, c->lateness) <= wm) s->late++;      /* isSkippedElement && isElementLate */
    }
    for (uint64_t q = 0; q < used; ++q) {
        SW *e = &t[list[q]];
        if (e->timer && !e->fired && e->fire < c->nb) emit(s, k, e->start, jadd(e->start, c->size), &e->acc, e->fire);
        memset(e, 0, sizeof(SW));
    }
}

/* ---- sessions: one key ------------------------------------------------------------------------------------------ */
typedef struct {
    int64_t start, end;
    Acc acc;
    int32_t has, fire_pending, cleanup_pending;
} SessW;

/* pending timers of the key's windows up to watermark wm (steps < b): fires, then cleanups */
static void sess_catch_up(Sub *s, int64_t k, SessW *w, int *nw, int64_t wm) {
    const Ctx *c = s->cx;
    int o = 0;
    for (int q = 0; q < *nw; ++q) {
        SessW *x = &w[q];
        const int64_t max_ts = jsub(x->end, 1);
        if (x->fire_pending && max_ts <= wm) {
            if (x->has) emit(s, k, x->start, x->end, &x->acc, fire_step(c, max_ts));
            x->fire_pending = 0;
        }
        if (x->cleanup_pending && cleanup_time(max_ts, c->lateness) <= wm) continue;   /* clearAllState + retire */
        w[o++] = *x;
    }
    *nw = o;
}

static void session_key(Sub *s, const int64_t *ix, int64_t m) {
    const Ctx *c = s->cx;
    const int64_t k = c->key[ix[0]];
    const int64_t bytes = (m + 2) * (int64_t)sizeof(SessW);
    if (s->scap < bytes) {
        free(s->scratch);
        s->scap = bytes;
        s->scratch = malloc((size_t)bytes);
    }
    SessW *w = (SessW *)s->scratch;   /* the key's in-flight windows, sorted by start, pairwise not intersecting */
    int nw = 0;
    for (int64_t r = 0; r < m; ++r) {
        const int64_t i = ix[r];
        const int64_t ts = c->ts[i], v = c->val ? c->val[i] : 0;
        const int64_t b = batch_of(c, i);
        const int64_t wm = wm_before(c, b);
        sess_catch_up(s, k, w, &nw, wm);
        SessW nwin = {ts, jadd(ts, c->gap), {0, 0, 0, 0}, 0, 0, 0};
        acc_init(&nwin.acc);
        /* TimeWindow.mergeWindows over the in-flight windows + the new one.  The in-flight windows are sorted by
         * start and pairwise not intersecting (touching windows were merged when the later one arrived), so the
         * sweep's only run of more than one window is the new window's: the window right before it (start <= the
         * new start; Collections.sort is stable and the new window comes last) joins if it reaches the new start,
         * and the windows after it join while the run's cover reaches their start (intersects()). */
        int pos = 0;
        while (pos < nw && w[pos].start <= nwin.start) ++pos;
        int lo = pos, hi = pos;
        int64_t cs = nwin.start, ce = nwin.end;
        if (pos > 0 && w[pos - 1].end >= nwin.start) {
            lo = pos - 1;
            cs = w[lo].start;
            ce = w[lo].end > ce ? w[lo].end : ce;
        }
        while (hi < nw && ce >= w[hi].start) {
            ce = w[hi].end > ce ? w[hi].end : ce;
            ++hi;
        }
        SessW *actual = NULL;
        if (hi - lo == 0) {   /* no merge: the new window enters the set */
            memmove(&w[pos + 1], &w[pos], (size_t)(nw - pos) * sizeof(SessW));
            w[pos] = nwin;
            nw++;
            actual = &w[pos];
        } else if (hi - lo == 1 && w[lo].start == cs && w[lo].end == ce) {
            /* the run's cover is one pre-existing window (the new window lies inside it, or equals it: the HashSet
             * of the run then holds one window): no merge callback, MergingWindowSet.java:199-211 */
            actual = &w[lo];
        } else {
            const int64_t rmax = jsub(ce, 1);
            if (jadd(rmax, c->lateness) <= wm) {   /* WindowOperator.java:318-323 */
                s->err = ERR_MERGE_LATE;
                return;
            }
            SessW R = {cs, ce, {0, 0, 0, 0}, 0, 0, 0};
            acc_init(&R.acc);
            for (int q = lo; q < hi; ++q) {   /* mergeNamespaces; the merged windows' timers are deleted */
                if (w[q].has) {
                    acc_merge(&R.acc, &w[q].acc);
                    R.has = 1;
                }
            }
            R.fire_pending = rmax > wm;       /* EventTimeTrigger.onMerge */
            memmove(&w[lo + 1], &w[hi], (size_t)(nw - hi) * sizeof(SessW));
            nw -= hi - lo - 1;
            w[lo] = R;
            actual = &w[lo];
        }
        const int64_t max_ts = jsub(actual->end, 1);
        const int64_t cu = cleanup_time(max_ts, c->lateness);
        if (cu <= wm) {   /* isWindowLate(actualWindow): retireWindow, element skipped */
            const int q = (int)(actual - w);
            memmove(&w[q], &w[q + 1], (size_t)(nw - q - 1) * sizeof(SessW));
            nw--;
            if (jadd(ts, c->lateness) <= wm) s->late++;
            continue;
        }
        acc_add(&actual->acc, v);
        actual->has = 1;
        if (max_ts <= wm) emit(s, k, actual->start, actual->end, &actual->acc, b);   /* onElement FIRE */
        else actual->fire_pending = 1;
        if (cu != LMAX) actual->cleanup_pending = 1;
    }
    sess_catch_up(s, k, w, &nw, c->nb ? c->wmax[c->nb - 1] : LMIN);
}

/* ---- subtasks ------------------------------------------------------------------------------------------------- */
typedef struct {
    int64_t key, i;
} KI;

static int cmp_ki(const void *a, const void *b) {
    const KI *x = (const KI *)a, *y = (const KI *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->i < y->i ? -1 : x->i > y->i;
}

static void *run_sub(void *arg) {
    Sub *s = (Sub *)arg;
    const Ctx *c = s->cx;
    KI *ki = (KI *)malloc((size_t)(s->nidx ? s->nidx : 1) * sizeof(KI));
    for (int64_t r = 0; r < s->nidx; ++r) {
        ki[r].key = c->key[s->idx[r]];
        ki[r].i = s->idx[r];
    }
    qsort(ki, (size_t)s->nidx, sizeof(KI), cmp_ki);
    int64_t *ix = (int64_t *)malloc((size_t)(s->nidx ? s->nidx : 1) * sizeof(int64_t));
    for (int64_t r = 0; r < s->nidx; ++r) ix[r] = ki[r].i;
    for (int64_t a = 0; a < s->nidx && !s->err;) {
        int64_t z = a + 1;
        while (z < s->nidx && ki[z].key == ki[a].key) ++z;
        if (c->sessions) session_key(s, ix + a, z - a);
        else slide_key(s, ix + a, z - a);
        a = z;
    }
    free(ki);
    free(ix);
    free(s->scratch);
    free(s->scratch2);
    s->scratch = s->scratch2 = NULL;
    return NULL;
}

/*
 * Runs the stream (records [bend[b-1], bend[b]) then watermark bwm[b], b < nb; records after bend[nb-1] get no
 * watermark).  step_rows / step_checksum: nb + 1 entries (step nb: rows of records after the last watermark).
 * keep: NULL or nb + 1 flags; the kept rows come back in *rows_out (malloc'd, (4 + naggs) words per row: key,
 * start, end, results..., step; free with wo_free) with their count in *n_rows.  Returns 0, or 7 when a merge
 * produced a late window (GWO_ERR_MERGE_LATE, WindowOperator.java:318-323), or -1 on bad arguments.
 */
static int run_sw(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const int64_t *bend,
                  const int64_t *bwm, int nb, int64_t size, int64_t slide, int64_t offset, int64_t gap,
                  int64_t lateness, int sessions, const int32_t *aggs, int naggs, int nthreads, int32_t max_par,
                  const uint8_t *keep, int64_t *step_rows, uint64_t *step_checksum, int64_t **rows_out,
                  int64_t *n_rows, int64_t *late) {
    if (naggs < 1 || naggs > 4 || nthreads < 1 || max_par < 1 || (!sessions && (size <= 0 || slide <= 0)) ||
        (sessions && gap <= 0))
        return -1;
    Ctx c = {key, ts, val, bend, NULL, nb, naggs, aggs, keep, size, slide, offset, gap, lateness, sessions};
    c.wmax = (int64_t *)malloc((size_t)(nb ? nb : 1) * sizeof(int64_t));
    int64_t run = LMIN;
    for (int b = 0; b < nb; ++b) {
        run = bwm[b] > run ? bwm[b] : run;
        c.wmax[b] = run;
    }
    int64_t *cnt = (int64_t *)calloc((size_t)nthreads + 1, sizeof(int64_t));
    int32_t *dst = (int32_t *)malloc((size_t)(n ? n : 1) * sizeof(int32_t));
    for (int64_t i = 0; i < n; ++i) {
        dst[i] = (int32_t)((int64_t)key_group(key[i], max_par) * nthreads / max_par);
        cnt[dst[i] + 1]++;
    }
    for (int t = 0; t < nthreads; ++t) cnt[t + 1] += cnt[t];
    int64_t *idx = (int64_t *)malloc((size_t)(n ? n : 1) * sizeof(int64_t));
    int64_t *fill = (int64_t *)malloc((size_t)nthreads * sizeof(int64_t));
    memcpy(fill, cnt, (size_t)nthreads * sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) idx[fill[dst[i]]++] = i;
    Sub *subs = (Sub *)calloc((size_t)nthreads, sizeof(Sub));
    pthread_t *th = (pthread_t *)malloc((size_t)nthreads * sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        subs[t].cx = &c;
        subs[t].idx = idx + cnt[t];
        subs[t].nidx = cnt[t + 1] - cnt[t];
        subs[t].step_rows = (int64_t *)calloc((size_t)nb + 1, sizeof(int64_t));
        subs[t].step_cs = (uint64_t *)calloc((size_t)nb + 1, sizeof(uint64_t));
        pthread_create(&th[t], NULL, run_sub, &subs[t]);
    }
    int err = 0;
    int64_t total_rows = 0, lt = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (subs[t].err) err = subs[t].err == ERR_MERGE_LATE ? ERR_MERGE_LATE : -1;
        total_rows += subs[t].nrows;
        lt += subs[t].late;
    }
    memset(step_rows, 0, ((size_t)nb + 1) * sizeof(int64_t));
    memset(step_checksum, 0, ((size_t)nb + 1) * sizeof(uint64_t));
    const int nw = 4 + naggs;
    int64_t *rows = rows_out ? (int64_t *)malloc((size_t)(total_rows ? total_rows : 1) * nw * sizeof(int64_t)) : NULL;
    int64_t at = 0;
    for (int t = 0; t < nthreads; ++t) {
        for (int b = 0; b <= nb; ++b) {
            step_rows[b] += subs[t].step_rows[b];
            step_checksum[b] += subs[t].step_cs[b];
        }
        if (rows && subs[t].nrows) memcpy(rows + at * nw, subs[t].rows, (size_t)subs[t].nrows * nw * sizeof(int64_t));
        at += subs[t].nrows;
        free(subs[t].step_rows);
        free(subs[t].step_cs);
        free(subs[t].rows);
    }
    if (rows_out) *rows_out = rows;
    if (n_rows) *n_rows = total_rows;
    if (late) *late = lt;
    free(c.wmax); free(cnt); free(dst); free(idx); free(fill); free(subs); free(th);
    return err;
}

int wo_sliding(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const int64_t *bend,
               const int64_t *bwm, int nb, int64_t size, int64_t slide, int64_t offset, int64_t lateness,
               const int32_t *aggs, int naggs, int nthreads, int32_t max_par, const uint8_t *keep, int64_t *step_rows,
               uint64_t *step_checksum, int64_t **rows_out, int64_t *n_rows, int64_t *late) {
    return run_sw(key, ts, val, n, bend, bwm, nb, size, slide, offset, 0, lateness, 0, aggs, naggs, nthreads, max_par,
                  keep, step_rows, step_checksum, rows_out, n_rows, late);
}

int wo_sessions(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const int64_t *bend,
                const int64_t *bwm, int nb, int64_t gap, int64_t lateness, const int32_t *aggs, int naggs,
                int nthreads, int32_t max_par, const uint8_t *keep, int64_t *step_rows, uint64_t *step_checksum,
                int64_t **rows_out, int64_t *n_rows, int64_t *late) {
    return run_sw(key, ts, val, n, bend, bwm, nb, 0, 0, 0, gap, lateness, 1, aggs, naggs, nthreads, max_par, keep,
                  step_rows, step_checksum, rows_out, n_rows, late);
}
