/*
 * window_oracle.c -- C restatement of Flink's WindowOperator for event-time TUMBLING windows with
 * EventTimeTrigger and an AggregatingState of sum/min/max/count -- TEST INFRASTRUCTURE ONLY.
 *
 * Used (1) by tests/ for parity at sizes the Python oracle cannot reach and (2) as bench.py's
 * cpu_baseline ("port": it restates the reference algorithm, it is not Flink).  Never linked into
 * or called by the product library.
 *
 * Structure follows the reference's heap state backend, not the GPU design:
 *   - records are routed to subtasks by key group (KeyGroupRangeAssignment.java:48-73,118-119;
 *     murmurHash CO/util/MathUtils.java:134-154), one thread per subtask;
 *   - per subtask: a hash map (key, window) -> accumulator  (StateTable/CopyOnWriteStateMap,
 *     RT/state/heap/CopyOnWriteStateMap.java:373-388) and a timer min-heap deduplicated on
 *     (timestamp, key, window) (InternalTimerServiceImpl.java:216-278, HeapPriorityQueueSet.java:120-135);
 *   - processElement: WindowOperator.java:386-427 (isWindowLate :578-580, isElementLate :588-591,
 *     EventTimeTrigger.onElement EventTimeTrigger.java:37-45, registerCleanupTimer :598-610);
 *   - processWatermark: fire timers <= wm in timestamp order, onEventTime :430-473 (FIRE iff
 *     time == maxTs, clear iff time == cleanupTime :639-653).
 * Integer semantics are Java's: wrap-around long sums, truncating '%'.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "jsem.h"

/* ---- per-subtask state ---------------------------------------------------------------------- */
typedef struct {
    int64_t key, start;
    int64_t acc[4];       /* sum, min, max, count */
    int32_t live;
} Entry;

typedef struct {
    int64_t ts;
    int64_t entry;        /* index into entries */
    int32_t kind;         /* bit0: fire (maxTs), bit1: cleanup */
} Timer;

typedef struct {
    Entry *e;
    int64_t ne, cape;
    int64_t *slot;        /* open addressing: entry index + 1, 0 = empty, -1 = deleted */
    uint64_t mask;
    int64_t used;         /* non-empty slots incl. tombstones */
    int64_t *free_list;
    int64_t nfree, capfree;
    Timer *heap;
    int64_t nh, caph;
    /* output */
    int64_t *out;         /* rows of 7 words: key, start, end, sum, min, max, count */
    int64_t nout, capout;
    int64_t late;
    uint64_t checksum;
    int store_rows;
} Sub;

static uint64_t mix2(int64_t k, int64_t s) {
    uint64_t x = (uint64_t)k * 0x9E3779B97F4A7C15ull ^ ((uint64_t)s + 0x632BE59BD9B4E019ull);
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

static void sub_rehash(Sub *s, uint64_t ncap) {
    int64_t *ns = (int64_t *)calloc(ncap, sizeof(int64_t));
    uint64_t m = ncap - 1;
    for (int64_t i = 0; i < s->ne; ++i) {
        if (!s->e[i].live) continue;
        uint64_t h = mix2(s->e[i].key, s->e[i].start) & m;
        while (ns[h]) h = (h + 1) & m;
        ns[h] = i + 1;
    }
    free(s->slot);
    s->slot = ns;
    s->mask = m;
    int64_t live = 0;
    for (int64_t i = 0; i < s->ne; ++i) live += s->e[i].live;
    s->used = live;
}

static int64_t sub_find(Sub *s, int64_t key, int64_t start, int create) {
    uint64_t h = mix2(key, start) & s->mask;
    int64_t tomb = -1;
    for (;;) {
        int64_t v = s->slot[h];
        if (v == 0) break;
        if (v > 0) {
            Entry *e = &s->e[v - 1];
            if (e->key == key && e->start == start) return v - 1;
        } else if (tomb < 0) {
            tomb = (int64_t)h;
        }
        h = (h + 1) & s->mask;
    }
    if (!create) return -1;
    int64_t idx;
    if (s->nfree) {
        idx = s->free_list[--s->nfree];
    } else {
        if (s->ne == s->cape) {
            s->cape = s->cape ? s->cape * 2 : 1024;
            s->e = (Entry *)realloc(s->e, s->cape * sizeof(Entry));
        }
        idx = s->ne++;
    }
    Entry *e = &s->e[idx];
    e->key = key; e->start = start; e->live = 1;
    e->acc[0] = 0; e->acc[1] = LMAX; e->acc[2] = LMIN; e->acc[3] = 0;
    if (tomb >= 0) {
        s->slot[tomb] = idx + 1;
    } else {
        s->slot[h] = idx + 1;
        s->used++;
    }
    if ((uint64_t)s->used * 10 > (s->mask + 1) * 7) sub_rehash(s, (s->mask + 1) * 2);
    return idx;
}

static void sub_remove(Sub *s, int64_t idx) {
    Entry *e = &s->e[idx];
    uint64_t h = mix2(e->key, e->start) & s->mask;
    while (s->slot[h] != idx + 1) h = (h + 1) & s->mask;
    s->slot[h] = -1;
    e->live = 0;
    if (s->nfree == s->capfree) {
        s->capfree = s->capfree ? s->capfree * 2 : 1024;
        s->free_list = (int64_t *)realloc(s->free_list, s->capfree * sizeof(int64_t));
    }
    s->free_list[s->nfree++] = idx;
}

static void heap_push(Sub *s, Timer t) {
    if (s->nh == s->caph) {
        s->caph = s->caph ? s->caph * 2 : 1024;
        s->heap = (Timer *)realloc(s->heap, s->caph * sizeof(Timer));
    }
    int64_t i = s->nh++;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (s->heap[p].ts <= t.ts) break;
        s->heap[i] = s->heap[p];
        i = p;
    }
    s->heap[i] = t;
}

static Timer heap_pop(Sub *s) {
    Timer top = s->heap[0];
    Timer last = s->heap[--s->nh];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= s->nh) break;
        if (c + 1 < s->nh && s->heap[c + 1].ts < s->heap[c].ts) c++;
        if (s->heap[c].ts >= last.ts) break;
        s->heap[i] = s->heap[c];
        i = c;
    }
    if (s->nh) s->heap[i] = last;
    return top;
}

static void emit(Sub *s, const Entry *e, int64_t size) {
    int64_t row[7] = {e->key, e->start, jadd(e->start, size), e->acc[0], e->acc[1], e->acc[2], e->acc[3]};
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 7; ++i) h = (h ^ (uint64_t)row[i]) * 1099511628211ull;
    s->checksum += h;   /* order-independent */
    if (s->store_rows) {
        if (s->nout == s->capout) {
            s->capout = s->capout ? s->capout * 2 : 4096;
            s->out = (int64_t *)realloc(s->out, s->capout * 7 * sizeof(int64_t));
        }
        memcpy(s->out + s->nout * 7, row, sizeof row);
    }
    s->nout++;
}

typedef struct {
    Sub *sub;
    const int64_t *key, *ts, *val;
    const int64_t *idx;    /* this subtask's record indices, arrival order */
    int64_t nidx;
    const int64_t *bend, *bwm;
    int nb;
    int64_t size, offset, lateness;
} Job;

static void advance(Sub *s, int64_t wm, int64_t size, int64_t lateness) {
    while (s->nh && s->heap[0].ts <= wm) {
        Timer t = heap_pop(s);
        Entry *e = &s->e[t.entry];
        if (!e->live) continue;
        int64_t max_ts = jsub(jadd(e->start, size), 1);
        if (t.ts == max_ts) emit(s, e, size);
        if (t.ts == cleanup_time(max_ts, lateness)) sub_remove(s, t.entry);
    }
}

static void *run_job(void *arg) {
    Job *j = (Job *)arg;
    Sub *s = j->sub;
    int64_t wm = LMIN;
    int64_t p = 0;
    for (int b = 0; b <= j->nb; ++b) {
        int64_t end = b < j->nb ? j->bend[b] : LMAX;
        while (p < j->nidx && j->idx[p] < end) {
            int64_t i = j->idx[p++];
            int64_t t = j->ts[i];
            int64_t start = jsub(t, jadd(jsub(t, j->offset), j->size) % j->size);
            int64_t max_ts = jsub(jadd(start, j->size), 1);
            int64_t cu = cleanup_time(max_ts, j->lateness);
            if (cu <= wm) {                                     /* isWindowLate */
                if (jadd(t, j->lateness) <= wm) s->late++;      /* isElementLate */
                continue;
            }
            int64_t id = sub_find(s, j->key[i], start, 1);
            Entry *e = &s->e[id];
            int fresh = e->acc[3] == 0;
            int64_t v = j->val ? j->val[i] : 0;
            e->acc[0] = jadd(e->acc[0], v);
            if (v < e->acc[1]) e->acc[1] = v;
            if (v > e->acc[2]) e->acc[2] = v;
            e->acc[3]++;
            if (max_ts <= wm) {
                emit(s, e, j->size);                            /* onElement FIRE */
            } else if (fresh) {
                Timer tm = {max_ts, id, 1};
                heap_push(s, tm);                               /* registerEventTimeTimer */
            }
            if (fresh && cu != LMAX && cu != max_ts) {
                Timer tm = {cu, id, 2};
                heap_push(s, tm);                               /* registerCleanupTimer */
            }
        }
        if (b < j->nb) {
            wm = j->bwm[b];
            advance(s, wm, j->size, j->lateness);
        }
    }
    return NULL;
}

/*
 * Runs the stream: records [bend[b-1], bend[b]) then watermark bwm[b].  Returns total output rows;
 * *checksum = sum of per-row FNV hashes (order independent); *late = numLateRecordsDropped.
 * If rows != NULL it must hold 7 * (returned rows) int64 (call once with NULL to size).
 */
static int64_t run(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const int64_t *bend,
                   const int64_t *bwm, int nb, int64_t size, int64_t offset, int64_t lateness, int nthreads,
                   int32_t max_par, int store, int64_t *rows, int64_t **rows_out, uint64_t *checksum, int64_t *late);

int64_t wo_tumbling(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const int64_t *bend,
                    const int64_t *bwm, int nb, int64_t size, int64_t offset, int64_t lateness, int nthreads,
                    int32_t max_par, int64_t *rows, uint64_t *checksum, int64_t *late) {
    return run(key, ts, val, n, bend, bwm, nb, size, offset, lateness, nthreads, max_par, rows != NULL, rows, NULL,
               checksum, late);
}

/* One pass that also returns the rows: *rows_out = malloc'd [returned rows][7] (free with wo_free). */
int64_t wo_tumbling_rows(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const int64_t *bend,
                         const int64_t *bwm, int nb, int64_t size, int64_t offset, int64_t lateness, int nthreads,
                         int32_t max_par, int64_t **rows_out, uint64_t *checksum, int64_t *late) {
    return run(key, ts, val, n, bend, bwm, nb, size, offset, lateness, nthreads, max_par, 1, NULL, rows_out,
               checksum, late);
}

void wo_free(void *p) { free(p); }

static int64_t run(const int64_t *key, const int64_t *ts, const int64_t *val, int64_t n, const int64_t *bend,
                   const int64_t *bwm, int nb, int64_t size, int64_t offset, int64_t lateness, int nthreads,
                   int32_t max_par, int store, int64_t *rows, int64_t **rows_out, uint64_t *checksum, int64_t *late) {
    if (nthreads < 1) nthreads = 1;
    /* keyBy routing: subtask = computeOperatorIndexForKeyGroup(kg) */
    int64_t *cnt = (int64_t *)calloc(nthreads + 1, sizeof(int64_t));
    int32_t *dst = (int32_t *)malloc(n * sizeof(int32_t));
    for (int64_t i = 0; i < n; ++i) {
        int32_t kg = key_group(key[i], max_par);
        dst[i] = (int32_t)((int64_t)kg * nthreads / max_par);
        cnt[dst[i] + 1]++;
    }
    for (int t = 0; t < nthreads; ++t) cnt[t + 1] += cnt[t];
    int64_t *idx = (int64_t *)malloc(n * sizeof(int64_t));
    int64_t *fill = (int64_t *)malloc(nthreads * sizeof(int64_t));
    memcpy(fill, cnt, nthreads * sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) idx[fill[dst[i]]++] = i;
    Sub *subs = (Sub *)calloc(nthreads, sizeof(Sub));
    Job *jobs = (Job *)calloc(nthreads, sizeof(Job));
    pthread_t *th = (pthread_t *)malloc(nthreads * sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        subs[t].mask = 1023;
        subs[t].slot = (int64_t *)calloc(1024, sizeof(int64_t));
        subs[t].store_rows = store;
        jobs[t] = (Job){&subs[t], key, ts, val, idx + cnt[t], cnt[t + 1] - cnt[t], bend, bwm, nb, size, offset, lateness};
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    int64_t total = 0;
    uint64_t cs = 0;
    int64_t lt = 0;
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    if (rows_out) {
        int64_t all = 0;
        for (int t = 0; t < nthreads; ++t) all += subs[t].nout;
        *rows_out = (int64_t *)malloc((size_t)(all ? all : 1) * 7 * sizeof(int64_t));
        rows = *rows_out;
    }
    for (int t = 0; t < nthreads; ++t) {
        if (rows) memcpy(rows + total * 7, subs[t].out, subs[t].nout * 7 * sizeof(int64_t));
        total += subs[t].nout;
        cs += subs[t].checksum;
        lt += subs[t].late;
        free(subs[t].e); free(subs[t].slot); free(subs[t].free_list); free(subs[t].heap); free(subs[t].out);
    }
    if (checksum) *checksum = cs;
    if (late) *late = lt;
    free(cnt); free(dst); free(idx); free(fill); free(subs); free(jobs); free(th);
    return total;
}
