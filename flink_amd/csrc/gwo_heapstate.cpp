// gwo_heapstate.cpp -- the keyed window state in the heap state backend's savepoint layout (include/gwo.h
// gwo_export_heap_state / gwo_import_heap_state).
//
// What WindowOperator leaves in a HeapKeyedStateBackend snapshot, per key group (HeapSnapshotStrategy.java:172-193):
// the "window-contents" state table (CopyOnWriteStateMapSnapshot.java:113-131: namespace, key, state), for merging
// assigners the "merging-window-set" list state (WindowOperator.java:265-271), and the timer service's two priority
// queues "_timer_state/event_window-timers" / "_timer_state/processing_window-timers" (InternalTimeServiceManager.java:
// 63-67, 132-133; KeyGroupPartitioner.java:251-264; TimerSerializer.java:158-162).  The rows come from gwo_snapshot
// and go to gwo_restore, so every layout is covered by the same code; this file only converts rows <-> bytes and
// accumulator words <-> GpuAggregates.Descriptor's long[] accumulator.
#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "gwo_handle.h"
#include "gwo_slide.h"

namespace gwo {

namespace {

constexpr int64_t kLongMax = (int64_t)0x7fffffffffffffffLL;

struct BE {   // big-endian writer (DataOutputView); counts bytes when buf is NULL
    uint8_t *p;
    int64_t n = 0, cap;
    bool over = false;
    void byte(uint8_t v) {
        if (p && n < cap) p[n] = v;
        else if (p) over = true;
        n++;
    }
    void i16(int16_t v) {
        for (int s = 8; s >= 0; s -= 8) byte((uint8_t)((uint16_t)v >> s));
    }
    void i32(int32_t v) {
        for (int s = 24; s >= 0; s -= 8) byte((uint8_t)((uint32_t)v >> s));
    }
    void i64(int64_t v) {
        for (int s = 56; s >= 0; s -= 8) byte((uint8_t)((uint64_t)v >> s));
    }
    void varint(uint32_t v) {   // StringValue.writeString's 7-bit groups, low first
        while (v >= 0x80) {
            byte((uint8_t)(v | 0x80));
            v >>= 7;
        }
        byte((uint8_t)v);
    }
};

struct Rd {   // big-endian reader (DataInputView)
    const uint8_t *p;
    int64_t n, at = 0;
    bool bad = false;
    uint8_t byte() {
        if (at >= n) {
            bad = true;
            return 0;
        }
        return p[at++];
    }
    int16_t i16() { return (int16_t)(((uint16_t)byte() << 8) | byte()); }
    int32_t i32() {
        uint32_t v = 0;
        for (int i = 0; i < 4; ++i) v = (v << 8) | byte();
        return (int32_t)v;
    }
    int64_t i64() {
        uint64_t v = 0;
        for (int i = 0; i < 8; ++i) v = (v << 8) | byte();
        return (int64_t)v;
    }
    uint32_t varint() {
        uint32_t v = byte();
        if (v < 0x80) return v;
        v &= 0x7f;
        for (int shift = 7; shift < 35; shift += 7) {
            const uint32_t c = byte();
            if (c < 0x80) return v | (c << shift);
            v |= (c & 0x7f) << shift;
        }
        bad = true;
        return 0;
    }
};

int64_t f64_order_key_h(int64_t bits) {   // Double.compareTo total order (the plan's MIN/MAX word for float64)
    if ((bits & 0x7ff0000000000000LL) == 0x7ff0000000000000LL && (bits & 0x000fffffffffffffLL) != 0)
        bits = 0x7ff8000000000000LL;
    return bits >= 0 ? bits : (bits ^ 0x7fffffffffffffffLL);
}
int64_t f64_from_order_key_h(int64_t k) { return k >= 0 ? k : (k ^ 0x7fffffffffffffffLL); }
}  // namespace

int64_t combine_h(int op, int64_t a, int64_t b) {
    switch (op) {
        case ACC_ADD_I64: return (int64_t)((uint64_t)a + (uint64_t)b);
        case ACC_ADD_F64: {
            double x, y;
            memcpy(&x, &a, 8);
            memcpy(&y, &b, 8);
            x += y;
            int64_t r;
            memcpy(&r, &x, 8);
            return r;
        }
        case ACC_MIN_I64: return b < a ? b : a;
        default: return b > a ? b : a;
    }
}

// accumulator words (the plan) -> GpuAggregates long[] (2 per aggregate), GpuAggregates.java createAccumulator/add
static void words_to_java(const ResultPlan &rp, const int64_t *w, int64_t *out) {
    for (int a = 0; a < rp.naggs; ++a) {
        const int64_t x = w[rp.word[a]];
        out[2 * a] = x;
        out[2 * a + 1] = 0;
        switch (rp.kind[a]) {
            case GWO_AGG_MIN:
            case GWO_AGG_MAX:
                if (rp.value_is_f64) {
                    out[2 * a] = f64_from_order_key_h(x);
                    out[2 * a + 1] = 1;   // "has a value": the f64 path of add() sets it
                }
                break;
            case GWO_AGG_AVG: out[2 * a + 1] = w[rp.word[a] + 1]; break;
            default: break;
        }
    }
}

static void java_to_words(const ResultPlan &rp, const AccPlan &p, const int64_t *j, int64_t *w) {
    for (int i = 0; i < p.nwords; ++i) w[i] = p.ident[i];
    for (int a = 0; a < rp.naggs; ++a) {
        const int wi = rp.word[a];
        switch (rp.kind[a]) {
            case GWO_AGG_MIN:
            case GWO_AGG_MAX: w[wi] = rp.value_is_f64 ? f64_order_key_h(j[2 * a]) : j[2 * a]; break;
            case GWO_AGG_AVG:
                w[wi] = j[2 * a];
                w[wi + 1] = j[2 * a + 1];
                break;
            default: w[wi] = j[2 * a]; break;
        }
    }
}

namespace {
struct WinEntry {   // one (key, window) of the export, in key-group order
    int32_t kg;
    int64_t key, start, end;
    std::vector<int64_t> words;
    bool pending;   // fire timer at maxTimestamp not yet fired
};
}  // namespace

gwo_status Handle::export_heap_state(const gwo_heap_state_ids *ids, uint8_t *buf, int64_t cap, int64_t *len,
                                     int64_t *kg_offsets, int64_t *wm_out) {
    if (!ids || !len) return fail(GWO_ERR_INVALID_ARGUMENT, "export_heap_state: ids and len are required");
    const bool merging = cfg.assigner == GWO_ASSIGNER_SESSION;
    if (merging && ids->merging_window_set < 0)
        return fail(GWO_ERR_INVALID_ARGUMENT, "export_heap_state: session windows need the merging-window-set id");
    int64_t bound = 0;
    GWO_TRY(snapshot_rows(&bound));
    const int NW = plan.nwords;
    const size_t m = (size_t)std::max<int64_t>(bound, 1);
    std::vector<int64_t> key(m), start(m), end(m), words(m * NW);
    std::vector<int32_t> kg(m), timer(m);
    gwo_state_rows rows{key.data(), start.data(), end.data(), words.data(), kg.data(), timer.data()};
    int64_t n = 0;
    GWO_TRY(snapshot(&rows, (int64_t)m, &n));
    // sliding windows restored from a per-window savepoint and not retired yet: rows n.. of `key`
    WindowRows RWn;
    if (cfg.assigner == GWO_ASSIGNER_SLIDING) GWO_TRY(slide_restored_rows(RWn));
    const int64_t nr = (int64_t)RWn.key.size();
    key.resize((size_t)n);
    key.insert(key.end(), RWn.key.begin(), RWn.key.end());
    // String keys: the Strings of the ids (StringValue.writeString writes their UTF-16 units)
    std::vector<int64_t> soff;
    std::vector<uint16_t> sch;
    if (cfg.key_kind == GWO_KEY_STRING && n + nr > 0) {
        soff.resize(n + nr + 1);
        int64_t need = 0;
        GWO_TRY(key_strings(key.data(), n + nr, soff.data(), nullptr, 0, &need));
        sch.resize(std::max<int64_t>(need, 1));
        GWO_TRY(key_strings(key.data(), n + nr, soff.data(), sch.data(), (int64_t)sch.size(), &need));
    }
    // (key, window) entries: rows as they are, or -- sliding -- each pane's windows that still hold state
    std::vector<WinEntry> es;
    std::vector<int64_t> row_of;   // entry -> a row of its key (String lookup)
    if (cfg.assigner == GWO_ASSIGNER_SLIDING) {
        const __int128 j_clean = first_uncleaned_window(wm);
        std::map<std::pair<int64_t, __int128>, size_t> at;
        for (int64_t i = 0; i < n; ++i) {
            const __int128 a = (__int128)start[i] - geom.unit_off_mod;
            __int128 u = a / geom.unit;
            if (a % geom.unit != 0 && a < 0) u -= 1;
            const __int128 ja = std::max(first_window_of_pane((long long)u), j_clean);
            __int128 jb = ((__int128)start[i] - slide->om) / cfg.slide;   // last window starting at or before the pane
            if (((__int128)start[i] - slide->om) % cfg.slide != 0 && (__int128)start[i] - slide->om < 0) jb -= 1;
            for (__int128 j = ja; j <= jb; ++j) {
                auto it = at.find({key[i], j});
                if (it == at.end()) {
                    WinEntry e;
                    e.kg = kg[i];
                    e.key = key[i];
                    e.start = win_start(j);
                    e.end = (int64_t)((uint64_t)e.start + (uint64_t)cfg.size);
                    e.words.assign(words.begin() + i * NW, words.begin() + (i + 1) * NW);
                    e.pending = (int64_t)((uint64_t)e.end - 1) > wm;
                    at[{key[i], j}] = es.size();
                    es.push_back(std::move(e));
                    row_of.push_back(i);
                } else {
                    WinEntry &e = es[it->second];
                    for (int w = 0; w < NW; ++w) e.words[w] = combine_h(plan.op[w], e.words[w], words[i * NW + w]);
                }
            }
        }
        // restored entries: a window with new records of the key has its timer again; one that only holds restored
        // entries keeps the timer state it was restored with (pending, or fired and waiting for the cleanup)
        for (int64_t r = 0; r < nr; ++r) {
            const __int128 j = RWn.j[r];
            auto it = at.find({RWn.key[r], j});
            const int64_t *rw = RWn.words.data() + (size_t)r * NW;
            if (it == at.end()) {
                WinEntry e;
                e.key = RWn.key[r];
                e.kg = key_group(e.key, cfg.key_kind, cfg.max_parallelism);
                e.start = win_start(j);
                e.end = (int64_t)((uint64_t)e.start + (uint64_t)cfg.size);
                e.words.assign(rw, rw + NW);
                e.pending = RWn.pending[r] != 0;
                at[{e.key, j}] = es.size();
                es.push_back(std::move(e));
                row_of.push_back(n + r);
            } else {
                WinEntry &e = es[it->second];
                for (int w = 0; w < NW; ++w) e.words[w] = combine_h(plan.op[w], e.words[w], rw[w]);
                e.pending = e.pending || RWn.pending[r] != 0;
            }
        }
        std::vector<size_t> ord(es.size());
        for (size_t q = 0; q < ord.size(); ++q) ord[q] = q;
        std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return es[x].kg < es[y].kg; });
        std::vector<WinEntry> s2;
        std::vector<int64_t> r2;
        for (size_t q : ord) {
            s2.push_back(std::move(es[q]));
            r2.push_back(row_of[q]);
        }
        es.swap(s2);
        row_of.swap(r2);
    } else {
        es.reserve(n);
        // a tumbling window restored with emitted entries (rdone) holds a key twice once the key got new records:
        // one heap entry, its accumulator the combination, its fire timer pending
        std::map<std::pair<int64_t, int64_t>, size_t> seen;
        const bool dedup = !rdone.empty();
        for (int64_t i = 0; i < n; ++i) {
            if (dedup) {
                auto it = seen.find({key[i], start[i]});
                if (it != seen.end()) {
                    WinEntry &e = es[it->second];
                    for (int w = 0; w < NW; ++w) e.words[w] = combine_h(plan.op[w], e.words[w], words[i * NW + w]);
                    e.pending = e.pending || timer[i] != 0;
                    continue;
                }
                seen[{key[i], start[i]}] = es.size();
            }
            WinEntry e;
            e.kg = kg[i];
            e.key = key[i];
            e.start = start[i];
            e.end = end[i];
            e.words.assign(words.begin() + i * NW, words.begin() + (i + 1) * NW);
            e.pending = timer[i] != 0;
            es.push_back(std::move(e));
            row_of.push_back(i);
        }
    }
    BE o{buf, 0, buf ? cap : 0};
    auto put_key = [&](size_t q) {
        if (cfg.key_kind == GWO_KEY_LONG) {
            o.i64(es[q].key);
        } else if (cfg.key_kind == GWO_KEY_INT) {
            o.i32((int32_t)es[q].key);
        } else {
            const int64_t r = row_of[q], b = soff[r], e = soff[r + 1];
            o.varint((uint32_t)(e - b + 1));
            for (int64_t c = b; c < e; ++c) o.varint(sch[c]);
        }
    };
    std::vector<int64_t> jacc(2 * rplan.naggs);
    size_t q0 = 0, q1 = 0;
    auto window_contents = [&]() {   // namespace (TimeWindow), key, accumulator (long[])
        o.i32((int32_t)(q1 - q0));
        for (size_t q = q0; q < q1; ++q) {
            o.i64(es[q].start);
            o.i64(es[q].end);
            put_key(q);
            words_to_java(rplan, es[q].words.data(), jacc.data());
            o.i32((int32_t)jacc.size());
            for (int64_t x : jacc) o.i64(x);
        }
    };
    auto merging_window_set = [&]() {   // one list per key of (window, state window); each window is its own
        std::map<int64_t, std::vector<size_t>> by_key;
        for (size_t q = q0; q < q1; ++q) by_key[es[q].key].push_back(q);
        o.i32((int32_t)by_key.size());
        for (auto &kv : by_key) {
            o.byte(0);   // VoidNamespaceSerializer: one byte
            put_key(kv.second[0]);
            o.i32((int32_t)kv.second.size());
            for (size_t q : kv.second) {
                o.i64(es[q].start);
                o.i64(es[q].end);
                o.i64(es[q].start);
                o.i64(es[q].end);
            }
        }
    };
    auto event_timers = [&]() {   // the fire timer of a pending window; its cleanup timer when that is later
        std::vector<std::pair<int64_t, size_t>> tm;
        for (size_t q = q0; q < q1; ++q) {
            const int64_t max_ts = (int64_t)((uint64_t)es[q].end - 1);
            const int64_t ct = cleanup_time_host(max_ts);
            if (es[q].pending) tm.push_back({max_ts, q});
            if (ct != max_ts && ct != kLongMax) tm.push_back({ct, q});
        }
        o.i32((int32_t)tm.size());
        for (auto &t : tm) {
            o.i64((int64_t)((uint64_t)t.first ^ 0x8000000000000000ull));   // MathUtils.flipSignBit
            put_key(t.second);
            o.i64(es[t.second].start);
            o.i64(es[t.second].end);
        }
    };
    auto processing_timers = [&]() { o.i32(0); };
    // HeapSnapshotStrategy writes every state of a key group in state-id order
    std::vector<std::pair<int, std::function<void()>>> sections = {
        {ids->window_contents, window_contents}, {ids->event_timers, event_timers},
        {ids->processing_timers, processing_timers}};
    if (merging) sections.push_back({ids->merging_window_set, merging_window_set});
    std::sort(sections.begin(), sections.end(),
              [](const std::pair<int, std::function<void()>> &x, const std::pair<int, std::function<void()>> &y) {
                  return x.first < y.first;
              });
    for (int g = cfg.key_group_start; g <= cfg.key_group_end; ++g) {
        if (kg_offsets) kg_offsets[g - cfg.key_group_start] = o.n;
        q1 = q0;
        while (q1 < es.size() && es[q1].kg == g) ++q1;
        if (q1 == q0 && q0 < es.size() && es[q0].kg < g)
            return poison(GWO_ERR_HIP, "export_heap_state: snapshot rows are not ordered by key group");
        o.i32(g);
        for (auto &sec : sections) {
            o.i16((int16_t)sec.first);
            sec.second();
        }
        q0 = q1;
    }
    if (q0 != es.size()) return poison(GWO_ERR_HIP, "export_heap_state: rows outside the key-group range");
    *len = o.n;
    if (wm_out) *wm_out = wm;
    if (buf && o.over) return fail(GWO_ERR_CAPACITY, "export_heap_state: %lld bytes, buffer holds %lld", (long long)o.n,
                                   (long long)cap);
    return GWO_OK;
}

gwo_status Handle::import_heap_state(const gwo_heap_state_ids *ids, const uint8_t *buf, int64_t len, int64_t new_wm) {
    if (!ids || (!buf && len > 0)) return fail(GWO_ERR_INVALID_ARGUMENT, "import_heap_state: ids and buf are required");
    const bool merging = cfg.assigner == GWO_ASSIGNER_SESSION;
    if (merging && ids->merging_window_set < 0)
        return fail(GWO_ERR_INVALID_ARGUMENT, "import_heap_state: session windows need the merging-window-set id");
    Rd r{buf, len};
    struct Entry {
        std::string skey;   // String keys: UTF-16 units as bytes
        int64_t key, start, end;
        std::vector<int64_t> jacc;
    };
    std::vector<Entry> contents;
    std::map<std::string, std::vector<std::pair<std::pair<int64_t, int64_t>, std::pair<int64_t, int64_t>>>> msets;
    std::map<std::tuple<std::string, int64_t, int64_t, int64_t>, int> timers;   // (key, start, end, ts)
    auto get_key = [&](std::string &sk, int64_t &k) {
        sk.clear();
        if (cfg.key_kind == GWO_KEY_LONG) k = r.i64();
        else if (cfg.key_kind == GWO_KEY_INT) k = r.i32();
        else {
            const uint32_t l = r.varint();
            if (l == 0) {
                r.bad = true;   // a null String key
                return;
            }
            for (uint32_t c = 0; c + 1 < l && !r.bad; ++c) {
                const uint32_t u = r.varint();
                sk.push_back((char)(u & 0xff));
                sk.push_back((char)(u >> 8));
            }
            k = 0;
        }
        if (cfg.key_kind != GWO_KEY_STRING) sk.assign((const char *)&k, 8);
    };
    // A key group's section holds every registered state once (HeapSnapshotStrategy.java:175-193 iterates the
    // backend's state tables): WindowOperator's three (four with a merging assigner) in the writer's id order.
    // Any other id is a keyed state this operator does not keep -- a custom trigger's (e.g. the reference's
    // session-with-stateful-trigger savepoint) or the user's -- whose entries it cannot even skip: UNSUPPORTED.
    const int nstates = merging ? 4 : 3;
    while (r.at < r.n && !r.bad) {
        const int32_t g = r.i32();
        const bool mine = g >= cfg.key_group_start && g <= cfg.key_group_end;
        unsigned seen = 0;
        for (int s = 0; s < nstates && !r.bad; ++s) {
            const int16_t id = r.i16();
            if (r.bad) break;
            const int bit = id == ids->window_contents ? 0 : id == ids->event_timers ? 1
                          : id == ids->processing_timers ? 2 : (merging && id == ids->merging_window_set) ? 3 : -1;
            if (bit < 0)
                return fail(GWO_ERR_UNSUPPORTED, "import_heap_state: key group %d holds state id %d, which is none of "
                                                 "the window operator's states (window-contents %d, event timers %d, "
                                                 "processing timers %d%s): a custom trigger's or another keyed state, "
                                                 "which this operator does not run", (int)g, (int)id,
                            (int)ids->window_contents, (int)ids->event_timers, (int)ids->processing_timers,
                            merging ? ", merging-window-set" : "");
            if (seen >> bit & 1u)
                return fail(GWO_ERR_INVALID_ARGUMENT, "import_heap_state: key group %d holds state id %d twice", (int)g,
                            (int)id);
            seen |= 1u << bit;
            const int32_t cnt = r.i32();
            if (cnt < 0) r.bad = true;
            for (int32_t e = 0; e < cnt && !r.bad; ++e) {
                if (id == ids->window_contents) {
                    Entry x;
                    x.start = r.i64();
                    x.end = r.i64();
                    get_key(x.skey, x.key);
                    const int32_t l = r.i32();
                    if (l != 2 * rplan.naggs) {
                        return fail(GWO_ERR_INVALID_ARGUMENT, "import_heap_state: accumulator of %d words, this "
                                                              "operator's aggregates use %d", l, 2 * rplan.naggs);
                    }
                    x.jacc.resize(l);
                    for (int32_t w = 0; w < l; ++w) x.jacc[w] = r.i64();
                    if (mine) contents.push_back(std::move(x));
                } else if (merging && id == ids->merging_window_set) {
                    if (r.byte() != 0) r.bad = true;   // VoidNamespace
                    std::string sk;
                    int64_t k;
                    get_key(sk, k);
                    const int32_t ml = r.i32();
                    for (int32_t i = 0; i < ml && !r.bad; ++i) {
                        const int64_t ws = r.i64(), we = r.i64(), ss = r.i64(), se = r.i64();
                        if (mine) msets[sk].push_back({{ws, we}, {ss, se}});
                    }
                } else if (id == ids->event_timers) {
                    const int64_t ts = (int64_t)((uint64_t)r.i64() ^ 0x8000000000000000ull);
                    std::string sk;
                    int64_t k;
                    get_key(sk, k);
                    const int64_t ws = r.i64(), we = r.i64();
                    if (mine) timers[std::make_tuple(sk, ws, we, ts)] = 1;
                } else {   // (id == ids->processing_timers)
                    return fail(GWO_ERR_UNSUPPORTED, "import_heap_state: processing-time timers in an event-time "
                                                     "window operator's state");
                }
            }
        }
    }
    if (r.bad) return fail(GWO_ERR_INVALID_ARGUMENT, "import_heap_state: truncated or malformed key-group data");
    // rows: (key, window, words, fire timer pending); sessions through their merging-window-set
    std::map<std::tuple<std::string, int64_t, int64_t>, size_t> by_ns;
    for (size_t i = 0; i < contents.size(); ++i)
        by_ns[std::make_tuple(contents[i].skey, contents[i].start, contents[i].end)] = i;
    RestoreRows R;
    R.nw = plan.nwords;
    std::vector<std::string> rkeys;
    auto add_row = [&](const Entry &c, int64_t ws, int64_t we) {
        R.key.push_back(c.key);
        R.start.push_back(ws);
        R.end.push_back(we);
        const int64_t max_ts = (int64_t)((uint64_t)we - 1);
        R.timer.push_back(timers.count(std::make_tuple(c.skey, ws, we, max_ts)) ? 1 : 0);
        std::vector<int64_t> w(plan.nwords);
        java_to_words(rplan, plan, c.jacc.data(), w.data());
        R.words.insert(R.words.end(), w.begin(), w.end());
        rkeys.push_back(c.skey);
    };
    if (merging) {
        for (auto &kv : msets)
            for (auto &pr : kv.second) {
                auto it = by_ns.find(std::make_tuple(kv.first, pr.second.first, pr.second.second));
                if (it == by_ns.end())   // a purging trigger's session: tracked, but with no contents
                    return fail(GWO_ERR_UNSUPPORTED, "import_heap_state: a session window without contents (state "
                                                     "of a purging trigger, which this operator does not run)");
                add_row(contents[it->second], pr.first.first, pr.first.second);
            }
    } else {
        for (auto &c : contents) add_row(c, c.start, c.end);
    }
    R.n = (int64_t)R.key.size();
    if (cfg.key_kind == GWO_KEY_STRING && R.n > 0) {   // the Strings become this handle's dictionary ids
        std::vector<int64_t> off(R.n + 1, 0);
        std::vector<uint16_t> ch;
        for (int64_t i = 0; i < R.n; ++i) {
            const std::string &s = rkeys[i];
            for (size_t b = 0; b + 1 < s.size(); b += 2) ch.push_back((uint16_t)((uint8_t)s[b] | ((uint8_t)s[b + 1] << 8)));
            off[i + 1] = (int64_t)ch.size();
        }
        if (ch.empty()) ch.push_back(0);
        const int64_t *idp = nullptr;
        GWO_TRY(intern_utf16(ch.data(), off.data(), R.n, &idp));
        GWO_TRY(hipcheck(copy_out(R.key.data(), idp, (size_t)R.n * 8, stream), "interned ids"));
    }
    std::vector<int32_t> kgs(R.n);
    gwo_state_rows rows{R.key.data(), R.start.data(), R.end.data(), R.words.data(), nullptr, R.timer.data()};
    if (R.n == 0) {
        static int64_t z[GWO_MAX_WORDS + 3] = {};
        static int32_t zt = 0;
        rows = gwo_state_rows{z, z, z, z, nullptr, &zt};
    }
    // sliding: the rows are windows (one accumulator per (key, window)), restored per window
    return restore_impl(&rows, plan.nwords, R.n, new_wm, cfg.assigner == GWO_ASSIGNER_SLIDING);
}

}  // namespace gwo

extern "C" {

gwo_status gwo_export_heap_state(gwo_handle *hh, const gwo_heap_state_ids *ids, uint8_t *buf, int64_t cap,
                                 int64_t *len, int64_t *kg_offsets, int64_t *watermark) {
    if (!hh) return GWO_ERR_INVALID_ARGUMENT;
    gwo::Handle *h = (gwo::Handle *)hh;
    if (h->poisoned) return h->poison_status;
    gwo::DeviceGuard g(h->cfg.device);
    return h->export_heap_state(ids, buf, cap, len, kg_offsets, watermark);
}

gwo_status gwo_import_heap_state(gwo_handle *hh, const gwo_heap_state_ids *ids, const uint8_t *buf, int64_t len,
                                 int64_t watermark) {
    if (!hh) return GWO_ERR_INVALID_ARGUMENT;
    gwo::Handle *h = (gwo::Handle *)hh;
    if (h->poisoned) return h->poison_status;
    gwo::DeviceGuard g(h->cfg.device);
    return h->import_heap_state(ids, buf, len, watermark);
}

gwo_status gwo_export_heap_state_begin(gwo_handle *hh, const gwo_heap_state_ids *ids, int64_t *len, int64_t *kg_offsets,
                                       int64_t *watermark) {
    if (!hh || !len) return GWO_ERR_INVALID_ARGUMENT;
    gwo::Handle *h = (gwo::Handle *)hh;
    if (h->poisoned) return h->poison_status;
    gwo::DeviceGuard g(h->cfg.device);
    std::vector<uint8_t>().swap(h->heap_img);   // a failed _begin leaves no stale image readable
    h->heap_img_open = false;
    int64_t n = 0;
    GWO_TRY(h->export_heap_state(ids, nullptr, 0, &n, nullptr, nullptr));
    std::vector<uint8_t> img((size_t)std::max<int64_t>(n, 1));
    GWO_TRY(h->export_heap_state(ids, img.data(), n, &n, kg_offsets, watermark));
    img.resize((size_t)n);
    h->heap_img.swap(img);
    h->heap_img_open = true;
    *len = n;
    return GWO_OK;
}

gwo_status gwo_export_heap_state_read(gwo_handle *hh, int64_t offset, uint8_t *buf, int64_t len) {
    if (!hh || len < 0 || offset < 0 || (len > 0 && !buf)) return GWO_ERR_INVALID_ARGUMENT;
    gwo::Handle *h = (gwo::Handle *)hh;
    if (!h->heap_img_open) return h->fail(GWO_ERR_STATE, "export_heap_state_read: no image (gwo_export_heap_state_begin)");
    if (offset > (int64_t)h->heap_img.size() || len > (int64_t)h->heap_img.size() - offset)
        return h->fail(GWO_ERR_INVALID_ARGUMENT, "export_heap_state_read: [%lld, %lld) past the image (%lld bytes)",
                       (long long)offset, (long long)(offset + len), (long long)h->heap_img.size());
    if (len) memcpy(buf, h->heap_img.data() + offset, (size_t)len);
    return GWO_OK;
}

gwo_status gwo_export_heap_state_end(gwo_handle *hh) {
    if (!hh) return GWO_ERR_INVALID_ARGUMENT;
    gwo::Handle *h = (gwo::Handle *)hh;
    std::vector<uint8_t>().swap(h->heap_img);
    h->heap_img_open = false;
    return GWO_OK;
}

}  // extern "C"
