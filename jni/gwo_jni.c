/*
 * gwo_jni.c -- JNI shim between GwoNative.java and the C ABI of include/gwo.h.  One function per native; columns
 * arrive as direct ByteBuffers (GetDirectBufferAddress: no copy); a failing gwo_status is thrown as the Java
 * exception the reference would raise (IllegalArgumentException for bad configuration, mirroring the assigners'
 * checks; UnsupportedOperationException for GWO_ERR_UNSUPPORTED and for GWO_ERR_MERGE_LATE, whose reference
 * counterpart is WindowOperator.java:318-323; RuntimeException otherwise).
 * Built by `make jni` only where jni.h exists (JAVA_HOME); this image has no JDK.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gwo.h"

#define JFN(name) Java_org_apache_flink_streaming_runtime_operators_windowing_gpu_GwoNative_##name
#define H(h) ((gwo_handle *)(intptr_t)(h))

static int fail(JNIEnv *env, gwo_handle *h, gwo_status s) {
    if (s == GWO_OK) return 0;
    const char *cls = s == GWO_ERR_INVALID_ARGUMENT ? "java/lang/IllegalArgumentException"
                      : (s == GWO_ERR_UNSUPPORTED || s == GWO_ERR_MERGE_LATE) ? "java/lang/UnsupportedOperationException"
                                                                               : "java/lang/RuntimeException";
    const char *msg = h ? gwo_last_error(h) : NULL;
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg && *msg ? msg : gwo_status_string(s));
    return 1;
}

static void *addr(JNIEnv *env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }

static void throw_arg(JNIEnv *env, const char *msg) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

/* A direct buffer that must hold `need` bytes: its address, or NULL with an IllegalArgumentException pending. */
static void *sized(JNIEnv *env, jobject buf, int64_t need, const char *what) {
    if (!buf) {
        if (need > 0) throw_arg(env, what);
        return NULL;
    }
    void *p = (*env)->GetDirectBufferAddress(env, buf);
    jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    if (!p || cap < 0 || (int64_t)cap < need) {
        throw_arg(env, what);
        return NULL;
    }
    return p;
}

/* A Java primitive array that must hold `need` elements. */
static int array_ok(JNIEnv *env, jarray a, int64_t need, const char *what) {
    if (!a || (int64_t)(*env)->GetArrayLength(env, a) < need) {
        throw_arg(env, what);
        return 0;
    }
    return 1;
}

JNIEXPORT jint JNICALL JFN(abiVersion)(JNIEnv *env, jclass c) {
    (void)env;
    (void)c;
    return GWO_ABI_VERSION;
}

JNIEXPORT jlong JNICALL JFN(create)(JNIEnv *env, jclass c, jint assigner, jlong size, jlong slide, jlong offset,
                                    jlong gap, jlong lateness, jintArray aggs, jint value_dtype, jint key_kind,
                                    jint max_par, jint kg_start, jint kg_end, jint device, jboolean side_output,
                                    jint layout, jlong expected_keys) {
    (void)c;
    gwo_config cfg;
    gwo_config_init(&cfg);
    cfg.assigner = assigner;
    cfg.size = size;
    cfg.slide = slide;
    cfg.offset = offset;
    cfg.gap = gap;
    cfg.allowed_lateness = lateness;
    jsize na = (*env)->GetArrayLength(env, aggs);
    if (na < 1 || na > GWO_MAX_AGGS) {
        fail(env, NULL, GWO_ERR_INVALID_ARGUMENT);
        return 0;
    }
    jint tmp[GWO_MAX_AGGS];
    (*env)->GetIntArrayRegion(env, aggs, 0, na, tmp);
    cfg.num_aggs = na;
    for (int i = 0; i < na; ++i) cfg.aggs[i] = tmp[i];
    cfg.value_dtype = value_dtype;
    cfg.key_kind = key_kind;
    cfg.max_parallelism = max_par;
    cfg.key_group_start = kg_start;
    cfg.key_group_end = kg_end;
    cfg.device = device;
    cfg.side_output = side_output ? 1 : 0;
    cfg.state_layout = layout;
    cfg.expected_keys = expected_keys;
    gwo_handle *h = NULL;
    if (fail(env, NULL, gwo_create(&cfg, &h))) return 0;
    return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL JFN(destroy)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    fail(env, NULL, gwo_destroy(H(h)));
}

/* gwo_host_register / gwo_host_unregister of a direct ByteBuffer's memory (the operator's columns, pinned once in
 * open(): its batches then reach the GPU by DMA). */
JNIEXPORT void JNICALL JFN(hostRegister)(JNIEnv *env, jclass c, jobject buf) {
    (void)c;
    void *p = sized(env, buf, 1, "direct buffer required");
    if ((*env)->ExceptionCheck(env)) return;
    fail(env, NULL, gwo_host_register(p, (int64_t)(*env)->GetDirectBufferCapacity(env, buf)));
}

JNIEXPORT void JNICALL JFN(hostUnregister)(JNIEnv *env, jclass c, jobject buf) {
    (void)c;
    void *p = sized(env, buf, 1, "direct buffer required");
    if ((*env)->ExceptionCheck(env)) return;
    fail(env, NULL, gwo_host_unregister(p));
}

JNIEXPORT void JNICALL JFN(submit)(JNIEnv *env, jclass c, jlong h, jobject k, jobject t, jobject v, jint n) {
    (void)c;
    if (n < 0) { throw_arg(env, "negative record count"); return; }
    void *pk = sized(env, k, 8LL * n, "keys buffer smaller than n records");
    if ((*env)->ExceptionCheck(env)) return;
    void *pt = sized(env, t, 8LL * n, "timestamps buffer smaller than n records");
    if ((*env)->ExceptionCheck(env)) return;
    void *pv = v ? sized(env, v, 8LL * n, "values buffer smaller than n records") : NULL;
    if ((*env)->ExceptionCheck(env)) return;
    fail(env, H(h), gwo_submit(H(h), pk, pt, pv, n));
}

JNIEXPORT void JNICALL JFN(submitUtf16)(JNIEnv *env, jclass c, jlong h, jobject chars, jobject offsets, jobject t,
                                        jobject v, jint n) {
    (void)c;
    if (n < 0) { throw_arg(env, "negative record count"); return; }
    const int64_t *off = sized(env, offsets, 8LL * (n + 1), "offsets buffer smaller than n + 1 entries");
    if ((*env)->ExceptionCheck(env)) return;
    if (off[0] != 0) { throw_arg(env, "offsets[0] must be 0"); return; }
    for (jint i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) { throw_arg(env, "decreasing offsets"); return; }
    void *pc = sized(env, chars, 2 * off[n], "chars buffer smaller than offsets[n] code units");
    if ((*env)->ExceptionCheck(env)) return;
    void *pt = sized(env, t, 8LL * n, "timestamps buffer smaller than n records");
    if ((*env)->ExceptionCheck(env)) return;
    void *pv = v ? sized(env, v, 8LL * n, "values buffer smaller than n records") : NULL;
    if ((*env)->ExceptionCheck(env)) return;
    fail(env, H(h), gwo_submit_utf16(H(h), pc, off, pt, pv, n));
}

/* gwo_sync: every submitted batch, exchange and fire completed (snapshots, close). */
JNIEXPORT void JNICALL JFN(sync)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    fail(env, H(h), gwo_sync(H(h)));
}

/* gwo_wait_fires: waits for a fire still running (sessions and the log layout fire asynchronously), so that
 * outputCount afterwards counts every row of the watermark just applied; batches stay in flight. */
JNIEXPORT void JNICALL JFN(waitFires)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    fail(env, H(h), gwo_wait_fires(H(h)));
}

JNIEXPORT void JNICALL JFN(advanceWatermark)(JNIEnv *env, jclass c, jlong h, jlong wm) {
    (void)c;
    fail(env, H(h), gwo_advance_watermark(H(h), wm));
}

JNIEXPORT jlong JNICALL JFN(outputCount)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    int64_t n = 0;
    fail(env, H(h), gwo_output_count(H(h), &n));
    return n;
}

JNIEXPORT jlong JNICALL JFN(drain)(JNIEnv *env, jclass c, jlong h, jobject k, jobject s, jobject e,
                                   jobjectArray results, jlong cap) {
    (void)c;
    if (cap < 0) {
        throw_arg(env, "negative capacity");
        return 0;
    }
    gwo_out o;
    memset(&o, 0, sizeof o);
    o.key = sized(env, k, 8 * cap, "keys buffer smaller than capacity");
    if (!(*env)->ExceptionCheck(env)) o.start = sized(env, s, 8 * cap, "starts buffer smaller than capacity");
    if (!(*env)->ExceptionCheck(env)) o.end = sized(env, e, 8 * cap, "ends buffer smaller than capacity");
    jsize nr = results ? (*env)->GetArrayLength(env, results) : 0;
    for (jsize i = 0; i < nr && i < GWO_MAX_AGGS && !(*env)->ExceptionCheck(env); ++i) {
        jobject b = (*env)->GetObjectArrayElement(env, results, i);
        o.result[i] = sized(env, b, 8 * cap, "result buffer smaller than capacity");
        (*env)->DeleteLocalRef(env, b);
    }
    if ((*env)->ExceptionCheck(env)) return 0;
    int64_t got = 0;
    fail(env, H(h), gwo_drain(H(h), &o, cap, &got));
    return got;
}

JNIEXPORT jint JNICALL JFN(resultDtype)(JNIEnv *env, jclass c, jlong h, jint agg) {
    (void)c;
    int32_t d = 0;
    fail(env, H(h), gwo_result_dtype(H(h), agg, &d));
    return d;
}

JNIEXPORT jlong JNICALL JFN(lateDropped)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    int64_t n = 0;
    fail(env, H(h), gwo_late_dropped(H(h), &n));
    return n;
}

JNIEXPORT jlong JNICALL JFN(sideOutputCount)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    int64_t n = 0;
    fail(env, H(h), gwo_side_output_count(H(h), &n));
    return n;
}

JNIEXPORT jlong JNICALL JFN(drainSideOutput)(JNIEnv *env, jclass c, jlong h, jobject k, jobject t, jobject v,
                                             jlong cap) {
    (void)c;
    if (cap < 0) {
        throw_arg(env, "negative capacity");
        return 0;
    }
    gwo_side_out o;
    o.key = sized(env, k, 8 * cap, "keys buffer smaller than capacity");
    o.ts = (*env)->ExceptionCheck(env) ? NULL : sized(env, t, 8 * cap, "timestamps buffer smaller than capacity");
    o.value = (*env)->ExceptionCheck(env) ? NULL : sized(env, v, 8 * cap, "values buffer smaller than capacity");
    if ((*env)->ExceptionCheck(env)) return 0;
    int64_t got = 0;
    fail(env, H(h), gwo_drain_side_output(H(h), &o, cap, &got));
    return got;
}

JNIEXPORT jlong JNICALL JFN(currentWatermark)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    int64_t wm = 0;
    fail(env, H(h), gwo_current_watermark(H(h), &wm));
    return wm;
}

JNIEXPORT jlong JNICALL JFN(stateSize)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    int64_t n = 0;
    fail(env, H(h), gwo_state_size(H(h), &n));
    return n;
}

JNIEXPORT jlongArray JNICALL JFN(snapshotRows)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    int64_t rows = 0;
    int32_t words = 0;
    if (fail(env, H(h), gwo_snapshot_rows(H(h), &rows, &words))) return NULL;
    jlongArray r = (*env)->NewLongArray(env, 2);
    jlong v[2] = {rows, words};
    (*env)->SetLongArrayRegion(env, r, 0, 2, v);
    return r;
}

/* gwo_snapshot into Java arrays (heap memory, as the heap backend's own snapshot is): capacity `cap` rows; words
 * holds cap * n_words longs.  Returns {rows, watermark}. */
JNIEXPORT jlongArray JNICALL JFN(snapshot)(JNIEnv *env, jclass c, jlong h, jlongArray k, jlongArray s, jlongArray e,
                                           jlongArray w, jintArray kg, jintArray tm, jint nw, jlong cap) {
    (void)c;
    if (cap < 0 || nw < 0) {
        throw_arg(env, "negative capacity");
        return NULL;
    }
    if (!array_ok(env, k, cap, "keys array smaller than capacity") || !array_ok(env, s, cap, "starts array") ||
        !array_ok(env, e, cap, "ends array") || !array_ok(env, w, cap * nw, "words array smaller than cap * n_words") ||
        !array_ok(env, kg, cap, "key groups array") || !array_ok(env, tm, cap, "timers array"))
        return NULL;
    jlong *pk = (*env)->GetLongArrayElements(env, k, NULL), *ps = (*env)->GetLongArrayElements(env, s, NULL),
          *pe = (*env)->GetLongArrayElements(env, e, NULL), *pw = (*env)->GetLongArrayElements(env, w, NULL);
    jint *pg = (*env)->GetIntArrayElements(env, kg, NULL), *pt = (*env)->GetIntArrayElements(env, tm, NULL);
    jlongArray r = NULL;
    if (pk && ps && pe && pw && pg && pt) {
        gwo_state_rows rows = {(int64_t *)pk, (int64_t *)ps, (int64_t *)pe, (int64_t *)pw, (int32_t *)pg, (int32_t *)pt};
        int64_t n = 0, wm = 0;
        if (!fail(env, H(h), gwo_snapshot(H(h), &rows, cap, &n, &wm))) {
            r = (*env)->NewLongArray(env, 2);
            jlong v[2] = {n, wm};
            if (r) (*env)->SetLongArrayRegion(env, r, 0, 2, v);
        }
    }
    const jint mode = r ? 0 : JNI_ABORT;
    if (pk) (*env)->ReleaseLongArrayElements(env, k, pk, mode);
    if (ps) (*env)->ReleaseLongArrayElements(env, s, ps, mode);
    if (pe) (*env)->ReleaseLongArrayElements(env, e, pe, mode);
    if (pw) (*env)->ReleaseLongArrayElements(env, w, pw, mode);
    if (pg) (*env)->ReleaseIntArrayElements(env, kg, pg, mode);
    if (pt) (*env)->ReleaseIntArrayElements(env, tm, pt, mode);
    return r;
}

JNIEXPORT void JNICALL JFN(restore)(JNIEnv *env, jclass c, jlong h, jlongArray k, jlongArray s, jlongArray e,
                                    jlongArray w, jintArray tm, jint nw, jlong n, jlong wm) {
    (void)c;
    if (n < 0 || nw < 0) { throw_arg(env, "negative row count"); return; }
    if (!array_ok(env, k, n, "keys array smaller than n") || !array_ok(env, s, n, "starts array") ||
        !array_ok(env, e, n, "ends array") || !array_ok(env, w, n * nw, "words array smaller than n * n_words") ||
        !array_ok(env, tm, n, "timers array"))
        return;
    jlong *pk = (*env)->GetLongArrayElements(env, k, NULL), *ps = (*env)->GetLongArrayElements(env, s, NULL),
          *pe = (*env)->GetLongArrayElements(env, e, NULL), *pw = (*env)->GetLongArrayElements(env, w, NULL);
    jint *pt = (*env)->GetIntArrayElements(env, tm, NULL);
    if (pk && ps && pe && pw && pt) {
        gwo_state_rows rows = {(int64_t *)pk, (int64_t *)ps, (int64_t *)pe, (int64_t *)pw, NULL, (int32_t *)pt};
        fail(env, H(h), gwo_restore(H(h), &rows, nw, n, wm));
    }
    if (pk) (*env)->ReleaseLongArrayElements(env, k, pk, JNI_ABORT);
    if (ps) (*env)->ReleaseLongArrayElements(env, s, ps, JNI_ABORT);
    if (pe) (*env)->ReleaseLongArrayElements(env, e, pe, JNI_ABORT);
    if (pw) (*env)->ReleaseLongArrayElements(env, w, pw, JNI_ABORT);
    if (pt) (*env)->ReleaseIntArrayElements(env, tm, pt, JNI_ABORT);
}

static int heap_ids(JNIEnv *env, jintArray ids, gwo_heap_state_ids *out) {
    if (!array_ok(env, ids, 4, "ids: {window-contents, merging-window-set, event timers, processing timers}")) return 0;
    jint v[4];
    (*env)->GetIntArrayRegion(env, ids, 0, 4, v);
    out->window_contents = (int16_t)v[0];
    out->merging_window_set = (int16_t)v[1];
    out->event_timers = (int16_t)v[2];
    out->processing_timers = (int16_t)v[3];
    return 1;
}

/* gwo_export_heap_state into a Java byte[] (sized by a first, counting call). */
JNIEXPORT jbyteArray JNICALL JFN(exportHeapState)(JNIEnv *env, jclass c, jlong h, jintArray ids, jlongArray kgOffsets,
                                                  jlongArray watermarkOut) {
    (void)c;
    gwo_heap_state_ids sid;
    gwo_config cfg;
    if (!heap_ids(env, ids, &sid) || !array_ok(env, watermarkOut, 1, "watermark array")) return NULL;
    if (fail(env, H(h), gwo_get_config(H(h), &cfg))) return NULL;
    /* one offset per key group of the subtask's KeyGroupRange (gwo_export_heap_state writes all of them) */
    if (!array_ok(env, kgOffsets, (jlong)cfg.key_group_end - cfg.key_group_start + 1,
                  "keyGroupOffsets smaller than the subtask's key-group count"))
        return NULL;
    int64_t need = 0, len = 0, wm = 0;
    if (fail(env, H(h), gwo_export_heap_state(H(h), &sid, NULL, 0, &need, NULL, NULL))) return NULL;
    if (need > 0x7fffffff - 8) {
        throw_arg(env, "heap-layout state exceeds one Java byte[]; checkpoint it with more subtasks");
        return NULL;
    }
    uint8_t *buf = (uint8_t *)malloc((size_t)(need > 0 ? need : 1));
    jlong *po = (*env)->GetLongArrayElements(env, kgOffsets, NULL);
    jbyteArray r = NULL;
    if (buf && po && !fail(env, H(h), gwo_export_heap_state(H(h), &sid, buf, need, &len, (int64_t *)po, &wm))) {
        r = (*env)->NewByteArray(env, (jsize)len);
        if (r) (*env)->SetByteArrayRegion(env, r, 0, (jsize)len, (const jbyte *)buf);
        jlong w = wm;
        (*env)->SetLongArrayRegion(env, watermarkOut, 0, 1, &w);
    } else if (!buf) {
        throw_arg(env, "out of host memory for the heap-layout state");
    }
    if (po) (*env)->ReleaseLongArrayElements(env, kgOffsets, po, r ? 0 : JNI_ABORT);
    free(buf);
    return r;
}

/* Staged export (gwo_export_heap_state_begin/_read/_end): the operator streams the image key group by key group into
 * its keyed state backend instead of holding it in one byte[]. */
JNIEXPORT jlong JNICALL JFN(exportHeapStateBegin)(JNIEnv *env, jclass c, jlong h, jintArray ids, jlongArray kgOffsets,
                                                 jlongArray watermarkOut) {
    (void)c;
    gwo_heap_state_ids sid;
    gwo_config cfg;
    if (!heap_ids(env, ids, &sid) || !array_ok(env, watermarkOut, 1, "watermark array")) return -1;
    if (fail(env, H(h), gwo_get_config(H(h), &cfg))) return -1;
    if (!array_ok(env, kgOffsets, (jlong)cfg.key_group_end - cfg.key_group_start + 1,
                  "keyGroupOffsets smaller than the subtask's key-group count"))
        return -1;
    jlong *po = (*env)->GetLongArrayElements(env, kgOffsets, NULL);
    if (!po) return -1;
    int64_t len = 0, wm = 0;
    const int bad = fail(env, H(h), gwo_export_heap_state_begin(H(h), &sid, &len, (int64_t *)po, &wm));
    (*env)->ReleaseLongArrayElements(env, kgOffsets, po, bad ? JNI_ABORT : 0);
    if (bad) return -1;
    jlong w = wm;
    (*env)->SetLongArrayRegion(env, watermarkOut, 0, 1, &w);
    return (jlong)len;
}

JNIEXPORT void JNICALL JFN(exportHeapStateRead)(JNIEnv *env, jclass c, jlong h, jlong offset, jbyteArray dst, jint len) {
    (void)c;
    if (len < 0 || !array_ok(env, dst, len, "destination smaller than len")) return;
    jbyte *p = (*env)->GetByteArrayElements(env, dst, NULL);
    if (!p) return;
    const int bad = fail(env, H(h), gwo_export_heap_state_read(H(h), offset, (uint8_t *)p, len));
    (*env)->ReleaseByteArrayElements(env, dst, p, bad ? JNI_ABORT : 0);
}

JNIEXPORT void JNICALL JFN(exportHeapStateEnd)(JNIEnv *env, jclass c, jlong h) {
    (void)c;
    fail(env, H(h), gwo_export_heap_state_end(H(h)));
}

JNIEXPORT void JNICALL JFN(importHeapState)(JNIEnv *env, jclass c, jlong h, jintArray ids, jbyteArray data,
                                            jlong watermark) {
    (void)c;
    gwo_heap_state_ids sid;
    if (!heap_ids(env, ids, &sid) || !array_ok(env, data, 0, "state bytes")) return;
    const jsize n = (*env)->GetArrayLength(env, data);
    jbyte *p = (*env)->GetByteArrayElements(env, data, NULL);
    if (!p) return;
    fail(env, H(h), gwo_import_heap_state(H(h), &sid, (const uint8_t *)p, n, watermark));
    (*env)->ReleaseByteArrayElements(env, data, p, JNI_ABORT);
}

/* Ids of a String-keyed handle (a Java long[]) back to Strings. */
JNIEXPORT jobjectArray JNICALL JFN(keyStrings)(JNIEnv *env, jclass c, jlong h, jlongArray ids, jint n) {
    (void)c;
    if (n < 0 || !array_ok(env, ids, n, "ids array smaller than n")) return NULL;
    jclass str = (*env)->FindClass(env, "java/lang/String");
    if (!str) return NULL;
    jlong *id = (*env)->GetLongArrayElements(env, ids, NULL);
    int64_t *off = (int64_t *)malloc(((size_t)n + 1) * sizeof(int64_t));
    jobjectArray out = NULL;
    uint16_t *u = NULL;
    int64_t need = 0;
    if (!id || !off) {
        throw_arg(env, "out of memory");
        goto done;
    }
    if (fail(env, H(h), gwo_key_strings(H(h), (const int64_t *)id, n, off, NULL, 0, &need))) goto done;
    u = (uint16_t *)malloc((size_t)(need > 0 ? need : 1) * 2);
    if (!u) {
        throw_arg(env, "out of memory");
        goto done;
    }
    if (fail(env, H(h), gwo_key_strings(H(h), (const int64_t *)id, n, off, u, need, &need))) goto done;
    out = (*env)->NewObjectArray(env, n, str, NULL);
    for (jint i = 0; out && i < n; ++i) {
        const int64_t len = off[i + 1] - off[i];
        if (len > INT32_MAX) {
            throw_arg(env, "String longer than 2^31 code units");
            out = NULL;
            break;
        }
        jstring js = (*env)->NewString(env, (const jchar *)(u + off[i]), (jsize)len);
        if (!js) {
            out = NULL;
            break;
        }
        (*env)->SetObjectArrayElement(env, out, i, js);
        (*env)->DeleteLocalRef(env, js);   /* n may exceed the 16 local references JNI guarantees */
    }
done:
    free(u);
    free(off);
    if (id) (*env)->ReleaseLongArrayElements(env, ids, id, JNI_ABORT);
    (*env)->DeleteLocalRef(env, str);
    return out;
}

JNIEXPORT void JNICALL JFN(internUtf16)(JNIEnv *env, jclass c, jlong h, jobject chars, jobject offsets, jint n,
                                        jlongArray ids) {
    (void)c;
    if (n < 0) { throw_arg(env, "negative count"); return; }
    const int64_t *off = sized(env, offsets, 8LL * (n + 1), "offsets buffer smaller than n + 1 entries");
    if ((*env)->ExceptionCheck(env)) return;
    if (off[0] != 0) { throw_arg(env, "offsets[0] must be 0"); return; }
    for (jint i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) { throw_arg(env, "decreasing offsets"); return; }
    void *pc = sized(env, chars, 2 * off[n], "chars buffer smaller than offsets[n] code units");
    if ((*env)->ExceptionCheck(env)) return;
    if (!array_ok(env, ids, n, "ids array smaller than n")) return;
    jlong *pi = (*env)->GetLongArrayElements(env, ids, NULL);
    if (!pi) return;
    const int bad = fail(env, H(h), gwo_intern_utf16(H(h), pc, off, n, (int64_t *)pi));
    (*env)->ReleaseLongArrayElements(env, ids, pi, bad ? JNI_ABORT : 0);
}
