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
    (*env)->ThrowNew(env, (*env)->FindClass(env, cls), msg && *msg ? msg : gwo_status_string(s));
    return 1;
}

static void *addr(JNIEnv *env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }

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

JNIEXPORT void JNICALL JFN(submit)(JNIEnv *env, jclass c, jlong h, jobject k, jobject t, jobject v, jint n) {
    (void)c;
    fail(env, H(h), gwo_submit(H(h), addr(env, k), addr(env, t), addr(env, v), n));
}

JNIEXPORT void JNICALL JFN(submitUtf16)(JNIEnv *env, jclass c, jlong h, jobject chars, jobject offsets, jobject t,
                                        jobject v, jint n) {
    (void)c;
    fail(env, H(h), gwo_submit_utf16(H(h), addr(env, chars), addr(env, offsets), addr(env, t), addr(env, v), n));
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
    gwo_out o;
    memset(&o, 0, sizeof o);
    o.key = addr(env, k);
    o.start = addr(env, s);
    o.end = addr(env, e);
    jsize nr = results ? (*env)->GetArrayLength(env, results) : 0;
    for (jsize i = 0; i < nr && i < GWO_MAX_AGGS; ++i) o.result[i] = addr(env, (*env)->GetObjectArrayElement(env, results, i));
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
    gwo_side_out o;
    o.key = addr(env, k);
    o.ts = addr(env, t);
    o.value = addr(env, v);
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

JNIEXPORT jlongArray JNICALL JFN(snapshot)(JNIEnv *env, jclass c, jlong h, jobject k, jobject s, jobject e,
                                           jobject w, jobject kg, jobject tm, jlong cap) {
    (void)c;
    gwo_state_rows rows = {addr(env, k), addr(env, s), addr(env, e), addr(env, w), addr(env, kg), addr(env, tm)};
    int64_t n = 0, wm = 0;
    if (fail(env, H(h), gwo_snapshot(H(h), &rows, cap, &n, &wm))) return NULL;
    jlongArray r = (*env)->NewLongArray(env, 2);
    jlong v[2] = {n, wm};
    (*env)->SetLongArrayRegion(env, r, 0, 2, v);
    return r;
}

JNIEXPORT void JNICALL JFN(restore)(JNIEnv *env, jclass c, jlong h, jobject k, jobject s, jobject e, jobject w,
                                    jobject tm, jint nw, jlong n, jlong wm) {
    (void)c;
    gwo_state_rows rows = {addr(env, k), addr(env, s), addr(env, e), addr(env, w), NULL, addr(env, tm)};
    fail(env, H(h), gwo_restore(H(h), &rows, nw, n, wm));
}

JNIEXPORT jobjectArray JNICALL JFN(keyStrings)(JNIEnv *env, jclass c, jlong h, jobject ids, jlong n) {
    (void)c;
    int64_t need = 0;
    int64_t *off = (int64_t *)(*env)->GetDirectBufferAddress(env, ids);   /* reused below only for the ids */
    jlongArray offs = (*env)->NewLongArray(env, (jsize)(n + 1));
    jlong *o = (*env)->GetLongArrayElements(env, offs, NULL);
    if (fail(env, H(h), gwo_key_strings(H(h), off, n, (int64_t *)o, NULL, 0, &need))) {
        (*env)->ReleaseLongArrayElements(env, offs, o, JNI_ABORT);
        return NULL;
    }
    jcharArray chars = (*env)->NewCharArray(env, (jsize)(need > 0 ? need : 1));
    jchar *u = (*env)->GetCharArrayElements(env, chars, NULL);
    gwo_status st = gwo_key_strings(H(h), off, n, (int64_t *)o, (uint16_t *)u, need, &need);
    jobjectArray out = NULL;
    if (!fail(env, H(h), st)) {
        out = (*env)->NewObjectArray(env, (jsize)n, (*env)->FindClass(env, "java/lang/String"), NULL);
        for (jsize i = 0; i < (jsize)n; ++i)
            (*env)->SetObjectArrayElement(env, out, i, (*env)->NewString(env, u + o[i], (jsize)(o[i + 1] - o[i])));
    }
    (*env)->ReleaseCharArrayElements(env, chars, u, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, offs, o, JNI_ABORT);
    return out;
}

JNIEXPORT void JNICALL JFN(internUtf16)(JNIEnv *env, jclass c, jlong h, jobject chars, jobject offsets, jint n,
                                        jobject ids) {
    (void)c;
    fail(env, H(h), gwo_intern_utf16(H(h), addr(env, chars), addr(env, offsets), n, addr(env, ids)));
}
