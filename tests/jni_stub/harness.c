/* TEST INFRASTRUCTURE ONLY (tests/test_java_binding.py): runs jni/gwo_jni.c's argument checks without a JVM.
 * A fake JNIEnv (the function table of tests/jni_stub/jni.h) backs Java arrays and direct buffers with plain C
 * structs and records the exception a call throws; fake gwo_* entry points record whether the shim reached the
 * library.  Each case prints "<name> <exception class or -> <library calls>". */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../jni/gwo_jni.c"

typedef struct { int kind; jsize len; void *data; } FakeArr;   /* kind 0: long[], 1: int[], 2: byte[], 3: direct */
static const char *thrown;
static int lib_calls;

static jclass f_FindClass(JNIEnv *e, const char *n) { (void)e; return (jclass)n; }
static jint f_ThrowNew(JNIEnv *e, jclass c, const char *m) { (void)e; (void)m; thrown = (const char *)c; return 0; }
static void *f_GetDirectBufferAddress(JNIEnv *e, jobject b) { (void)e; return b ? ((FakeArr *)b)->data : NULL; }
static jlong f_GetDirectBufferCapacity(JNIEnv *e, jobject b) { (void)e; return b ? ((FakeArr *)b)->len : -1; }
static jsize f_GetArrayLength(JNIEnv *e, jarray a) { (void)e; return ((FakeArr *)a)->len; }
static void f_GetIntArrayRegion(JNIEnv *e, jintArray a, jsize s, jsize n, jint *d) {
    (void)e; memcpy(d, (jint *)((FakeArr *)a)->data + s, (size_t)n * 4);
}
static jboolean f_ExceptionCheck(JNIEnv *e) { (void)e; return thrown != NULL; }
static jlong *f_GetLongArrayElements(JNIEnv *e, jlongArray a, jboolean *c) { (void)e; (void)c; return ((FakeArr *)a)->data; }
static void f_ReleaseLongArrayElements(JNIEnv *e, jlongArray a, jlong *p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jbyte *f_GetByteArrayElements(JNIEnv *e, jbyteArray a, jboolean *c) { (void)e; (void)c; return ((FakeArr *)a)->data; }
static void f_ReleaseByteArrayElements(JNIEnv *e, jbyteArray a, jbyte *p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jbyteArray f_NewByteArray(JNIEnv *e, jsize n) {
    (void)e; FakeArr *a = calloc(1, sizeof *a); a->kind = 2; a->len = n; a->data = calloc((size_t)n + 1, 1); return a;
}
static void f_SetByteArrayRegion(JNIEnv *e, jbyteArray a, jsize s, jsize n, const jbyte *d) {
    (void)e; memcpy((jbyte *)((FakeArr *)a)->data + s, d, (size_t)n);
}
static void f_SetLongArrayRegion(JNIEnv *e, jlongArray a, jsize s, jsize n, const jlong *d) {
    (void)e; memcpy((jlong *)((FakeArr *)a)->data + s, d, (size_t)n * 8);
}

/* the library side: only what these cases reach */
static gwo_config g_cfg;
gwo_status gwo_get_config(const gwo_handle *h, gwo_config *out) { (void)h; *out = g_cfg; return GWO_OK; }
gwo_status gwo_export_heap_state(gwo_handle *h, const gwo_heap_state_ids *ids, uint8_t *buf, int64_t cap, int64_t *len,
                                 int64_t *kg_offsets, int64_t *wm) {
    (void)h; (void)ids; (void)cap;
    lib_calls++;
    *len = 16;
    if (buf) memset(buf, 7, 16);
    if (kg_offsets)   /* writes every key group's offset, as the library does */
        for (int g = 0; g <= g_cfg.key_group_end - g_cfg.key_group_start; ++g) kg_offsets[g] = g;
    if (wm) *wm = 42;
    return GWO_OK;
}
gwo_status gwo_import_heap_state(gwo_handle *h, const gwo_heap_state_ids *ids, const uint8_t *b, int64_t l, int64_t w) {
    (void)h; (void)ids; (void)b; (void)l; (void)w; lib_calls++; return GWO_OK;
}
gwo_status gwo_host_register(void *p, int64_t n) { (void)p; (void)n; lib_calls++; return GWO_OK; }
gwo_status gwo_host_unregister(void *p) { (void)p; lib_calls++; return GWO_OK; }
const char *gwo_last_error(const gwo_handle *h) { (void)h; return ""; }
const char *gwo_status_string(gwo_status s) { (void)s; return "status"; }

static FakeArr *arr(int kind, jsize len, size_t elem) {
    FakeArr *a = calloc(1, sizeof *a); a->kind = kind; a->len = len; a->data = calloc((size_t)len + 1, elem); return a;
}
static void report(const char *name) {
    printf("%s %s %d\n", name, thrown ? thrown : "-", lib_calls);
    thrown = NULL;
    lib_calls = 0;
}

int main(void) {
    struct JNINativeInterface_ fns = {0};
    fns.FindClass = f_FindClass; fns.ThrowNew = f_ThrowNew; fns.GetDirectBufferAddress = f_GetDirectBufferAddress;
    fns.GetDirectBufferCapacity = f_GetDirectBufferCapacity; fns.GetArrayLength = f_GetArrayLength;
    fns.GetIntArrayRegion = f_GetIntArrayRegion; fns.ExceptionCheck = f_ExceptionCheck;
    fns.GetLongArrayElements = f_GetLongArrayElements; fns.ReleaseLongArrayElements = f_ReleaseLongArrayElements;
    fns.GetByteArrayElements = f_GetByteArrayElements; fns.ReleaseByteArrayElements = f_ReleaseByteArrayElements;
    fns.NewByteArray = f_NewByteArray; fns.SetByteArrayRegion = f_SetByteArrayRegion;
    fns.SetLongArrayRegion = f_SetLongArrayRegion;
    const struct JNINativeInterface_ *tbl = &fns;
    JNIEnv *env = &tbl;
    g_cfg.key_group_start = 10;
    g_cfg.key_group_end = 17;   /* 8 key groups */
    FakeArr *ids = arr(1, 4, 4), *wm = arr(0, 1, 8);
    jint *iv = ids->data; iv[0] = 0; iv[1] = -1; iv[2] = 1; iv[3] = 2;
    JFN(exportHeapState)(env, NULL, 1, ids, NULL, wm);
    report("export_null_offsets");
    JFN(exportHeapState)(env, NULL, 1, ids, arr(0, 7, 8), wm);
    report("export_short_offsets");
    FakeArr *off = arr(0, 8, 8);
    jbyteArray r = JFN(exportHeapState)(env, NULL, 1, ids, off, wm);
    printf("export_ok_len %d wm %lld last_offset %lld\n", r ? ((FakeArr *)r)->len : -1, (long long)((jlong *)wm->data)[0],
           (long long)((jlong *)off->data)[7]);
    report("export_ok");
    JFN(importHeapState)(env, NULL, 1, ids, NULL, 0);
    report("import_null_data");
    JFN(importHeapState)(env, NULL, 1, ids, arr(2, 16, 1), 0);
    report("import_ok");
    JFN(hostRegister)(env, NULL, NULL);
    report("register_null");
    JFN(hostRegister)(env, NULL, arr(3, 64, 1));
    report("register_ok");
    return 0;
}
