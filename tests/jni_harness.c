/* Runtime check of the JNI shim's argument validation without a JVM (tests/test_jni_shim.py).
 *
 * java/jni/titan_gpu_olap_jni.c is linked into this program together with a fake JNIEnv whose
 * arrays are plain C buffers (tests/jni_stub/jni.h declares the table), and this program's own
 * tgo_load_csr, which records the call instead of touching a device (the executable's
 * definition is the one the shim's call binds to).  Each case calls the loadCsr entry point
 * as TgoNative.loadCsr would and checks the status and whether tgo_load_csr was reached.
 * Prints one line per case; exit status = failed cases. */
#include <jni.h>
#include <stdio.h>
#include <string.h>
#include "titan_gpu_olap.h"

typedef struct { jsize len; void* data; } FakeArr;
#define ARR(a) ((jarray)(void*)(a))

static jsize get_len(JNIEnv* env, jarray a) { (void)env; return ((FakeArr*)(void*)a)->len; }
static jint* get_ints(JNIEnv* env, jintArray a, jboolean* c) { (void)env; (void)c; return (jint*)((FakeArr*)(void*)a)->data; }
static jlong* get_longs(JNIEnv* env, jlongArray a, jboolean* c) { (void)env; (void)c; return (jlong*)((FakeArr*)(void*)a)->data; }
static void rel_ints(JNIEnv* env, jintArray a, jint* p, jint m) { (void)env; (void)a; (void)p; (void)m; }
static void rel_longs(JNIEnv* env, jlongArray a, jlong* p, jint m) { (void)env; (void)a; (void)p; (void)m; }
static int region_oob = 0;
static void long_region(JNIEnv* env, jlongArray a, jsize start, jsize len, jlong* buf) {
    (void)env;
    FakeArr* f = (FakeArr*)(void*)a;
    if (start < 0 || len < 0 || start + len > f->len) { region_oob = 1; return; }   /* JNI: ArrayIndexOutOfBounds */
    memcpy(buf, (jlong*)f->data + start, (size_t)len * sizeof(jlong));
}

static struct JNINativeInterface_ table;
static int csr_calls = 0;
static int64_t csr_n = -1;

/* the shim's call lands here (no device) */
int tgo_load_csr(tgo_ctx* ctx, int64_t n, const int64_t* titan_ids, const int64_t* out_off, const int32_t* out_idx,
                 const int32_t* out_w, const int64_t* in_off, const int32_t* in_idx, const int32_t* in_w,
                 const tgo_load_opts* opts) {
    (void)ctx; (void)titan_ids; (void)out_off; (void)out_idx; (void)out_w; (void)in_off; (void)in_idx; (void)in_w;
    (void)opts;
    ++csr_calls;
    csr_n = n;
    return TGO_OK;
}

jint Java_com_thinkaurelius_titan_graphdb_olap_gpu_TgoNative_loadCsr(JNIEnv* env, jclass cls, jlong h, jlongArray ids,
        jlongArray out_off, jintArray out_idx, jintArray out_w, jlongArray in_off, jintArray in_idx, jintArray in_w,
        jint scope, jlong weight_key, jboolean column_order);

static int failures = 0;
static void expect(const char* name, jint rc, jint want_rc, int want_calls) {
    const int ok = rc == want_rc && csr_calls == want_calls && !region_oob;
    printf("%s %s: rc=%d calls=%d\n", ok ? "ok  " : "FAIL", name, (int)rc, csr_calls);
    failures += !ok;
    csr_calls = 0;
    region_oob = 0;
}

int main(void) {
    table.GetArrayLength = get_len;
    table.GetIntArrayElements = get_ints;
    table.GetLongArrayElements = get_longs;
    table.ReleaseIntArrayElements = rel_ints;
    table.ReleaseLongArrayElements = rel_longs;
    table.GetLongArrayRegion = long_region;
    JNIEnv envp = &table;
    JNIEnv* env = &envp;
    /* 3 rows: 0 -> 1, 1 -> 2 (OUT); the IN lists their transposes */
    jlong ids_d[3] = {8, 16, 24}, oo_d[4] = {0, 1, 2, 2}, io_d[4] = {0, 0, 1, 2}, bad0_d[4] = {1, 1, 2, 2};
    jint oi_d[2] = {1, 2}, ii_d[2] = {0, 1}, w_d[2] = {3, 4};
    FakeArr ids = {3, ids_d}, ids2 = {2, ids_d}, oo = {4, oo_d}, io = {4, io_d}, bad0 = {4, bad0_d};
    FakeArr oi = {2, oi_d}, ii = {2, ii_d}, oi_short = {1, oi_d}, ii_short = {1, ii_d}, w = {2, w_d}, w_short = {1, w_d};
    FakeArr empty_off = {0, oo_d};
#define CALL(i, o, oix, ow, in, iix, iw, wk) \
    Java_com_thinkaurelius_titan_graphdb_olap_gpu_TgoNative_loadCsr(env, NULL, 1, ARR(i), ARR(o), ARR(oix), ARR(ow), \
                                                                    ARR(in), ARR(iix), ARR(iw), 2, wk, 0)
    expect("consistent rows reach tgo_load_csr", CALL(&ids, &oo, &oi, NULL, &io, &ii, NULL, 0), TGO_OK, 1);
    if (csr_n != 3) { printf("FAIL n passed as %lld\n", (long long)csr_n); ++failures; }
    expect("weighted rows with both weight arrays", CALL(&ids, &oo, &oi, &w, &io, &ii, &w, 7), TGO_OK, 1);
    expect("out index array shorter than out_off[n]", CALL(&ids, &oo, &oi_short, NULL, &io, &ii, NULL, 0), TGO_E_INVALID, 0);
    expect("in index array shorter than in_off[n]", CALL(&ids, &oo, &oi, NULL, &io, &ii_short, NULL, 0), TGO_E_INVALID, 0);
    expect("null out index array", CALL(&ids, &oo, NULL, NULL, &io, &ii, NULL, 0), TGO_E_INVALID, 0);
    expect("null in index array", CALL(&ids, &oo, &oi, NULL, &io, NULL, NULL, 0), TGO_E_INVALID, 0);
    expect("null offsets", CALL(&ids, NULL, &oi, NULL, &io, &ii, NULL, 0), TGO_E_INVALID, 0);
    expect("weight key without an out weight array", CALL(&ids, &oo, &oi, NULL, &io, &ii, &w, 7), TGO_E_INVALID, 0);
    expect("weight key with a short in weight array", CALL(&ids, &oo, &oi, &w, &io, &ii, &w_short, 7), TGO_E_INVALID, 0);
    expect("offsets not starting at 0", CALL(&ids, &bad0, &oi, NULL, &io, &ii, NULL, 0), TGO_E_INVALID, 0);
    expect("ids length disagrees with the offsets", CALL(&ids2, &oo, &oi, NULL, &io, &ii, NULL, 0), TGO_E_INVALID, 0);
    expect("empty offset array", CALL(&ids, &empty_off, &oi, NULL, &empty_off, &ii, NULL, 0), TGO_E_INVALID, 0);
    return failures;
}
