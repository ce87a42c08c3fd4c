/* Runtime check of the JNI shim without a JVM (tests/test_jni_shim.py).
 *
 * java/jni/titan_gpu_olap_jni.c is linked into this program together with a fake JNIEnv whose
 * arrays are plain C buffers (tests/jni_stub/jni.h declares the table), and this program's own
 * tgo_load_csr, which records the call instead of touching a device (the executable's
 * definition is the one the shim's call binds to); every other entry point is the real
 * library's.  The loadCsr cases call the entry point as TgoNative.loadCsr would and check the
 * status and whether tgo_load_csr was reached; the multi-GPU cases check the argument
 * validation of the partition / exchange natives and run tgo_part_layout (host work).
 * `jni_harness gpu` (a GPU box) then drives the Java multi-GPU path end to end at world 1:
 * create, partLayout, loadPartition, exchangeRcclId / exchangeRcclCreate and the three native
 * loops through the shim, against the one-GPU engine on the same graph.
 * Prints one line per case; exit status = failed cases. */
#include <jni.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "titan_gpu_olap.h"
#include "titan_gpu_olap_part.h"

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

/* arrays the shim creates (New*Array) and region copies with the JNI bounds rule */
static int thrown = 0;
static jclass find_class(JNIEnv* env, const char* name) { (void)env; (void)name; return (jclass)(void*)&thrown; }
static jint throw_new(JNIEnv* env, jclass c, const char* msg) { (void)env; (void)c; (void)msg; thrown = 1; return 0; }
static jstring new_string(JNIEnv* env, const char* utf) { (void)env; return (jstring)(void*)utf; }
static jarray new_arr(jsize len, size_t es) {
    FakeArr* f = (FakeArr*)calloc(1, sizeof(FakeArr));
    f->len = len;
    f->data = calloc((size_t)(len > 0 ? len : 1), es);
    return (jarray)(void*)f;
}
static jbyteArray new_bytes(JNIEnv* env, jsize len) { (void)env; return new_arr(len, 1); }
static jintArray new_ints(JNIEnv* env, jsize len) { (void)env; return new_arr(len, 4); }
static jlongArray new_longs(JNIEnv* env, jsize len) { (void)env; return new_arr(len, 8); }
static jdoubleArray new_doubles(JNIEnv* env, jsize len) { (void)env; return new_arr(len, 8); }
static jdouble* get_doubles(JNIEnv* env, jdoubleArray a, jboolean* c) { (void)env; (void)c; return (jdouble*)((FakeArr*)(void*)a)->data; }
static void rel_doubles(JNIEnv* env, jdoubleArray a, jdouble* p, jint m) { (void)env; (void)a; (void)p; (void)m; }
static void region(jarray a, jsize start, jsize len, void* buf, size_t es, int to_array) {
    FakeArr* f = (FakeArr*)(void*)a;
    if (start < 0 || len < 0 || start + len > f->len) { region_oob = 1; return; }
    if (to_array) memcpy((char*)f->data + (size_t)start * es, buf, (size_t)len * es);
    else memcpy(buf, (char*)f->data + (size_t)start * es, (size_t)len * es);
}
static void get_byte_region(JNIEnv* env, jbyteArray a, jsize s, jsize l, jbyte* b) { (void)env; region(a, s, l, b, 1, 0); }
static void set_byte_region(JNIEnv* env, jbyteArray a, jsize s, jsize l, const jbyte* b) { (void)env; region(a, s, l, (void*)b, 1, 1); }
static void set_long_region(JNIEnv* env, jlongArray a, jsize s, jsize l, const jlong* b) { (void)env; region(a, s, l, (void*)b, 8, 1); }

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

#define JFN(name) Java_com_thinkaurelius_titan_graphdb_olap_gpu_TgoNative_##name
jlong JFN(create)(JNIEnv*, jclass, jint, jint, jint, jlong);
void JFN(destroy)(JNIEnv*, jclass, jlong);
jintArray JFN(partLayout)(JNIEnv*, jclass, jintArray, jintArray, jlong, jlong, jlong, jint);
jint JFN(loadPartition)(JNIEnv*, jclass, jlong, jlong, jlong, jlong, jintArray, jintArray, jintArray, jint, jboolean,
                        jintArray);
jbyteArray JFN(exchangeRcclId)(JNIEnv*, jclass);
jlong JFN(exchangeRcclCreate)(JNIEnv*, jclass, jint, jint, jbyteArray, jint);
void JFN(exchangeDestroy)(JNIEnv*, jclass, jlong);
jlongArray JFN(partBfsRun)(JNIEnv*, jclass, jlong, jlong, jlong, jint, jdouble, jdouble);
jlongArray JFN(partSsspRun)(JNIEnv*, jclass, jlong, jlong, jlong, jlong);
jdoubleArray JFN(partPageRankRun)(JNIEnv*, jclass, jlong, jlong, jdouble, jlong, jint, jint);
jlongArray JFN(partMsbfsRun)(JNIEnv*, jclass, jlong, jlong, jlongArray, jint, jdouble, jlong);
jlongArray JFN(partMsLevels)(JNIEnv*, jclass, jlong, jint);
jint JFN(loadRows)(JNIEnv*, jclass, jlong, jlongArray, jlongArray, jlongArray, jobject, jlongArray, jlongArray, jlongArray,
                   jint, jboolean, jlongArray, jlong);
jlongArray JFN(finishPartitionRows)(JNIEnv*, jclass, jlong, jlong, jboolean);
jlongArray JFN(partWeightMin)(JNIEnv*, jclass, jlong);
#include "tgo_synth.h"
static void* direct_address(JNIEnv* env, jobject b) { (void)env; return ((FakeArr*)(void*)b)->data; }

static int failures = 0;
static void check(const char* name, int ok) {
    printf("%s %s\n", ok ? "ok  " : "FAIL", name);
    failures += !ok;
}

/* the test graph of the multi-GPU cases: a ring 0 -> 1 -> ... -> n-1 -> 0 plus chords
 * v -> 3v+1 mod n, weights 1 + (v * 7 + u) % 13 */
enum { GN = 256 };
static jint g_src[2 * GN], g_dst[2 * GN], g_w[2 * GN];
static int graph_edges(void) {
    int m = 0;
    for (int v = 0; v < GN; ++v) {
        const int t[2] = {(v + 1) % GN, (3 * v + 1) % GN};
        for (int k = 0; k < 2; ++k) { g_src[m] = v; g_dst[m] = t[k]; g_w[m] = 1 + (v * 7 + t[k]) % 13; ++m; }
    }
    return m;
}

static void partition_cases(JNIEnv* env) {
    const int m = graph_edges();
    FakeArr src = {m, g_src}, dst = {m, g_dst}, w = {m, g_w}, short_dst = {m - 1, g_dst}, w_short = {m - 2, g_w};
    jint lay_d[GN];
    FakeArr lay_short = {GN - 1, lay_d};
    /* partLayout (host work): a permutation of the owned range */
    jintArray lay = JFN(partLayout)(env, NULL, ARR(&src), ARR(&dst), GN, 64, 192, 2);
    int perm_ok = lay != NULL && ((FakeArr*)(void*)lay)->len == 128;
    if (perm_ok) {
        int seen[GN] = {0};
        const jint* p = (const jint*)((FakeArr*)(void*)lay)->data;
        for (int i = 0; i < 128; ++i) perm_ok &= p[i] >= 64 && p[i] < 192 && !seen[p[i]]++;
    }
    check("partLayout returns a permutation of [lo, hi)", perm_ok);
    check("partLayout rejects src / dst of different lengths",
          JFN(partLayout)(env, NULL, ARR(&src), ARR(&short_dst), GN, 0, GN, 2) == NULL);
    check("partLayout rejects an empty range", JFN(partLayout)(env, NULL, ARR(&src), ARR(&dst), GN, 64, 64, 2) == NULL);
    check("partLayout rejects a range past n_global", JFN(partLayout)(env, NULL, ARR(&src), ARR(&dst), GN, 0, GN + 64, 2) == NULL);
    /* loadPartition validates before the C-ABI (the ctx handle is fake: reaching it would crash) */
    check("loadPartition rejects src / dst of different lengths",
          JFN(loadPartition)(env, NULL, 1, GN, 0, GN, ARR(&src), ARR(&short_dst), NULL, 1, 1, NULL) == TGO_E_INVALID);
    check("loadPartition rejects a short weight array",
          JFN(loadPartition)(env, NULL, 1, GN, 0, GN, ARR(&src), ARR(&dst), ARR(&w_short), 1, 1, NULL) == TGO_E_INVALID);
    check("loadPartition rejects a layout shorter than n_global",
          JFN(loadPartition)(env, NULL, 1, GN, 0, GN, ARR(&src), ARR(&dst), ARR(&w), 1, 1, ARR(&lay_short)) == TGO_E_INVALID);
    check("loadPartition rejects null edges",
          JFN(loadPartition)(env, NULL, 1, GN, 0, GN, NULL, ARR(&dst), NULL, 1, 1, NULL) == TGO_E_INVALID);
    /* exchange creation: 128 id bytes, 0 <= rank < world */
    jbyte idb[128] = {0};
    FakeArr id_short = {127, idb}, id = {128, idb};
    check("exchangeRcclCreate rejects a 127-byte id", JFN(exchangeRcclCreate)(env, NULL, 1, 0, ARR(&id_short), 0) == 0);
    check("exchangeRcclCreate rejects rank >= world", JFN(exchangeRcclCreate)(env, NULL, 2, 2, ARR(&id), 0) == 0);
    /* the loops need an exchange; the sweep takes 1..64 seeds */
    jlong sd[65] = {0};
    FakeArr seeds65 = {65, sd}, seeds0 = {0, sd};
    check("partBfsRun without an exchange", JFN(partBfsRun)(env, NULL, 1, 0, 0, 4, 15.0, 18.0) == NULL);
    check("partMsbfsRun rejects 65 seeds", JFN(partMsbfsRun)(env, NULL, 1, 1, ARR(&seeds65), 4, 12.0, 0) == NULL);
    check("partMsbfsRun rejects no seeds", JFN(partMsbfsRun)(env, NULL, 1, 1, ARR(&seeds0), 4, 12.0, 0) == NULL);
    /* the rows partition reports its status instead of throwing (E_UNSUPPORTED -> one device) */
    jlongArray st = JFN(finishPartitionRows)(env, NULL, 0, 0, 1);
    check("finishPartitionRows without a ctx: {E_INVALID, 0, 0, 0}",
          st != NULL && ((FakeArr*)(void*)st)->len == 4 && ((jlong*)((FakeArr*)(void*)st)->data)[0] == TGO_E_INVALID);
    jlongArray wm = JFN(partWeightMin)(env, NULL, 0);
    check("partWeightMin without a ctx: {E_INVALID, 0}",
          wm != NULL && ((FakeArr*)(void*)wm)->len == 2 && ((jlong*)((FakeArr*)(void*)wm)->data)[0] == TGO_E_INVALID);
}

/* world 1 on a GPU, the Java multi-GPU ROW path (PartitionedRun: loadRows blocks + the collective
 * finishPartitionRows): synthetic edgestore rows of the test graph at a hard limit of 3 (every
 * row is cut: a vertex has 2 OUT + 2 IN user-edge entries), so the push rows come from the pull
 * entries sent through the exchange; SSSP (unit weights) and PageRank against tgo_load_rows. */
static void gpu_rows_case(JNIEnv* env) {
    const int m = graph_edges();
    const int64_t label = (1 << 6) | 21;
    int64_t sz[3];
    if (tgo_synth_rows(GN, m, (const int32_t*)g_src, (const int32_t*)g_dst, NULL, label, 5, 2, sz, NULL, NULL, NULL, NULL,
                       NULL) != TGO_OK) { check("synth rows sizes", 0); return; }
    static jlong keys[GN], eb[GN + 1], bb[GN + 1];
    jlong* lv = (jlong*)calloc((size_t)sz[1] + 1, 8);
    uint8_t* bytes = (uint8_t*)calloc((size_t)sz[2] + 1, 1);
    int ok = tgo_synth_rows(GN, m, (const int32_t*)g_src, (const int32_t*)g_dst, NULL, label, 5, 2, sz, (int64_t*)keys,
                            (int64_t*)eb, (int64_t*)bb, bytes, (int64_t*)lv) == TGO_OK;
    check("synth rows", ok);
    jlong types_d[5] = {label, TGO_MULTI, 0, 0, 0}, none_d[1] = {0};
    FakeArr fk = {(jsize)sz[0], keys}, feb = {(jsize)sz[0] + 1, eb}, fbb = {(jsize)sz[0] + 1, bb}, fby = {(jsize)sz[2], bytes};
    FakeArr flv = {(jsize)sz[1], lv}, types = {5, types_d}, none = {0, none_d};
    jlong h = JFN(create)(env, NULL, 0, 5, 4, 3);
    jint rc = ok && h ? JFN(loadRows)(env, NULL, h, ARR(&fk), ARR(&feb), ARR(&fbb), (jobject)(void*)&fby, ARR(&flv),
                                      ARR(&types), ARR(&none), TGO_SCOPE_IN_E, 1, ARR(&none), 0) : TGO_E_INVALID;
    check("loadRows (a worker's block)", rc == TGO_OK);
    jbyteArray id = JFN(exchangeRcclId)(env, NULL);
    jlong x = (rc == TGO_OK && id) ? JFN(exchangeRcclCreate)(env, NULL, 1, 0, id, 0) : 0;
    jlongArray part = x ? JFN(finishPartitionRows)(env, NULL, h, x, 1) : NULL;
    const jlong* p = part ? (const jlong*)((FakeArr*)(void*)part)->data : NULL;
    check("finishPartitionRows (world 1): {0, 256, 256, 256}", p && p[0] == 0 && p[1] == GN && p[2] == GN && p[3] == GN);
    tgo_options o;
    tgo_default_options(&o);
    o.hard_query_limit = 3;
    tgo_ctx* one = NULL;
    tgo_rows r = {sz[0], (const int64_t*)keys, (const int64_t*)eb, (const int64_t*)bb, bytes, (const int64_t*)lv};
    tgo_edge_type et;
    memset(&et, 0, sizeof et);
    et.type_id = label;
    et.multiplicity = TGO_MULTI;
    tgo_schema sc = {1, &et, 0, NULL};
    tgo_load_opts lo;
    memset(&lo, 0, sizeof lo);
    lo.scope = TGO_SCOPE_IN_E;
    lo.apply_cap = 1;
    int ref_ok = tgo_create(&o, &one) == TGO_OK && tgo_load_rows(one, &r, &sc, &lo) == TGO_OK && tgo_finish_load(one) == TGO_OK;
    tgo_stats s1;
    ref_ok = ref_ok && tgo_stats_get(one, &s1) == TGO_OK && s1.truncated_results == GN;
    check("one-GPU tgo_load_rows reference (every row cut)", ref_ok);
    if (p && p[0] == 0 && ref_ok) {
        static int64_t ref[GN];
        tgo_sssp_args sa;
        memset(&sa, 0, sizeof sa);
        sa.seed = 5; sa.seed_is_dense = 1; sa.max_depth = GN; sa.scope = TGO_SCOPE_IN_E; sa.mode = TGO_SSSP_DELTA;
        jlongArray d = JFN(partSsspRun)(env, NULL, h, x, 5, 0);
        int same = d != NULL && tgo_sssp(one, &sa, ref) == TGO_OK;
        for (int v = 0; same && v < GN; ++v) same = ((jlong*)((FakeArr*)(void*)d)->data)[v] == ref[v];
        check("rows partition: partSsspRun == tgo_sssp (cut rows, pushed pull entries)", same);
        tgo_pr_args pa;
        memset(&pa, 0, sizeof pa);
        pa.alpha = 0.85; pa.vertex_count = GN; pa.max_iterations = 9;
        static double pref[GN];
        jdoubleArray pp = JFN(partPageRankRun)(env, NULL, h, x, 0.85, GN, 9, 1);
        int close = pp != NULL && tgo_pagerank(one, &pa, pref) == TGO_OK;
        double l1 = 0;
        for (int v = 0; close && v < GN; ++v) l1 += fabs(((jdouble*)((FakeArr*)(void*)pp)->data)[v] - pref[v]);
        check("rows partition: partPageRankRun within 1e-12 L1 of tgo_pagerank", close && l1 <= 1e-12);
        jlongArray wm = JFN(partWeightMin)(env, NULL, h);
        check("partWeightMin (unweighted: {0, 0})", wm && ((jlong*)((FakeArr*)(void*)wm)->data)[0] == 0 &&
                                                      ((jlong*)((FakeArr*)(void*)wm)->data)[1] == 0);
    }
    if (x) JFN(exchangeDestroy)(env, NULL, x);
    if (h) JFN(destroy)(env, NULL, h);
    tgo_destroy(one);
    free(lv);
    free(bytes);
}

/* world 1 on a GPU: the Java multi-GPU calls through the shim against the one-GPU engine */
static void gpu_cases(JNIEnv* env) {
    const int m = graph_edges();
    FakeArr src = {m, g_src}, dst = {m, g_dst}, w = {m, g_w};
    jlong h = JFN(create)(env, NULL, 0, 5, 4, 100000);
    check("create (device 0)", h != 0);
    if (!h) return;
    jintArray lay = JFN(partLayout)(env, NULL, ARR(&src), ARR(&dst), GN, 0, GN, 4);
    check("partLayout (world 1)", lay != NULL);
    jint rc = JFN(loadPartition)(env, NULL, h, GN, 0, GN, ARR(&src), ARR(&dst), ARR(&w), TGO_SCOPE_IN_E, 1, lay);
    check("loadPartition (weighted inE, layout)", rc == TGO_OK);
    jbyteArray id = JFN(exchangeRcclId)(env, NULL);
    check("exchangeRcclId", id != NULL);
    jlong x = id ? JFN(exchangeRcclCreate)(env, NULL, 1, 0, id, 0) : 0;
    check("exchangeRcclCreate (world 1)", x != 0);
    /* the one-GPU engine on the same edges */
    tgo_options o;
    tgo_default_options(&o);
    tgo_ctx* one = NULL;
    int ok = tgo_create(&o, &one) == TGO_OK;
    tgo_edges e;
    memset(&e, 0, sizeof e);
    e.n = GN; e.m = m; e.src = (const int32_t*)g_src; e.dst = (const int32_t*)g_dst; e.weight = (const int32_t*)g_w;
    tgo_load_opts lo;
    memset(&lo, 0, sizeof lo);
    lo.scope = TGO_SCOPE_IN_E;
    lo.apply_cap = 1;
    ok = ok && tgo_load_edges(one, &e, &lo) == TGO_OK;
    check("one-GPU reference engine", ok);
    if (x && ok && rc == TGO_OK) {
        static int64_t ref[GN];
        tgo_sssp_args sa;
        memset(&sa, 0, sizeof sa);
        sa.seed = 5; sa.seed_is_dense = 1; sa.max_depth = GN; sa.scope = TGO_SCOPE_IN_E; sa.mode = TGO_SSSP_DELTA;
        jlongArray d = JFN(partSsspRun)(env, NULL, h, x, 5, 0);
        int same = d != NULL && tgo_sssp(one, &sa, ref) == TGO_OK;
        for (int v = 0; same && v < GN; ++v) same = ((jlong*)((FakeArr*)(void*)d)->data)[v] == ref[v];
        check("partSsspRun == tgo_sssp (delta, converged)", same);
        tgo_pr_args pa;
        memset(&pa, 0, sizeof pa);
        pa.alpha = 0.85; pa.vertex_count = GN; pa.max_iterations = 12;
        static double pref[GN];
        for (int mode = 0; mode < 2; ++mode) {
            jdoubleArray p = JFN(partPageRankRun)(env, NULL, h, x, 0.85, GN, 12, mode);
            int close = p != NULL && tgo_pagerank(one, &pa, pref) == TGO_OK;
            double l1 = 0;
            for (int v = 0; close && v < GN; ++v) l1 += fabs(((jdouble*)((FakeArr*)(void*)p)->data)[v] - pref[v]);
            printf("     pagerank mode %d L1 vs one GPU %.3g\n", mode, l1);
            check(mode ? "partPageRankRun (ghost) within 1e-12 L1 of tgo_pagerank"
                       : "partPageRankRun (all-gather) within 1e-12 L1 of tgo_pagerank", close && l1 <= 1e-12);
        }
    }
    if (x) JFN(exchangeDestroy)(env, NULL, x);
    JFN(destroy)(env, NULL, h);
    /* unweighted bothE: BFS and the multi-source sweep against tgo_bfs */
    h = JFN(create)(env, NULL, 0, 5, 4, 100000);
    lo.scope = TGO_SCOPE_BOTH_E;
    lo.apply_cap = 0;
    e.weight = NULL;
    tgo_ctx* oneb = NULL;
    ok = h != 0 && tgo_create(&o, &oneb) == TGO_OK && tgo_load_edges(oneb, &e, &lo) == TGO_OK &&
         JFN(loadPartition)(env, NULL, h, GN, 0, GN, ARR(&src), ARR(&dst), NULL, TGO_SCOPE_BOTH_E, 0, NULL) == TGO_OK;
    check("bothE partition + reference", ok);
    id = JFN(exchangeRcclId)(env, NULL);                   /* one unique id per communicator */
    x = (ok && id) ? JFN(exchangeRcclCreate)(env, NULL, 1, 0, id, 0) : 0;
    check("second exchange (a fresh id)", x != 0);
    if (ok && x) {
        static int64_t ref[GN];
        tgo_bfs_args ba;
        memset(&ba, 0, sizeof ba);
        ba.seed = 7; ba.seed_is_dense = 1; ba.max_depth = GN; ba.scope = TGO_SCOPE_BOTH_E;
        jlongArray d = JFN(partBfsRun)(env, NULL, h, x, 7, GN, 15.0, 18.0);
        int same = d != NULL && tgo_bfs(oneb, &ba, ref) == TGO_OK;
        for (int v = 0; same && v < GN; ++v) same = ((jlong*)((FakeArr*)(void*)d)->data)[v] == ref[v];
        check("partBfsRun == tgo_bfs", same);
        jlong sdv[3] = {7, 100, 200};
        FakeArr seeds = {3, sdv};
        jlongArray r = JFN(partMsbfsRun)(env, NULL, h, x, ARR(&seeds), GN, 12.0, 1 << 20);
        jlongArray lv = r ? JFN(partMsLevels)(env, NULL, h, 0) : NULL;
        same = r != NULL && lv != NULL && ((FakeArr*)(void*)r)->len == 7;
        for (int v = 0; same && v < GN; ++v) same = ((jlong*)((FakeArr*)(void*)lv)->data)[v] == ref[v];
        check("partMsbfsRun + partMsLevels(0) == tgo_bfs", same);
    }
    if (x) JFN(exchangeDestroy)(env, NULL, x);
    if (h) JFN(destroy)(env, NULL, h);
    tgo_destroy(one);
    tgo_destroy(oneb);
}
static void expect(const char* name, jint rc, jint want_rc, int want_calls) {
    const int ok = rc == want_rc && csr_calls == want_calls && !region_oob;
    printf("%s %s: rc=%d calls=%d\n", ok ? "ok  " : "FAIL", name, (int)rc, csr_calls);
    failures += !ok;
    csr_calls = 0;
    region_oob = 0;
}

int main(int argc, char** argv) {
    table.FindClass = find_class;
    table.ThrowNew = throw_new;
    table.NewStringUTF = new_string;
    table.NewByteArray = new_bytes;
    table.NewIntArray = new_ints;
    table.NewLongArray = new_longs;
    table.NewDoubleArray = new_doubles;
    table.GetDoubleArrayElements = get_doubles;
    table.ReleaseDoubleArrayElements = rel_doubles;
    table.GetByteArrayRegion = get_byte_region;
    table.SetByteArrayRegion = set_byte_region;
    table.SetLongArrayRegion = set_long_region;
    table.GetArrayLength = get_len;
    table.GetIntArrayElements = get_ints;
    table.GetLongArrayElements = get_longs;
    table.ReleaseIntArrayElements = rel_ints;
    table.ReleaseLongArrayElements = rel_longs;
    table.GetLongArrayRegion = long_region;
    table.GetDirectBufferAddress = direct_address;
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
    partition_cases(env);
    if (argc > 1 && strcmp(argv[1], "gpu") == 0) {
        gpu_cases(env);
        gpu_rows_case(env);
    }
    return failures;
}
