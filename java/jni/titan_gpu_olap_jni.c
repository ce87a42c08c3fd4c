/*
 * titan_gpu_olap_jni.c — JNI shim between TgoNative.java and the C-ABI of
 * libtitan_gpu_olap.so (include/titan_gpu_olap.h).  The only native glue of the Java host
 * layer: arrays are pinned for the duration of one call (the ABI never retains caller
 * buffers), the flattened schema is unpacked into tgo_schema, statuses come back as ints and
 * TgoNative.check() turns a failure into TitanException with tgo_last_error().
 *
 * Built only where a JDK is present (java/Makefile; this image has none).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "titan_gpu_olap.h"
#include "titan_gpu_olap_part.h"

#define JFN(name) Java_com_thinkaurelius_titan_graphdb_olap_gpu_TgoNative_##name
#define CTX(h) ((tgo_ctx*)(intptr_t)(h))

/* Java arrays are indexed by jsize (int32): a result larger than that cannot be handed back
 * as one array.  Raise IllegalStateException (pending on return) instead of truncating. */
static int fits_jsize(JNIEnv* env, int64_t n, const char* what) {
    if (n >= 0 && n <= INT32_MAX) return 1;
    jclass ex = (*env)->FindClass(env, "java/lang/IllegalStateException");
    if (ex) (*env)->ThrowNew(env, ex, what);
    return 0;
}

JNIEXPORT jlong JNICALL JFN(create)(JNIEnv* env, jclass cls, jint device, jint pb, jint threads, jlong limit) {
    (void)env; (void)cls;
    tgo_options o;
    tgo_default_options(&o);
    o.device = device;
    o.partition_bits = pb;
    o.host_threads = threads;
    o.hard_query_limit = limit;
    tgo_ctx* ctx = NULL;
    return tgo_create(&o, &ctx) == TGO_OK ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT void JNICALL JFN(destroy)(JNIEnv* env, jclass cls, jlong h) {
    (void)env; (void)cls;
    tgo_destroy(CTX(h));
}

JNIEXPORT jstring JNICALL JFN(lastError)(JNIEnv* env, jclass cls, jlong h) {
    (void)cls;
    return (*env)->NewStringUTF(env, h ? tgo_last_error(CTX(h)) : "tgo_create failed: no usable gfx950 device");
}

/* Flattened edge labels: {typeId, multiplicity, sortOrder, nSortKey, sortKeyIds..., nSignature, signatureIds...}*. */
static int unpack_schema(const jlong* et, jsize net, const jlong* pk, jsize npk, tgo_schema* s,
                         tgo_edge_type** types_out, tgo_property_key** keys_out) {
    int n = 0;
    for (jsize i = 0; i < net;) {
        if (i + 4 > net) return TGO_E_INVALID;
        jsize nsk = (jsize)et[i + 3];
        if (i + 4 + nsk + 1 > net) return TGO_E_INVALID;
        jsize nsig = (jsize)et[i + 4 + nsk];
        i += 4 + nsk + 1 + nsig;
        if (i > net) return TGO_E_INVALID;
        n++;
    }
    tgo_edge_type* t = (tgo_edge_type*)calloc((size_t)(n > 0 ? n : 1), sizeof(tgo_edge_type));
    tgo_property_key* k = (tgo_property_key*)calloc((size_t)(npk / 2 > 0 ? npk / 2 : 1), sizeof(tgo_property_key));
    if (!t || !k) { free(t); free(k); return TGO_E_OOM; }
    int j = 0;
    for (jsize i = 0; i < net; j++) {
        t[j].type_id = et[i];
        t[j].multiplicity = (int32_t)et[i + 1];
        t[j].sort_order = (int32_t)et[i + 2];
        t[j].n_sort_key = (int32_t)et[i + 3];
        t[j].sort_key_ids = (const int64_t*)&et[i + 4];
        jsize sig = i + 4 + t[j].n_sort_key;
        t[j].n_signature = (int32_t)et[sig];
        t[j].signature_ids = (const int64_t*)&et[sig + 1];
        i = sig + 1 + t[j].n_signature;
    }
    for (jsize i = 0; i + 1 < npk; i += 2) {
        k[i / 2].key_id = pk[i];
        k[i / 2].datatype = (int32_t)pk[i + 1];
    }
    s->n_edge_types = n;
    s->edge_types = t;
    s->n_property_keys = (int32_t)(npk / 2);
    s->property_keys = k;
    *types_out = t;
    *keys_out = k;
    return TGO_OK;
}

JNIEXPORT jint JNICALL JFN(loadRows)(JNIEnv* env, jclass cls, jlong h, jlongArray keys, jlongArray eb, jlongArray bb,
                                     jobject bytes, jlongArray lvp, jlongArray types, jlongArray pkeys, jint scope,
                                     jboolean apply_cap, jlongArray labels, jlong weight_key) {
    (void)cls;
    const uint8_t* data = (const uint8_t*)(*env)->GetDirectBufferAddress(env, bytes);
    if (!data) return TGO_E_INVALID;                       /* entryBytes must be a direct buffer */
    jlong* k = (*env)->GetLongArrayElements(env, keys, NULL);
    jlong* e = (*env)->GetLongArrayElements(env, eb, NULL);
    jlong* b = (*env)->GetLongArrayElements(env, bb, NULL);
    jlong* v = (*env)->GetLongArrayElements(env, lvp, NULL);
    jlong* et = (*env)->GetLongArrayElements(env, types, NULL);
    jlong* pk = (*env)->GetLongArrayElements(env, pkeys, NULL);
    jlong* lab = (*env)->GetLongArrayElements(env, labels, NULL);
    int rc = TGO_E_OOM;
    tgo_schema s;
    tgo_edge_type* t = NULL;
    tgo_property_key* pkk = NULL;
    if (k && e && b && v && et && pk && lab) {
        rc = unpack_schema(et, (*env)->GetArrayLength(env, types), pk, (*env)->GetArrayLength(env, pkeys), &s, &t, &pkk);
        if (rc == TGO_OK) {
            tgo_rows r;
            r.nrows = (*env)->GetArrayLength(env, keys);
            r.row_keys = (const int64_t*)k;
            r.row_entry_begin = (const int64_t*)e;
            r.row_byte_begin = (const int64_t*)b;
            r.entry_bytes = data;
            r.entry_limit_valpos = (const int64_t*)v;
            tgo_load_opts o;
            memset(&o, 0, sizeof o);
            o.scope = scope;
            o.apply_cap = apply_cap ? 1 : 0;
            o.n_labels = (int32_t)(*env)->GetArrayLength(env, labels);
            o.label_ids = o.n_labels ? (const int64_t*)lab : NULL;
            o.weight_key = weight_key;
            rc = tgo_load_rows(CTX(h), &r, &s, &o);
        }
    }
    free(t);
    free(pkk);
    if (k) (*env)->ReleaseLongArrayElements(env, keys, k, JNI_ABORT);
    if (e) (*env)->ReleaseLongArrayElements(env, eb, e, JNI_ABORT);
    if (b) (*env)->ReleaseLongArrayElements(env, bb, b, JNI_ABORT);
    if (v) (*env)->ReleaseLongArrayElements(env, lvp, v, JNI_ABORT);
    if (et) (*env)->ReleaseLongArrayElements(env, types, et, JNI_ABORT);
    if (pk) (*env)->ReleaseLongArrayElements(env, pkeys, pk, JNI_ABORT);
    if (lab) (*env)->ReleaseLongArrayElements(env, labels, lab, JNI_ABORT);
    return rc;
}

JNIEXPORT jint JNICALL JFN(finishLoad)(JNIEnv* env, jclass cls, jlong h) {
    (void)env; (void)cls;
    return tgo_finish_load(CTX(h));
}

/* tgo_load_csr: the rows a Java CSR collector already holds (dense neighbour indices); the
 * weight arrays may be null when weightKey == 0. */
JNIEXPORT jint JNICALL JFN(loadCsr)(JNIEnv* env, jclass cls, jlong h, jlongArray ids, jlongArray out_off,
                                    jintArray out_idx, jintArray out_w, jlongArray in_off, jintArray in_idx,
                                    jintArray in_w, jint scope, jlong weight_key, jboolean column_order) {
    (void)cls;
    if (!ids || !out_off || !in_off || !out_idx || !in_idx) return TGO_E_INVALID;
    const jsize n1 = (*env)->GetArrayLength(env, out_off);
    if (n1 < 1 || (*env)->GetArrayLength(env, in_off) != n1 || (*env)->GetArrayLength(env, ids) != n1 - 1)
        return TGO_E_INVALID;
    /* tgo_load_csr stages out_off[n] / in_off[n] entries from the pinned index (and weight)
     * arrays: arrays shorter than the offsets say would be read past their end */
    jlong ends[4];
    (*env)->GetLongArrayRegion(env, out_off, 0, 1, &ends[0]);
    (*env)->GetLongArrayRegion(env, out_off, n1 - 1, 1, &ends[1]);
    (*env)->GetLongArrayRegion(env, in_off, 0, 1, &ends[2]);
    (*env)->GetLongArrayRegion(env, in_off, n1 - 1, 1, &ends[3]);
    if (ends[0] != 0 || ends[2] != 0 || ends[1] < 0 || ends[3] < 0 ||
        ends[1] > (jlong)(*env)->GetArrayLength(env, out_idx) || ends[3] > (jlong)(*env)->GetArrayLength(env, in_idx))
        return TGO_E_INVALID;
    if (weight_key != 0 &&
        (!out_w || !in_w || ends[1] > (jlong)(*env)->GetArrayLength(env, out_w) ||
         ends[3] > (jlong)(*env)->GetArrayLength(env, in_w)))
        return TGO_E_INVALID;
    if (weight_key == 0) { out_w = NULL; in_w = NULL; }
    jlong* t = (*env)->GetLongArrayElements(env, ids, NULL);
    jlong* oo = (*env)->GetLongArrayElements(env, out_off, NULL);
    jlong* io = (*env)->GetLongArrayElements(env, in_off, NULL);
    jint* oi = (*env)->GetIntArrayElements(env, out_idx, NULL);
    jint* ii = (*env)->GetIntArrayElements(env, in_idx, NULL);
    jint* ow = out_w ? (*env)->GetIntArrayElements(env, out_w, NULL) : NULL;
    jint* iw = in_w ? (*env)->GetIntArrayElements(env, in_w, NULL) : NULL;
    int rc = TGO_E_OOM;
    if (t && oo && io && oi && ii && (!out_w || ow) && (!in_w || iw)) {
        tgo_load_opts o;
        memset(&o, 0, sizeof o);
        o.scope = scope;
        o.weight_key = weight_key;
        o.flags = column_order ? TGO_LOAD_COLUMN_ORDER : 0;
        rc = tgo_load_csr(CTX(h), (int64_t)(n1 - 1), (const int64_t*)t, (const int64_t*)oo, (const int32_t*)oi,
                          (const int32_t*)ow, (const int64_t*)io, (const int32_t*)ii, (const int32_t*)iw, &o);
    }
    if (t) (*env)->ReleaseLongArrayElements(env, ids, t, JNI_ABORT);
    if (oo) (*env)->ReleaseLongArrayElements(env, out_off, oo, JNI_ABORT);
    if (io) (*env)->ReleaseLongArrayElements(env, in_off, io, JNI_ABORT);
    if (oi) (*env)->ReleaseIntArrayElements(env, out_idx, oi, JNI_ABORT);
    if (ii) (*env)->ReleaseIntArrayElements(env, in_idx, ii, JNI_ABORT);
    if (ow) (*env)->ReleaseIntArrayElements(env, out_w, ow, JNI_ABORT);
    if (iw) (*env)->ReleaseIntArrayElements(env, in_w, iw, JNI_ABORT);
    return rc;
}

JNIEXPORT jlongArray JNICALL JFN(vertexIds)(JNIEnv* env, jclass cls, jlong h) {
    (void)cls;
    if (!fits_jsize(env, tgo_num_vertices(CTX(h)), "more vertices than a Java array holds")) return NULL;
    jsize n = (jsize)tgo_num_vertices(CTX(h));
    jlongArray out = (*env)->NewLongArray(env, n);
    if (!out) return NULL;
    jlong* p = (*env)->GetLongArrayElements(env, out, NULL);
    int rc = tgo_vertex_ids(CTX(h), (int64_t*)p);
    (*env)->ReleaseLongArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}

static jlongArray distances(JNIEnv* env, jlong h, int (*run)(tgo_ctx*, const void*, int64_t*), const void* args) {
    if (!fits_jsize(env, tgo_num_vertices(CTX(h)), "more vertices than a Java array holds")) return NULL;
    jsize n = (jsize)tgo_num_vertices(CTX(h));
    jlongArray out = (*env)->NewLongArray(env, n);
    if (!out) return NULL;
    jlong* p = (*env)->GetLongArrayElements(env, out, NULL);
    int rc = run(CTX(h), args, (int64_t*)p);
    (*env)->ReleaseLongArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}
static int run_bfs(tgo_ctx* c, const void* a, int64_t* o) { return tgo_bfs(c, (const tgo_bfs_args*)a, o); }
static int run_sssp(tgo_ctx* c, const void* a, int64_t* o) { return tgo_sssp(c, (const tgo_sssp_args*)a, o); }

JNIEXPORT jlongArray JNICALL JFN(bfs)(JNIEnv* env, jclass cls, jlong h, jlong seed, jint max_depth, jint scope) {
    (void)cls;
    tgo_bfs_args a;
    memset(&a, 0, sizeof a);
    a.seed = seed;
    a.max_depth = max_depth;
    a.scope = scope;
    return distances(env, h, run_bfs, &a);
}

JNIEXPORT jlongArray JNICALL JFN(sssp)(JNIEnv* env, jclass cls, jlong h, jlong seed, jint max_depth, jint scope,
                                       jint mode, jlong delta) {
    (void)cls;
    tgo_sssp_args a;
    memset(&a, 0, sizeof a);
    a.seed = seed;
    a.max_depth = max_depth;
    a.scope = scope;
    a.mode = mode;
    a.delta = delta;
    return distances(env, h, run_sssp, &a);
}

JNIEXPORT jdoubleArray JNICALL JFN(pageRank)(JNIEnv* env, jclass cls, jlong h, jdouble alpha, jlong vertex_count,
                                             jint iterations) {
    (void)cls;
    if (!fits_jsize(env, tgo_num_vertices(CTX(h)), "more vertices than a Java array holds")) return NULL;
    jsize n = (jsize)tgo_num_vertices(CTX(h));
    jdoubleArray out = (*env)->NewDoubleArray(env, n);
    if (!out) return NULL;
    jdouble* p = (*env)->GetDoubleArrayElements(env, out, NULL);
    tgo_pr_args a;
    memset(&a, 0, sizeof a);
    a.alpha = alpha;
    a.vertex_count = vertex_count;
    a.max_iterations = iterations;
    int rc = tgo_pagerank(CTX(h), &a, (double*)p);
    (*env)->ReleaseDoubleArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}

JNIEXPORT jintArray JNICALL JFN(walkCount)(JNIEnv* env, jclass cls, jlong h, jint length) {
    (void)cls;
    if (!fits_jsize(env, tgo_num_vertices(CTX(h)), "more vertices than a Java array holds")) return NULL;
    jsize n = (jsize)tgo_num_vertices(CTX(h));
    jintArray out = (*env)->NewIntArray(env, n);
    if (!out) return NULL;
    jint* p = (*env)->GetIntArrayElements(env, out, NULL);
    int rc = tgo_walkcount(CTX(h), length, (int32_t*)p);
    (*env)->ReleaseIntArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}

/* tgo_result_rows: Object[5] = {long[] rowKeys, long[] rowEntryBegin, long[] rowByteBegin,
 * long[] entryLimitValuePos, byte[] entryBytes}, or NULL on error (status: lastError; a result
 * beyond the int32 index range of a Java array: IllegalStateException). */
JNIEXPORT jobjectArray JNICALL JFN(resultRows)(JNIEnv* env, jclass cls, jlong h, jint kind, jlongArray jkeys,
                                              jintArray jtypes, jlong relationIdBase) {
    (void)cls;
    tgo_result_args a;
    memset(&a, 0, sizeof a);
    a.kind = kind;
    a.relation_id_base = relationIdBase;
    jsize nk = (*env)->GetArrayLength(env, jkeys);
    if (nk < 1 || nk > 2 || (*env)->GetArrayLength(env, jtypes) != nk) return NULL;
    (*env)->GetLongArrayRegion(env, jkeys, 0, nk, (jlong*)a.key_ids);
    (*env)->GetIntArrayRegion(env, jtypes, 0, nk, (jint*)a.datatypes);
    tgo_result_size sz;
    memset(&sz, 0, sizeof sz);
    if (tgo_result_rows(CTX(h), &a, &sz, NULL) != TGO_OK) return NULL;
    if (!fits_jsize(env, sz.nrows + 1, "result rows exceed a Java array") ||
        !fits_jsize(env, sz.nentries, "result entries exceed a Java array") ||
        !fits_jsize(env, sz.nbytes, "result bytes exceed a Java array (write back in smaller batches)"))
        return NULL;
    int64_t* keys = (int64_t*)malloc((size_t)(sz.nrows + 1) * 8);
    int64_t* eb = (int64_t*)malloc((size_t)(sz.nrows + 1) * 8);
    int64_t* bb = (int64_t*)malloc((size_t)(sz.nrows + 1) * 8);
    int64_t* lv = (int64_t*)malloc((size_t)(sz.nentries + 1) * 8);
    uint8_t* bytes = (uint8_t*)malloc((size_t)(sz.nbytes + 1));
    jobjectArray out = NULL;
    tgo_rows_buf buf = {keys, eb, bb, bytes, lv};
    if (keys && eb && bb && lv && bytes && tgo_result_rows(CTX(h), &a, &sz, &buf) == TGO_OK) {
        jclass la = (*env)->FindClass(env, "java/lang/Object");
        out = (*env)->NewObjectArray(env, 5, la, NULL);
        const int64_t* parts[4] = {keys, eb, bb, lv};
        const jsize lens[4] = {(jsize)sz.nrows, (jsize)sz.nrows + 1, (jsize)sz.nrows + 1, (jsize)sz.nentries};
        for (int i = 0; out && i < 4; ++i) {
            jlongArray arr = (*env)->NewLongArray(env, lens[i]);
            if (!arr) { out = NULL; break; }
            (*env)->SetLongArrayRegion(env, arr, 0, lens[i], (const jlong*)parts[i]);
            (*env)->SetObjectArrayElement(env, out, i, arr);
        }
        if (out) {
            jbyteArray data = (*env)->NewByteArray(env, (jsize)sz.nbytes);
            if (!data) {
                out = NULL;                                  /* OutOfMemoryError is pending */
            } else {
                (*env)->SetByteArrayRegion(env, data, 0, (jsize)sz.nbytes, (const jbyte*)bytes);
                (*env)->SetObjectArrayElement(env, out, 4, data);
            }
        }
    }
    free(keys); free(eb); free(bb); free(lv); free(bytes);
    return out;
}

JNIEXPORT jdoubleArray JNICALL JFN(stats)(JNIEnv* env, jclass cls, jlong h) {
    (void)cls;
    tgo_stats st;
    if (tgo_stats_get(CTX(h), &st) != TGO_OK) return NULL;
    jdouble v[6] = {(jdouble)st.ghost_vertices, (jdouble)st.truncated_results, (jdouble)st.skipped_rows,
                    (jdouble)st.iterations, st.load_ms, st.last_kernel_ms};
    jdoubleArray out = (*env)->NewDoubleArray(env, 6);
    if (out) (*env)->SetDoubleArrayRegion(env, out, 0, 6, v);
    return out;
}

/* ---- multi-GPU (include/titan_gpu_olap_part.h): one ctx + one exchange per GPU worker ----
 * GpuGraphComputer.devices(...) runs one worker thread per device in the JVM; every worker
 * loads its 1-D vertex range [lo, hi) of the global dense ids from an edge list that holds
 * every edge with an endpoint in the range, and the program runs as ONE native call per
 * worker whose collectives go over its RCCL communicator (tgo_exchange_rccl_*). */
#define XCH(h) ((tgo_exchange*)(intptr_t)(h))

/* edge arrays: src / dst (and weight, may be null) of equal length m */
static int edge_lengths(JNIEnv* env, jintArray src, jintArray dst, jintArray w, jsize* m) {
    if (!src || !dst) return TGO_E_INVALID;
    *m = (*env)->GetArrayLength(env, src);
    if ((*env)->GetArrayLength(env, dst) != *m) return TGO_E_INVALID;
    if (w && (*env)->GetArrayLength(env, w) != *m) return TGO_E_INVALID;
    return TGO_OK;
}

/* tgo_part_layout: the degree-grouped ids of the owned vertices [lo, hi) (int[hi - lo]) or
 * null on failure; every worker's slice goes into one layoutGlobal array (n_global). */
JNIEXPORT jintArray JNICALL JFN(partLayout)(JNIEnv* env, jclass cls, jintArray src, jintArray dst, jlong n_global,
                                            jlong lo, jlong hi, jint threads) {
    (void)cls;
    jsize m = 0;
    if (edge_lengths(env, src, dst, NULL, &m) != TGO_OK || lo < 0 || hi <= lo || hi > n_global) return NULL;
    if (!fits_jsize(env, hi - lo, "a partition larger than a Java array holds")) return NULL;
    jintArray out = (*env)->NewIntArray(env, (jsize)(hi - lo));
    if (!out) return NULL;
    jint* s = (*env)->GetIntArrayElements(env, src, NULL);
    jint* d = (*env)->GetIntArrayElements(env, dst, NULL);
    jint* o = (*env)->GetIntArrayElements(env, out, NULL);
    int rc = TGO_E_OOM;
    if (s && d && o) {
        tgo_edges e;
        memset(&e, 0, sizeof e);
        e.n = n_global;
        e.m = m;
        e.src = (const int32_t*)s;
        e.dst = (const int32_t*)d;
        rc = tgo_part_layout(&e, n_global, lo, hi, threads, (int32_t*)o);
    }
    if (s) (*env)->ReleaseIntArrayElements(env, src, s, JNI_ABORT);
    if (d) (*env)->ReleaseIntArrayElements(env, dst, d, JNI_ABORT);
    if (o) (*env)->ReleaseIntArrayElements(env, out, o, 0);
    return rc == TGO_OK ? out : NULL;
}

/* tgo_load_partition(_layout): weight may be null (unweighted); layoutGlobal null = the
 * caller's ids as they are, else int[n_global] (every worker the same array). */
JNIEXPORT jint JNICALL JFN(loadPartition)(JNIEnv* env, jclass cls, jlong h, jlong n_global, jlong lo, jlong hi,
                                          jintArray src, jintArray dst, jintArray weight, jint scope, jboolean apply_cap,
                                          jintArray layout_global) {
    (void)cls;
    jsize m = 0;
    if (edge_lengths(env, src, dst, weight, &m) != TGO_OK || lo < 0 || hi <= lo || hi > n_global) return TGO_E_INVALID;
    if (layout_global && (jlong)(*env)->GetArrayLength(env, layout_global) != n_global) return TGO_E_INVALID;
    jint* s = (*env)->GetIntArrayElements(env, src, NULL);
    jint* d = (*env)->GetIntArrayElements(env, dst, NULL);
    jint* w = weight ? (*env)->GetIntArrayElements(env, weight, NULL) : NULL;
    jint* lg = layout_global ? (*env)->GetIntArrayElements(env, layout_global, NULL) : NULL;
    int rc = TGO_E_OOM;
    if (s && d && (!weight || w) && (!layout_global || lg)) {
        tgo_edges e;
        memset(&e, 0, sizeof e);
        e.n = n_global;
        e.m = m;
        e.src = (const int32_t*)s;
        e.dst = (const int32_t*)d;
        e.weight = (const int32_t*)w;
        tgo_load_opts o;
        memset(&o, 0, sizeof o);
        o.scope = scope;
        o.apply_cap = apply_cap ? 1 : 0;
        rc = tgo_load_partition_layout(CTX(h), n_global, lo, hi, &e, &o, (const int32_t*)lg);
    }
    if (s) (*env)->ReleaseIntArrayElements(env, src, s, JNI_ABORT);
    if (d) (*env)->ReleaseIntArrayElements(env, dst, d, JNI_ABORT);
    if (w) (*env)->ReleaseIntArrayElements(env, weight, w, JNI_ABORT);
    if (lg) (*env)->ReleaseIntArrayElements(env, layout_global, lg, JNI_ABORT);
    return rc;
}

/* tgo_exchange_rccl_id: the 128-byte RCCL unique id (worker 0 makes it, every worker of the
 * JVM creates its communicator from the same bytes), null on failure. */
JNIEXPORT jbyteArray JNICALL JFN(exchangeRcclId)(JNIEnv* env, jclass cls) {
    (void)cls;
    uint8_t id[128];
    if (tgo_exchange_rccl_id(id) != TGO_OK) return NULL;
    jbyteArray out = (*env)->NewByteArray(env, 128);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, 128, (const jbyte*)id);
    return out;
}

/* tgo_exchange_rccl_create: 0 on failure.  Every rank of `world` must call it concurrently
 * (one thread per device): RCCL's communicator set-up is collective. */
JNIEXPORT jlong JNICALL JFN(exchangeRcclCreate)(JNIEnv* env, jclass cls, jint world, jint rank, jbyteArray id,
                                                jint device) {
    (void)cls;
    if (!id || (*env)->GetArrayLength(env, id) != 128 || world < 1 || rank < 0 || rank >= world) return 0;
    uint8_t b[128];
    (*env)->GetByteArrayRegion(env, id, 0, 128, (jbyte*)b);
    tgo_exchange* x = NULL;
    return tgo_exchange_rccl_create(world, rank, b, device, &x) == TGO_OK ? (jlong)(intptr_t)x : 0;
}

JNIEXPORT void JNICALL JFN(exchangeDestroy)(JNIEnv* env, jclass cls, jlong x) {
    (void)env; (void)cls;
    if (x) tgo_exchange_destroy(XCH(x));
}

JNIEXPORT jstring JNICALL JFN(exchangeLastError)(JNIEnv* env, jclass cls, jlong x) {
    (void)cls;
    return (*env)->NewStringUTF(env, x ? tgo_exchange_last_error(XCH(x)) : "no exchange");
}

/* The partitioned programs as one call each; outputs are the owned vertices in row order
 * (n_local = tgo_num_vertices of the partition ctx), null on failure (see lastError). */
static jsize owned(JNIEnv* env, jlong h) {
    const int64_t n = tgo_num_vertices(CTX(h));
    return fits_jsize(env, n, "a partition larger than a Java array holds") ? (jsize)n : -1;
}

JNIEXPORT jlongArray JNICALL JFN(partBfsRun)(JNIEnv* env, jclass cls, jlong h, jlong x, jlong seed, jint max_depth,
                                             jdouble alpha, jdouble beta) {
    (void)cls;
    if (!h || !x) return NULL;                            /* validated before the ctx is touched */
    const jsize n = owned(env, h);
    if (n < 0) return NULL;
    jlongArray out = (*env)->NewLongArray(env, n);
    if (!out) return NULL;
    jlong* p = (*env)->GetLongArrayElements(env, out, NULL);
    int32_t levels = 0;
    const int rc = p ? tgo_part_bfs_run(CTX(h), XCH(x), seed, max_depth, alpha, beta, (int64_t*)p, NULL, &levels) : TGO_E_OOM;
    if (p) (*env)->ReleaseLongArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}

JNIEXPORT jlongArray JNICALL JFN(partSsspRun)(JNIEnv* env, jclass cls, jlong h, jlong x, jlong seed, jlong delta) {
    (void)cls;
    if (!h || !x) return NULL;                            /* validated before the ctx is touched */
    const jsize n = owned(env, h);
    if (n < 0) return NULL;
    jlongArray out = (*env)->NewLongArray(env, n);
    if (!out) return NULL;
    jlong* p = (*env)->GetLongArrayElements(env, out, NULL);
    int32_t phases = 0;
    const int rc = p ? tgo_part_sssp_run(CTX(h), XCH(x), seed, delta, (int64_t*)p, NULL, &phases) : TGO_E_OOM;
    if (p) (*env)->ReleaseLongArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}

JNIEXPORT jdoubleArray JNICALL JFN(partPageRankRun)(JNIEnv* env, jclass cls, jlong h, jlong x, jdouble alpha,
                                                    jlong vertex_count, jint iterations, jint exchange_mode) {
    (void)cls;
    if (!h || !x) return NULL;                            /* validated before the ctx is touched */
    const jsize n = owned(env, h);
    if (n < 0) return NULL;
    jdoubleArray out = (*env)->NewDoubleArray(env, n);
    if (!out) return NULL;
    jdouble* p = (*env)->GetDoubleArrayElements(env, out, NULL);
    tgo_pr_args a;
    memset(&a, 0, sizeof a);
    a.alpha = alpha;
    a.vertex_count = vertex_count;
    a.max_iterations = iterations;
    int64_t moved = 0;
    const int rc = p ? tgo_part_pagerank_run(CTX(h), XCH(x), &a, exchange_mode, (double*)p, &moved) : TGO_E_OOM;
    if (p) (*env)->ReleaseDoubleArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}

/* tgo_part_msbfs_run: long[1 + 2 * nseeds] = {levels, reached per seed..., entries per seed...}
 * (global counts), null on failure; the owned levels of source i then come from partMsLevels. */
JNIEXPORT jlongArray JNICALL JFN(partMsbfsRun)(JNIEnv* env, jclass cls, jlong h, jlong x, jlongArray seeds,
                                               jint max_depth, jdouble ms_alpha, jlong fixed_bytes) {
    (void)cls;
    if (!seeds || !x) return NULL;
    const jsize ns = (*env)->GetArrayLength(env, seeds);
    if (ns < 1 || ns > 64) return NULL;
    jlong sd[64], re[64], en[64];
    (*env)->GetLongArrayRegion(env, seeds, 0, ns, sd);
    int32_t levels = 0;
    if (tgo_part_msbfs_run(CTX(h), XCH(x), (const int64_t*)sd, ns, max_depth, ms_alpha, fixed_bytes, (int64_t*)re,
                           (int64_t*)en, &levels) != TGO_OK)
        return NULL;
    jlongArray out = (*env)->NewLongArray(env, 1 + 2 * ns);
    if (!out) return NULL;
    const jlong lv = levels;
    (*env)->SetLongArrayRegion(env, out, 0, 1, &lv);
    (*env)->SetLongArrayRegion(env, out, 1, ns, re);
    (*env)->SetLongArrayRegion(env, out, 1 + ns, ns, en);
    return out;
}

JNIEXPORT jlongArray JNICALL JFN(partMsLevels)(JNIEnv* env, jclass cls, jlong h, jint source) {
    (void)cls;
    const jsize n = owned(env, h);
    if (n < 0) return NULL;
    jlongArray out = (*env)->NewLongArray(env, n);
    if (!out) return NULL;
    jlong* p = (*env)->GetLongArrayElements(env, out, NULL);
    const int rc = p ? tgo_part_ms_levels(CTX(h), source, (int64_t*)p) : TGO_E_OOM;
    if (p) (*env)->ReleaseLongArrayElements(env, out, p, 0);
    return rc == TGO_OK ? out : NULL;
}

/* tgo_finish_partition_rows after this worker's loadRows blocks (collective over the exchange):
 * long[4] = {status, live rows here, slot size S, live rows of every worker}; the status is
 * returned rather than thrown so that the caller can tell TGO_E_UNSUPPORTED (vertex cuts, a
 * non-Integer weight key: the graph runs on one device) from a failure.  null only without
 * memory for the array. */
JNIEXPORT jlongArray JNICALL JFN(finishPartitionRows)(JNIEnv* env, jclass cls, jlong h, jlong x, jboolean layout) {
    (void)cls;
    jlong out[4] = {TGO_E_INVALID, 0, 0, 0};
    if (h && x) {
        int64_t part[3] = {0, 0, 0};
        out[0] = tgo_finish_partition_rows(CTX(h), XCH(x), layout ? 1 : 0, part);
        out[1] = part[0]; out[2] = part[1]; out[3] = part[2];
    }
    jlongArray a = (*env)->NewLongArray(env, 4);
    if (a) (*env)->SetLongArrayRegion(env, a, 0, 4, out);
    return a;
}

/* tgo_part_weight_min: long[2] = {status, smallest weight of this worker's load (0 unweighted)}. */
JNIEXPORT jlongArray JNICALL JFN(partWeightMin)(JNIEnv* env, jclass cls, jlong h) {
    (void)cls;
    int64_t w = 0;
    jlong out[2] = {h ? tgo_part_weight_min(CTX(h), &w) : TGO_E_INVALID, 0};
    out[1] = w;
    jlongArray a = (*env)->NewLongArray(env, 2);
    if (a) (*env)->SetLongArrayRegion(env, a, 0, 2, out);
    return a;
}
