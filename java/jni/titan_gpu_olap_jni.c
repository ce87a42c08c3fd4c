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
