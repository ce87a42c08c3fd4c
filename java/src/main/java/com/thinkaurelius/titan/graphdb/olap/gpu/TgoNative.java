package com.thinkaurelius.titan.graphdb.olap.gpu;

import com.thinkaurelius.titan.core.TitanException;

import java.nio.ByteBuffer;

/**
 * JNI binding of the MI355X engine's C-ABI (include/titan_gpu_olap.h), implemented by
 * java/jni/titan_gpu_olap_jni.c over libtitan_gpu_olap.so.  Every call maps one C entry point;
 * a non-zero status becomes a TitanException carrying tgo_last_error(), which is how the
 * reference reports executor failures (FulgoraGraphComputer.java:165-174; the future of
 * submit() then fails with ExecutionException, OLAPTest.java:222-239).
 *
 * Handles are opaque tgo_ctx pointers.  A handle is used by one thread at a time (the ABI's
 * rule); CsrCollectingScanJob serialises its work-block flushes on the handle.
 */
public final class TgoNative {

    static {
        System.loadLibrary("titan_gpu_olap_jni");
    }

    private TgoNative() {}

    /* tgo_scope: MessageScope.Local(__::outE / __::inE / __::bothE) */
    public static final int SCOPE_OUT_E = 0, SCOPE_IN_E = 1, SCOPE_BOTH_E = 2;
    /* tgo_sssp_mode */
    public static final int SSSP_HOP_BOUNDED = 0, SSSP_DELTA = 1;
    /* tgo_multiplicity (core/Multiplicity.java:21-75) */
    public static final int MULTI = 0, SIMPLE = 1, MANY2ONE = 2, ONE2MANY = 3, ONE2ONE = 4;
    /* tgo_datatype */
    public static final int DT_BYTE = 1, DT_SHORT = 2, DT_INTEGER = 3, DT_LONG = 4, DT_FLOAT = 5, DT_DOUBLE = 6,
            DT_BOOLEAN = 7, DT_DATE = 8, DT_CHARACTER = 9, DT_STRING = 10;
    /** TGO_DIST_ABSENT: no DISTANCE property was set (the vertex was not reached). */
    public static final long DIST_ABSENT = Long.MIN_VALUE;

    /** tgo_default_options + tgo_create; returns 0 when no gfx950 device is usable (no CPU fallback). */
    public static native long create(int device, int partitionBits, int hostThreads, long hardQueryLimit);

    public static native void destroy(long ctx);

    public static native String lastError(long ctx);

    /**
     * tgo_load_rows: one work block of scanned rows in StaticArrayEntryList form
     * (StaticArrayEntryList.java:15-50).  {@code entryBytes} must be a direct buffer.
     * The schema is flattened: per edge label {typeId, multiplicity, sortOrder (0 ASC, 1 DESC),
     * nSortKey, sortKeyIds...,
     * nSignature, signatureIds...}; per property key {keyId, datatype}.
     */
    public static native int loadRows(long ctx, long[] rowKeys, long[] rowEntryBegin, long[] rowByteBegin,
                                      ByteBuffer entryBytes, long[] entryLimitValuePos, long[] edgeTypes,
                                      long[] propertyKeys, int scope, boolean applyCap, long[] labelIds,
                                      long weightKey);

    public static native int finishLoad(long ctx);

    /**
     * tgo_load_csr: rows already collected as CSR (row v = titanIds[v]; OUT entries
     * outIdx[outOff[v]..outOff[v+1]), IN entries inIdx[inOff[v]..inOff[v+1]) as dense indices;
     * weights null when weightKey == 0).  The rows as preloaded: no cap is applied again.
     */
    public static native int loadCsr(long ctx, long[] titanIds, long[] outOff, int[] outIdx, int[] outWeight,
                                     long[] inOff, int[] inIdx, int[] inWeight, int scope, long weightKey,
                                     boolean columnOrder);

    public static native long[] vertexIds(long ctx);

    /** tgo_bfs with the unit edge function; null on failure (see lastError). */
    public static native long[] bfs(long ctx, long seedId, int maxDepth, int scope);

    public static native long[] sssp(long ctx, long seedId, int maxDepth, int scope, int mode, long delta);

    public static native double[] pageRank(long ctx, double alpha, long vertexCount, int maxIterations);

    public static native int[] walkCount(long ctx, int length);

    /** tgo_stats_get: {ghostVertices, truncatedResults, skippedRows, iterations, loadMs, lastKernelMs}. */
    public static native double[] stats(long ctx);

    /** tgo_result_kind */
    public static final int RESULT_DISTANCE = 0, RESULT_PAGERANK = 1, RESULT_DEGREE = 2;
    /**
     * tgo_result_rows: the edgestore entries (single-cardinality property entries) of the last
     * program's compute keys, as {long[] rowKeys, long[] rowEntryBegin, long[] rowByteBegin,
     * long[] entryLimitValuePos, byte[] entryBytes}; null on error (see lastError).
     */
    public static native Object[] resultRows(long ctx, int kind, long[] keyIds, int[] datatypes, long relationIdBase);

    /* ---- multi-GPU (include/titan_gpu_olap_part.h; PartitionedRun): one ctx + one exchange per
     * GPU worker thread, the ranks' vertex ranges [lo, hi) of the global dense ids. ---- */

    /** tgo_part_layout: the degree-grouped ids of the owned vertices (int[hi - lo]); null on failure. */
    public static native int[] partLayout(int[] src, int[] dst, long nGlobal, long lo, long hi, int threads);

    /**
     * tgo_load_partition_layout: edges (dense global ids) holding every edge with an endpoint in
     * [lo, hi); weight null when unweighted; layoutGlobal null = ids as given, else every
     * worker's partLayout slice gathered (int[nGlobal]).
     */
    public static native int loadPartition(long ctx, long nGlobal, long lo, long hi, int[] src, int[] dst, int[] weight,
                                           int scope, boolean applyCap, int[] layoutGlobal);

    /**
     * tgo_finish_partition_rows (collective: every worker calls it after staging ITS rows with
     * {@link #loadRows}): {status, live rows here, slot size S, live rows of every worker}.  The
     * worker's results are the first "live" entries of the partSsspRun / partPageRankRun outputs,
     * whose ids are the first "live" of vertexIds; rank r's global ids are r * S + i.
     * status TGO_E_UNSUPPORTED: the graph has vertex cuts or a non-Integer weight key.
     */
    public static native long[] finishPartitionRows(long ctx, long exchange, boolean layout);

    /** tgo_part_weight_min: {status, smallest weight of this worker's load (0 unweighted)}. */
    public static native long[] partWeightMin(long ctx);

    /** tgo_status values the Java layer branches on. */
    public static final int E_INVALID = -1, E_UNSUPPORTED = -7;

    /** tgo_exchange_rccl_id: the 128-byte RCCL unique id (made once, shared by every worker). */
    public static native byte[] exchangeRcclId();

    /** tgo_exchange_rccl_create (collective: every rank calls it concurrently); 0 on failure. */
    public static native long exchangeRcclCreate(int world, int rank, byte[] id, int device);

    public static native void exchangeDestroy(long exchange);

    public static native String exchangeLastError(long exchange);

    /** tgo_part_bfs_run: the owned distances in row order; null on failure (see lastError). */
    public static native long[] partBfsRun(long ctx, long exchange, long seedGlobal, int maxDepth, double alpha,
                                           double beta);

    /** tgo_part_sssp_run (delta-stepping, converged distances): owned distances; null on failure. */
    public static native long[] partSsspRun(long ctx, long exchange, long seedGlobal, long delta);

    /** tgo_part_pagerank_run: owned ranks; null on failure.  exchangeMode 0 all-gather, 1 ghost. */
    public static native double[] partPageRankRun(long ctx, long exchange, double alpha, long vertexCount,
                                                  int maxIterations, int exchangeMode);

    /** tgo_part_msbfs_run: {levels, reached per seed..., entries per seed...} (global); null on failure. */
    public static native long[] partMsbfsRun(long ctx, long exchange, long[] seedsGlobal, int maxDepth, double msAlpha,
                                             long fixedExchangeBytes);

    /** tgo_part_ms_levels: source i's owned distances after partMsbfsRun; null on failure. */
    public static native long[] partMsLevels(long ctx, int source);

    /** A non-zero status of a C-ABI call as a TitanException carrying tgo_last_error(). */
    public static void check(long ctx, int rc) {
        if (rc != 0) throw new TitanException("[" + rc + "] " + lastError(ctx));
    }

    /** A null result of a C-ABI call (its status was non-zero) as a TitanException. */
    public static <T> T checked(long ctx, T result) {
        if (result == null) throw new TitanException(lastError(ctx));
        return result;
    }
}
