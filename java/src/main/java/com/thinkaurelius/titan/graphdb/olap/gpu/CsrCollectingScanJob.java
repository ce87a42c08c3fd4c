package com.thinkaurelius.titan.graphdb.olap.gpu;

import com.thinkaurelius.titan.diskstorage.Entry;
import com.thinkaurelius.titan.diskstorage.EntryList;
import com.thinkaurelius.titan.diskstorage.StaticBuffer;
import com.thinkaurelius.titan.diskstorage.configuration.Configuration;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.SliceQuery;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.scan.ScanJob;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.scan.ScanMetrics;
import com.thinkaurelius.titan.graphdb.database.idhandling.IDHandler;
import com.thinkaurelius.titan.graphdb.idmanagement.IDManager;
import com.thinkaurelius.titan.graphdb.internal.RelationCategory;
import com.thinkaurelius.titan.graphdb.olap.VertexJobConverter;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.List;
import java.util.Map;
import java.util.function.Predicate;

/**
 * The one edgestore scan of the GPU path: a {@link ScanJob} (ScanJob.java:17-130) run by the
 * unchanged StandardScanner (Backend.buildEdgeScanJob(), Backend.java:336-355) that collects
 * every row and hands it, in work blocks, to tgo_load_rows.  It replaces Fulgora's rescan of
 * the edgestore in every superstep (FulgoraGraphComputer.java:151-189).
 *
 * Queries: the grounded VertexExists slice first (the executor rejects a non-grounded first
 * query, StandardScannerExecutor.java:92-101; VertexJobConverter.java:39), then the whole
 * user-edge slice [0x60, 0x80) (IDHandler.getBounds(EDGE), IDHandler.java:158-179) WITHOUT a
 * limit: the device loader applies the QueryContainer cap of the program's scope itself
 * (QueryContainer.java:28,122) so that the truncated-results counter stays exact.  The row
 * key filter drops Invisible ids like VertexJobConverter.getKeyFilter (:156-162); ghosts and
 * vertex cuts are classified by the loader from the rows' first entries.
 *
 * Rows are appended as (key, entries) in StaticArrayEntryList form; each processor thread owns
 * a clone (StandardScannerExecutor clones the job per work block, :259-265) and flushes a
 * full block under the shared handle's monitor (a tgo_ctx is single-threaded).
 */
public class CsrCollectingScanJob implements ScanJob {

    /** FulgoraGraphComputer.readBatchSize default: 10 x storage.buffer-size (FulgoraGraphComputer.java:76-81). */
    public static final int DEFAULT_BLOCK_ROWS = 10 * 1024;

    private static final SliceQuery EDGE_SLICE = new SliceQuery(
            IDHandler.getBounds(RelationCategory.EDGE, false)[0],
            IDHandler.getBounds(RelationCategory.EDGE, false)[1]);

    private final Handle handle;
    private final int blockRows;

    // the current work block (per clone)
    private long[] keys, entryBegin, byteBegin, limitValuePos;
    private ByteBuffer bytes;
    private int rows, entries;

    /**
     * Where full blocks go instead of one ctx: the multi-GPU path keeps the scan's blocks and
     * hands each worker its row range ({@link PartitionedRun.RowBlocks}).  {@code bytes} holds
     * {@code byteCount} bytes from position 0 and is reused after the call: copy it.
     */
    public interface BlockSink {
        void accept(long[] keys, long[] entryBegin, long[] byteBegin, ByteBuffer bytes, int byteCount, long[] limitValuePos);
    }

    /** Shared by all clones: the native context and what every tgo_load_rows call needs. */
    public static final class Handle {
        final long ctx;
        final BlockSink sink;           // non-null: blocks go here, not to tgo_load_rows
        final IDManager idManager;
        final long[] edgeTypes, propertyKeys, labelIds;
        final int scope;
        final boolean applyCap;
        final long weightKey;
        // the first failed flush: a TitanException thrown from workerIterationEnd escapes a
        // processor's finally, where StandardScannerExecutor only logs it (:278-282) and counts
        // no FAILURE, so the submitting thread must check it before tgo_finish_load
        private volatile Throwable failure;

        /** Throws the first flush failure of any clone (sticky). */
        public void rethrowFailure() {
            Throwable f = failure;
            if (f != null) throw new com.thinkaurelius.titan.core.TitanException("a work block failed to load", f);
        }

        public Handle(long ctx, IDManager idManager, long[] edgeTypes, long[] propertyKeys, int scope,
                      boolean applyCap, long[] labelIds, long weightKey) {
            this(ctx, null, idManager, edgeTypes, propertyKeys, scope, applyCap, labelIds, weightKey);
        }

        public Handle(long ctx, BlockSink sink, IDManager idManager, long[] edgeTypes, long[] propertyKeys, int scope,
                      boolean applyCap, long[] labelIds, long weightKey) {
            this.ctx = ctx;
            this.sink = sink;
            this.idManager = idManager;
            this.edgeTypes = edgeTypes;
            this.propertyKeys = propertyKeys;
            this.scope = scope;
            this.applyCap = applyCap;
            this.labelIds = labelIds;
            this.weightKey = weightKey;
        }
    }

    public CsrCollectingScanJob(Handle handle) {
        this(handle, DEFAULT_BLOCK_ROWS);
    }

    public CsrCollectingScanJob(Handle handle, int blockRows) {
        this.handle = handle;
        this.blockRows = blockRows;
        reset();
    }

    private void reset() {
        keys = new long[blockRows];
        entryBegin = new long[blockRows + 1];
        byteBegin = new long[blockRows + 1];
        limitValuePos = new long[Math.max(1024, blockRows * 4)];
        if (bytes == null) bytes = ByteBuffer.allocateDirect(1 << 20).order(ByteOrder.BIG_ENDIAN);
        bytes.clear();
        rows = 0;
        entries = 0;
    }

    @Override
    public List<SliceQuery> getQueries() {
        List<SliceQuery> q = new ArrayList<>(2);
        q.add(VertexJobConverter.VERTEX_EXISTS_QUERY);
        q.add(EDGE_SLICE);
        return q;
    }

    @Override
    public Predicate<StaticBuffer> getKeyFilter() {
        // VertexJobConverter.getKeyFilter (:156-162): skip Invisible ids (schema rows etc.)
        return buffer -> !IDManager.VertexIDType.Invisible.is(handle.idManager.getKeyID(buffer));
    }

    @Override
    public void process(StaticBuffer key, Map<SliceQuery, EntryList> slices, ScanMetrics metrics) {
        EntryList exists = slices.get(VertexJobConverter.VERTEX_EXISTS_QUERY);
        EntryList edges = slices.get(EDGE_SLICE);
        int n = (exists == null ? 0 : exists.size()) + (edges == null ? 0 : edges.size());
        ensureEntries(n);
        keys[rows] = key.getLong(0);
        entryBegin[rows] = entries;
        byteBegin[rows] = bytes.position();
        int rowStart = bytes.position();
        // column order: the VertexExists entry (system property, 0x02...) precedes user edges
        if (exists != null) for (Entry e : exists) append(e, rowStart);
        if (edges != null) for (Entry e : edges) append(e, rowStart);
        rows++;
        entryBegin[rows] = entries;
        byteBegin[rows] = bytes.position();
        if (rows == blockRows) flush();
    }

    private void append(Entry e, int rowStart) {
        int len = e.length();
        ensureBytes(len);
        for (int i = 0; i < len; i++) bytes.put(e.getByte(i));
        long limit = bytes.position() - rowStart;           // StaticArrayEntryList: end offset in the row
        limitValuePos[entries++] = (limit << 32) | (e.getValuePosition() & 0xFFFFFFFFL);
    }

    private void ensureEntries(int more) {
        if (entries + more <= limitValuePos.length) return;
        long[] x = new long[Math.max(limitValuePos.length * 2, entries + more)];
        System.arraycopy(limitValuePos, 0, x, 0, entries);
        limitValuePos = x;
    }

    private void ensureBytes(int more) {
        if (bytes.remaining() >= more) return;
        ByteBuffer b = ByteBuffer.allocateDirect(Math.max(bytes.capacity() * 2, bytes.position() + more))
                .order(ByteOrder.BIG_ENDIAN);
        bytes.flip();
        b.put(bytes);
        bytes = b;
    }

    /** Hands the current block to tgo_load_rows (one native call per block, serialised per ctx). */
    public void flush() {
        if (rows == 0) return;
        long[] k = java.util.Arrays.copyOf(keys, rows);
        long[] eb = java.util.Arrays.copyOf(entryBegin, rows + 1);
        long[] bb = java.util.Arrays.copyOf(byteBegin, rows + 1);
        long[] lv = java.util.Arrays.copyOf(limitValuePos, Math.max(entries, 1));
        synchronized (handle) {
            try {
                if (handle.failure != null) return;       // the load is lost already: stop feeding it
                if (handle.sink != null) {
                    handle.sink.accept(k, eb, bb, bytes, (int) byteBegin[rows], lv);
                    return;
                }
                TgoNative.check(handle.ctx, TgoNative.loadRows(handle.ctx, k, eb, bb, bytes, lv, handle.edgeTypes,
                        handle.propertyKeys, handle.scope, handle.applyCap, handle.labelIds, handle.weightKey));
            } catch (RuntimeException e) {
                if (handle.failure == null) handle.failure = e;
                throw e;
            } finally {
                reset();
            }
        }
    }

    @Override
    public void workerIterationStart(Configuration jobConfiguration, Configuration graphConfiguration,
                                     ScanMetrics metrics) {
        reset();
    }

    @Override
    public void workerIterationEnd(ScanMetrics metrics) {
        flush();
    }

    @Override
    public CsrCollectingScanJob clone() {
        // every clone flushes its own block; the handle (native ctx) is shared
        return new CsrCollectingScanJob(handle, blockRows);
    }
}
