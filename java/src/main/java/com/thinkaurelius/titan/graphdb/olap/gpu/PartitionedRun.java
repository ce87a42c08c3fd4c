package com.thinkaurelius.titan.graphdb.olap.gpu;

import com.thinkaurelius.titan.core.TitanException;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.CyclicBarrier;
import java.util.concurrent.ExecutorService;
import java.util.concurrent.Executors;
import java.util.concurrent.Future;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.atomic.AtomicBoolean;

/**
 * The multi-GPU form of the GPU path ({@code GpuGraphComputer.devices(...)}): the graph is
 * 1-D vertex-partitioned over the node's GPUs (include/titan_gpu_olap_part.h), one worker
 * thread per device inside this JVM, each with its own tgo_ctx and RCCL communicator.  The
 * reference has no multi-device executor (Fulgora is one JVM, FulgoraGraphComputer.java:117-311);
 * the job API in front of it is unchanged (TitanGraphComputer.java:8-43).
 *
 * <ol>
 * <li>ONE edgestore scan: the single-device path's {@link CsrCollectingScanJob} with a
 *     {@link RowBlocks} sink, so the rows stay raw (StaticArrayEntryList form) and in scan
 *     order, in work blocks.</li>
 * <li>A Titan row holds its vertex's OUT and IN entries, so the 1-D vertex partition is a
 *     row-range partition of the scan: worker r takes a contiguous range of blocks, balanced
 *     by rows + entries ({@link #blockRanges}; titan_amd/distributed.py balanced_row_ranges is
 *     the same rule over rows, and tests/test_java_partition.py pins this one).</li>
 * <li>Worker r stages its blocks with tgo_load_rows (exactly the single-device decode: key
 *     filter, ghosts, typed scopes, and the QueryContainer cap per row in column order,
 *     QueryContainer.java:28,122 / ColumnValueStore.java:47-69), joins the RCCL exchange, and
 *     finishes with tgo_finish_partition_rows (collective: global ids, layout, the push rows of
 *     a cut scope); then the program as ONE native call (tgo_part_pagerank_run /
 *     tgo_part_sssp_run); its results are its live rows' values, ids from tgo_vertex_ids.</li>
 * </ol>
 * Graphs the partitioned programs do not cover — vertex cuts (they fold into the canonical
 * vertex on one device, VertexProgramScanJob.java:76-92), a non-Integer weight key, a negative
 * weight for delta-stepping, a ShortestDistance depth that can cut a path, no vertex at all —
 * raise {@link NotPartitionable} on every worker together; the caller then runs the single-
 * device path on the same {@link RowBlocks} (no second scan).  A worker that fails before the
 * exchange exists breaks the phase barrier, so the others stop too; the native calls after it
 * agree on failure among themselves; the job's future fails after {@link #RUN_TIMEOUT_MINUTES}
 * if a peer still stays blocked in a collective (RCCL does not notify peers of an aborted
 * communicator).
 */
public final class PartitionedRun {

    public static final int RUN_TIMEOUT_MINUTES = 60;
    /** titan_gpu_olap_part.h tgo_part_pagerank_run exchange modes */
    public static final int PR_EXCHANGE_ALLGATHER = 0, PR_EXCHANGE_GHOST = 1;

    private PartitionedRun() {}

    /** What a program runs on each worker: the native call over the loaded partition. */
    public interface Program {
        int scope();
        boolean applyCap();
        /** Whether the program has a partitioned form for a job of n live vertices (ShortestDistance:
         *  only when its depth cannot cut a path). */
        boolean partitions(long n);
        /** Whether it needs non-negative weights (delta-stepping). */
        boolean needsNonNegativeWeights();
        /** The worker's results (long[] or double[], at least ownIds.length entries, row order):
         *  ownIds = this worker's live vertex ids in row order, lo = the global id of the first. */
        Object run(long ctx, long exchange, long[] ownIds, long lo);
    }

    /** The graph cannot run partitioned; every worker raised it, the caller runs one device. */
    public static final class NotPartitionable extends TitanException {
        public NotPartitionable(String why) { super(why); }
    }

    // ------------------------------------------------------------------ the scanned rows
    /** One work block of the scan, copied out of the collector. */
    static final class Block {
        final long[] keys, entryBegin, byteBegin, limitValuePos;
        final ByteBuffer bytes;
        Block(long[] keys, long[] entryBegin, long[] byteBegin, ByteBuffer bytes, long[] limitValuePos) {
            this.keys = keys; this.entryBegin = entryBegin; this.byteBegin = byteBegin; this.bytes = bytes;
            this.limitValuePos = limitValuePos;
        }
        /** rows + entries: the balance weight of the block */
        long weight() { return keys.length + entryBegin[keys.length]; }
    }

    /** The scan's blocks in arrival order (a {@link CsrCollectingScanJob.BlockSink}). */
    public static final class RowBlocks implements CsrCollectingScanJob.BlockSink {
        final List<Block> blocks = new ArrayList<>();
        long rows = 0;

        @Override
        public synchronized void accept(long[] keys, long[] entryBegin, long[] byteBegin, ByteBuffer bytes, int byteCount,
                                        long[] limitValuePos) {
            ByteBuffer b = ByteBuffer.allocateDirect(Math.max(byteCount, 1)).order(ByteOrder.BIG_ENDIAN);
            ByteBuffer src = bytes.duplicate();
            src.position(0);
            src.limit(byteCount);
            b.put(src);
            b.flip();
            blocks.add(new Block(keys, entryBegin, byteBegin, b, limitValuePos));
            rows += keys.length;
        }

        public long rows() { return rows; }

        /** Stages blocks [from, to) into one ctx with tgo_load_rows (a worker, or the single-
         *  device fallback before tgo_finish_load). */
        public void loadInto(long ctx, CsrCollectingScanJob.Handle h, int from, int to) {
            for (int i = from; i < to; i++) {
                Block b = blocks.get(i);
                TgoNative.check(ctx, TgoNative.loadRows(ctx, b.keys, b.entryBegin, b.byteBegin, b.bytes, b.limitValuePos,
                        h.edgeTypes, h.propertyKeys, h.scope, h.applyCap, h.labelIds, h.weightKey));
            }
        }

        public void loadInto(long ctx, CsrCollectingScanJob.Handle h) { loadInto(ctx, h, 0, blocks.size()); }
    }

    /**
     * Contiguous block ranges for `world` workers balanced by rows + entries: range r ends at the
     * first block boundary whose prefix weight reaches ceil(total * (r + 1) / world); returns
     * world + 1 cut points (cut[r] .. cut[r + 1] is worker r's range, possibly empty).
     */
    static int[] blockRanges(long[] weights, int world) {
        final int nb = weights.length;
        long[] prefix = new long[nb + 1];
        for (int i = 0; i < nb; i++) prefix[i + 1] = prefix[i] + weights[i];
        final long total = prefix[nb];
        int[] cut = new int[world + 1];
        for (int r = 1; r < world; r++) {
            final long target = (total * r + world - 1) / world;
            int lo = 0, hi = nb;                 // the first boundary with prefix >= target
            while (lo < hi) {
                int mid = (lo + hi) >>> 1;
                if (prefix[mid] < target) lo = mid + 1; else hi = mid;
            }
            cut[r] = Math.max(cut[r - 1], Math.min(nb, lo));
        }
        cut[world] = nb;
        return cut;
    }

    // ------------------------------------------------------------------ partition + run
    /**
     * Runs `program` over the scanned rows on `devices` (one worker each).  Returns the live
     * vertices' Titan ids (worker-major row order) and the program's results in that order.
     */
    public static Object[] run(RowBlocks rows, CsrCollectingScanJob.Handle schema, Program program, int[] devices,
                               int partitionBits, int hostThreads, long hardQueryLimit) throws Exception {
        final int world = devices.length;
        long[] w = new long[rows.blocks.size()];
        for (int i = 0; i < w.length; i++) w[i] = rows.blocks.get(i).weight();
        final int[] cut = blockRanges(w, world);
        final byte[] rcclId = TgoNative.exchangeRcclId();
        if (rcclId == null) throw new TitanException("tgo_exchange_rccl_id failed");
        final CyclicBarrier phase = new CyclicBarrier(world);
        final AtomicBoolean notPartitionable = new AtomicBoolean(false);
        final String[] why = new String[1];
        final long[] minWeight = new long[world];
        final long[][] ownIds = new long[world][];
        final Object[] owned = new Object[world];
        ExecutorService pool = Executors.newFixedThreadPool(world);
        try {
            List<Future<?>> fs = new ArrayList<>();
            for (int r = 0; r < world; r++) {
                final int rank = r;
                fs.add(pool.submit(() -> {
                    worker(rank, world, devices[rank], rows, cut[rank], cut[rank + 1], schema, rcclId, phase, program,
                            minWeight, notPartitionable, why, ownIds, owned, partitionBits, hostThreads, hardQueryLimit);
                    return null;
                }));
            }
            for (Future<?> f : fs) f.get(RUN_TIMEOUT_MINUTES, TimeUnit.MINUTES);
        } finally {
            pool.shutdownNow();
        }
        if (notPartitionable.get()) throw new NotPartitionable(why[0]);
        long n = 0;
        for (long[] ids : ownIds) n += ids.length;
        if (n > Integer.MAX_VALUE - 8) throw new TitanException("more live vertices than one Java array holds");
        long[] ids = new long[(int) n];
        Object values = owned[0] instanceof double[] ? new double[(int) n] : new long[(int) n];
        int at = 0;
        for (int r = 0; r < world; r++) {
            System.arraycopy(ownIds[r], 0, ids, at, ownIds[r].length);
            System.arraycopy(owned[r], 0, values, at, ownIds[r].length);
            at += ownIds[r].length;
        }
        return new Object[]{ids, values};
    }

    /** A phase barrier that gives up with the job (a peer that died never arrives). */
    private static void await(CyclicBarrier phase) throws Exception {
        phase.await(RUN_TIMEOUT_MINUTES, TimeUnit.MINUTES);
    }

    private static void worker(int rank, int world, int device, RowBlocks rows, int from, int to,
                               CsrCollectingScanJob.Handle schema, byte[] rcclId, CyclicBarrier phase, Program program,
                               long[] minWeight, AtomicBoolean notPartitionable, String[] why, long[][] ownIds,
                               Object[] owned, int partitionBits, int hostThreads, long hardQueryLimit) throws Exception {
        long ctx = 0, x = 0;
        try {
            ctx = TgoNative.create(device, partitionBits, hostThreads, hardQueryLimit);
            if (ctx == 0) throw new TitanException("no usable gfx950 device " + device);
            // staging is local; a block that fails to stage is reported by the collective finish
            RuntimeException staged = null;
            try {
                rows.loadInto(ctx, schema, from, to);
            } catch (RuntimeException e) {
                staged = e;
            }
            await(phase);                                      // every ctx exists: the communicator may form
            x = TgoNative.exchangeRcclCreate(world, rank, rcclId, device);
            if (x == 0) throw new TitanException("tgo_exchange_rccl_create failed on worker " + rank);
            long[] part = TgoNative.finishPartitionRows(ctx, x, true);
            if (part == null) throw new TitanException("out of memory on worker " + rank);
            // the load's status is agreed (every worker failed it, or none did)
            if (part[0] != 0) {
                if (part[0] == TgoNative.E_UNSUPPORTED) {        // vertex cuts / a non-Integer weight key
                    why[0] = TgoNative.lastError(ctx);
                    notPartitionable.set(true);
                }
                await(phase);                                    // every worker's reason is in
                if (notPartitionable.get()) return;
                if (staged != null) throw staged;
                TgoNative.check(ctx, (int) part[0]);
            }
            final long live = part[1], slot = part[2], total = part[3];
            // the program's own conditions, decided from agreed values: every worker alike
            if (!program.partitions(total)) {
                notPartitionable.set(true);
                why[0] = "the program has no partitioned form for " + total + " vertices";
                return;
            }
            if (program.needsNonNegativeWeights()) {
                long[] wm = TgoNative.partWeightMin(ctx);
                TgoNative.check(ctx, (int) wm[0]);
                minWeight[rank] = wm[1];
                await(phase);                                    // every worker's minimum is in
                for (long m : minWeight)
                    if (m < 0) {
                        notPartitionable.set(true);
                        why[0] = "a negative weight: delta-stepping needs non-negative weights";
                        return;
                    }
            }
            long[] allIds = TgoNative.vertexIds(ctx);
            long[] ids = java.util.Arrays.copyOf(allIds, (int) live);
            Object res = TgoNative.checked(ctx, program.run(ctx, x, ids, rank * slot));
            ownIds[rank] = ids;
            owned[rank] = res;
        } catch (Exception e) {
            phase.reset();                                     // the peers waiting on a phase fail too
            throw e;
        } finally {
            if (x != 0) TgoNative.exchangeDestroy(x);
            if (ctx != 0) TgoNative.destroy(ctx);
        }
    }
}
