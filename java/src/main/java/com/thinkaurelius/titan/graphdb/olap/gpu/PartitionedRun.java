package com.thinkaurelius.titan.graphdb.olap.gpu;

import com.thinkaurelius.titan.core.TitanException;
import com.thinkaurelius.titan.diskstorage.Entry;
import com.thinkaurelius.titan.diskstorage.EntryList;
import com.thinkaurelius.titan.diskstorage.StaticBuffer;
import com.thinkaurelius.titan.diskstorage.configuration.Configuration;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.SliceQuery;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.scan.ScanJob;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.scan.ScanMetrics;
import com.thinkaurelius.titan.graphdb.database.StandardTitanGraph;
import com.thinkaurelius.titan.graphdb.database.idhandling.IDHandler;
import com.thinkaurelius.titan.graphdb.idmanagement.IDManager;
import com.thinkaurelius.titan.graphdb.internal.RelationCategory;
import com.thinkaurelius.titan.graphdb.olap.VertexJobConverter;
import com.thinkaurelius.titan.graphdb.relations.RelationCache;
import com.thinkaurelius.titan.graphdb.transaction.StandardTitanTx;
import org.apache.tinkerpop.gremlin.structure.Direction;

import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import java.util.Map;
import java.util.concurrent.CyclicBarrier;
import java.util.concurrent.ExecutorService;
import java.util.concurrent.Executors;
import java.util.concurrent.Future;
import java.util.concurrent.TimeUnit;
import java.util.function.Predicate;

/**
 * The multi-GPU form of the GPU path ({@code GpuGraphComputer.devices(...)}): the graph is
 * 1-D vertex-partitioned over the node's GPUs (include/titan_gpu_olap_part.h), one worker
 * thread per device inside this JVM, each with its own tgo_ctx and RCCL communicator.  The
 * reference has no multi-device executor (Fulgora is one JVM, FulgoraGraphComputer.java:117-311);
 * the job API in front of it is unchanged (TitanGraphComputer.java:8-43).
 *
 * <ol>
 * <li>ONE edgestore scan ({@link EdgeCollectingScanJob}) decodes every row with the graph's own
 *     EdgeSerializer (EdgeSerializer.java:73-166), as VertexJobConverter.process does per row
 *     (:109-129): ghost rows (no VertexExists entry) are skipped, vertex cuts fold into their
 *     canonical vertex (PartitionedVertexProgramExecutor.java:47-103), and every user edge is
 *     kept once, from its OUT entry.</li>
 * <li>The live vertices' Titan ids, sorted, are the global dense ids; edges to vertices that
 *     never execute are dropped (PreloadedVertex, VertexState.java:103-137).  The dense range
 *     is cut into {@code world} equal 64-aligned slices (padding ids are entry-less).</li>
 * <li>Worker r: tgo_part_layout of its slice (the degree-grouped order, gathered into one
 *     array every worker loads with), tgo_load_partition_layout of the edges with an endpoint
 *     in its slice (the program's scope and QueryContainer cap applied by the load), an RCCL
 *     exchange (worker 0's id, created by all workers together), then the program as ONE
 *     native call (tgo_part_pagerank_run / tgo_part_sssp_run), owned results into the
 *     global result arrays.</li>
 * </ol>
 * A worker that fails before the exchange exists breaks the phase barrier, so the others stop
 * too; a failure inside a running program is reported by that worker, and the job's future
 * fails after {@link #RUN_TIMEOUT_MINUTES} if a peer stays blocked in a collective (RCCL does
 * not notify peers of an aborted communicator).
 */
public final class PartitionedRun {

    public static final int RUN_TIMEOUT_MINUTES = 60;
    /** titan_gpu_olap_part.h tgo_part_pagerank_run exchange modes */
    public static final int PR_EXCHANGE_ALLGATHER = 0, PR_EXCHANGE_GHOST = 1;
    /** TGO_DIST_ABSENT / the Integer weight of an edge without the weight property (kMissingWeight). */
    static final int MISSING_WEIGHT = Integer.MIN_VALUE;

    private PartitionedRun() {}

    /** What a program runs on each worker: the native call, and how its owned results land. */
    public interface Program {
        int scope();
        boolean applyCap();
        /** The owned results of this worker (long[] or double[] of the slice length); live = the
         *  sorted live vertex ids (global dense id = index), for seeds given as Titan ids. */
        Object run(long ctx, long exchange, long[] live);
        /** The global result array of n live vertices. */
        Object newResult(int n);
    }

    // ------------------------------------------------------------------ the scanned graph
    /** Growable int storage past the 2^31 element limit of one Java array. */
    static final class IntChunks {
        static final int CHUNK = 1 << 24;
        final List<int[]> chunks = new ArrayList<>();
        long size = 0;
        void add(int v) {
            if ((size & (CHUNK - 1)) == 0 && size / CHUNK == chunks.size()) chunks.add(new int[CHUNK]);
            chunks.get((int) (size / CHUNK))[(int) (size & (CHUNK - 1))] = v;
            size++;
        }
        int get(long i) { return chunks.get((int) (i / CHUNK))[(int) (i & (CHUNK - 1))]; }
        void set(long i, int v) { chunks.get((int) (i / CHUNK))[(int) (i & (CHUNK - 1))] = v; }
    }
    static final class LongChunks {
        static final int CHUNK = 1 << 23;
        final List<long[]> chunks = new ArrayList<>();
        long size = 0;
        void add(long v) {
            if ((size & (CHUNK - 1)) == 0 && size / CHUNK == chunks.size()) chunks.add(new long[CHUNK]);
            chunks.get((int) (size / CHUNK))[(int) (size & (CHUNK - 1))] = v;
            size++;
        }
        long get(long i) { return chunks.get((int) (i / CHUNK))[(int) (i & (CHUNK - 1))]; }
    }

    /** Shared by the scan's clones: every clone's rows are appended under its monitor. */
    public static final class Collected {
        final LongChunks vertices = new LongChunks();       // live (canonical) vertex ids
        final LongChunks src = new LongChunks(), dst = new LongChunks();   // Titan ids, OUT entries
        final IntChunks weight = new IntChunks();
        final boolean weighted;
        public Collected(boolean weighted) { this.weighted = weighted; }
    }

    /**
     * The scan: the grounded VertexExists slice, then the user-edge slice [0x60, 0x80) without a
     * limit (the partition load applies the scope's cap), as CsrCollectingScanJob asks.
     */
    public static final class EdgeCollectingScanJob implements ScanJob {
        private static final SliceQuery EDGE_SLICE = new SliceQuery(
                IDHandler.getBounds(RelationCategory.EDGE, false)[0],
                IDHandler.getBounds(RelationCategory.EDGE, false)[1]);
        private final StandardTitanGraph graph;
        private final IDManager idManager;
        private final long weightKey;
        private final Collected out;
        private StandardTitanTx tx;
        private LongChunks v, s, d;
        private IntChunks w;

        public EdgeCollectingScanJob(StandardTitanGraph graph, long weightKey, Collected out) {
            this.graph = graph;
            this.idManager = graph.getIDManager();
            this.weightKey = weightKey;
            this.out = out;
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
            return buffer -> !IDManager.VertexIDType.Invisible.is(idManager.getKeyID(buffer));
        }

        @Override
        public void workerIterationStart(Configuration jobConfiguration, Configuration graphConfiguration,
                                         ScanMetrics metrics) {
            tx = VertexJobConverter.startTransaction(graph);
            v = new LongChunks();
            s = new LongChunks();
            d = new LongChunks();
            w = new IntChunks();
        }

        @Override
        public void process(StaticBuffer key, Map<SliceQuery, EntryList> slices, ScanMetrics metrics) {
            long vid = idManager.getKeyID(key);
            final boolean cut = idManager.isPartitionedVertex(vid);
            EntryList exists = slices.get(VertexJobConverter.VERTEX_EXISTS_QUERY);
            if (!cut && (exists == null || exists.isEmpty())) return;      // a ghost (VertexJobConverter.java:132)
            if (cut) vid = idManager.getCanonicalVertexId(vid);
            v.add(vid);
            EntryList edges = slices.get(EDGE_SLICE);
            if (edges == null) return;
            for (Entry e : edges) {
                RelationCache rc = tx.getEdgeSerializer().parseRelation(e, weightKey == 0, tx);
                if (rc.direction != Direction.OUT) continue;               // each edge once, from its tail
                long other = rc.getOtherVertexId();
                if (idManager.isPartitionedVertex(other)) other = idManager.getCanonicalVertexId(other);
                s.add(vid);
                d.add(other);
                if (weightKey != 0) {
                    Object x = rc.hasProperties() ? rc.get(weightKey) : null;
                    // ShortestDistanceVertexProgram.java:53 reads edge.<Integer>value(weight)
                    w.add(x instanceof Integer ? (Integer) x : MISSING_WEIGHT);
                }
            }
        }

        @Override
        public void workerIterationEnd(ScanMetrics metrics) {
            synchronized (out) {
                for (long i = 0; i < v.size; i++) out.vertices.add(v.get(i));
                for (long i = 0; i < s.size; i++) {
                    out.src.add(s.get(i));
                    out.dst.add(d.get(i));
                    if (out.weighted) out.weight.add(w.get(i));
                }
            }
            if (tx != null && tx.isOpen()) tx.rollback();
        }

        @Override
        public EdgeCollectingScanJob clone() {
            return new EdgeCollectingScanJob(graph, weightKey, out);
        }
    }

    // ------------------------------------------------------------------ partition + run
    /**
     * Runs `program` over the collected graph on `devices` (one worker each).  Returns the live
     * vertices' Titan ids (row order) and the program's results in that order.
     */
    public static Object[] run(Collected c, Program program, int[] devices, int partitionBits, int hostThreads,
                               long hardQueryLimit) throws Exception {
        final int world = devices.length;
        // (2) global dense ids: the sorted live vertex ids
        if (c.vertices.size > Integer.MAX_VALUE - 64) throw new TitanException("too many vertices for one job");
        long[] ids = new long[(int) c.vertices.size];
        for (int i = 0; i < ids.length; i++) ids[i] = c.vertices.get(i);
        Arrays.sort(ids);
        int n = 0;
        for (int i = 0; i < ids.length; i++) if (i == 0 || ids[i] != ids[i - 1]) ids[n++] = ids[i];  // cut rows repeat
        final long[] live = Arrays.copyOf(ids, n);
        final long nLocal = ((n + world - 1L) / world + 63) / 64 * 64;
        final long nGlobal = nLocal * world;
        // every edge once, in dense ids; bucketed per worker by its endpoints' owners
        final IntChunks[] bs = new IntChunks[world], bd = new IntChunks[world], bw = new IntChunks[world];
        for (int r = 0; r < world; r++) { bs[r] = new IntChunks(); bd[r] = new IntChunks(); bw[r] = new IntChunks(); }
        for (long i = 0; i < c.src.size; i++) {
            int a = Arrays.binarySearch(live, c.src.get(i)), b = Arrays.binarySearch(live, c.dst.get(i));
            if (a < 0 || b < 0) continue;                      // an endpoint never executes
            int ra = (int) (a / nLocal), rb = (int) (b / nLocal);
            int wt = c.weighted ? c.weight.get(i) : 0;
            bs[ra].add(a); bd[ra].add(b); if (c.weighted) bw[ra].add(wt);
            if (rb != ra) { bs[rb].add(a); bd[rb].add(b); if (c.weighted) bw[rb].add(wt); }
        }
        final int[] layoutGlobal = new int[(int) nGlobal];
        final Object result = program.newResult(n);
        final byte[] rcclId = TgoNative.exchangeRcclId();
        if (rcclId == null) throw new TitanException("tgo_exchange_rccl_id failed");
        final CyclicBarrier phase = new CyclicBarrier(world);
        ExecutorService pool = Executors.newFixedThreadPool(world);
        try {
            List<Future<?>> fs = new ArrayList<>();
            for (int r = 0; r < world; r++) {
                final int rank = r;
                fs.add(pool.submit(() -> {
                    worker(rank, world, devices[rank], nGlobal, nLocal, live, toArray(bs[rank]), toArray(bd[rank]),
                            c.weighted ? toArray(bw[rank]) : null, layoutGlobal, rcclId, phase, program, result,
                            partitionBits, hostThreads, hardQueryLimit);
                    return null;
                }));
            }
            for (Future<?> f : fs) f.get(RUN_TIMEOUT_MINUTES, TimeUnit.MINUTES);
        } finally {
            pool.shutdownNow();
        }
        return new Object[]{live, result};
    }

    static int[] toArray(IntChunks x) {
        if (x.size > Integer.MAX_VALUE - 8) throw new TitanException("a partition holds more edges than a Java array");
        int[] out = new int[(int) x.size];
        for (int i = 0; i < out.length; i++) out[i] = x.get(i);
        return out;
    }

    private static void worker(int rank, int world, int device, long nGlobal, long nLocal, long[] live, int[] src, int[] dst,
                               int[] weight, int[] layoutGlobal, byte[] rcclId, CyclicBarrier phase, Program program,
                               Object result, int partitionBits, int hostThreads, long hardQueryLimit) throws Exception {
        final long lo = rank * nLocal, hi = lo + nLocal;
        long ctx = 0, x = 0;
        try {
            int[] lay = TgoNative.partLayout(src, dst, nGlobal, lo, hi, hostThreads);
            if (lay == null) throw new TitanException("tgo_part_layout failed on worker " + rank);
            System.arraycopy(lay, 0, layoutGlobal, (int) lo, lay.length);
            phase.await();                                     // every slice in layoutGlobal
            ctx = TgoNative.create(device, partitionBits, hostThreads, hardQueryLimit);
            if (ctx == 0) throw new TitanException("no usable gfx950 device " + device);
            TgoNative.check(ctx, TgoNative.loadPartition(ctx, nGlobal, lo, hi, src, dst, weight, program.scope(),
                    program.applyCap(), layoutGlobal));
            phase.await();                                     // every worker loaded: the communicator may form
            x = TgoNative.exchangeRcclCreate(world, rank, rcclId, device);
            if (x == 0) throw new TitanException("tgo_exchange_rccl_create failed on worker " + rank);
            Object owned = TgoNative.checked(ctx, program.run(ctx, x, live));
            int count = (int) Math.max(0, Math.min(hi, live.length) - lo);
            if (count > 0) System.arraycopy(owned, 0, result, (int) lo, count);
        } catch (Exception e) {
            phase.reset();                                     // the peers waiting on a phase fail too
            throw e;
        } finally {
            if (x != 0) TgoNative.exchangeDestroy(x);
            if (ctx != 0) TgoNative.destroy(ctx);
        }
    }
}
