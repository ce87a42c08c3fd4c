package com.thinkaurelius.titan.graphdb.olap.computer;

import com.google.common.base.Preconditions;
import com.thinkaurelius.titan.core.TitanException;
import com.thinkaurelius.titan.core.TitanGraphComputer;
import com.thinkaurelius.titan.core.PropertyKey;
import com.thinkaurelius.titan.core.schema.TitanManagement;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.scan.ScanMetrics;
import com.thinkaurelius.titan.diskstorage.keycolumnvalue.scan.StandardScanner;
import com.thinkaurelius.titan.graphdb.database.StandardTitanGraph;
import com.thinkaurelius.titan.graphdb.olap.QueryContainer;
import com.thinkaurelius.titan.graphdb.olap.gpu.CsrCollectingScanJob;
import com.thinkaurelius.titan.graphdb.olap.gpu.TgoNative;
import org.apache.commons.configuration.BaseConfiguration;
import org.apache.tinkerpop.gremlin.process.computer.ComputerResult;
import org.apache.tinkerpop.gremlin.process.computer.GraphComputer;
import org.apache.tinkerpop.gremlin.process.computer.MapReduce;
import org.apache.tinkerpop.gremlin.process.computer.VertexProgram;
import org.apache.tinkerpop.gremlin.process.computer.util.DefaultComputerResult;
import org.apache.tinkerpop.gremlin.process.computer.util.GraphComputerHelper;

import java.lang.reflect.Field;
import java.util.HashSet;
import java.util.Map;
import java.util.HashMap;
import java.util.Set;
import java.util.concurrent.CompletableFuture;
import java.util.concurrent.Future;

/**
 * Drop-in for {@link FulgoraGraphComputer} on the OLAP path (core/TitanGraphComputer.java:8-43):
 * the same builder API (program / mapReduce / workers / resultMode / submit), executed by the
 * MI355X engine through {@link TgoNative}.
 *
 * submit() runs ONE edgestore scan ({@link CsrCollectingScanJob} through the unchanged
 * StandardScanner, Backend.java:336-355) instead of Fulgora's scan per superstep
 * (FulgoraGraphComputer.java:151-189), runs the recognised program on the device, and hands
 * the per-vertex results to the MapReducers through FulgoraMapEmitter, reduce and
 * addResultToMemory exactly as Fulgora's map phase does (:192-246).  Programs the device does
 * not implement fail with TitanException (as ExecutionException from get()).
 *
 * Supported: tmain's PageRankVertexProgram, ShortestDistanceVertexProgram and
 * OLAPTest.DegreeCounter (matched by class name; their parameters are read from
 * storeState(), or the DegreeCounter's length field).  ResultMode NONE only: PERSIST and
 * LOCALTX write the compute keys back through batched transactions in the reference
 * (:248-305) and are rejected here.
 */
public class GpuGraphComputer implements TitanGraphComputer {

    private final StandardTitanGraph graph;
    private VertexProgram<?> vertexProgram;
    private final Set<MapReduce> mapReduces = new HashSet<>();
    private int numThreads = 1;
    private int device = 0;
    private ResultGraph resultGraphMode = null;
    private Persist persistMode = null;
    private boolean executed = false;

    public GpuGraphComputer(StandardTitanGraph graph) {
        this.graph = graph;
    }

    public GpuGraphComputer device(int ordinal) {
        this.device = ordinal;
        return this;
    }

    @Override
    public GraphComputer result(ResultGraph mode) {
        this.resultGraphMode = mode;
        return this;
    }

    @Override
    public GraphComputer persist(Persist mode) {
        this.persistMode = mode;
        return this;
    }

    @Override
    public TitanGraphComputer workers(int threads) {
        Preconditions.checkArgument(threads > 0, "Invalid number of threads: %s", threads);
        numThreads = threads;
        return this;
    }

    @Override
    public TitanGraphComputer program(VertexProgram vertexProgram) {
        Preconditions.checkState(this.vertexProgram == null, "A vertex program has already been set");
        this.vertexProgram = vertexProgram;
        return this;
    }

    @Override
    public TitanGraphComputer mapReduce(MapReduce mapReduce) {
        this.mapReduces.add(mapReduce);
        return this;
    }

    @Override
    public Future<ComputerResult> submit() {
        if (executed) throw Exceptions.computerHasAlreadyBeenSubmittedAVertexProgram();
        executed = true;
        if (null == vertexProgram && mapReduces.isEmpty())
            throw GraphComputer.Exceptions.computerHasNoVertexProgramNorMapReducers();
        if (null != vertexProgram) {
            GraphComputerHelper.validateProgramOnComputer(this, vertexProgram);
            mapReduces.addAll(vertexProgram.getMapReducers());
        }
        final Persist persist = persistMode == null ? Persist.NOTHING : persistMode;
        if (persist != Persist.NOTHING)
            throw new TitanException("GpuGraphComputer supports ResultMode.NONE only (no property write-back)");
        final DeviceProgram program = DeviceProgram.recognise(vertexProgram);
        final FulgoraMemory memory = new FulgoraMemory(vertexProgram, mapReduces);
        return CompletableFuture.<ComputerResult>supplyAsync(() -> {
            final long start = System.currentTimeMillis();
            long ctx = TgoNative.create(device, graph.getIDManager().getPartitionBits(), numThreads,
                    QueryContainer.DEFAULT_HARD_QUERY_LIMIT);
            if (ctx == 0) throw new TitanException("no usable gfx950 device (the GPU engine has no CPU fallback)");
            try {
                // (1) one scan collects the rows the program's scope preloads
                CsrCollectingScanJob.Handle handle = new CsrCollectingScanJob.Handle(ctx, graph.getIDManager(),
                        Schemas.edgeTypes(graph), Schemas.propertyKeys(graph), program.scope(), true, new long[0],
                        program.weightKey(graph));
                StandardScanner.Builder scan = graph.getBackend().buildEdgeScanJob();
                scan.setJobId("gpu-olap#load");
                scan.setNumProcessingThreads(numThreads);
                scan.setWorkBlockSize(CsrCollectingScanJob.DEFAULT_BLOCK_ROWS);
                scan.setJob(new CsrCollectingScanJob(handle));
                ScanMetrics m = scan.execute().get();
                if (m.get(ScanMetrics.Metric.FAILURE) > 0)
                    throw new TitanException("Failed to process [" + m.get(ScanMetrics.Metric.FAILURE) + "] rows");
                TgoNative.check(ctx, TgoNative.finishLoad(ctx));
                // (2) the program on the device; memory reports its iteration (FulgoraMemory.java:73-76)
                long[] ids = TgoNative.vertexIds(ctx);
                Map<String, Object> values = program.run(ctx);
                for (int i = 0; i < program.iterations(); i++) memory.incrIteration();
                // (3) map / reduce / addResultToMemory as Fulgora's map phase
                for (MapReduce mr : mapReduces) {
                    FulgoraMapEmitter emitter = new FulgoraMapEmitter<>(mr.doStage(MapReduce.Stage.REDUCE));
                    program.emit(ids, values, emitter);
                    emitter.complete(mr);
                    if (mr.doStage(MapReduce.Stage.REDUCE)) {
                        FulgoraReduceEmitter reduce = new FulgoraReduceEmitter<>();
                        mr.workerStart(MapReduce.Stage.REDUCE);
                        for (Object e : emitter.reduceMap.entrySet()) {
                            Map.Entry entry = (Map.Entry) e;
                            mr.reduce(entry.getKey(), ((Iterable) entry.getValue()).iterator(), reduce);
                        }
                        mr.workerEnd(MapReduce.Stage.REDUCE);
                        reduce.complete(mr);
                        mr.addResultToMemory(memory, reduce.reduceQueue.iterator());
                    } else {
                        mr.addResultToMemory(memory, emitter.mapQueue.iterator());
                    }
                }
                memory.setRuntime(System.currentTimeMillis() - start);
                memory.complete();
                return new DefaultComputerResult(graph, memory.asImmutable());
            } catch (TitanException e) {
                throw e;
            } catch (Exception e) {
                throw new TitanException(e);
            } finally {
                TgoNative.destroy(ctx);
            }
        });
    }

    @Override
    public GraphComputer.Features features() {
        return new GraphComputer.Features() {
            @Override public boolean supportsWorkerPersistenceBetweenIterations() { return false; }
            @Override public boolean supportsResultGraphPersistCombination(ResultGraph r, Persist p) {
                return p == Persist.NOTHING;
            }
        };
    }

    /** Flattened schema for tgo_load_rows (layout documented in TgoNative.loadRows). */
    static final class Schemas {
        static long[] edgeTypes(StandardTitanGraph graph) {
            TitanManagement mgmt = graph.openManagement();
            try {
                java.util.List<Long> out = new java.util.ArrayList<>();
                for (com.thinkaurelius.titan.core.EdgeLabel l : mgmt.getRelationTypes(com.thinkaurelius.titan.core.EdgeLabel.class)) {
                    com.thinkaurelius.titan.graphdb.internal.InternalRelationType t =
                            (com.thinkaurelius.titan.graphdb.internal.InternalRelationType) l;
                    out.add(t.longId());
                    out.add((long) t.multiplicity().ordinal());
                    out.add(t.getSortOrder() == com.thinkaurelius.titan.graphdb.internal.Order.DESC ? 1L : 0L);
                    long[] sk = t.getSortKey();
                    out.add((long) sk.length);
                    for (long k : sk) out.add(k);
                    long[] sig = t.getSignature();
                    out.add((long) sig.length);
                    for (long k : sig) out.add(k);
                }
                return out.stream().mapToLong(Long::longValue).toArray();
            } finally {
                mgmt.rollback();
            }
        }

        static long[] propertyKeys(StandardTitanGraph graph) {
            TitanManagement mgmt = graph.openManagement();
            try {
                java.util.List<Long> out = new java.util.ArrayList<>();
                for (PropertyKey k : mgmt.getRelationTypes(PropertyKey.class)) {
                    out.add(((com.thinkaurelius.titan.graphdb.internal.InternalRelationType) k).longId());
                    out.add((long) datatype(k.dataType()));
                }
                return out.stream().mapToLong(Long::longValue).toArray();
            } finally {
                mgmt.rollback();
            }
        }

        static int datatype(Class<?> c) {
            if (c == Byte.class) return TgoNative.DT_BYTE;
            if (c == Short.class) return TgoNative.DT_SHORT;
            if (c == Integer.class) return TgoNative.DT_INTEGER;
            if (c == Long.class) return TgoNative.DT_LONG;
            if (c == Float.class) return TgoNative.DT_FLOAT;
            if (c == Double.class) return TgoNative.DT_DOUBLE;
            if (c == Boolean.class) return TgoNative.DT_BOOLEAN;
            if (c == java.util.Date.class) return TgoNative.DT_DATE;
            if (c == Character.class) return TgoNative.DT_CHARACTER;
            if (c == String.class) return TgoNative.DT_STRING;
            return 0;   // unknown: the decoder fails loudly if such a property must be skipped
        }
    }

    /**
     * A vertex program the device implements: its scope, its parameters, the C-ABI call and
     * the (id, value) pairs its MapReducer emits — the canonical id and the compute key's
     * value (PageRankMapReduce / ShortestDistanceMapReduce / DegreeMapper all do exactly that).
     */
    abstract static class DeviceProgram {
        abstract int scope();
        abstract int iterations();
        long weightKey(StandardTitanGraph graph) { return 0; }
        abstract Map<String, Object> run(long ctx);
        abstract void emit(long[] ids, Map<String, Object> values, FulgoraMapEmitter emitter);

        static DeviceProgram recognise(VertexProgram<?> p) {
            if (p == null) throw new TitanException("the GPU path needs a vertex program");
            BaseConfiguration conf = new BaseConfiguration();
            p.storeState(conf);
            switch (p.getClass().getName()) {
                case "com.thinkaurelius.titan.olap.PageRankVertexProgram":
                    return new PageRank(conf.getDouble("titan.pageRank.dampingFactor", 0.85D),
                            conf.getInt("titan.pageRank.maxIterations", 10), conf.getLong("titan.pageRank.vertexCount", 1L));
                case "com.thinkaurelius.titan.olap.ShortestDistanceVertexProgram":
                    return new ShortestDistance(conf.getLong("titan.shortestDistanceVertexProgram.seedID"),
                            conf.getInt("titan.shortestDistanceVertexProgram.maxDepth"),
                            conf.getString("titan.shortestDistanceVertexProgram.weightProperty", "distance"));
                case "com.thinkaurelius.titan.olap.OLAPTest$DegreeCounter":
                    return new DegreeCount(lengthOf(p));
                default:
                    throw new TitanException("vertex program " + p.getClass().getName() + " is not supported on the GPU path");
            }
        }

        private static int lengthOf(VertexProgram<?> p) {
            try {
                Field f = p.getClass().getDeclaredField("length");
                f.setAccessible(true);
                return f.getInt(p);
            } catch (ReflectiveOperationException e) {
                throw new TitanException(e);
            }
        }
    }

    static final class PageRank extends DeviceProgram {
        final double alpha; final int maxIterations; final long vertexCount;
        PageRank(double alpha, int maxIterations, long vertexCount) {
            this.alpha = alpha; this.maxIterations = maxIterations; this.vertexCount = vertexCount;
        }
        int scope() { return TgoNative.SCOPE_IN_E; }
        int iterations() { return maxIterations; }
        Map<String, Object> run(long ctx) {
            Map<String, Object> v = new HashMap<>();
            v.put("titan.pageRank.pageRank", TgoNative.checked(ctx, TgoNative.pageRank(ctx, alpha, vertexCount, maxIterations)));
            return v;
        }
        void emit(long[] ids, Map<String, Object> values, FulgoraMapEmitter emitter) {
            double[] pr = (double[]) values.get("titan.pageRank.pageRank");
            for (int i = 0; i < ids.length; i++) if (!Double.isNaN(pr[i])) emitter.emit(ids[i], pr[i]);
        }
    }

    static final class ShortestDistance extends DeviceProgram {
        final long seed; final int maxDepth; final String weightProperty;
        ShortestDistance(long seed, int maxDepth, String weightProperty) {
            this.seed = seed; this.maxDepth = maxDepth; this.weightProperty = weightProperty;
        }
        int scope() { return TgoNative.SCOPE_IN_E; }       // Local(inE, m + e.value(weight)) (:53)
        int iterations() { return maxDepth; }
        long weightKey(StandardTitanGraph graph) {
            TitanManagement mgmt = graph.openManagement();
            try {
                PropertyKey k = mgmt.getPropertyKey(weightProperty);
                if (k == null) throw new TitanException("weight property '" + weightProperty + "' does not exist");
                return ((com.thinkaurelius.titan.graphdb.internal.InternalRelationType) k).longId();
            } finally {
                mgmt.rollback();
            }
        }
        Map<String, Object> run(long ctx) {
            Map<String, Object> v = new HashMap<>();
            v.put("titan.shortestDistanceVertexProgram.distance", TgoNative.checked(ctx,
                    TgoNative.sssp(ctx, seed, maxDepth, scope(), TgoNative.SSSP_HOP_BOUNDED, 0)));
            return v;
        }
        void emit(long[] ids, Map<String, Object> values, FulgoraMapEmitter emitter) {
            long[] d = (long[]) values.get("titan.shortestDistanceVertexProgram.distance");
            for (int i = 0; i < ids.length; i++) if (d[i] != TgoNative.DIST_ABSENT) emitter.emit(ids[i], d[i]);
        }
    }

    static final class DegreeCount extends DeviceProgram {
        final int length;
        DegreeCount(int length) { this.length = length; }
        int scope() { return TgoNative.SCOPE_IN_E; }        // DEG_MSG = Local(inE) (OLAPTest.java:338)
        int iterations() { return length; }
        Map<String, Object> run(long ctx) {
            Map<String, Object> v = new HashMap<>();
            v.put("degree", TgoNative.checked(ctx, TgoNative.walkCount(ctx, length)));
            return v;
        }
        void emit(long[] ids, Map<String, Object> values, FulgoraMapEmitter emitter) {
            int[] d = (int[]) values.get("degree");
            for (int i = 0; i < ids.length; i++) emitter.emit(ids[i], d[i]);
        }
    }
}
