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
import com.thinkaurelius.titan.graphdb.olap.gpu.PartitionedRun;
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
import java.util.Optional;
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
 * storeState(), or the DegreeCounter's length field).
 *
 * Write-back (FulgoraGraphComputer.java:248-305): with Persist.VERTEX_PROPERTIES the compute
 * keys are encoded on the device (tgo_result_rows: single-cardinality property entries, one
 * row per vertex holding a value) and written to the edgestore as column overwrites in
 * batches of writeBatchSize rows (ResultGraph.ORIGINAL); ResultGraph.NEW sets them in a new,
 * uncommitted transaction instead, as Fulgora does.  The compute keys must exist as typed
 * property keys (Long distance, Double pageRank / edgeCount, Integer degree).
 */
public class GpuGraphComputer implements TitanGraphComputer {

    private final StandardTitanGraph graph;
    private VertexProgram<?> vertexProgram;
    private final Set<MapReduce> mapReduces = new HashSet<>();
    private int numThreads = 1;
    private int device = 0;
    private int[] devices = null;       // > 1: the multi-GPU path (PartitionedRun)
    private ResultGraph resultGraphMode = null;
    private Persist persistMode = null;
    private boolean executed = false;

    public GpuGraphComputer(StandardTitanGraph graph) {
        this.graph = graph;
    }

    public GpuGraphComputer device(int ordinal) {
        this.device = ordinal;
        this.devices = null;
        return this;
    }

    /**
     * Several GPUs of this node: programs that partition (PageRank, and ShortestDistance when its
     * depth bound cannot cut a path — the converged distances) run 1-D vertex-partitioned, one
     * worker thread per device with an RCCL communicator each ({@link PartitionedRun}); the
     * others run on the first device alone.
     */
    public GpuGraphComputer devices(int... ordinals) {
        Preconditions.checkArgument(ordinals != null && ordinals.length > 0, "no devices");
        this.device = ordinals[0];
        this.devices = ordinals.length > 1 ? ordinals.clone() : null;
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
        // unset modes come from the program's preference (FulgoraGraphComputer.java:133-135):
        // PageRank / ShortestDistance persist into the original graph, DegreeCounter into NEW
        final Persist persist = GraphComputerHelper.getPersistState(Optional.ofNullable(vertexProgram),
                Optional.ofNullable(persistMode));
        final ResultGraph resultGraph = GraphComputerHelper.getResultGraphState(Optional.ofNullable(vertexProgram),
                Optional.ofNullable(resultGraphMode));
        if (!features().supportsResultGraphPersistCombination(resultGraph, persist))
            throw GraphComputer.Exceptions.resultGraphPersistCombinationNotSupported(resultGraph, persist);
        final DeviceProgram program = DeviceProgram.recognise(vertexProgram);
        final FulgoraMemory memory = new FulgoraMemory(vertexProgram, mapReduces);
        if (devices != null && program.partitioned() != null)
            return CompletableFuture.<ComputerResult>supplyAsync(() -> submitPartitioned(program, memory, persist,
                    resultGraph));
        return CompletableFuture.<ComputerResult>supplyAsync(() -> {
            final long start = System.currentTimeMillis();
            long ctx = TgoNative.create(device, graph.getIDManager().getPartitionBits(), numThreads,
                    QueryContainer.DEFAULT_HARD_QUERY_LIMIT);
            if (ctx == 0) throw new TitanException("no usable gfx950 device (the GPU engine has no CPU fallback)");
            try {
                // (1) one scan collects the rows the program's scope preloads
                CsrCollectingScanJob.Handle handle = handle(ctx, null, program);
                scan(handle, "gpu-olap#load");
                // a block whose flush failed in workerIterationEnd is only logged by the scanner
                // (StandardScannerExecutor.java:278-282): the handle keeps that failure
                handle.rethrowFailure();
                TgoNative.check(ctx, TgoNative.finishLoad(ctx));
                return runLoaded(ctx, program, memory, persist, resultGraph, start);
            } catch (TitanException e) {
                throw e;
            } catch (Exception e) {
                throw new TitanException(e);
            } finally {
                TgoNative.destroy(ctx);
            }
        });
    }

    /** The collecting scan's shared handle: rows to tgo_load_rows on ctx, or to sink. */
    private CsrCollectingScanJob.Handle handle(long ctx, CsrCollectingScanJob.BlockSink sink, DeviceProgram program) {
        return new CsrCollectingScanJob.Handle(ctx, sink, graph.getIDManager(), Schemas.edgeTypes(graph),
                Schemas.propertyKeys(graph), program.scope(), true, new long[0], program.weightKey(graph));
    }

    /** The one edgestore scan (StandardScanner over the edgestore, Backend.buildEdgeScanJob). */
    private void scan(CsrCollectingScanJob.Handle handle, String jobId) throws Exception {
        StandardScanner.Builder scan = graph.getBackend().buildEdgeScanJob();
        scan.setJobId(jobId);
        scan.setNumProcessingThreads(numThreads);
        scan.setWorkBlockSize(CsrCollectingScanJob.DEFAULT_BLOCK_ROWS);
        scan.setJob(new CsrCollectingScanJob(handle));
        ScanMetrics m = scan.execute().get();
        if (m.get(ScanMetrics.Metric.FAILURE) > 0)
            throw new TitanException("Failed to process [" + m.get(ScanMetrics.Metric.FAILURE) + "] rows");
    }

    /**
     * Steps (2)-(4) on a loaded ctx: the program on the device, the map phase, the write-back.
     * Fulgora runs supersteps 0..T (T = the first iteration whose terminate() holds: maxIterations,
     * maxDepth, length) and increments the iteration after each of them, the terminating one
     * included (FulgoraGraphComputer.java:181-188); complete() then steps back once
     * (FulgoraMemory.java:73-76), so getIteration() reports T (OLAPTest.java:219,255).
     */
    private ComputerResult runLoaded(long ctx, DeviceProgram program, FulgoraMemory memory, Persist persist,
                                     ResultGraph resultGraph, long start) throws Exception {
        long[] ids = TgoNative.vertexIds(ctx);
        Map<String, Object> values = program.run(ctx);
        for (int i = 0; i <= program.iterations(); i++) memory.incrIteration();
        mapPhase(program, ids, values, memory);
        org.apache.tinkerpop.gremlin.structure.Graph result = graph;
        if (persist == Persist.VERTEX_PROPERTIES) {
            if (resultGraph == ResultGraph.NEW) result = WriteBack.localTx(graph, ids, values, program);
            else if (WriteBack.directWriteSafe(graph, program)) WriteBack.persist(graph, ctx, program);
            else WriteBack.transactional(graph, ids, values, program, numThreads);
        }
        memory.setRuntime(System.currentTimeMillis() - start);
        memory.complete();
        return new DefaultComputerResult(result, memory.asImmutable());
    }

    /** (3) map / reduce / addResultToMemory as Fulgora's map phase (FulgoraGraphComputer.java:192-246). */
    private void mapPhase(DeviceProgram program, long[] ids, Map<String, Object> values, FulgoraMemory memory) {
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
    }

    /**
     * The multi-GPU path: one scan keeps the raw rows in work blocks (PartitionedRun.RowBlocks),
     * then one worker per device loads its row range and runs the program; the map phase and
     * the write-back are the single-GPU path's, on the gathered results.  A graph the
     * partitioned programs do not cover (PartitionedRun.NotPartitionable: vertex cuts, a
     * non-Integer weight key, a negative weight, a depth bound that can cut a path, no vertex)
     * runs on the first device from the same rows, without a second scan.  The device-encoded
     * write-back needs one ctx holding every vertex, so results persist transactionally.
     */
    private ComputerResult submitPartitioned(DeviceProgram program, FulgoraMemory memory, Persist persist,
                                             ResultGraph resultGraph) {
        final long start = System.currentTimeMillis();
        try {
            PartitionedRun.RowBlocks rows = new PartitionedRun.RowBlocks();
            CsrCollectingScanJob.Handle handle = handle(0, rows, program);
            scan(handle, "gpu-olap#partitioned-load");
            handle.rethrowFailure();
            Object[] out;
            try {
                out = PartitionedRun.run(rows, handle, program.partitioned(), devices, graph.getIDManager().getPartitionBits(),
                        numThreads, QueryContainer.DEFAULT_HARD_QUERY_LIMIT);
            } catch (PartitionedRun.NotPartitionable e) {
                long ctx = TgoNative.create(device, graph.getIDManager().getPartitionBits(), numThreads,
                        QueryContainer.DEFAULT_HARD_QUERY_LIMIT);
                if (ctx == 0) throw new TitanException("no usable gfx950 device (the GPU engine has no CPU fallback)");
                try {
                    rows.loadInto(ctx, handle);
                    TgoNative.check(ctx, TgoNative.finishLoad(ctx));
                    return runLoaded(ctx, program, memory, persist, resultGraph, start);
                } finally {
                    TgoNative.destroy(ctx);
                }
            }
            long[] ids = (long[]) out[0];
            Map<String, Object> values = new HashMap<>();
            values.put(program.computeKeys()[0], out[1]);
            for (int i = 0; i <= program.iterations(); i++) memory.incrIteration();
            mapPhase(program, ids, values, memory);
            org.apache.tinkerpop.gremlin.structure.Graph result = graph;
            if (persist == Persist.VERTEX_PROPERTIES) {
                if (resultGraph == ResultGraph.NEW) result = WriteBack.localTx(graph, ids, values, program);
                else WriteBack.transactional(graph, ids, values, program, numThreads);
            }
            memory.setRuntime(System.currentTimeMillis() - start);
            memory.complete();
            return new DefaultComputerResult(result, memory.asImmutable());
        } catch (TitanException e) {
            throw e;
        } catch (Exception e) {
            throw new TitanException(e);
        }
    }

    @Override
    public GraphComputer.Features features() {
        return new GraphComputer.Features() {
            @Override public boolean supportsWorkerPersistenceBetweenIterations() { return false; }
            @Override public boolean supportsResultGraphPersistCombination(ResultGraph r, Persist p) {
                return p == Persist.NOTHING || p == Persist.VERTEX_PROPERTIES;
            }
        };
    }

    /** Compute-key write-back (FulgoraGraphComputer.java:248-305). */
    static final class WriteBack {
        static final int WRITE_BATCH_ROWS = 10000;

        /**
         * The device-encoded entries may go straight to the store only when nothing above the
         * store keeps a copy of the properties: no graph index over a compute key (the
         * transaction path maintains indexes) and no edgestore cache (cache.db-cache), which
         * would keep serving the old values.  Otherwise {@link #transactional} writes them.
         */
        static boolean directWriteSafe(StandardTitanGraph graph, DeviceProgram program) {
            if (graph.getConfiguration().getConfiguration()
                    .get(com.thinkaurelius.titan.graphdb.configuration.GraphDatabaseConfiguration.DB_CACHE))
                return false;
            Set<String> keys = new HashSet<>(java.util.Arrays.asList(program.computeKeys()));
            TitanManagement mgmt = graph.openManagement();
            try {
                for (com.thinkaurelius.titan.core.schema.TitanGraphIndex idx :
                        mgmt.getGraphIndexes(org.apache.tinkerpop.gremlin.structure.Vertex.class))
                    for (PropertyKey k : idx.getFieldKeys())
                        if (keys.contains(k.name())) return false;
                return true;
            } finally {
                mgmt.rollback();
            }
        }

        /**
         * Fulgora's own write path (VertexPropertyWriter, FulgoraGraphComputer.java:314-342):
         * batched transactions of v.property(single, key, value), committed, so indexes and
         * caches are maintained; a failed batch fails the job (:285-292).
         */
        static void transactional(StandardTitanGraph graph, long[] ids, Map<String, Object> values,
                                  DeviceProgram program, int threads) {
            for (int r0 = 0; r0 < ids.length; r0 += WRITE_BATCH_ROWS) {
                com.thinkaurelius.titan.core.TitanTransaction tx = graph.buildTransaction().enableBatchLoading().start();
                try {
                    for (int i = r0; i < Math.min(ids.length, r0 + WRITE_BATCH_ROWS); i++) {
                        org.apache.tinkerpop.gremlin.structure.Vertex v = null;
                        for (Map.Entry<String, Object> kv : values.entrySet()) {
                            Object x = program.valueAt(kv.getValue(), i);
                            if (x == null) continue;
                            if (v == null) v = tx.getVertex(ids[i]);
                            v.property(org.apache.tinkerpop.gremlin.structure.VertexProperty.Cardinality.single,
                                    kv.getKey(), x);
                        }
                    }
                    tx.commit();
                } catch (Exception e) {
                    throw new TitanException("Could not persist program results to graph", e);
                } finally {
                    if (tx.isOpen()) tx.rollback();
                }
            }
        }

        /** ResultGraph.ORIGINAL: device-encoded property entries as edgestore column overwrites. */
        static void persist(StandardTitanGraph graph, long ctx, DeviceProgram program) throws Exception {
            long[] keys = program.computeKeyIds(graph);
            int[] types = program.computeKeyTypes();
            long base = RelationIds.reserve(graph, keys.length * (long) TgoNative.vertexIds(ctx).length);
            Object[] rows = TgoNative.checked(ctx, TgoNative.resultRows(ctx, program.resultKind(), keys, types, base));
            long[] rowKeys = (long[]) rows[0], eb = (long[]) rows[1], bb = (long[]) rows[2], lv = (long[]) rows[3];
            byte[] data = (byte[]) rows[4];
            com.thinkaurelius.titan.diskstorage.keycolumnvalue.KeyColumnValueStoreManager mgr =
                    graph.getBackend().getStoreManager();
            String store = com.thinkaurelius.titan.diskstorage.Backend.EDGESTORE_NAME;
            for (int r0 = 0; r0 < rowKeys.length; r0 += WRITE_BATCH_ROWS) {
                Map<String, Map<com.thinkaurelius.titan.diskstorage.StaticBuffer,
                        com.thinkaurelius.titan.diskstorage.keycolumnvalue.KCVMutation>> batch = new HashMap<>();
                Map<com.thinkaurelius.titan.diskstorage.StaticBuffer,
                        com.thinkaurelius.titan.diskstorage.keycolumnvalue.KCVMutation> muts = new HashMap<>();
                for (int r = r0; r < Math.min(rowKeys.length, r0 + WRITE_BATCH_ROWS); r++) {
                    java.util.List<com.thinkaurelius.titan.diskstorage.Entry> adds = new java.util.ArrayList<>();
                    long start = 0;
                    for (int e = (int) eb[r]; e < eb[r + 1]; e++) {
                        int end = (int) (lv[e] >>> 32), vpos = (int) (lv[e] & 0x7FFFFFFF);
                        byte[] entry = java.util.Arrays.copyOfRange(data, (int) (bb[r] + start), (int) (bb[r] + end));
                        adds.add(com.thinkaurelius.titan.diskstorage.util.StaticArrayEntry.of(
                                new com.thinkaurelius.titan.diskstorage.util.StaticArrayBuffer(entry, 0, vpos),
                                new com.thinkaurelius.titan.diskstorage.util.StaticArrayBuffer(entry, vpos, entry.length)));
                        start = end;
                    }
                    muts.put(com.thinkaurelius.titan.diskstorage.util.BufferUtil.getLongBuffer(rowKeys[r]),
                            new com.thinkaurelius.titan.diskstorage.keycolumnvalue.KCVMutation(adds,
                                    java.util.Collections.emptyList()));
                }
                batch.put(store, muts);
                com.thinkaurelius.titan.diskstorage.keycolumnvalue.StoreTransaction tx =
                        mgr.beginTransaction(com.thinkaurelius.titan.diskstorage.util.StandardBaseTransactionConfig.of(
                                graph.getConfiguration().getTimestampProvider()));
                try {
                    mgr.mutateMany(batch, tx);
                    tx.commit();
                } catch (Exception e) {
                    tx.rollback();
                    throw new TitanException("Could not persist program results to graph", e);
                }
            }
        }

        /** ResultGraph.NEW: a new transaction holding the properties, not committed (:296-305). */
        static org.apache.tinkerpop.gremlin.structure.Graph localTx(StandardTitanGraph graph, long[] ids,
                                                                     Map<String, Object> values, DeviceProgram program) {
            com.thinkaurelius.titan.core.TitanTransaction tx = graph.newTransaction();
            for (Map.Entry<String, Object> kv : values.entrySet()) {
                for (int i = 0; i < ids.length; i++) {
                    Object v = program.valueAt(kv.getValue(), i);
                    if (v != null) tx.getVertex(ids[i]).property(
                            org.apache.tinkerpop.gremlin.structure.VertexProperty.Cardinality.single, kv.getKey(), v);
                }
            }
            return tx;
        }
    }

    /**
     * First id of a block of `count` consecutive relation ids for the written properties.  Titan
     * hands relation ids out of IDAuthority blocks per partition (VertexIDAssigner.java); the
     * device numbers entries base + i, so the host takes one block large enough from the
     * authority's relation namespace (the hook a maintainer wires to IDAuthority.getIDBlock).
     */
    static final class RelationIds {
        static long reserve(StandardTitanGraph graph, long count) {
            com.thinkaurelius.titan.diskstorage.IDBlock block = graph.getBackend().getIDAuthority()
                    .getIDBlock(0, com.thinkaurelius.titan.graphdb.database.idassigner.VertexIDAssigner.RELATION_NAMESPACE,
                            java.time.Duration.ofMinutes(1));
            if (block.numIds() < count)
                throw new TitanException("relation-id block of " + block.numIds() + " ids is smaller than " + count);
            return block.getId(0);
        }
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
        /** Write-back: tgo_result_kind, the compute keys (typed property keys) and their datatypes. */
        abstract int resultKind();
        abstract String[] computeKeys();
        abstract int[] computeKeyTypes();
        long[] computeKeyIds(StandardTitanGraph graph) {
            TitanManagement mgmt = graph.openManagement();
            try {
                String[] names = computeKeys();
                long[] out = new long[names.length];
                for (int i = 0; i < names.length; i++) {
                    PropertyKey k = mgmt.getPropertyKey(names[i]);
                    if (k == null || Schemas.datatype(k.dataType()) != computeKeyTypes()[i])
                        throw new TitanException("compute key '" + names[i] + "' must be a typed property key");
                    out[i] = ((com.thinkaurelius.titan.graphdb.internal.InternalRelationType) k).longId();
                }
                return out;
            } finally {
                mgmt.rollback();
            }
        }
        /** The multi-GPU form of the program, or null when it has none (then it runs on one device). */
        PartitionedRun.Program partitioned() { return null; }
        /** The value of compute-key array `values` at row i, null when the vertex holds none. */
        Object valueAt(Object values, int i) {
            if (values instanceof long[]) { long d = ((long[]) values)[i]; return d == TgoNative.DIST_ABSENT ? null : d; }
            if (values instanceof double[]) { double d = ((double[]) values)[i]; return Double.isNaN(d) ? null : d; }
            return ((int[]) values)[i];
        }

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
        int resultKind() { return TgoNative.RESULT_PAGERANK; }
        String[] computeKeys() { return new String[]{"titan.pageRank.pageRank", "titan.pageRank.edgeCount"}; }
        int[] computeKeyTypes() { return new int[]{TgoNative.DT_DOUBLE, TgoNative.DT_DOUBLE}; }
        Map<String, Object> run(long ctx) {
            Map<String, Object> v = new HashMap<>();
            v.put("titan.pageRank.pageRank", TgoNative.checked(ctx, TgoNative.pageRank(ctx, alpha, vertexCount, maxIterations)));
            return v;
        }
        PartitionedRun.Program partitioned() {
            return new PartitionedRun.Program() {
                public int scope() { return TgoNative.SCOPE_IN_E; }
                public boolean applyCap() { return true; }
                public boolean partitions(long n) { return n > 0; }
                public boolean needsNonNegativeWeights() { return false; }
                public Object run(long ctx, long x, long[] ownIds, long lo) {
                    return TgoNative.partPageRankRun(ctx, x, alpha, vertexCount, maxIterations,
                            PartitionedRun.PR_EXCHANGE_GHOST);
                }
            };
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
        int resultKind() { return TgoNative.RESULT_DISTANCE; }
        String[] computeKeys() { return new String[]{"titan.shortestDistanceVertexProgram.distance"}; }
        int[] computeKeyTypes() { return new int[]{TgoNative.DT_LONG}; }
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
        /**
         * Partitioned: delta-stepping's converged distances, which equal the hop-bounded result
         * only when no shortest path can exceed maxDepth hops — maxDepth >= n - 1 (a shortest
         * path visits each vertex once), n = the job's live vertices (known after the load) —
         * and only for non-negative weights (the reference's hop-bounded Jacobi takes any).
         */
        PartitionedRun.Program partitioned() {
            return new PartitionedRun.Program() {
                public int scope() { return TgoNative.SCOPE_IN_E; }
                public boolean applyCap() { return true; }
                public boolean partitions(long n) { return n > 0 && maxDepth >= n - 1; }
                public boolean needsNonNegativeWeights() { return true; }
                public Object run(long ctx, long x, long[] ownIds, long lo) {
                    // every worker runs the same phases (collectives); only the seed's owner
                    // seeds (a seed that is no live vertex reaches nobody: TGO_DIST_ABSENT)
                    long s = -1;
                    for (int i = 0; i < ownIds.length && s < 0; i++) if (ownIds[i] == seed) s = lo + i;
                    return TgoNative.partSsspRun(ctx, x, s, 0);
                }
            };
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
        int resultKind() { return TgoNative.RESULT_DEGREE; }
        String[] computeKeys() { return new String[]{"degree"}; }
        int[] computeKeyTypes() { return new int[]{TgoNative.DT_INTEGER}; }
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
