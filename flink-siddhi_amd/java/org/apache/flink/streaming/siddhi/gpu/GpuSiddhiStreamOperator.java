package org.apache.flink.streaming.siddhi.gpu;

import java.nio.ByteBuffer;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.LinkedHashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;

import org.apache.flink.api.common.state.ListState;
import org.apache.flink.api.common.state.ListStateDescriptor;
import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.common.typeutils.base.array.BytePrimitiveArraySerializer;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.runtime.state.StateInitializationContext;
import org.apache.flink.runtime.state.StateSnapshotContext;
import org.apache.flink.streaming.api.TimeCharacteristic;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.streaming.siddhi.control.ControlEvent;
import org.apache.flink.streaming.siddhi.control.ControlEventListener;
import org.apache.flink.streaming.siddhi.control.MetadataControlEvent;
import org.apache.flink.streaming.siddhi.control.OperationControlEvent;
import org.apache.flink.streaming.siddhi.operator.SiddhiOperatorContext;
import org.apache.flink.streaming.siddhi.router.StreamRoute;
import org.apache.flink.streaming.siddhi.schema.StreamSchema;

/**
 * Drop-in for SiddhiStreamOperator (operator/SiddhiStreamOperator.java) that
 * runs every execution plan on libcep (MI355X) instead of Siddhi.
 *
 * It keeps the reference operator's contract: input {@code Tuple2<StreamRoute, IN>},
 * the control stream (onEventReceived, AbstractSiddhiOperator.java:400-467),
 * event time through watermarks, output records formatted by type
 * (StreamOutputHandler.java:63-92) and the state names
 * "siddhiRuntimeState" / "queuedRecordsState" (AbstractSiddhiOperator.java:97-98).
 * It is a sibling of AbstractSiddhiOperator rather than a subclass: that
 * class creates its Siddhi runtimes in private code (startSiddhiManager,
 * :301-313) and keeps its PriorityQueue private.
 *
 * Where the work goes:
 *   processEvent (SiddhiStreamOperator.java:52-54)  -> the record's fields
 *       written straight into each reading plan's columnar batch (RowWriter
 *       into ColumnBatch: no getRow boxing, no per-event send).  Everything
 *       per (plan, stream) — the runtime, its input handle, the attribute
 *       types, the batch — is resolved once when the plan starts, so an event
 *       costs no JNI call and (for POJOs with primitive fields) no allocation;
 *   processElement, event time (:222-231)       -> full batches go to
 *       cep_buffer_batch: the device holds the out-of-order rows, not a
 *       PriorityQueue serialised on every event (:231);
 *   processWatermark (:238-247)                 -> cep_watermark (stable device
 *       sort by (ts, arrival), rows <= mark released), cep_flush (callbacks
 *       collect the matches), then emitWatermark;
 *   snapshotState (:331-393)                    -> cep_snapshot per plan into
 *       "siddhiRuntimeState"; initializeState restores it (a TODO upstream,
 *       :341).  The device reorder buffer is part of that snapshot, so
 *       "queuedRecordsState" stays empty, as after the reference's
 *       checkpointSiddhiRuntimeState (:379).
 * Processing time stamps rows with the wall clock (:218-219) and delivers a
 * batch's matches when the batch is sent (batch full, watermark, checkpoint
 * barrier or close) instead of inside every send.
 *
 * A plan outside the engine subset (joins, windows, tables) throws
 * CepStatus.UnsupportedPlanException from the constructor, so a factory can
 * build the stock SiddhiStreamOperator instead:
 * <pre>
 *   try { op = new GpuSiddhiStreamOperator<>(ctx); }
 *   catch (CepStatus.UnsupportedPlanException e) { op = new SiddhiStreamOperator<>(ctx); }
 * </pre>
 * (utils/SiddhiStreamFactory.java:33-38 is where that choice goes.)
 */
public class GpuSiddhiStreamOperator<IN, OUT> extends AbstractStreamOperator<OUT>
    implements OneInputStreamOperator<Tuple2<StreamRoute, IN>, OUT>, ControlEventListener {

    private static final String SIDDHI_RUNTIME_STATE_NAME = "siddhiRuntimeState";
    private static final String QUEUED_RECORDS_STATE_NAME = "queuedRecordsState";
    private static final int BATCH_ROWS = 1 << 16;

    private final SiddhiOperatorContext siddhiPlan;
    private final boolean isProcessingTime;
    private final long[] engineOptions;

    private transient long op;                                // cep_operator*
    private transient Dictionary dict;                         // the operator's string dictionary
    private transient Map<String, ColumnBatch> batches;        // per (plan id, attribute layout)
    private transient Map<String, Map<String, Target>> planInputs;  // plan id -> stream -> target
    private transient Map<String, Target[]> routes;            // input stream -> the plans reading it
    private transient Map<String, RowWriter<IN>> writers;      // input stream -> field writer
    private transient List<CepNative.RowSink> sinks;           // kept reachable while native code holds them
    private transient ListState<byte[]> siddhiRuntimeState;
    private transient ListState<byte[]> queuedRecordsState;
    private transient Map<String, byte[]> restored;            // plan id -> engine snapshot

    public GpuSiddhiStreamOperator(SiddhiOperatorContext siddhiPlan) {
        this(siddhiPlan, new long[] {16, 1L << 20, 1L << 22, 1, 0, 1});
    }

    /** engineOptions = {pending_slots, key_capacity, chunk_events,
     *  ordered_output, late_policy, sparse_keys} (cep_options). */
    public GpuSiddhiStreamOperator(SiddhiOperatorContext siddhiPlan, long[] engineOptions) {
        // fail fast at DAG build, as AbstractSiddhiOperator.validate (:292-299)
        final String[] err = new String[1];
        CepStatus.check(CepNative.validate(siddhiPlan.getAllEnrichedExecutionPlan(), err), err[0]);
        this.siddhiPlan = siddhiPlan;
        this.isProcessingTime = siddhiPlan.getTimeCharacteristic() == TimeCharacteristic.ProcessingTime;
        this.engineOptions = engineOptions.clone();
    }

    // ---- lifecycle ------------------------------------------------------------
    @Override
    public void open() throws Exception {
        super.open();
        final String[] err = new String[1];
        op = CepNative.operatorCreate(0, engineOptions, err);
        if (op == 0) throw new IllegalStateException("libcep: " + err[0]);
        dict = new Dictionary(op);
        batches = new HashMap<>();
        planInputs = new HashMap<>();
        routes = new HashMap<>();
        writers = new HashMap<>();
        sinks = new ArrayList<>();
        for (String id : siddhiPlan.getExecutionPlanMap().keySet()) startPlan(id, false);
        if (restored != null) {
            for (Map.Entry<String, byte[]> e : restored.entrySet()) {
                final long app = CepNative.operatorPlan(op, e.getKey());
                if (app != 0) CepStatus.check(CepNative.restore(app, e.getValue()), CepNative.lastError(app));
            }
            restored = null;
        }
    }

    @Override
    public void close() throws Exception {
        sendAll();
        flushAll();
        CepNative.operatorDestroy(op);
        op = 0;
        super.close();
    }

    // ---- input -----------------------------------------------------------------
    @Override
    public void processElement(StreamRecord<Tuple2<StreamRoute, IN>> element) throws Exception {
        final Tuple2<StreamRoute, IN> value = element.getValue();
        final String streamId = value.f0.getInputStreamId();
        if (ControlEvent.DEFAULT_INTERNAL_CONTROL_STREAM.equals(streamId)) {
            // rows before the control event reach the plans that were live then
            sendAll();
            onEventReceived((ControlEvent) value.f1);
            return;
        }
        final Target[] targets = routes.get(streamId);
        if (targets == null) {
            // UndefinedStreamException for an unknown stream (SiddhiOperatorContext.java:151);
            // a known stream no plan reads is dropped
            siddhiPlan.getInputStreamSchema(streamId);
            return;
        }
        final long ts = isProcessingTime ? System.currentTimeMillis() : element.getTimestamp();
        final RowWriter<IN> w = writers.get(streamId);
        // every plan reading the stream gets the event (AbstractSiddhiOperator.java:283-287)
        for (int i = 0; i < targets.length; ++i) {
            final Target t = targets[i];
            final ColumnBatch b = t.batch;
            w.write(value.f1, b, b.begin(t.input, ts));
            b.commit();
            if (b.full()) send(b);
        }
    }

    /** One (plan, input stream) pair, resolved once in startPlan. */
    private static final class Target {
        final String planId;
        final int input;          // cep_input handle
        final ColumnBatch batch;  // the plan's batch for the stream's attribute layout

        Target(String planId, int input, ColumnBatch batch) {
            this.planId = planId;
            this.input = input;
            this.batch = batch;
        }
    }

    @Override
    public void processWatermark(Watermark mark) throws Exception {
        sendAll();
        if (!isProcessingTime) {
            for (String id : siddhiPlan.getExecutionPlanMap().keySet()) {
                final long app = CepNative.operatorPlan(op, id);
                CepStatus.check(CepNative.watermark(app, mark.getTimestamp()), CepNative.lastError(app));
            }
        }
        flushAll();   // matches precede the watermark (:246)
        output.emitWatermark(mark);
    }

    /** A plan's batch to its runtime (disabled plans drop the rows at
     *  release time, as QueryRuntimeHandler.send does, :127-132). */
    private void send(ColumnBatch b) {
        final int rc = b.send(!isProcessingTime);
        if (rc != CepStatus.OK) CepStatus.check(rc, CepNative.lastError(b.app));
        b.clear();
        if (isProcessingTime) {
            final int f = CepNative.flush(b.app);
            if (f != CepStatus.OK) CepStatus.check(f, CepNative.lastError(b.app));
        }
    }

    private void sendAll() {
        for (ColumnBatch b : batches.values()) {
            if (b.size() > 0) send(b);
        }
    }

    /** routes (stream -> targets) from planInputs, after a plan change. */
    private void rebuildRoutes() {
        final Map<String, List<Target>> m = new HashMap<>();
        for (Map<String, Target> byStream : planInputs.values())
            for (Map.Entry<String, Target> e : byStream.entrySet())
                m.computeIfAbsent(e.getKey(), k -> new ArrayList<>()).add(e.getValue());
        routes = new HashMap<>();
        for (Map.Entry<String, List<Target>> e : m.entrySet())
            routes.put(e.getKey(), e.getValue().toArray(new Target[0]));
    }

    private static String layoutOf(int[] types) {
        final StringBuilder sb = new StringBuilder();
        for (int t : types) sb.append(t).append(',');
        return sb.toString();
    }

    private void flushAll() {
        for (String id : siddhiPlan.getExecutionPlanMap().keySet()) {
            final long app = CepNative.operatorPlan(op, id);
            if (app != 0) CepStatus.check(CepNative.flush(app), CepNative.lastError(app));
        }
    }

    private static int[] inputTypes(long app, String streamId) {
        final String[] names = new String[64];
        final int[] types = new int[64];
        final int[] n = new int[1];
        CepStatus.check(CepNative.streamSchema(app, streamId, names, types, n), CepNative.lastError(app));
        final int[] t = new int[n[0]];
        System.arraycopy(types, 0, t, 0, n[0]);
        return t;
    }

    // ---- plans -------------------------------------------------------------------
    /** new QueryRuntimeHandler(plan).start() (:120-142): the runtime, its
     *  output callbacks (registerInputAndOutput, :159-175) and its inputs. */
    @SuppressWarnings("unchecked")
    private void startPlan(String id, boolean update) {
        final String plan = siddhiPlan.getEnrichedExecutionPlan(id);
        final int rc = update ? CepNative.operatorUpdatePlan(op, id, plan) : CepNative.operatorAddPlan(op, id, plan);
        CepStatus.check(rc, CepNative.operatorLastError(op));
        final long app = CepNative.operatorPlan(op, id);
        for (Map.Entry<String, TypeInformation> e : siddhiPlan.getOutputStreamTypes().entrySet()) {
            final String[] names = new String[64];
            final int[] types = new int[64];
            final int[] n = new int[1];
            if (CepNative.streamSchema(app, e.getKey(), names, types, n) != CepStatus.OK) continue;   // not this plan's
            final String[] nm = new String[n[0]];
            final int[] ty = new int[n[0]];
            System.arraycopy(names, 0, nm, 0, n[0]);
            System.arraycopy(types, 0, ty, 0, n[0]);
            final GpuOutputHandler<OUT> h = new GpuOutputHandler<>(e.getKey(), (TypeInformation<OUT>) e.getValue(), nm, ty,
                                                                   (org.apache.flink.streaming.api.operators.Output) output, dict);
            sinks.add(h);
            CepStatus.check(CepNative.setCallback(app, e.getKey(), h), CepNative.lastError(app));
        }
        forget(id);
        // resolve everything an event of each input stream needs, once
        final Set<String> layouts = new LinkedHashSet<>();
        final Map<String, Target> byStream = new HashMap<>();
        for (String stream : CepNative.planInputStreams(plan).split("\n")) {
            if (stream.isEmpty()) continue;
            final int[] types = inputTypes(app, stream);
            final String layout = layoutOf(types);
            layouts.add(layout);
            final int h = CepNative.input(app, stream);
            if (h < 0) CepStatus.check(-h, CepNative.lastError(app));
            ColumnBatch b = batches.get(id + "|" + layout);
            if (b == null) {
                b = new ColumnBatch(app, id, layout, types, BATCH_ROWS, dict);
                batches.put(id + "|" + layout, b);
            }
            RowWriter<IN> w = writers.get(stream);
            if (w == null) {
                final StreamSchema<IN> schema = siddhiPlan.getInputStreamSchema(stream);
                w = new RowWriter<>(schema);
                writers.put(stream, w);
            }
            if (w.arity() != b.arity())
                throw new IllegalArgumentException("stream " + stream + ": " + w.arity() + " fields, plan " + id
                                                   + " defines " + b.arity() + " attributes");
            byStream.put(stream, new Target(id, h, b));
        }
        // the device event-time buffer holds one attribute layout between two
        // watermarks (cep_buffer_batch): streams of one definition mix freely
        if (!isProcessingTime && layouts.size() > 1)
            throw new CepStatus.UnsupportedPlanException(
                "plan " + id + " reads input streams of different definitions in event time");
        planInputs.put(id, byStream);
        rebuildRoutes();
    }

    /** A plan's routing entries, input handles and batches (removed / replaced). */
    private void forget(String id) {
        planInputs.remove(id);
        batches.keySet().removeIf(k -> k.startsWith(id + "|"));
        rebuildRoutes();
    }

    @Override
    public void onEventReceived(ControlEvent event) {
        if (event instanceof MetadataControlEvent) {
            final MetadataControlEvent m = (MetadataControlEvent) event;
            if (m.getDeletedExecutionPlanId() != null) {
                for (String id : m.getDeletedExecutionPlanId()) {
                    siddhiPlan.removeExecutionPlan(id);
                    CepNative.operatorRemovePlan(op, id);   // unknown ids are ignored
                    forget(id);
                }
            }
            if (m.getAddedExecutionPlanMap() != null) {
                for (Map.Entry<String, String> e : m.getAddedExecutionPlanMap().entrySet()) {
                    siddhiPlan.addExecutionPlan(e.getKey(), e.getValue());
                    startPlan(e.getKey(), false);
                }
            }
            if (m.getUpdatedExecutionPlanMap() != null) {
                for (Map.Entry<String, String> e : m.getUpdatedExecutionPlanMap().entrySet()) {
                    siddhiPlan.updateExecutionPlan(e.getKey(), e.getValue());
                    flushOne(e.getKey());   // the old runtime's matches go out before it is replaced
                    startPlan(e.getKey(), true);
                }
            }
        } else if (event instanceof OperationControlEvent) {
            final OperationControlEvent o = (OperationControlEvent) event;
            if (o.getAction() == null) return;
            switch (o.getAction()) {
                case ENABLE_QUERY:
                    CepNative.operatorEnable(op, o.getQueryId(), true);
                    break;
                case DISABLE_QUERY:
                    CepNative.operatorEnable(op, o.getQueryId(), false);
                    break;
                default:
                    throw new IllegalStateException("Illegal action type " + o.getAction() + ": " + event);
            }
        } else {
            throw new IllegalStateException("Illegal event type " + event);
        }
    }

    private void flushOne(String id) {
        final long app = CepNative.operatorPlan(op, id);
        if (app != 0) CepStatus.check(CepNative.flush(app), CepNative.lastError(app));
    }

    // ---- state -------------------------------------------------------------------
    @Override
    public void prepareSnapshotPreBarrier(long checkpointId) throws Exception {
        super.prepareSnapshotPreBarrier(checkpointId);
        // buffered rows into the engine (its reorder buffer is snapshotted) and
        // every match so far out before the barrier
        sendAll();
        flushAll();
    }

    @Override
    public void snapshotState(StateSnapshotContext context) throws Exception {
        super.snapshotState(context);
        siddhiRuntimeState.clear();
        final int subtask = getRuntimeContext().getIndexOfThisSubtask();
        for (String id : siddhiPlan.getExecutionPlanMap().keySet()) {
            final long app = CepNative.operatorPlan(op, id);
            final byte[] s = CepNative.snapshot(app);
            if (s == null) throw new IllegalStateException("cep_snapshot: " + CepNative.lastError(app));
            siddhiRuntimeState.add(frame(subtask, id, s));
        }
        queuedRecordsState.clear();
    }

    @Override
    public void initializeState(StateInitializationContext context) throws Exception {
        super.initializeState(context);
        siddhiRuntimeState = context.getOperatorStateStore().getUnionListState(
            new ListStateDescriptor<>(SIDDHI_RUNTIME_STATE_NAME, new BytePrimitiveArraySerializer()));
        queuedRecordsState = context.getOperatorStateStore().getListState(
            new ListStateDescriptor<>(QUEUED_RECORDS_STATE_NAME, new BytePrimitiveArraySerializer()));
        if (context.isRestored()) {
            // union state hands every subtask all entries: take this subtask's
            // (same parallelism; a rescale would need the engine state split by key)
            restored = new HashMap<>();
            final int subtask = getRuntimeContext().getIndexOfThisSubtask();
            for (byte[] f : siddhiRuntimeState.get()) {
                final ByteBuffer b = ByteBuffer.wrap(f);
                final int st = b.getInt();
                final byte[] idb = new byte[b.getInt()];
                b.get(idb);
                final byte[] s = new byte[b.remaining()];
                b.get(s);
                if (st == subtask) restored.put(new String(idb, StandardCharsets.UTF_8), s);
            }
        }
    }

    /** [subtask i32][plan id length i32][plan id utf-8][engine snapshot] */
    private static byte[] frame(int subtask, String id, byte[] s) {
        final byte[] idb = id.getBytes(StandardCharsets.UTF_8);
        final ByteBuffer b = ByteBuffer.allocate(8 + idb.length + s.length);
        b.putInt(subtask).putInt(idb.length).put(idb).put(s);
        return b.array();
    }
}
