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
 *   processEvent (SiddhiStreamOperator.java:52-54)  -> a row appended to the
 *       stream's columnar batch (ColumnBatch), no per-event send;
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
    private transient Map<String, ColumnBatch> batches;        // per (plan id, attribute layout)
    private transient Map<String, Set<String>> plansOfStream;  // input stream -> plan ids reading it
    private transient Map<String, Integer> inputs;             // (plan id, stream) -> cep_input handle
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
        batches = new HashMap<>();
        plansOfStream = new HashMap<>();
        inputs = new HashMap<>();
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
        // UndefinedStreamException for an unknown stream (SiddhiOperatorContext.java:151)
        final StreamSchema<IN> schema = siddhiPlan.getInputStreamSchema(streamId);
        final long ts = isProcessingTime ? System.currentTimeMillis() : element.getTimestamp();
        final Set<String> plans = plansOfStream.get(streamId);
        if (plans == null || plans.isEmpty()) return;   // no plan reads it
        final Object[] row = schema.getStreamSerializer().getRow(value.f1);
        // every plan reading the stream gets the event (AbstractSiddhiOperator.java:283-287)
        for (String id : plans) {
            final long app = CepNative.operatorPlan(op, id);
            final int[] types = inputTypes(app, streamId);
            final String layout = layoutOf(types);
            ColumnBatch b = batches.get(id + "|" + layout);
            if (b == null) {
                b = new ColumnBatch(app, layout, types, BATCH_ROWS, op);
                batches.put(id + "|" + layout, b);
            }
            b.append(inputOf(id, app, streamId), row, ts);
            if (b.full()) send(id, b);
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
    private void send(String id, ColumnBatch b) {
        CepStatus.check(b.send(!isProcessingTime), CepNative.lastError(b.app));
        b.clear();
        if (isProcessingTime) flushOne(id);
    }

    private void sendAll() {
        for (Map.Entry<String, ColumnBatch> e : batches.entrySet()) {
            if (e.getValue().size() > 0) send(e.getKey().substring(0, e.getKey().lastIndexOf('|')), e.getValue());
        }
    }

    private int inputOf(String id, long app, String streamId) {
        final String k = id + "|" + streamId;
        Integer h = inputs.get(k);
        if (h == null) {
            final int x = CepNative.input(app, streamId);
            if (x < 0) CepStatus.check(-x, CepNative.lastError(app));
            h = x;
            inputs.put(k, h);
        }
        return h;
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
                                                                   (org.apache.flink.streaming.api.operators.Output) output, op);
            sinks.add(h);
            CepStatus.check(CepNative.setCallback(app, e.getKey(), h), CepNative.lastError(app));
        }
        forget(id);
        final Set<String> layouts = new LinkedHashSet<>();
        for (String stream : CepNative.planInputStreams(plan).split("\n")) {
            if (stream.isEmpty()) continue;
            plansOfStream.computeIfAbsent(stream, k -> new LinkedHashSet<>()).add(id);
            layouts.add(layoutOf(inputTypes(app, stream)));
        }
        // the device event-time buffer holds one attribute layout between two
        // watermarks (cep_buffer_batch): streams of one definition mix freely
        if (!isProcessingTime && layouts.size() > 1)
            throw new CepStatus.UnsupportedPlanException(
                "plan " + id + " reads input streams of different definitions in event time");
    }

    /** A plan's routing entries, input handles and batches (removed / replaced). */
    private void forget(String id) {
        for (Set<String> s : plansOfStream.values()) s.remove(id);
        inputs.keySet().removeIf(k -> k.startsWith(id + "|"));
        batches.keySet().removeIf(k -> k.startsWith(id + "|"));
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
