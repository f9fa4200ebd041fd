package org.apache.flink.streaming.siddhi.gpu;

import java.nio.ByteBuffer;

/**
 * JNI entry points of libcep.so (include/cep.h), implemented by
 * flink-siddhi_amd/jni/cep_jni.c.  Handles are the C pointers as longs.
 * Status codes are returned as ints (0 = CEP_OK) and mapped onto the
 * reference's exceptions by {@link CepStatus#check}.
 *
 * Each method names the Siddhi call it replaces in
 * core/src/main/java/org/apache/flink/streaming/siddhi/operator/AbstractSiddhiOperator.java.
 */
final class CepNative {
    static {
        System.loadLibrary("cep_jni");   // libcep_jni.so, linked against libcep.so
    }

    private CepNative() {}

    /** Receives one output stream's rows during {@link #flush}: direct
     *  buffers over the engine's pinned delivery memory, valid only during the
     *  call (StreamCallback.receive, StreamOutputHandler.java:63). */
    interface RowSink {
        void receive(long n, ByteBuffer ts, ByteBuffer[] cols);
    }

    // ---- cep_operator: the QueryRuntimeHandler map (:112-176) ---------------
    /** cep_operator_create; options = {pending_slots, key_capacity, chunk_events,
     *  ordered_output, late_policy, sparse_keys}; err[0] receives the message. */
    static native long operatorCreate(int device, long[] options, String[] err);
    static native void operatorDestroy(long op);
    /** new QueryRuntimeHandler(enrichedPlan) + start() (:120-142, :416-424). */
    static native int operatorAddPlan(long op, String planId, String enrichedPlan);
    /** updated plans (:426-438): the old runtime is shut down. */
    static native int operatorUpdatePlan(long op, String planId, String enrichedPlan);
    /** deleted plans (:406-414). */
    static native int operatorRemovePlan(long op, String planId);
    /** OperationControlEvent ENABLE_QUERY / DISABLE_QUERY (:445-460). */
    static native int operatorEnable(long op, String planId, boolean enabled);
    /** The plan's runtime (cep_app*), 0 if unknown. */
    static native long operatorPlan(long op, String planId);
    static native int operatorIntern(long op, String s);
    static native String operatorLookup(long op, int id);
    static native String operatorLastError(long op);

    // ---- plan-level ----------------------------------------------------------
    /** The input streams a plan reads, newline separated (AddRouteOperator.java:159-175). */
    static native String planInputStreams(String plan);
    /** validateSiddhiApp (:292-299): status, message in err[0]. */
    static native int validate(String plan, String[] err);

    // ---- one plan's runtime (cep_app*) ----------------------------------------
    /** getStreamDefinitionMap().get(id) (:160-163): attribute names and cep_type codes. */
    static native int streamSchema(long app, String streamId, String[] names, int[] types, int[] n);
    /** getInputHandler (:172): handle >= 0 or -CEP_E_UNDEFINED_STREAM. */
    static native int input(long app, String streamId);
    /** addCallback(outId, StreamOutputHandler) (:165-166). */
    static native int setCallback(long app, String outId, RowSink sink);
    /** A batch of InputHandler.send(ts, row) (:130): columns in definition
     *  order, `stream` one input handle per row (u8). */
    static native int sendBatch(long app, int input, long n, ByteBuffer ts, ByteBuffer stream, ByteBuffer[] cols);
    /** processElement's PriorityQueue.offer (:222-231), on the device. */
    static native int bufferBatch(long app, int input, long n, ByteBuffer ts, ByteBuffer stream, ByteBuffer[] cols);
    /** processWatermark's drain (:238-245), on the device. */
    static native int watermark(long app, long mark);
    /** Deliver every match so far to the sinks (before emitWatermark :246). */
    static native int flush(long app);
    /** SiddhiAppRuntime.snapshot() (:374-380); null on failure. */
    static native byte[] snapshot(long app);
    /** The restore the reference leaves as a TODO (:341). */
    static native int restore(long app, byte[] state);
    static native String lastError(long app);
}
