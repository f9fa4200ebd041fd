package org.apache.flink.streaming.siddhi.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/**
 * Structure-of-arrays batch of one plan's input events: one direct buffer
 * per attribute (stream-definition order, the row order of
 * schema/StreamSerializer.java:38-66), the event timestamps and a per-row
 * input handle, so the streams of one definition (the Event type of the
 * ITCases feeding inputStream1 and inputStream2) share one batch in arrival
 * order — what the engine's event-time buffer needs between two watermarks.
 * It replaces the per-event {@code Object[]} + {@code InputHandler.send} of
 * SiddhiStreamOperator.processEvent (operator/SiddhiStreamOperator.java:52-54):
 * a {@link RowWriter} stores each record's fields here with typed puts (no
 * boxing) and the rows go to libcep a batch at a time.
 *
 * Element layouts follow include/cep.h: INT int32, LONG int64, FLOAT float,
 * DOUBLE double, BOOL uint8, STRING int32 dictionary id (the operator's
 * shared {@link Dictionary}: a repeated string costs no JNI call).
 * Conversions between a field's Java type and the attribute type follow
 * Java's primitive conversions, as Siddhi's Number.xxxValue() reads do.
 */
final class ColumnBatch {
    static final int INT = 0, LONG = 1, FLOAT = 2, DOUBLE = 3, BOOL = 4, STRING = 5;
    private static final int[] WIDTH = {4, 8, 4, 8, 1, 4};

    final long app;           // the plan's runtime (cep_app*)
    final String planId;
    final String layout;      // attribute types, e.g. "0,5,3,1"
    private final int[] types;
    private final ByteBuffer ts;
    private final ByteBuffer stream;   // per-row input handle (cep_input)
    private int firstInput = -1;
    private final ByteBuffer[] cols;
    private final int capacity;
    private int n;
    private final Dictionary dict;

    ColumnBatch(long app, String planId, String layout, int[] types, int capacity, Dictionary dict) {
        this.app = app;
        this.planId = planId;
        this.layout = layout;
        this.types = types.clone();
        this.capacity = capacity;
        this.dict = dict;
        this.ts = ByteBuffer.allocateDirect(capacity * 8).order(ByteOrder.nativeOrder());
        this.stream = ByteBuffer.allocateDirect(capacity);
        this.cols = new ByteBuffer[types.length];
        for (int c = 0; c < types.length; ++c) {
            if (types[c] < INT || types[c] > STRING)
                throw new CepStatus.UnsupportedPlanException("attribute type OBJECT in layout " + layout);
            cols[c] = ByteBuffer.allocateDirect(capacity * WIDTH[types[c]]).order(ByteOrder.nativeOrder());
        }
    }

    int size() {
        return n;
    }

    int arity() {
        return types.length;
    }

    boolean full() {
        return n == capacity;
    }

    /** Open the next row (event of input `input` at `timestamp`); the caller
     *  writes its attributes with the put methods, then {@link #commit}s. */
    int begin(int input, long timestamp) {
        if (firstInput < 0) firstInput = input;
        ts.putLong(n * 8, timestamp);
        stream.put(n, (byte) input);
        return n;
    }

    void commit() {
        ++n;
    }

    void putLong(int c, int r, long v) {
        final ByteBuffer b = cols[c];
        switch (types[c]) {
            case INT:
            case STRING:   // not reached for well-typed plans; an id is an int
                b.putInt(r * 4, (int) v);
                break;
            case LONG:
                b.putLong(r * 8, v);
                break;
            case FLOAT:
                b.putFloat(r * 4, (float) v);
                break;
            case DOUBLE:
                b.putDouble(r * 8, (double) v);
                break;
            default:
                b.put(r, (byte) (v != 0 ? 1 : 0));
                break;
        }
    }

    void putDouble(int c, int r, double v) {
        final ByteBuffer b = cols[c];
        switch (types[c]) {
            case FLOAT:
                b.putFloat(r * 4, (float) v);
                break;
            case DOUBLE:
                b.putDouble(r * 8, v);
                break;
            case LONG:
                b.putLong(r * 8, (long) v);
                break;
            case BOOL:
                b.put(r, (byte) (v != 0 ? 1 : 0));
                break;
            default:
                b.putInt(r * 4, (int) v);
                break;
        }
    }

    void putBool(int c, int r, boolean v) {
        if (types[c] == BOOL) cols[c].put(r, (byte) (v ? 1 : 0));
        else putLong(c, r, v ? 1 : 0);
    }

    /** A field that is already an object (Tuple / Row fields, atomic records,
     *  String or boxed POJO fields).  Null numeric values are stored as 0 (the
     *  engine has no null columns). */
    void putObject(int c, int r, Object v) {
        switch (types[c]) {
            case STRING:
                cols[c].putInt(r * 4, dict.intern(v == null ? "" : v.toString()));
                break;
            case BOOL:
                cols[c].put(r, (byte) (Boolean.TRUE.equals(v) ? 1 : 0));
                break;
            case FLOAT:
            case DOUBLE:
                putDouble(c, r, v == null ? 0.0 : ((Number) v).doubleValue());
                break;
            default:
                putLong(c, r, v == null ? 0L : ((Number) v).longValue());
                break;
        }
    }

    /** The batch to one plan's runtime: a device-side PriorityQueue offer
     *  (event time) or direct sends (processing time). */
    int send(boolean eventTime) {
        if (n == 0) return CepStatus.OK;
        return eventTime ? CepNative.bufferBatch(app, firstInput, n, ts, stream, cols)
                         : CepNative.sendBatch(app, firstInput, n, ts, stream, cols);
    }

    /** libcep has consumed the rows (cep_send_batch / cep_buffer_batch copy
     *  host batches before returning): the buffers are reused. */
    void clear() {
        n = 0;
        firstInput = -1;
    }
}
