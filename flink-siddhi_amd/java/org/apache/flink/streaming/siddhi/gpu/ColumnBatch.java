package org.apache.flink.streaming.siddhi.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.HashMap;
import java.util.Map;

/**
 * Structure-of-arrays batch of one plan's input events: one direct buffer
 * per attribute (stream-definition order, the row order of
 * schema/StreamSerializer.java:38-66), the event timestamps and a per-row
 * input handle, so the streams of one definition (the Event type of the
 * ITCases feeding inputStream1 and inputStream2) share one batch in arrival
 * order — what the engine's event-time buffer needs between two watermarks.  It replaces
 * the per-event {@code Object[]} + {@code InputHandler.send} of
 * SiddhiStreamOperator.processEvent (operator/SiddhiStreamOperator.java:52-54):
 * rows are appended here and handed to libcep a batch at a time.
 *
 * Element layouts follow include/cep.h: INT int32, LONG int64, FLOAT float,
 * DOUBLE double, BOOL uint8, STRING int32 dictionary id (the operator's
 * shared dictionary, cached on this side so a repeated string costs no JNI
 * call).
 */
final class ColumnBatch {
    static final int INT = 0, LONG = 1, FLOAT = 2, DOUBLE = 3, BOOL = 4, STRING = 5;
    private static final int[] WIDTH = {4, 8, 4, 8, 1, 4};

    final long app;           // the plan's runtime (cep_app*)
    final String layout;      // attribute types, e.g. "0,5,3,1"
    private final int[] types;
    private final ByteBuffer ts;
    private final ByteBuffer stream;   // per-row input handle (cep_input)
    private int firstInput = -1;
    private final ByteBuffer[] cols;
    private final int capacity;
    private int n;
    private final long op;   // cep_operator* (string dictionary)
    private final Map<String, Integer> dict = new HashMap<>();

    ColumnBatch(long app, String layout, int[] types, int capacity, long op) {
        this.app = app;
        this.layout = layout;
        this.types = types.clone();
        this.capacity = capacity;
        this.op = op;
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

    boolean full() {
        return n == capacity;
    }

    /** One event of input `input` in StreamSerializer.getRow order. */
    void append(int input, Object[] row, long timestamp) {
        if (firstInput < 0) firstInput = input;
        ts.putLong(n * 8, timestamp);
        stream.put(n, (byte) input);
        for (int c = 0; c < types.length; ++c) {
            final Object v = row[c];
            final ByteBuffer b = cols[c];
            switch (types[c]) {
                case INT:
                    b.putInt(n * 4, v == null ? 0 : ((Number) v).intValue());
                    break;
                case LONG:
                    b.putLong(n * 8, v == null ? 0L : ((Number) v).longValue());
                    break;
                case FLOAT:
                    b.putFloat(n * 4, v == null ? 0f : ((Number) v).floatValue());
                    break;
                case DOUBLE:
                    b.putDouble(n * 8, v == null ? 0.0 : ((Number) v).doubleValue());
                    break;
                case BOOL:
                    b.put(n, (byte) (Boolean.TRUE.equals(v) ? 1 : 0));
                    break;
                default:
                    b.putInt(n * 4, intern(v == null ? "" : v.toString()));
                    break;
            }
        }
        ++n;
    }

    private int intern(String s) {
        Integer id = dict.get(s);
        if (id == null) {
            id = CepNative.operatorIntern(op, s);
            dict.put(s, id);
        }
        return id;
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
