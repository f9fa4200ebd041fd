package org.apache.flink.streaming.siddhi.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.Map;
import java.util.TreeMap;

import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.java.tuple.Tuple;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.typeutils.PojoTypeInfo;
import org.apache.flink.shaded.jackson2.com.fasterxml.jackson.databind.DeserializationFeature;
import org.apache.flink.shaded.jackson2.com.fasterxml.jackson.databind.ObjectMapper;
import org.apache.flink.streaming.api.operators.Output;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.streaming.siddhi.utils.GenericRecord;
import org.apache.flink.streaming.siddhi.utils.SiddhiTupleFactory;
import org.apache.flink.types.Row;

/**
 * Columnar libcep output -> Flink records, formatted exactly as
 * StreamOutputHandler.receive formats Siddhi events
 * (operator/StreamOutputHandler.java:63-92): Map / GenericRecord with keys
 * sorted by attribute name (a TreeMap, :103-109), Row in definition order,
 * Tuple, POJO through Jackson, else IllegalArgumentException (:89).  Each
 * record is collected with the completing event's timestamp.  Rows arrive in
 * Siddhi's emission order (cep_options.ordered_output = 1).  STRING cells
 * are dictionary ids resolved through the operator's cached {@link
 * Dictionary}: a string seen before costs no JNI call and no new String.
 */
final class GpuOutputHandler<R> implements CepNative.RowSink {
    private final String outputStreamId;
    private final TypeInformation<R> typeInfo;
    private final String[] names;
    private final int[] types;
    private final Output<StreamRecord<R>> output;
    private final Dictionary dict;   // the operator's string dictionary (cached: no JNI per cell)
    private final ObjectMapper objectMapper = new ObjectMapper();

    GpuOutputHandler(String outputStreamId, TypeInformation<R> typeInfo, String[] names, int[] types,
                     Output<StreamRecord<R>> output, Dictionary dict) {
        this.outputStreamId = outputStreamId;
        this.typeInfo = typeInfo;
        this.names = names;
        this.types = types;
        this.output = output;
        this.dict = dict;
        this.objectMapper.configure(DeserializationFeature.FAIL_ON_UNKNOWN_PROPERTIES, false);
    }

    @Override
    @SuppressWarnings("unchecked")
    public void receive(long n, ByteBuffer ts, ByteBuffer[] cols) {
        ts.order(ByteOrder.nativeOrder());
        for (ByteBuffer c : cols) c.order(ByteOrder.nativeOrder());
        final StreamRecord<R> reusable = new StreamRecord<>(null, 0L);
        final Object[] data = new Object[names.length];
        for (int i = 0; i < (int) n; ++i) {
            for (int c = 0; c < names.length; ++c) data[c] = value(cols[c], types[c], i);
            final long t = ts.getLong(i * 8);
            final Object out;
            final Class<?> cls = typeInfo == null ? null : typeInfo.getTypeClass();
            if (typeInfo == null || Map.class.isAssignableFrom(cls) || GenericRecord.class.isAssignableFrom(cls)) {
                out = new GenericRecord(map(data));
            } else if (Row.class.isAssignableFrom(cls)) {
                out = Row.of(data.clone());
            } else if (typeInfo.isTupleType()) {
                final Tuple tuple = SiddhiTupleFactory.newTuple(data.clone());
                out = tuple;
            } else if (typeInfo instanceof PojoTypeInfo) {
                out = objectMapper.convertValue(map(data), cls);
            } else {
                throw new IllegalArgumentException("Unable to format row of " + outputStreamId + " as type " + typeInfo);
            }
            reusable.replace((R) Tuple2.of(outputStreamId, out), t);
            output.collect(reusable);
        }
    }

    private TreeMap<String, Object> map(Object[] data) {
        final TreeMap<String, Object> m = new TreeMap<>();
        for (int c = 0; c < names.length; ++c) m.put(names[c], data[c]);
        return m;
    }

    private Object value(ByteBuffer b, int type, int i) {
        switch (type) {
            case ColumnBatch.INT:
                return b.getInt(i * 4);
            case ColumnBatch.LONG:
                return b.getLong(i * 8);
            case ColumnBatch.FLOAT:
                return b.getFloat(i * 4);
            case ColumnBatch.DOUBLE:
                return b.getDouble(i * 8);
            case ColumnBatch.BOOL:
                return b.get(i) != 0;
            default:
                return dict.lookup(b.getInt(i * 4));
        }
    }
}
