package org.apache.flink.streaming.siddhi.gpu;

import java.lang.reflect.Field;

import org.apache.flink.api.java.tuple.Tuple;
import org.apache.flink.api.java.typeutils.TypeExtractor;
import org.apache.flink.streaming.siddhi.schema.StreamSchema;
import org.apache.flink.types.Row;

/**
 * Writes one input record straight into a {@link ColumnBatch} row, in the
 * attribute order of StreamSerializer.getRow
 * (core/.../schema/StreamSerializer.java:38-66), without building the boxed
 * {@code Object[]} that getRow returns.
 *
 * Built once per input stream.  POJO and case-class fields are resolved once
 * (the reference looks every field up reflectively per event: "TODO: Cache
 * Field Accessor", StreamSerializer.java:68-82) and primitive fields are read
 * with the primitive accessors ({@code Field.getInt/getLong/getDouble/...}),
 * so an event of the ITCases' Event POJO costs no allocation at all.  Tuple
 * and Row fields are already objects inside the record and are read as they
 * are.
 */
final class RowWriter<T> {
    private static final int ATOMIC = 0, TUPLE = 1, ROW = 2, FIELDS = 3;
    private static final int P_OBJECT = 0, P_INT = 1, P_LONG = 2, P_FLOAT = 3, P_DOUBLE = 4, P_BOOL = 5,
        P_SHORT = 6, P_BYTE = 7;

    private final int kind;
    private final Class<?> typeClass;
    private final String typeName;
    private final int[] index;        // TUPLE / ROW: field positions (StreamSchema.getFieldIndexes)
    private final Field[] fields;     // FIELDS: accessors, resolved once
    private final int[] prim;         // FIELDS: primitive accessor per field

    RowWriter(StreamSchema<T> schema) {
        this.typeClass = schema.getTypeInfo().getTypeClass();
        this.typeName = String.valueOf(schema.getTypeInfo());
        this.index = schema.getFieldIndexes().clone();
        if (schema.isAtomicType()) {
            kind = ATOMIC;
            fields = null;
            prim = null;
        } else if (schema.isTupleType()) {
            kind = TUPLE;
            fields = null;
            prim = null;
        } else if (schema.isRowType()) {
            kind = ROW;
            fields = null;
            prim = null;
        } else if (schema.isPojoType() || schema.isCaseClassType()) {
            kind = FIELDS;
            final String[] names = schema.getFieldNames();
            fields = new Field[names.length];
            prim = new int[names.length];
            for (int i = 0; i < names.length; ++i) {
                final Field f = TypeExtractor.getDeclaredField(typeClass, names[i]);
                if (f == null) throw new IllegalArgumentException(names[i] + " is not found in " + typeName);
                if (!f.isAccessible()) f.setAccessible(true);
                fields[i] = f;
                final Class<?> c = f.getType();
                prim[i] = c == int.class ? P_INT : c == long.class ? P_LONG : c == float.class ? P_FLOAT
                    : c == double.class ? P_DOUBLE : c == boolean.class ? P_BOOL : c == short.class ? P_SHORT
                    : c == byte.class ? P_BYTE : P_OBJECT;
            }
        } else {
            throw new IllegalArgumentException("Failed to get field values from " + typeName);
        }
    }

    /** Number of attributes a record yields (the stream definition's arity). */
    int arity() {
        return kind == ATOMIC ? 1 : kind == FIELDS ? fields.length : index.length;
    }

    /** Record `input` into row `r` of `b`. */
    void write(T input, ColumnBatch b, int r) {
        // the type check of StreamSerializer.getRow (:39-40); its message is
        // built only on failure
        if (input.getClass() != typeClass)
            throw new IllegalArgumentException("Invalid input type: " + input + ", expected: " + typeName);
        switch (kind) {
            case ATOMIC:
                b.putObject(0, r, input);
                return;
            case TUPLE: {
                final Tuple t = (Tuple) input;
                for (int i = 0; i < index.length; ++i) b.putObject(i, r, t.getField(index[i]));
                return;
            }
            case ROW: {
                final Row row = (Row) input;
                for (int i = 0; i < index.length; ++i) b.putObject(i, r, row.getField(index[i]));
                return;
            }
            default:
                try {
                    for (int i = 0; i < fields.length; ++i) {
                        final Field f = fields[i];
                        switch (prim[i]) {
                            case P_INT:
                                b.putLong(i, r, f.getInt(input));
                                break;
                            case P_LONG:
                                b.putLong(i, r, f.getLong(input));
                                break;
                            case P_SHORT:
                                b.putLong(i, r, f.getShort(input));
                                break;
                            case P_BYTE:
                                b.putLong(i, r, f.getByte(input));
                                break;
                            case P_FLOAT:
                                b.putDouble(i, r, f.getFloat(input));
                                break;
                            case P_DOUBLE:
                                b.putDouble(i, r, f.getDouble(input));
                                break;
                            case P_BOOL:
                                b.putBool(i, r, f.getBoolean(input));
                                break;
                            default:
                                b.putObject(i, r, f.get(input));
                                break;
                        }
                    }
                } catch (IllegalAccessException e) {
                    throw new IllegalStateException(e.getMessage(), e);
                }
        }
    }
}
