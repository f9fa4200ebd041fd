package org.apache.flink.streaming.siddhi.gpu;

import java.util.ArrayList;
import java.util.HashMap;
import java.util.Map;

/**
 * The operator's string dictionary (cep_operator_intern / cep_operator_lookup),
 * cached on the Java side in both directions: a string seen before costs a
 * HashMap lookup on input and an array read on output, no JNI crossing and
 * no new String.  Only the first occurrence of a string (or of an id the
 * engine produced, e.g. a constant in a select) goes through JNI.
 *
 * Siddhi keeps strings as Java objects inside its events; the engine keeps
 * them as int32 ids in its columns (include/cep.h, CEP_STRING).
 */
final class Dictionary {
    private final long op;   // cep_operator*
    private final Map<String, Integer> ids = new HashMap<>();
    private final ArrayList<String> strings = new ArrayList<>();

    Dictionary(long op) {
        this.op = op;
    }

    int intern(String s) {
        final Integer id = ids.get(s);
        if (id != null) return id;
        final int x = CepNative.operatorIntern(op, s);
        ids.put(s, x);
        remember(x, s);
        return x;
    }

    String lookup(int id) {
        if (id >= 0 && id < strings.size()) {
            final String s = strings.get(id);
            if (s != null) return s;
        }
        final String s = CepNative.operatorLookup(op, id);
        if (s != null && id >= 0) {
            remember(id, s);
            ids.putIfAbsent(s, id);
        }
        return s;
    }

    private void remember(int id, String s) {
        if (id < 0) return;
        while (strings.size() <= id) strings.add(null);
        strings.set(id, s);
    }
}
