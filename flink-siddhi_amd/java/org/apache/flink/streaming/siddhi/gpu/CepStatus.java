package org.apache.flink.streaming.siddhi.gpu;

import org.apache.flink.streaming.siddhi.exception.DuplicatedStreamException;
import org.apache.flink.streaming.siddhi.exception.UndefinedStreamException;

/** libcep status codes (include/cep.h) -> the reference's exceptions. */
final class CepStatus {
    static final int OK = 0, PARSE = 1, UNDEFINED_STREAM = 2, DUPLICATED_STREAM = 3,
        UNSUPPORTED = 4, ARG = 5, DEVICE = 6, CAPACITY = 7, STATE = 8;

    private CepStatus() {}

    /** Thrown for valid SiddhiQL outside the engine subset (joins, windows,
     *  tables): the stream factory then builds the stock SiddhiStreamOperator. */
    static final class UnsupportedPlanException extends RuntimeException {
        UnsupportedPlanException(String msg) {
            super(msg);
        }
    }

    static void check(int rc, String msg) {
        switch (rc) {
            case OK:
                return;
            case PARSE:   // SiddhiAppCreationException at DAG build (AbstractSiddhiOperator.java:292-299)
                throw new org.wso2.siddhi.core.exception.SiddhiAppCreationException(msg);
            case UNDEFINED_STREAM:   // exception/UndefinedStreamException.java:20
                throw new UndefinedStreamException(msg);
            case DUPLICATED_STREAM:
                throw new DuplicatedStreamException(msg);
            case UNSUPPORTED:
                throw new UnsupportedPlanException(msg);
            case ARG:   // StreamOutputHandler.java:89
                throw new IllegalArgumentException(msg);
            default:
                throw new IllegalStateException("libcep status " + rc + ": " + msg);
        }
    }
}
