"""GPU: the reference's own test fixtures sent through libcep (the HIP path).

These are every result the reference's test suite pins at the Siddhi
boundary.  `test_oracle_golden.py` checks the same fixtures
on the CPU oracle; here the engine must reproduce them:
  * SiddhiSyntaxTest.java:47-82 — order-preserving pass-through of three rows
    and the UndefinedStreamException for an unknown stream;
  * SiddhiCEPITCase.java:362-382 — `every s1=inputStream1[id == 2]+,
    s2=inputStream2[id == 3]? within 1000 second` produces exactly one line;
  * SiddhiCEPITCase.java:115-179 (5 and 6 lines from one stream) and
    :280-300 (three unioned streams x 10 events = 30 lines);
  * SiddhiCEPITCase.java:332-357 — the config-1 golden row (also in
    test_gpu_parity.py::test_itcase_config1_golden_through_engine, run here
    once more with one event per send call, as the ITCase's source emits).
"""
import numpy as np
import pytest

import flink_siddhi as fs
from helpers import engine_rows, oracle_run
from test_oracle_golden import EVENT_DDL, ITCASE_GOLDEN, ITCASE_PLAN, itcase_events

pytestmark = pytest.mark.gpu


def _event_cols(rt, ids, ts):
    """Event rows (id int, name string, price double, timestamp long) as
    columns; name is "test_event" (RandomEventSource.java:60-63)."""
    name = rt.intern("test_event")
    n = len(ids)
    return [np.asarray(ids, np.int32), np.full(n, name, np.int32), np.full(n, 0.5, np.float64),
            np.asarray(ts, np.int64)]


def test_syntax_passthrough_order_through_engine():
    # SiddhiSyntaxTest.java:47-82: three rows in, the same three rows out, in order
    plan = "define stream inStream (name string, value double);from inStream insert into outStream"
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("outStream")
    names = [rt.intern(s) for s in ("a", "b", "c")]
    rt.send("inStream", np.zeros(3, np.int64), [np.asarray(names, np.int32), np.array([1.1, 1.2, 1.3])])
    rt.flush()
    rows = rt.collect("outStream").rows()
    assert [(rt.lookup(r[0]), r[1]) for r in rows] == [("a", 1.1), ("b", 1.2), ("c", 1.3)]
    # the unknown stream of the same test: UndefinedStreamException
    with pytest.raises(fs.UndefinedStreamException):
        rt.send("unknownStream", np.zeros(1, np.int64), [np.zeros(1, np.int32), np.zeros(1)])
    rt.shutdown()


def test_syntax_passthrough_one_row_per_send():
    # the reference sends the rows one InputHandler.send at a time
    plan = "define stream inStream (name string, value double);from inStream insert into outStream"
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("outStream")
    for s, v in (("a", 1.1), ("b", 1.2), ("c", 1.3)):
        rt.send("inStream", np.zeros(1, np.int64), [np.array([rt.intern(s)], np.int32), np.array([v])])
    rt.flush()
    rows = rt.collect("outStream").rows()
    assert [(rt.lookup(r[0]), r[1]) for r in rows] == [("a", 1.1), ("b", 1.2), ("c", 1.3)]
    rt.shutdown()


def _sequence_plan():
    return ("define stream inputStream1 %s;define stream inputStream2 %s;"
            "from every s1 = inputStream1[id == 2]+ , s2 = inputStream2[id == 3]? "
            "within 1000 second select s1[0].name as n1, s2.name as n2 "
            "insert into outputStream" % (EVENT_DDL, EVENT_DDL))


@pytest.mark.parametrize("batched", [True, False])
def test_itcase_sequence_kleene_one_line_through_engine(batched):
    # SiddhiCEPITCase.java:362-382: the same 5-event source feeds both streams
    # (id = 0..4, ts = 1000 n); the Kleene + / optional ? sequence yields 1 line
    plan = _sequence_plan()
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("outputStream")
    ids = [n for n in range(5) for _ in (0, 1)]
    ts = [1000 * n for n in range(5) for _ in (0, 1)]
    st = np.array([0, 1] * 5, np.uint8)
    if batched:
        rt.send("inputStream1", np.asarray(ts, np.int64), _event_cols(rt, ids, ts), streams=st)
    else:
        for i in range(len(ids)):
            sid = "inputStream1" if st[i] == 0 else "inputStream2"
            rt.send(sid, np.asarray(ts[i:i + 1], np.int64), _event_cols(rt, ids[i:i + 1], ts[i:i + 1]))
    rt.flush()
    out = rt.collect("outputStream")
    assert len(out) == 1
    # and the content agrees with the oracle's restatement
    ev = [("inputStream1" if st[i] == 0 else "inputStream2", ts[i], (ids[i], "test_event", 0.5, ts[i]))
          for i in range(len(ids))]
    want = oracle_run(plan, ev)["outputStream"]
    got = engine_rows(out)
    assert len(want) == 1
    assert [(t, s) for t, s, _ in got] == [(t, s) for t, s, _ in want]
    assert [tuple(rt.lookup(v) for v in d) for _, _, d in got] == [d for _, _, d in want]
    rt.shutdown()


@pytest.mark.parametrize("n_streams,per,expected", [(1, 5, 5), (1, 6, 6), (3, 10, 30)])
def test_itcase_passthrough_line_counts_through_engine(n_streams, per, expected):
    # SiddhiCEPITCase.java:115-179 (5 / 6 lines) and :280-300 (3 unions x 10 = 30)
    plan = "".join("define stream inputStream%d %s;" % (i + 1, EVENT_DDL) for i in range(n_streams))
    plan += "".join("from inputStream%d select timestamp, id, name, price insert into outputStream;" % (i + 1)
                    for i in range(n_streams))
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("outputStream")
    for i in range(n_streams):
        ids = [n % 50 for n in range(per)]
        ts = [1000 * n for n in range(per)]
        rt.send("inputStream%d" % (i + 1), np.asarray(ts, np.int64), _event_cols(rt, ids, ts))
    rt.flush()
    out = rt.collect("outputStream")
    assert len(out) == expected
    # select timestamp, id, name, price: every row carries its event's values
    rows = out.rows()
    assert sorted(r[0] for r in rows) == sorted(1000 * n for n in range(per) for _ in range(n_streams))
    assert all(rt.lookup(r[2]) == "test_event" and r[3] == 0.5 for r in rows)
    rt.shutdown()


def test_itcase_config1_golden_one_event_per_send():
    # SiddhiCEPITCase.java:332-357 with the source's one-event-per-send cadence
    rt = fs.SiddhiAppRuntime(ITCASE_PLAN)
    rt.add_callback("outputStream")
    name = rt.intern("test_event")
    for sid, ts, row in itcase_events():
        rt.send(sid, np.array([ts], np.int64),
                [np.array([row[0]], np.int32), np.array([name], np.int32), np.array([row[2]]),
                 np.array([row[3]], np.int64)])
    rt.flush()
    rows = rt.collect("outputStream").rows()
    assert len(rows) == 1
    defs = rt.stream_definition("outputStream")
    m = {}
    for (k, t), v in zip(defs, rows[0]):
        m[k] = rt.lookup(v) if t == 5 else v
    assert "{" + ", ".join("%s=%s" % (k, m[k]) for k in sorted(m)) + "}" == ITCASE_GOLDEN
    rt.shutdown()
