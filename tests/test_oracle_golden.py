"""CPU: the oracle against the reference's own fixtures + App. A KATs.

Reference-pinned:
  * SiddhiCEPITCase.java:332-357 — config-1 pattern golden row;
  * SiddhiSyntaxTest.java:47-82 — order-preserving pass-through;
  * SiddhiExecutionPlanSchemaTest.java:47 — DDL text;
  * SiddhiCEPITCase.java:115-300 — pass-through line counts.
Everything tagged `App.A.x` is a hand-derived known-answer test for a Siddhi
semantic the reference's tests do not pin ("parity unpinned").
"""
import json
import random
from pathlib import Path

import pytest

import siddhi_oracle as O

GOLDEN_DIR = Path(__file__).parent / "golden"

EVENT_DDL = "(id int,name string,price double,timestamp long)"
ITCASE_PLAN = (
    "define stream inputStream1 %s;define stream inputStream2 %s;"
    "from every s1 = inputStream1[id == 2]  -> s2 = inputStream2[id == 3] "
    "select s1.id as id_1, s1.name as name_1, s2.id as id_2, s2.name as name_2 "
    "insert into outputStream" % (EVENT_DDL, EVENT_DDL))
ITCASE_GOLDEN = "{id_1=2, id_2=3, name_1=test_event, name_2=test_event}"


def itcase_events():
    """Two RandomEventSource(50) streams (RandomEventSource.java:56-66):
    id = n % 50, name = test_event, ts = T0 + 1000 n, merged by event time
    (AbstractSiddhiOperator.java:238-245), ties stream1 first."""
    fx = json.loads((GOLDEN_DIR / "config1_itcase.json").read_text())
    return [(e[0], e[1], tuple(e[2])) for e in fx["events"]]


def test_config1_itcase_golden_fixture_matches_generator():
    fx = json.loads((GOLDEN_DIR / "config1_itcase.json").read_text())
    assert fx["plan"] == ITCASE_PLAN
    assert fx["expected"] == [ITCASE_GOLDEN]
    ev = itcase_events()
    assert len(ev) == 100
    assert [e[2][0] for e in ev if e[0] == "inputStream1"] == [n % 50 for n in range(50)]


def test_config1_itcase_golden():
    rt = O.OracleRuntime(ITCASE_PLAN)
    outs = []
    for sid, ts, row in itcase_events():
        outs.extend(rt.send(sid, ts, row))
    od = rt.stream_def("outputStream")
    assert [O.format_map(od, o.data) for o in outs] == [ITCASE_GOLDEN]


def test_syntax_passthrough_order():
    # SiddhiSyntaxTest.java:47-82
    rt = O.OracleRuntime("define stream inStream (name string, value double);"
                         "from inStream insert into outStream")
    got = []
    for row in [("a", 1.1), ("b", 1.2), ("c", 1.3)]:
        got += [o.data for o in rt.send("inStream", 0, row)]
    assert got == [("a", 1.1), ("b", 1.2), ("c", 1.3)]
    with pytest.raises(O.SiddhiError):
        rt.send("unknownStream", 0, ("x", 1.0))


def test_ddl_format():
    # SiddhiExecutionPlanSchemaTest.java:47
    s = O.stream_definition_expression(
        "test_stream", [("id", "int"), ("timestamp", "long"), ("name", "string"),
                        ("price", "double")])
    assert s == "define stream test_stream (id int,timestamp long,name string,price double);"
    app = O.parse_app(s)
    assert [(a.name, a.type) for a in app.streams["test_stream"].attrs] == \
        [("id", "int"), ("timestamp", "long"), ("name", "string"), ("price", "double")]


@pytest.mark.parametrize("n_streams,per,expected", [(1, 5, 5), (1, 6, 6), (3, 10, 30)])
def test_itcase_passthrough_line_counts(n_streams, per, expected):
    # SiddhiCEPITCase.java:115-179 (5/6 lines) and :280-300 (3 unions x 10 = 30)
    plan = "".join("define stream inputStream%d %s;" % (i + 1, EVENT_DDL)
                   for i in range(n_streams))
    plan += "".join("from inputStream%d select timestamp, id, name, price insert into "
                    "outputStream;" % (i + 1) for i in range(n_streams))
    rt = O.OracleRuntime(plan)
    lines = 0
    for n in range(per):
        for i in range(n_streams):
            lines += len(rt.send("inputStream%d" % (i + 1), 1000 * n,
                                 (n % 50, "test_event", 0.5, 1000 * n)))
    assert lines == expected


P2 = ("define stream A (k int, v double);define stream B (k int, v double);")


def _run(plan, evs, out="O"):
    rt = O.OracleRuntime(plan)
    res = []
    for sid, ts, row in evs:
        res += [(o.ts, o.data) for o in rt.send(sid, ts, row) if o.stream == out]
    return res


def test_appA3_within_boundary_inclusive():
    plan = P2 + "from every a=A -> b=B within 10 ms select a.v as x, b.v as y insert into O;"
    assert _run(plan, [("A", 0, (1, 1.0)), ("B", 10, (1, 2.0))]) == [(10, (1.0, 2.0))]
    assert _run(plan, [("A", 0, (1, 1.0)), ("B", 11, (1, 2.0))]) == []


def test_appA3_one_b_completes_all_pending_in_order():
    plan = P2 + "from every a=A -> b=B select a.v as x, b.v as y insert into O;"
    evs = [("A", 0, (1, 1.0)), ("A", 1, (1, 2.0)), ("A", 2, (1, 3.0)),
           ("B", 3, (1, 9.0)), ("B", 4, (1, 8.0))]
    assert _run(plan, evs) == [(3, (1.0, 9.0)), (3, (2.0, 9.0)), (3, (3.0, 9.0))]


def test_appA3_condition_on_s1_leaves_others_pending():
    plan = P2 + "from every a=A -> b=B[v > a.v] select a.v as x, b.v as y insert into O;"
    evs = [("A", 0, (1, 5.0)), ("A", 1, (1, 1.0)), ("B", 2, (1, 3.0)),
           ("B", 3, (1, 6.0))]
    assert _run(plan, evs) == [(2, (1.0, 3.0)), (3, (5.0, 6.0))]


def test_appA3_new_partial_not_visible_to_same_event():
    plan = ("define stream S (x int);"
            "from every a=S[x > 0] -> b=S[x > 0] select a.x as p, b.x as q insert into O;")
    evs = [("S", 0, (1,)), ("S", 1, (2,)), ("S", 2, (3,))]
    assert _run(plan, evs) == [(1, (1, 2)), (2, (2, 3))]


def test_appA3_without_every_one_shot():
    plan = P2 + "from a=A -> b=B select a.v as x, b.v as y insert into O;"
    evs = [("A", 0, (1, 1.0)), ("A", 1, (1, 2.0)), ("B", 2, (1, 3.0)),
           ("A", 3, (1, 4.0)), ("B", 4, (1, 5.0))]
    assert _run(plan, evs) == [(2, (1.0, 3.0))]


def test_appA3_partition_isolates_keys():
    plan = P2 + ("partition with (k of A, k of B) begin from every a=A -> b=B "
                 "select a.k as k, a.v as x, b.v as y insert into O; end;")
    evs = [("A", 0, (1, 1.0)), ("A", 1, (2, 2.0)), ("B", 2, (2, 3.0)),
           ("B", 3, (1, 4.0))]
    assert _run(plan, evs) == [(2, (2, 2.0, 3.0)), (3, (1, 1.0, 4.0))]


def test_appA2_java_integer_semantics():
    plan = ("define stream S (a int, b int, l long);"
            "from S select a / b as q, a % b as r, a * b as m, l * 3 as lm insert into O;")
    rt = O.OracleRuntime(plan)
    d = rt.send("S", 0, (-7, 2, 1 << 62))[0].data
    assert d[:2] == (-3, -1)
    assert d[3] == O._wrap64((1 << 62) * 3)
    d = rt.send("S", 0, (7, 0, 0))[0].data
    assert d[0] is None and d[1] is None          # App. A.2: int div/mod by zero -> null
    d = rt.send("S", 0, (-2147483648, -1, 0))[0].data
    assert d[0] == -2147483648 and d[1] == 0      # Java wraps INT_MIN / -1
    d = rt.send("S", 0, (65536, 65536, 0))[0].data
    assert d[2] == 0                              # int overflow wraps


def test_appA2_null_compare_is_false():
    plan = "define stream S (a int, b int);from S[a / b > 0 or a / b <= 0] select a insert into O;"
    rt = O.OracleRuntime(plan)
    assert rt.send("S", 0, (1, 0)) == []
    assert len(rt.send("S", 0, (1, 1))) == 1


def test_appA6_running_aggregates_group_by_having():
    plan = ("define stream S (k int, p double);"
            "from S select k, sum(p) as total, count() as n group by k having total > 1.0 "
            "insert into O;")
    evs = [("S", 0, (1, 0.6)), ("S", 1, (2, 0.9)), ("S", 2, (1, 0.6)), ("S", 3, (2, 0.2)),
           ("S", 4, (1, 0.1))]
    assert _run(plan, evs) == [(2, (1, 1.2, 2)), (3, (2, 1.1, 2)), (4, (1, 1.3, 3))]


def test_appA5_sequence_strict_contiguity():
    plan = P2 + "from every a=A, b=B select a.v as x, b.v as y insert into O;"
    evs = [("A", 0, (1, 1.0)), ("B", 1, (1, 2.0)), ("A", 2, (1, 3.0)), ("A", 3, (1, 4.0)),
           ("B", 4, (1, 5.0))]
    assert _run(plan, evs) == [(1, (1.0, 2.0)), (4, (4.0, 5.0))]


def test_itcase_sequence_line_count():
    # SiddhiCEPITCase.java:362-382 — the same 5-event source registered as two
    # streams; `every s1=inputStream1[id == 2]+, s2=inputStream2[id == 3]?` -> 1 line
    plan = ("define stream inputStream1 %s;define stream inputStream2 %s;"
            "from every s1 = inputStream1[id == 2]+ , s2 = inputStream2[id == 3]? "
            "within 1000 second select s1[0].name as n1, s2.name as n2 "
            "insert into outputStream" % (EVENT_DDL, EVENT_DDL))
    rt = O.OracleRuntime(plan)
    lines = 0
    for n in range(5):
        for sid in ("inputStream1", "inputStream2"):
            lines += len(rt.send(sid, 1000 * n, (n, "test_event", 0.5, 1000 * n)))
    assert lines == 1


def test_java_double_formatting():
    assert O.java_double_str(0.5) == "0.5"
    assert O.java_double_str(1.0e7) == "1.0E7"
    assert O.java_double_str(1.0e-5) == "1.0E-5"
    assert O.java_double_str(123.0) == "123.0"


def test_oracle_parser_rejects_what_siddhi_rejects():
    for bad in ["define stream A (x int); from A[x + 'a' > 1] select x insert into O;",
                "define stream A (x int); from A select y insert into O;",
                "define stream A (x int); from every a=A -> b=B select a.x insert into O;",
                "define stream A (x int); from A select x, x insert into O;"]:
        with pytest.raises(O.SiddhiError):
            O.parse_app(bad)
