"""Config 5 of BASELINE.json on the device: one Siddhi app holding 64 queries
(32 `every s1=A, s2=B+, s3=C within` sequences in one partition block, outputs
Seq0..Seq31, and 32 group-by/having aggregations, outputs Agg0..Agg31) over
three keyed streams, compared output by output with the CPU oracle, bit-exact.

This is the reference's multi-query operator case (several `cql(...)`
statements sharing one AbstractSiddhiOperator, AbstractSiddhiOperator.java:130).
The sequence conditions use `id % 10` instead of config 5's `id == q % 50` so
that strictly contiguous sequences complete often enough on a stream the Python
oracle finishes in seconds; the query shape (three states, Kleene `+`,
`[last]`, within, partition) is the config's.
"""
import numpy as np
import pytest

import flink_siddhi as fs
from flink_siddhi import workload
from helpers import assert_same_rows, engine_rows, oracle_run

pytestmark = pytest.mark.gpu

EV3 = ("define stream A (k int, ts long, id int, price double);"
       "define stream B (k int, ts long, id int, price double);"
       "define stream C (k int, ts long, id int, price double);")
NAMES = ("A", "B", "C")
NQ = 32


def config5_plan():
    seq = ["partition with (k of A, k of B, k of C) begin "]
    for q in range(NQ):
        seq.append("from every s1=A[price > %s], s2=B[id %% 10 == %d]+, s3=C[id %% 10 == %d] "
                   "within 10 sec select s1.k as k, s1.price as p1, s2[last].price as p2, "
                   "s3.ts as t3 insert into Seq%d;" % (repr(q / 64.0), q % 10, (q + 1) % 10, q))
    seq.append(" end;")
    agg = []
    for q in range(NQ):
        agg.append("from %s[id >= %d] select k, sum(price) as total, count() as n "
                   "group by k having total > %s insert into Agg%d;"
                   % (NAMES[q % 3], q, repr(1.0 + q / 8.0), q))
    return EV3 + "".join(seq) + "".join(agg)


def three_streams(n, keys):
    w = workload.generate(0, n, keys, rate=1)
    w["stream"] = ((w["price"] * 1000).astype(np.int64) % 3).astype(np.uint8)
    return w


def events(w):
    k, ts, i, p, st = (w[c].tolist() for c in ("k", "ts", "id", "price", "stream"))
    return [(NAMES[st[j]], ts[j], (k[j], ts[j], i[j], p[j])) for j in range(len(ts))]


def outputs():
    return ["Seq%d" % q for q in range(NQ)] + ["Agg%d" % q for q in range(NQ)]


def test_config5_64_queries_two_batches():
    plan = config5_plan()
    w = three_streams(8000, 48)
    want = oracle_run(plan, events(w))
    rt = fs.SiddhiAppRuntime(plan, key_capacity=64)
    for o in outputs():
        rt.add_callback(o)
    n = len(w["ts"])
    h = n // 2
    for s, e in ((0, h), (h, n)):
        rt.send("A", w["ts"][s:e], [w["k"][s:e], w["ts"][s:e], w["id"][s:e], w["price"][s:e]],
                streams=w["stream"][s:e])
        rt.flush()
    got = {o: engine_rows(rt.collect(o)) for o in outputs()}
    rt.shutdown()
    seq_rows = agg_rows = 0
    for o in outputs():
        assert_same_rows(got[o], want.get(o, []), o)
        if o.startswith("Seq"):
            seq_rows += len(got[o])
        else:
            agg_rows += len(got[o])
    assert seq_rows > 20 and agg_rows > 1000, (seq_rows, agg_rows)


def config5_exact_plan():
    return workload.config5_plan()


def test_config5_exact_predicates():
    plan = config5_exact_plan()
    # few keys, many events per key: strictly contiguous A, B+, C runs with
    # id == q % 50 complete now and then; the aggregates emit on most A's
    w = three_streams(24000, 4)
    want = oracle_run(plan, events(w))
    outs = ["Seq%d" % q for q in range(32)] + ["Agg%d" % q for q in range(32, 64)]
    rt = fs.SiddhiAppRuntime(plan, key_capacity=64)
    for o in outs:
        rt.add_callback(o)
    n = len(w["ts"])
    for s, e in ((0, n // 3), (n // 3, n)):
        rt.send("A", w["ts"][s:e], [w["k"][s:e], w["ts"][s:e], w["id"][s:e], w["price"][s:e]],
                streams=w["stream"][s:e])
        rt.flush()
    got = {o: engine_rows(rt.collect(o)) for o in outs}
    rt.shutdown()
    for o in outs:
        assert_same_rows(got[o], want.get(o, []), o)
    assert sum(len(got[o]) for o in outs if o.startswith("Agg")) > 10000
    assert sum(len(want.get(o, [])) for o in outs if o.startswith("Seq")) > 0
