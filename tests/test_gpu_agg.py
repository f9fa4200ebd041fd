"""Group-by / having on the device (SURVEY.md §8 row a3, config 5's
aggregation half) vs the CPU oracle, bit-exact: running aggregates per group
in arrival order, fp64 sums accumulated sequentially per group (so no
tolerance is needed: the device adds in the oracle's order)."""
import numpy as np
import pytest

import flink_siddhi as fs
from flink_siddhi import workload
from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

pytestmark = pytest.mark.gpu

EV2 = ("define stream A (k int, ts long, id int, price double);"
       "define stream B (k int, ts long, id int, price double);")


def run(plan, w, batches=1, **opts):
    rt = fs.SiddhiAppRuntime(plan, **opts)
    rt.add_callback("O")
    n = len(w["ts"])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        rt.send("A", w["ts"][s:e], [w["k"][s:e], w["ts"][s:e], w["id"][s:e], w["price"][s:e]],
                streams=w["stream"][s:e])
        rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    return got


def agg_case(query, n=30000, keys=512, batches=1, **opts):
    plan = EV2 + query
    w = workload.generate(0, n, keys, rate=1)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    got = run(plan, w, batches=batches, **opts)
    assert_same_rows(got, want, query)
    return len(want)


def test_config5_group_by_having():
    m = agg_case("from A[price > 0.5] select k, sum(price) as total, count() as n "
                 "group by k having total > 1.0 insert into O;")
    assert m > 1000


def test_group_by_all_aggregates_int_and_double():
    m = agg_case("from A[id < 40] select k, sum(id) as si, avg(id) as ai, min(price) as mn, "
                 "max(id) as mx, avg(price) as ap, count() as c group by k insert into O;")
    assert m > 1000


def test_group_by_multi_chunk_multi_batch():
    m = agg_case("from A select k, sum(price) as s, max(price) as m group by k insert into O;",
                 n=40000, keys=1024, batches=3, chunk_events=4096)
    assert m > 10000


def test_global_aggregate_without_group_by():
    m = agg_case("from A[id == 3] select sum(price) as s, count() as c insert into O;",
                 n=20000, keys=64)
    assert m > 100


def test_partitioned_group_by_with_current_attributes():
    m = agg_case("partition with (k of A) begin from A[price < 0.3] select k, id, price, "
                 "sum(price) as s group by k having s > 0.5 and id > 10 insert into O; end;")
    assert m > 100


def test_group_by_snapshot_restore():
    plan = EV2 + ("from A select k, sum(price) as s, count() as c group by k insert into O;")
    w = workload.generate(0, 20000, 256, rate=1)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    h = 10000
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    rt.send("A", w["ts"][:h], [w["k"][:h], w["ts"][:h], w["id"][:h], w["price"][:h]],
            streams=w["stream"][:h])
    rt.flush()
    first = engine_rows(rt.collect("O"))
    snap = rt.snapshot()
    rt.shutdown()
    rt2 = fs.SiddhiAppRuntime(plan)
    rt2.add_callback("O")
    rt2.restore(snap)
    rt2.send("A", w["ts"][h:], [w["k"][h:], w["ts"][h:], w["id"][h:], w["price"][h:]],
             streams=w["stream"][h:])
    rt2.flush()
    second = engine_rows(rt2.collect("O"))
    rt2.shutdown()
    # the snapshot carries the arrival counter: seq continues across restore
    assert_same_rows(first + second, want, "group-by snapshot/restore")
