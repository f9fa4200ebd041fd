"""Timestamps that go backwards, on the device, vs the oracle (VERDICT r04
items 3 / Missing 3-4).

The reference never drops a late row: processElement offers every record to
its PriorityQueue and the next watermark's drain hands it to Siddhi with that
watermark's rows, smallest ts first — behind rows Siddhi has already
processed (core/.../operator/AbstractSiddhiOperator.java:222-231, 238-245).
Processing time (:218-219) and direct callers can also hand Siddhi a ts
below one it has seen.  Siddhi then prunes a partial when |ts(event) -
ts(s1)| > W on every event of the stream the partial waits on (SURVEY App.
A.3, the rule both oracles implement).  With cep_options.ts_order = 0 (the
default) the engine runs every `within` pattern on its order-tolerant form
(the closed form's TOL build for `every A -> B`, tests/test_gpu_ooo_cf.py; the
N-state walk otherwise); ts_order = 1 keeps the event-time fast paths and
reports a descent.  late_policy = 2 (default) delivers late rows as the
reference's drain does.

Every case is bit-exact against oracle/siddhi_oracle.py fed exactly the
sequence the reference would hand Siddhi.
"""
import numpy as np
import pytest

import flink_siddhi as fs
from flink_siddhi import workload
from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

pytestmark = pytest.mark.gpu

COLS = ("k", "ts", "id", "price", "stream")


def _take(w, idx):
    return {c: w[c][idx] for c in COLS}


def _cols(w, s=0, e=None):
    e = len(w["ts"]) if e is None else e
    return [w["k"][s:e], w["ts"][s:e], w["id"][s:e], w["price"][s:e]]


def reference_drains(w, cuts, marks):
    """The order AbstractSiddhiOperator hands rows to Siddhi: rows arrive in
    index order, batch b = [cuts[b], cuts[b+1]); after batch b the watermark
    marks[b] drains every buffered row with ts <= mark, in (ts, arrival)
    order (the engine's stable order; the reference PQ breaks ties
    arbitrarily).  Returns each watermark's release (arrival
    indices in drain order)."""
    buf = []
    out = []
    for b in range(len(marks)):
        buf.extend(range(cuts[b], cuts[b + 1]))
        m = marks[b]
        rel = sorted((i for i in buf if w["ts"][i] <= m), key=lambda i: (w["ts"][i], i))
        relset = set(rel)
        buf = [i for i in buf if i not in relset]
        out.append(rel)
    assert not buf
    return out


def reference_drain(w, cuts, marks):
    return np.array([i for rel in reference_drains(w, cuts, marks) for i in rel], dtype=np.int64)


def laggy_stream(n, keys, rate, jitter, seed):
    """Arrival = index + U[0, jitter) (bounded disorder)."""
    w = workload.generate(0, n, keys, rate=rate)
    rng = np.random.default_rng(seed)
    arrival = np.argsort(np.arange(n) + rng.integers(0, jitter, n), kind="stable")
    return _take(w, arrival)


def run_event_time(plan, w, cuts, marks, out="O", **opts):
    rt = fs.SiddhiAppRuntime(plan, **opts)
    rt.add_callback(out)
    for b in range(len(marks)):
        s, e = cuts[b], cuts[b + 1]
        rt.process_elements("A", w["ts"][s:e], _cols(w, s, e), streams=w["stream"][s:e])
        rt.process_watermark(int(marks[b]))
    rt.flush()
    got = engine_rows(rt.collect(out))
    late = rt.stats().late_events
    rt.shutdown()
    return got, late


PLAN_1S = workload.PATTERN_PLAN.replace("within 10 sec", "within 1 sec")


@pytest.mark.parametrize("plan", [workload.PATTERN_PLAN, PLAN_1S])
def test_late_rows_reach_the_pattern_like_the_reference_drain(plan):
    # watermarks lag the largest ts seen by less than the disorder: rows keep
    # arriving below an earlier watermark (late), and the reference hands
    # them to Siddhi with the next drain
    n, batches = 60000, 12
    w = laggy_stream(n, 512, 8, jitter=4000, seed=21)
    cuts = np.linspace(0, n, batches + 1).astype(int)
    marks = [int(w["ts"][:cuts[b + 1]].max()) - 100 for b in range(batches - 1)] + [int(w["ts"].max())]
    order = reference_drain(w, cuts, marks)
    want = oracle_run(plan, workload_events(_take(w, order))).get("O", [])
    got, late = run_event_time(plan, w, cuts, marks)
    assert late > 100, "the stream must hold late rows"
    assert len(want) > 500
    assert_same_rows(got, want, "late rows delivered")


def test_late_rows_dropped_with_policy_0():
    n, batches = 30000, 6
    w = laggy_stream(n, 512, 8, jitter=4000, seed=22)
    cuts = np.linspace(0, n, batches + 1).astype(int)
    marks = [int(w["ts"][:cuts[b + 1]].max()) - 100 for b in range(batches - 1)] + [int(w["ts"].max())]
    # the oracle without the late rows: a released row is late when its ts
    # is below the largest ts an earlier watermark released
    on_time, nlate, top = [], 0, np.iinfo(np.int64).min
    for rel in reference_drains(w, cuts, marks):
        for i in rel:
            if w["ts"][i] < top:
                nlate += 1
            else:
                on_time.append(i)
        if rel:
            top = max(top, int(max(w["ts"][i] for i in rel)))
    want = oracle_run(workload.PATTERN_PLAN, workload_events(_take(w, np.array(on_time)))).get("O", [])
    got, late = run_event_time(workload.PATTERN_PLAN, w, cuts, marks, late_policy=0)
    assert late == nlate > 50
    assert_same_rows(got, want, "late rows dropped")


def test_late_rows_reach_the_filter():
    plan = workload.FILTER_PLAN
    n, batches = 40000, 8
    g = workload.generate(0, n, 1, single_stream=True, rate=4)
    rng = np.random.default_rng(5)
    arrival = np.argsort(np.arange(n) + rng.integers(0, 3000, n), kind="stable")
    w = {c: g[c][arrival] for c in ("id", "price", "ts")}
    cuts = np.linspace(0, n, batches + 1).astype(int)
    marks = [int(w["ts"][:cuts[b + 1]].max()) - 50 for b in range(batches - 1)] + [int(w["ts"].max())]
    order = reference_drain(w, cuts, marks)
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    name = rt.intern("test_event")
    names = np.full(n, name, np.int32)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        rt.process_elements("inputStream", w["ts"][s:e], [w["id"][s:e], names[s:e], w["price"][s:e], w["ts"][s:e]])
        rt.process_watermark(marks[b])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    assert rt.stats().late_events > 100
    rt.shutdown()
    ev = [("inputStream", int(w["ts"][i]), (int(w["id"][i]), name, float(w["price"][i]), int(w["ts"][i])))
          for i in order]
    want = oracle_run(plan, ev)["O"]
    assert_same_rows(got, want, "late rows through the filter")


@pytest.mark.parametrize("device", [False, True])
def test_reversed_ts_under_within_matches_oracle(device):
    # processing-time-like input with ts going backwards inside one batch
    # (VERDICT r04 Missing 4: the engine used to raise here)
    w = workload.generate(0, 5000, 16, rate=1)
    w["ts"] = w["ts"][::-1].copy()
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt.add_callback("O")
    if device:
        import torch
        d = {c: torch.from_numpy(np.ascontiguousarray(w[c])).cuda() for c in COLS}
        rt.send("A", d["ts"], _cols(d), streams=d["stream"])
    else:
        rt.send("A", w["ts"], _cols(w), streams=w["stream"])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    assert len(want) > 20
    assert_same_rows(got, want, "reversed ts")


def test_strict_ts_order_still_reports_a_descent():
    w = workload.generate(0, 5000, 16, rate=1)
    w["ts"] = w["ts"][::-1].copy()
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, ts_order=1)
    rt.add_callback("O")
    rt.send("A", w["ts"], _cols(w), streams=w["stream"])
    with pytest.raises(ValueError, match="order"):
        rt.flush()
    rt.shutdown()


@pytest.mark.parametrize("chunk", [1 << 15, 1 << 22])
def test_descent_mid_batch_multi_chunk(chunk):
    # a block of rows shifted back by 30 s in the middle of a batch that the
    # engine splits into several chunks: the chunks before it stay on the
    # fast path, the rest is re-run tolerant; every row vs the oracle
    n = 200000
    w = workload.generate(0, n, 4096, rate=4)
    w["ts"] = w["ts"].copy()
    w["ts"][120000:126000] -= 30000
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, chunk_events=chunk)
    rt.add_callback("O")
    rt.send("A", w["ts"], _cols(w), streams=w["stream"])
    # a second, ordered batch afterwards goes back to the fast path
    w2 = workload.generate(n, 40000, 4096, rate=4)
    rt.send("A", w2["ts"], _cols(w2), streams=w2["stream"])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    want2 = oracle_run(workload.PATTERN_PLAN,
                       workload_events(w) + workload_events(w2)).get("O", [])
    assert len(want2) > len(want) > 1000
    assert_same_rows(got, want2, "descent mid batch")


def test_descent_across_device_batches():
    # the second device batch starts 20 s before the first one ended: the
    # engine keeps the last ts of a batch on the device for the next check
    import torch
    n = 60000
    w = workload.generate(0, n, 1024, rate=2)
    w["ts"] = w["ts"].copy()
    h = n // 2
    w["ts"][h:] -= 20000
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    d = {c: torch.from_numpy(np.ascontiguousarray(w[c])).cuda() for c in COLS}
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt.add_callback("O")
    rt.send("A", d["ts"][:h], [x[:h] for x in _cols(d)], streams=d["stream"][:h])
    rt.send("A", d["ts"][h:], [x[h:] for x in _cols(d)], streams=d["stream"][h:])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    assert_same_rows(got, want, "descent across device batches")


EV3 = ("define stream A (k int, ts long, id int, price double);"
       "define stream B (k int, ts long, id int, price double);"
       "define stream C (k int, ts long, id int, price double);")
P3 = "partition with (k of A, k of B, k of C) begin "


def _three(n, keys, seed):
    w = workload.generate(0, n, keys, rate=1)
    w["stream"] = ((w["price"] * 1000).astype(np.int64) % 3).astype(np.uint8)
    rng = np.random.default_rng(seed)
    w["ts"] = w["ts"] + rng.integers(-3000, 3000, n)   # any order
    return w


def _events3(w):
    k, ts, i, p, st = (w[c].tolist() for c in COLS)
    return [("ABC"[st[j]], ts[j], (k[j], ts[j], i[j], p[j])) for j in range(len(ts))]


@pytest.mark.parametrize("query", [
    # N-state pattern (general walk; rows failing every condition still prune)
    "from every s1=A[price > 0.5] -> s2=B[id % 4 == 0] -> s3=C[id % 3 == 0] within 2 sec "
    "select s1.k as k, s1.price as p1, s2.id as i2, s3.ts as t3 insert into O;",
    # 2-state pattern whose B condition reads s1 (N-state walk)
    "from every s1=A[price > 0.3] -> s2=B[price < s1.price] within 2 sec "
    "select s1.k as k, s1.price as p1, s2.price as p2 insert into O;",
    # sequence with a Kleene state (order-agnostic walk, no order check)
    "from every s1=A[price > 0.25], s2=B[id < 30]+, s3=C[id > 20] within 2 sec "
    "select s1.k as k, s1.price as p1, s2[last].price as p2, s3.price as p3 insert into O;",
])
def test_any_order_general_paths(query):
    plan = EV3 + P3 + query + " end;"
    w = _three(30000, 64, seed=3)
    want = oracle_run(plan, _events3(w)).get("O", [])
    rt = fs.SiddhiAppRuntime(plan, chunk_events=4096)
    rt.add_callback("O")
    rt.send("A", w["ts"], _cols(w), streams=w["stream"])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    assert len(want) > 10
    assert_same_rows(got, want, query[:40])


def test_any_order_multi_query_group():
    # config 5's shape (32 sequences + 32 aggregations: one multi-query
    # group) over timestamps in any order
    import config5_cases as C5
    plan = C5.variant_plan()
    w = _three(8000, 48, seed=4)
    want = oracle_run(plan, _events3(w))
    rt = fs.SiddhiAppRuntime(plan, key_capacity=64)
    outs = C5.variant_outputs()
    for o in outs:
        rt.add_callback(o)
    rt.send("A", w["ts"], _cols(w), streams=w["stream"])
    rt.flush()
    seq_rows = 0
    for o in outs:
        got = engine_rows(rt.collect(o))
        assert_same_rows(got, want.get(o, []), o)
        seq_rows += len(got) if o.startswith("Seq") else 0
    rt.shutdown()
    assert seq_rows > 10
