"""GPU parity: libcep (HIP, gfx950) vs the CPU oracle on identical inputs.

Bit-exact for every output column, timestamp, sequence number and the global
emission order (cep_options.ordered_output = 1 delivers Siddhi's order:
completing event, then pending-creation order — SURVEY.md App. A.4).
"""
import numpy as np
import pytest

from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

pytestmark = pytest.mark.gpu

import flink_siddhi as fs  # noqa: E402
from flink_siddhi import workload  # noqa: E402

EV2 = ("define stream A (k int, ts long, id int, price double);"
       "define stream B (k int, ts long, id int, price double);")


def run_engine(plan, w, out="O", batches=1, names=("A", "B"), **opts):
    rt = fs.SiddhiAppRuntime(plan, **opts)
    rt.add_callback(out)
    n = len(w["ts"])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        rt.send(names[0], w["ts"][s:e], [w["k"][s:e], w["ts"][s:e], w["id"][s:e],
                                         w["price"][s:e]], streams=w["stream"][s:e])
        rt.flush()
    got = engine_rows(rt.collect(out))
    rt.shutdown()
    return got


def pattern_case(plan, n=20000, keys=64, rate=1, batches=1, **opts):
    w = workload.generate(0, n, keys, rate=rate)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    got = run_engine(plan, w, batches=batches, **opts)
    assert_same_rows(got, want, plan)
    return len(want)


def test_config3_keyed_pattern_small():
    m = pattern_case(workload.PATTERN_PLAN, n=30000, keys=4096, rate=1)
    assert m > 100


def test_config3_multi_chunk_multi_batch():
    m = pattern_case(workload.PATTERN_PLAN, n=40000, keys=2048, rate=1, batches=3,
                     chunk_events=4096)
    assert m > 50


def test_pattern_bucket_window_overflow():
    # 4 keys -> every record of a chunk lands in 4 buckets: several LDS windows
    plan = workload.PATTERN_PLAN.replace("within 10 sec", "within 100 milliseconds")
    m = pattern_case(plan, n=30000, keys=4, rate=1, chunk_events=1 << 16)
    assert m > 100


def test_pattern_condition_on_s1():
    plan = EV2 + ("partition with (k of A, k of B) begin "
                  "from every s1=A[id < 25] -> s2=B[price > s1.price and id != s1.id] "
                  "within 3 sec select s1.id as i1, s2.id as i2, s1.price as p1, "
                  "s2.price - s1.price as d insert into O; end;")
    m = pattern_case(plan, n=20000, keys=512, rate=1)
    assert m > 20


def test_pattern_condition_on_s1_long_pending_lists():
    # an s1-dependent condition keeps ~150 live partials
    # per key (16 keys, 1 event/ms, 10 s window; B[id > s1.id + 47] is rare)
    # with 16 inline slots: the N-state walk continues the lists in the
    # pending pool instead of failing with CEP_E_CAPACITY
    plan = EV2 + ("partition with (k of A, k of B) begin "
                  "from every s1=A[price > 0.2] -> s2=B[id > s1.id + 47] within 10 sec "
                  "select s1.id as i1, s2.id as i2, s1.price as p1, s2.ts as t insert into O; end;")
    w = workload.generate(0, 40000, 16, rate=1)
    a = (w["stream"] == 0) & (w["price"] > 0.2)
    per_key = max(int(((w["k"] == k) & a & (w["ts"] < w["ts"][0] + 10000)).sum()) for k in range(16))
    assert per_key >= 40
    want = oracle_run(plan, workload_events(w)).get("O", [])
    got = run_engine(plan, w, batches=2, pending_slots=16, chunk_events=8192)
    assert len(want) > 200
    assert_same_rows(got, want, plan)


def test_pattern_without_every_is_one_shot_per_key():
    plan = EV2 + ("partition with (k of A, k of B) begin "
                  "from s1=A[price > 0.9] -> s2=B[id == 7] select s1.k as k, s2.ts as t "
                  "insert into O; end;")
    m = pattern_case(plan, n=20000, keys=32, rate=1)
    assert 0 < m <= 32


def test_pattern_without_within_or_partition():
    plan = EV2 + ("from every s1=A[id == 2] -> s2=B[id == 3] "
                  "select s1.id as id_1, s2.id as id_2, s1.k as k1, s2.k as k2 insert into O;")
    pattern_case(plan, n=3000, keys=8, rate=1, pending_slots=16)


def test_same_stream_pattern():
    plan = ("define stream A (k int, ts long, id int, price double);"
            "partition with (k of A) begin "
            "from every s1=A[id % 5 == 1] -> s2=A[id % 5 == 2 or id == 11] within 4 sec "
            "select s1.id as a, s2.id as b, s2.ts as t insert into O; end;")
    w = workload.generate(0, 20000, 1024, rate=1, single_stream=True)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    got = run_engine(plan, w)
    assert_same_rows(got, want, plan)
    assert len(want) > 10


def test_config2_filter_parity():
    w = workload.generate(0, 200000, 1 << 20, single_stream=True)
    plan = workload.FILTER_PLAN
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    name = rt.intern("test_event")
    names = np.full(len(w["ts"]), name, np.int32)
    rt.send("inputStream", w["ts"], [w["id"], names, w["price"], w["ts"]])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    ev = [("inputStream", t, (i, name, p, t)) for i, p, t in
          zip(w["id"].tolist(), w["price"].tolist(), w["ts"].tolist())]
    want = oracle_run(plan, ev)["O"]
    assert_same_rows(got, want, "config-2 filter")
    assert abs(len(want) / 200000 - 0.08) < 0.01


def test_config2_filter_many_tiles_vs_c_oracle():
    """3 * 2^20 events in three batches: ~130 tiles of 8192 rows per batch,
    so the look-back walks past its 64-tile window; every selected row (its
    columns, ts and arrival number, in order) vs oracle/cep_oracle.c."""
    import cep_oracle as CO
    n, batches = 3 << 20, 3
    w = workload.generate(0, n, 1 << 20, single_stream=True)
    rt = fs.SiddhiAppRuntime(workload.FILTER_PLAN)
    rt.add_callback("O")
    name = rt.intern("test_event")
    names = np.full(n, name, np.int32)
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        rt.send("inputStream", w["ts"][s:e], [w["id"][s:e], names[s:e], w["price"][s:e], w["ts"][s:e]])
    rt.flush()
    out = rt.collect("O")
    rt.shutdown()
    sel = CO.filter_indices(w["id"], w["price"], CO.cond(("price", 0, ">", 0.5), ("id", 7, "==", 0)))
    assert len(sel) > 0.07 * n
    np.testing.assert_array_equal(out.seq, sel)
    np.testing.assert_array_equal(out.ts, w["ts"][sel])
    np.testing.assert_array_equal(out.cols[0], w["id"][sel])
    np.testing.assert_array_equal(out.cols[1], names[sel])
    np.testing.assert_array_equal(out.cols[2], w["price"][sel])
    np.testing.assert_array_equal(out.cols[3], w["ts"][sel])


def test_filter_expression_semantics():
    plan = ("define stream S (a int, b long, c float, d double, e bool);"
            "from S[(a % 3 == -1 or a / 4 > 2) and not e or d / 0.0 > 1.0e300] "
            "select a * 7 - b as x, c * 2.5f as y, d % 1.5 as z, a / (a % 5) as q, "
            "b + a as w insert into O;")
    rng = np.random.default_rng(7)
    n = 5000
    a = rng.integers(-50, 50, n).astype(np.int32)
    b = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    c = rng.standard_normal(n).astype(np.float32)
    d = rng.standard_normal(n) * 10
    e = rng.integers(0, 2, n).astype(np.uint8)
    ts = np.arange(n, dtype=np.int64)
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    rt.send("S", ts, [a, b, c, d, e])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    ev = [("S", int(ts[i]), (int(a[i]), int(b[i]), float(c[i]), float(d[i]), bool(e[i])))
          for i in range(n)]
    want = oracle_run(plan, ev)["O"]
    # the engine writes a null int (a / 0) as 0; the oracle keeps None
    want = [(t, s, tuple(0 if v is None else v for v in d)) for t, s, d in want]
    got = [(t, s, (x, float(np.float32(y)), z, q, wv)) for t, s, (x, y, z, q, wv) in got]
    assert_same_rows(got, want, "expression semantics")


def test_itcase_config1_golden_through_engine():
    from test_oracle_golden import itcase_events, ITCASE_PLAN, ITCASE_GOLDEN
    rt = fs.SiddhiAppRuntime(ITCASE_PLAN)
    rt.add_callback("outputStream")
    name = rt.intern("test_event")
    ev = itcase_events()
    ts = np.array([e[1] for e in ev], np.int64)
    st = np.array([0 if e[0] == "inputStream1" else 1 for e in ev], np.uint8)
    cols = [np.array([e[2][0] for e in ev], np.int32), np.full(len(ev), name, np.int32),
            np.array([e[2][2] for e in ev], np.float64), ts]
    rt.send("inputStream1", ts, cols, streams=st)
    rt.flush()
    out = rt.collect("outputStream")
    rows = out.rows()
    assert len(rows) == 1
    defs = rt.stream_definition("outputStream")
    m = {defs[i][0]: v for i, v in enumerate(rows[0])}
    m = {k: (rt.lookup(v) if defs[[d[0] for d in defs].index(k)][1] == 5 else v)
         for k, v in m.items()}
    text = "{" + ", ".join("%s=%s" % (k, m[k]) for k in sorted(m)) + "}"
    assert text == ITCASE_GOLDEN


def test_snapshot_restore_roundtrip():
    plan = workload.PATTERN_PLAN
    w = workload.generate(0, 30000, 4096, rate=1)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    assert len(want) > 100
    half = 17000
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    rt.send("A", w["ts"][:half], [w["k"][:half], w["ts"][:half], w["id"][:half],
                                  w["price"][:half]], streams=w["stream"][:half])
    rt.flush()
    first = engine_rows(rt.collect("O"))
    snap = rt.snapshot()
    rt.shutdown()
    rt2 = fs.SiddhiAppRuntime(plan)
    rt2.add_callback("O")
    rt2.restore(snap)
    rt2.send("A", w["ts"][half:], [w["k"][half:], w["ts"][half:], w["id"][half:],
                                   w["price"][half:]], streams=w["stream"][half:])
    rt2.flush()
    second = engine_rows(rt2.collect("O"))
    assert_same_rows(first + second, want, "snapshot/restore")


def test_disabled_runtime_drops_events():
    rt = fs.SiddhiAppRuntime(workload.FILTER_PLAN)
    rt.add_callback("O")
    rt.set_enabled(False)
    w = workload.generate(0, 1000, 10, single_stream=True)
    rt.send("inputStream", w["ts"], [w["id"], w["id"], w["price"], w["ts"]])
    rt.flush()
    assert len(rt.collect("O")) == 0


def test_device_resident_batch_matches_host_batch():
    import torch
    n, keys = 50000, 8192
    d = workload.generate_device(0, n, keys, rate=2)
    torch.cuda.synchronize()
    h = workload.generate(0, n, keys, rate=2)
    for k in ("k", "ts", "id", "price", "stream"):
        assert np.array_equal(d[k].cpu().numpy(), h[k]), k
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt.add_callback("O")
    rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    want = run_engine(workload.PATTERN_PLAN, h)
    assert_same_rows(got, want, "device vs host batch")


def test_pending_overflow_general_path_is_reported(monkeypatch):
    # g never holds: every key keeps ~39 live partials inside the 10 s window
    # (64 keys, 1 event/ms), more than 16 slots.  The general walk keeps
    # per-key lists in LDS and reports capacity (the closed-form path spills
    # to the pending pool: test_gpu_cf.py::test_pending_lists_longer_than_pending_slots)
    monkeypatch.setenv("CEP_NO_CF", "1")
    w = workload.generate(0, 30000, 64, rate=1)
    plan = workload.PATTERN_PLAN.replace("id % 7 == 0", "id == 1000")
    rt = fs.SiddhiAppRuntime(plan, pending_slots=16)
    rt.add_callback("O")
    rt.send("A", w["ts"], [w["k"], w["ts"], w["id"], w["price"]], streams=w["stream"])
    with pytest.raises(fs.CepCapacityError):
        rt.flush()


def test_pending_slots_full_capacity_denser_keys():
    m = pattern_case(workload.PATTERN_PLAN.replace("within 10 sec", "within 2 sec"),
                     n=30000, keys=256, rate=1, pending_slots=16)
    assert m > 100


def test_pending_slots_above_limit_rejected():
    with pytest.raises(fs.CepCapacityError):
        fs.SiddhiAppRuntime(workload.PATTERN_PLAN, pending_slots=32)
