"""k_filterc (filter.hip), the coalesced compaction filter, against the
oracle: ragged batch lengths around its 2048-row tiles and 512-row wave
slabs, multi-stream batches, 1 / 2 / 3 predicate columns (bool, int, float,
double), OR term lists, no predicate, and selections dense enough that a
wave projects more than 64 rows (several projection rounds).  The
FilterProcessor semantics are the reference's (AbstractSiddhiOperator.java:130
-> Siddhi `from S[cond] select ...`)."""
import numpy as np
import pytest

import flink_siddhi as fs
from flink_siddhi import _lib as L
from flink_siddhi import workload
from helpers import assert_same_rows, engine_rows, oracle_run

pytestmark = pytest.mark.gpu

S_DEF = "define stream S (a int, b long, c float, d double, e bool);"


def _cols(n, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(-50, 50, n).astype(np.int32),
            rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64),
            rng.standard_normal(n).astype(np.float32),
            rng.standard_normal(n) * 3,
            rng.integers(0, 2, n).astype(np.uint8)]


def _events(sid, ts, cols):
    return [(sid, int(ts[i]), (int(cols[0][i]), int(cols[1][i]), float(cols[2][i]), float(cols[3][i]),
                               bool(cols[4][i]))) for i in range(len(ts))]


def _run(plan, n, seed=3, batches=1, device=False):
    cols = _cols(n, seed)
    ts = np.arange(n, dtype=np.int64) * 3
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        if device:
            import torch
            rt.send("S", torch.from_numpy(ts[s:e].copy()).cuda(),
                    [torch.from_numpy(c[s:e].copy()).cuda() for c in cols])
        else:
            rt.send("S", ts[s:e], [c[s:e] for c in cols])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    launches = rt.stats().kernel_launches[L.K_FILTER]
    rt.shutdown()
    want = oracle_run(plan, _events("S", ts, cols)).get("O", [])
    return got, want, launches


@pytest.mark.parametrize("n", [1, 2, 3, 511, 512, 513, 2047, 2048, 2049, 4097, 20001])
def test_ragged_lengths(n):
    plan = S_DEF + "from S[a > 10 and d < 1.5] select * insert into O;"
    got, want, k = _run(plan, n)
    assert k >= 1
    assert_same_rows(got, want, "ragged n=%d" % n)


@pytest.mark.parametrize("cond", ["e and a > 0 and d < 0.5",        # 3 columns, bool
                                  "a > 40 or d < -2.0",             # OR
                                  "c > 0.25",                       # float
                                  "b % 3 == 1",                     # long arithmetic
                                  "a > -1000"])                     # every row: many projection rounds
def test_predicate_shapes(cond):
    plan = S_DEF + "from S[%s] select d, a, e, b, c insert into O;" % cond
    got, want, _ = _run(plan, 9000, batches=3)
    assert len(want) > 0
    assert_same_rows(got, want, cond)


def test_no_predicate_projection():
    plan = S_DEF + "from S select b, a insert into O;"
    got, want, _ = _run(plan, 5000)
    assert len(want) == 5000
    assert_same_rows(got, want, "no predicate")


def test_device_batches_with_odd_lengths():
    plan = S_DEF + "from S[a % 7 == 0 and d > 0.0] select * insert into O;"
    got, want, _ = _run(plan, 30011, batches=7, device=True)
    assert_same_rows(got, want, "device batches")


def test_multi_stream_batch_selects_its_stream():
    plan = ("define stream S1 (a int, b long, c float, d double, e bool);"
            "define stream S2 (a int, b long, c float, d double, e bool);"
            "from S2[a > 0] select a, d insert into O;")
    n = 12345
    cols = _cols(n, 11)
    ts = np.arange(n, dtype=np.int64)
    st = (np.arange(n) % 3 == 1).astype(np.uint8)   # handle 1 = S2
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    assert rt.input_handle("S2") == 1
    rt.send("S1", ts, cols, streams=st)
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    ev = [("S2" if st[i] else "S1", int(ts[i]), (int(cols[0][i]), int(cols[1][i]), float(cols[2][i]),
                                                 float(cols[3][i]), bool(cols[4][i]))) for i in range(n)]
    want = oracle_run(plan, ev).get("O", [])
    assert len(want) > 1000
    assert_same_rows(got, want, "multi-stream")


def test_config2_large_batch_vs_c_oracle():
    import cep_oracle as CO
    n = (1 << 22) + 77
    w = workload.generate(0, n, 1 << 20, single_stream=True)
    rt = fs.SiddhiAppRuntime(workload.FILTER_PLAN)
    rt.add_callback("O")
    name = rt.intern("test_event")
    names = np.full(n, name, np.int32)
    rt.send("inputStream", w["ts"], [w["id"], names, w["price"], w["ts"]])
    rt.flush()
    out = rt.collect("O")
    rt.shutdown()
    sel = CO.filter_indices(w["id"], w["price"], CO.cond(("price", 0, ">", 0.5), ("id", 7, "==", 0)))
    np.testing.assert_array_equal(out.seq, sel)
    np.testing.assert_array_equal(out.ts, w["ts"][sel])
    np.testing.assert_array_equal(out.cols[0], w["id"][sel])
    np.testing.assert_array_equal(out.cols[2], w["price"][sel])
