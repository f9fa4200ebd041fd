"""CPU: the C restatement (oracle/cep_oracle.c) agrees with the independent
Python oracle on seeded streams of the config-2 and config-3 shapes."""
import numpy as np
import pytest

import cep_oracle as CO
from helpers import oracle_run, workload_events

from flink_siddhi import workload

F3 = CO.cond(("price", 0, ">", 0.5))
G3 = CO.cond(("id", 7, "==", 0))


@pytest.mark.parametrize("keys,rate,n", [(64, 1, 20000), (4, 1, 5000), (1000, 40, 30000)])
def test_c_oracle_matches_python_oracle_config3(keys, rate, n):
    w = workload.generate(0, n, keys, rate=rate)
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    po = CO.PatternOracle(keys, F3, G3, every=True, within=10000)
    a, b, m = po.run(w)
    assert m == len(want)
    got = [(int(w["ts"][j]), int(j), (int(w["k"][i]), float(w["price"][i]),
                                      float(w["price"][j]), int(w["ts"][j])))
           for i, j in zip(a.tolist(), b.tolist())]
    assert got == want


def test_c_oracle_state_carries_across_calls():
    w = workload.generate(0, 20000, 32, rate=1)
    po = CO.PatternOracle(32, F3, G3, within=10000)
    a1, b1, _ = po.run({k: v[:7000] for k, v in w.items()})
    a2, b2, _ = po.run({k: v[7000:] for k, v in w.items()})
    full = CO.PatternOracle(32, F3, G3, within=10000)
    a, b, _ = full.run(w)
    assert np.array_equal(np.concatenate([a1, a2]), a)
    assert np.array_equal(np.concatenate([b1, b2]), b)


def test_c_oracle_filter_matches_python():
    w = workload.generate(0, 20000, 10, single_stream=True)
    sel = CO.filter_indices(w["id"], w["price"], CO.cond(("price", 0, ">", 0.5), ("id", 7, "==", 0)))
    ev = [("inputStream", t, (i, 0, p, t)) for i, p, t in
          zip(w["id"].tolist(), w["price"].tolist(), w["ts"].tolist())]
    want = oracle_run(workload.FILTER_PLAN, ev)["O"]
    assert [s for _, s, _ in want] == sel.tolist()


def test_c_generator_and_sharded_digest():
    """oracle_generate == workload.generate; the key-sharded C oracle gives
    the same matches and order-sensitive digest at every thread count; the
    torch digest (bench.py's engine side) equals the C digest of the
    single-thread oracle's pairs."""
    import numpy as np
    import torch
    import cep_oracle as CO
    from flink_siddhi import workload
    w = workload.generate(1000, 150000, 4096, rate=3)
    w2 = CO.generate(1000, 150000, 4096, rate=3, threads=5)
    for c in w:
        assert np.array_equal(w[c], w2[c]), c
    f, g = CO.cond(("price", 0, ">", 0.5)), CO.cond(("id", 7, "==", 0))
    res = {T: CO.pattern_mt(w, 4096, f, g, True, 100, threads=T, idx0=1000)[:2] for T in (1, 3, 8)}
    assert len(set(res.values())) == 1, res
    po = CO.PatternOracle(4096, f, g, True, 100)
    po.idx = 1000
    a, b, m = po.run(w)
    assert (m, ) == (res[1][0], ) and m > 100
    ai, bi = a - 1000, b - 1000
    t = torch.from_numpy
    d = workload.rows_digest(t(w["k"][ai]), t(w["price"][ai]), t(w["price"][bi]), t(w["ts"][bi]), t(b))
    assert d == res[1][1]
    # order sensitivity: swapping two rows of one key changes the digest
    k = w["k"][ai]
    dup = np.nonzero(np.bincount(k) >= 2)[0][0]
    i, j = np.nonzero(k == dup)[0][:2]
    perm = np.arange(len(ai))
    perm[[i, j]] = perm[[j, i]]
    d2 = workload.rows_digest(t(k[perm]), t(w["price"][ai][perm]), t(w["price"][bi][perm]),
                              t(w["ts"][bi][perm]), t(b[perm]))
    assert d2 != d


# ---- config 5 family: oracle/mq_oracle.c vs the Python oracle -------------
@pytest.mark.parametrize("case,n,keys,rate", [("exact", 9000, 4, 1), ("variant", 6000, 24, 1),
                                              ("variant", 6000, 6, 3)])
def test_mq_oracle_matches_python_config5(case, n, keys, rate):
    import config5_cases as C5
    if case == "exact":
        plan, qs, outs = workload.config5_plan(), CO.config5_queries(), workload.CONFIG5_OUTPUTS
    else:
        plan, qs, outs = C5.variant_plan(), C5.variant_queries(), C5.variant_outputs()
    w = C5.three_streams(n, keys, rate=rate)
    want = oracle_run(plan, C5.events(w))
    got = CO.mq_rows(qs, w, keys)
    seq_rows = 0
    for i, o in enumerate(outs):
        assert got[i] == C5.as_words(want.get(o, [])), o
        seq_rows += len(got[i]) if o.startswith("Seq") else 0
    assert seq_rows > 0
    # sharded digests: independent of the thread count, equal to the rows' digest
    ref = None
    for T in (1, 3):
        c, d, _ = CO.mq_mt(qs, w, keys, threads=T)
        assert c == [len(r) for r in got]
        ref = ref or d
        assert d == ref
    for i in (0, 1, 32, 63):
        rank, dig = {}, 0
        for ts, seq, ws in got[i]:
            k = int(np.int64(np.uint64(ws[0])))
            r = rank.get(k, 0)
            rank[k] = r + 1
            dig = (dig + CO.mq_row_digest(k, r, ws, ts, seq)) & ((1 << 64) - 1)
        assert dig == ref[i], outs[i]


def test_mq_oracle_nfa_shapes():
    """Patterns (->), optional / bounded count states, non-every starts and
    first / last captures on a small 3-stream stream, against the Python oracle."""
    import config5_cases as C5
    plan = C5.EV3 + (
        "partition with (k of A, k of B, k of C) begin "
        "from every s1=A[price > 0.3] -> s2=B[id % 3 == 0] -> s3=C[price < 0.5] within 30 sec "
        "select s1.k as k, s1.price as p1, s2.id as i2, s3.ts as t insert into P;"
        "from every s1=A[id > 10], s2=B[price > 0.2]<1:3>, s3=C? "
        "select s1.k as k, s2[0].price as f, s2[last].price as l insert into S;"
        "from s1=B[id % 2 == 0], s2=A+, s3=C[id < 25] within 5 sec "
        "select s1.k as k, s2[last].id as i, s3.price as p insert into T; end;")
    qs = [CO.nfa_query([(0, 1, 1, [("price", 0, ">", 0.3)]), (1, 1, 1, [("id", 3, "==", 0)]),
                        (2, 1, 1, [("price", 0, "<", 0.5)])],
                       [(0, 0, "k"), (0, 0, "price"), (1, 0, "id"), (2, 0, "ts")], within=30000, sequence=False),
          CO.nfa_query([(0, 1, 1, [("id", 0, ">", 10)]), (1, 1, 3, [("price", 0, ">", 0.2)]), (2, 0, 1, [])],
                       [(0, 0, "k"), (1, 0, "price"), (1, -1, "price")]),
          CO.nfa_query([(1, 1, 1, [("id", 2, "==", 0)]), (0, 1, -1, []), (2, 1, 1, [("id", 0, "<", 25)])],
                       [(0, 0, "k"), (1, -1, "id"), (2, 0, "price")], within=5000, every=False)]
    w = C5.three_streams(5000, 16, rate=2)
    want = oracle_run(plan, C5.events(w))
    got = CO.mq_rows(qs, w, 16)
    for i, o in enumerate(("P", "S", "T")):
        assert got[i] == C5.as_words(want.get(o, [])), o
        assert len(got[i]) > 0, o
