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
