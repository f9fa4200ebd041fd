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
