"""Sparse partition keys (cep_options.sparse_keys): any int / long partition
value, mapped on the device to dense key slots (keymap.hip).  Siddhi's
`partition with` takes any attribute value and flink-siddhi's router hashes
whatever the group-by value is (router/AddRouteOperator.java:83-92); these
tests feed values far outside [0, key_capacity) — negative, 64-bit, the
encoding edge cases -1, 0, INT64_MIN / MAX — and compare rows (with the
original key values) and per-key order against the Python oracle.
"""
import numpy as np
import pytest

from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

pytestmark = pytest.mark.gpu

import flink_siddhi as fs  # noqa: E402
from flink_siddhi import workload  # noqa: E402

LONG_PLAN = workload.PATTERN_PLAN.replace("(k int,", "(k long,")


def run(plan, w, batches=2, device=False, **opts):
    rt = fs.SiddhiAppRuntime(plan, ts_order=1, sparse_keys=1, **opts)
    rt.add_callback("O")
    n = len(w["ts"])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        cols = {c: np.ascontiguousarray(w[c][s:e]) for c in ("k", "ts", "id", "price", "stream")}
        if device:
            import torch
            cols = {c: torch.from_numpy(v).cuda() for c, v in cols.items()}
        rt.send("A", cols["ts"], [cols["k"], cols["ts"], cols["id"], cols["price"]], streams=cols["stream"])
        rt.flush()
    got = engine_rows(rt.collect("O"))
    return rt, got


def by_key(rows):
    d = {}
    for r in rows:
        d.setdefault(r[2][0], []).append(r)
    return d


def long_values(nkeys, seed):
    rng = np.random.default_rng(seed)
    vals = rng.integers(-(1 << 63), (1 << 63) - 1, nkeys, dtype=np.int64)
    vals[:5] = [-1, 0, np.iinfo(np.int64).min, np.iinfo(np.int64).max, 1]
    return vals


@pytest.mark.parametrize("device", [False, True])
def test_long_keys_match_oracle(device):
    w = workload.generate(0, 60000, 3000, rate=1)
    w["k"] = long_values(3000, 5)[w["k"]]
    want = oracle_run(LONG_PLAN, workload_events(w)).get("O", [])
    rt, got = run(LONG_PLAN, w, batches=3, device=device, key_capacity=4096)
    rt.shutdown()
    assert len(want) > 300
    assert by_key(got) == by_key(want)


def test_int_keys_outside_key_capacity():
    w = workload.generate(0, 60000, 2000, rate=1)
    rng = np.random.default_rng(9)
    vals = rng.integers(-(1 << 31), (1 << 31) - 1, 2000, dtype=np.int64).astype(np.int32)
    vals[0] = -1
    w["k"] = vals[w["k"]]
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    rt, got = run(workload.PATTERN_PLAN, w, key_capacity=2048, ordered_output=1)
    rt.shutdown()
    assert_same_rows(got, want, "sparse int keys, Siddhi emission order")


def test_more_values_than_key_capacity_is_reported():
    w = workload.generate(0, 20000, 3000, rate=1)
    w["k"] = long_values(3000, 6)[w["k"]]
    rt = fs.SiddhiAppRuntime(LONG_PLAN, ts_order=1, sparse_keys=1, key_capacity=1024)
    rt.add_callback("O")
    rt.send("A", w["ts"], [w["k"], w["ts"], w["id"], w["price"]], streams=w["stream"])
    with pytest.raises(fs.CepCapacityError, match="distinct"):
        rt.flush()
    rt.shutdown()


def test_sparse_key_map_survives_snapshot():
    w = workload.generate(0, 60000, 3000, rate=1)
    w["k"] = long_values(3000, 7)[w["k"]]
    want = oracle_run(LONG_PLAN, workload_events(w)).get("O", [])
    h = 27000
    rt, first = run(LONG_PLAN, {c: v[:h] for c, v in w.items()}, batches=1, key_capacity=4096)
    snap = rt.snapshot()
    rt.shutdown()
    rt2 = fs.SiddhiAppRuntime(LONG_PLAN, ts_order=1, sparse_keys=1, key_capacity=4096)
    rt2.add_callback("O")
    rt2.restore(snap)
    rt2.send("A", w["ts"][h:], [w["k"][h:], w["ts"][h:], w["id"][h:], w["price"][h:]], streams=w["stream"][h:])
    rt2.flush()
    second = engine_rows(rt2.collect("O"))
    rt2.shutdown()
    assert by_key(first + second) == by_key(want)


def test_key_in_a_filter_is_unsupported():
    plan = workload.PATTERN_PLAN.replace("A[price > 0.5]", "A[price > 0.5 and k > 3]")
    with pytest.raises(fs.UnsupportedPlanException):
        fs.SiddhiAppRuntime(plan, ts_order=1, sparse_keys=1)
