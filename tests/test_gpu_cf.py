"""GPU parity of the closed-form fast path (k_cfpart / k_cfwalk,
flink-siddhi_amd/csrc/cf_kernels.hip) and of the general path it replaces
(k_partition / k_walk, CEP_NO_CF=1), both against the CPU oracle.

Bit-exact on every output column, ts, seq and the emission order.  The cases
push the fast path's edges: several chunks and batches, buckets whose records
overflow one LDS window (hot keys), pending partials carried across chunks,
batches where a carried column aliases the event-ts buffer (1 physical
carried word) or not (2), sharded key ownership, and snapshot/restore across
the two paths (same per-key state layout).
"""
import os

import numpy as np
import pytest

from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

pytestmark = pytest.mark.gpu

import flink_siddhi as fs  # noqa: E402
from flink_siddhi import _lib as L  # noqa: E402
from flink_siddhi import workload  # noqa: E402


@pytest.fixture(params=["cf", "general"])
def path(request, monkeypatch):
    """cf: k_cfpart + k_cfwalk; general: k_partition + k_walk (CEP_NO_CF=1)."""
    if request.param == "general":
        monkeypatch.setenv("CEP_NO_CF", "1")
    else:
        monkeypatch.delenv("CEP_NO_CF", raising=False)
    return request.param


def send_all(rt, w, batches=1, device=False):
    n = len(w["ts"])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        cols = {k: w[k][s:e] for k in ("k", "ts", "id", "price", "stream")}
        if device:
            import torch
            cols = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in cols.items()}
        rt.send("A", cols["ts"], [cols["k"], cols["ts"], cols["id"], cols["price"]],
                streams=cols["stream"])
        rt.flush()


def check_path(rt, path):
    st = rt.stats()
    cf = st.kernel_launches[L.K_CF_WALK]
    gen = st.kernel_launches[L.K_WALK]
    if path == "cf":
        assert cf > 0 and gen == 0, (cf, gen)
    else:
        assert cf == 0 and gen > 0, (cf, gen)


def run(plan, w, path, batches=1, device=False, **opts):
    rt = fs.SiddhiAppRuntime(plan, ts_order=1, **opts)
    rt.add_callback("O")
    send_all(rt, w, batches, device)
    got = engine_rows(rt.collect("O"))
    check_path(rt, path)
    rt.shutdown()
    return got


def case(plan, w, path, **kw):
    want = oracle_run(plan, workload_events(w)).get("O", [])
    got = run(plan, w, path, **kw)
    assert_same_rows(got, want, "%s path" % path)
    return len(want)


def test_config3_small(path):
    w = workload.generate(0, 60000, 4096, rate=1)
    assert case(workload.PATTERN_PLAN, w, path) > 300


def test_many_chunks_and_batches(path):
    # chunk 8192 rows (one fast-path tile): partials cross many chunk borders
    w = workload.generate(0, 50000, 1024, rate=2)
    assert case(workload.PATTERN_PLAN, w, path, batches=3, chunk_events=8192) > 200


def test_device_batch_aliases_ts(path):
    # device columns are used in place: the `ts` attribute IS the event-ts
    # buffer, so the fast path carries 1 physical word instead of 2
    w = workload.generate(0, 40000, 2048, rate=1)
    assert case(workload.PATTERN_PLAN, w, path, device=True, batches=2) > 100


def test_hot_keys_overflow_one_window(path):
    # 2 keys: each bucket holds ~13 k records per chunk -> several LDS windows,
    # long key runs (arrival sort), many pending partials
    plan = workload.PATTERN_PLAN.replace("within 10 sec", "within 15 milliseconds")
    w = workload.generate(0, 80000, 2, rate=1)
    assert case(plan, w, path, chunk_events=1 << 17) > 1000


def test_skewed_keys(path):
    # a heavy hitter (30 % of events) among 5000 uniform keys
    w = workload.generate(0, 60000, 5000, rate=4)
    rng = np.random.default_rng(11)
    hot = rng.random(len(w["k"])) < 0.3
    w["k"] = np.where(hot, 17, w["k"]).astype(np.int32)
    plan = workload.PATTERN_PLAN.replace("within 10 sec", "within 20 milliseconds")
    assert case(plan, w, path) > 500


def test_sharded_ownership(path):
    # this shard owns keys with k % 3 == 1 (cep_options key_stride / key_offset)
    w = workload.generate(0, 60000, 3000, rate=1)
    keep = (w["k"] % 3) == 1
    w = {k: v[keep] for k, v in w.items()}
    assert case(workload.PATTERN_PLAN, w, path, key_capacity=1000, key_stride=3,
                key_offset=1) > 100


def test_within_boundary_exact(path):
    # ts step 1 ms per event, within 5 ms: pairs exactly W apart match,
    # W + 1 apart do not (SURVEY App. A.3 inclusivity)
    plan = workload.PATTERN_PLAN.replace("within 10 sec", "within 5 milliseconds")
    w = workload.generate(0, 30000, 16, rate=1)
    assert case(plan, w, path) > 50


def test_select_key_and_captures_only():
    # s1.ts captured (aliases the event ts on device batches) + key
    plan = workload.EV2 if hasattr(workload, "EV2") else (
        "define stream A (k int, ts long, id int, price double);"
        "define stream B (k int, ts long, id int, price double);")
    plan += ("partition with (k of A, k of B) begin "
             "from every s1=A[price > 0.7] -> s2=B[id < 10] within 2 sec "
             "select s1.k as k, s1.ts as t1, s2.ts as t2, s1.price as p insert into O; end;")
    w = workload.generate(0, 40000, 512, rate=1)
    for dev in (False, True):
        assert case(plan, w, "cf", device=dev) > 100


def test_snapshot_cf_restore_general(monkeypatch):
    plan = workload.PATTERN_PLAN
    w = workload.generate(0, 40000, 2048, rate=1)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    half = 23000
    first_w = {k: v[:half] for k, v in w.items()}
    second_w = {k: v[half:] for k, v in w.items()}
    monkeypatch.delenv("CEP_NO_CF", raising=False)
    rt = fs.SiddhiAppRuntime(plan, ts_order=1)
    rt.add_callback("O")
    send_all(rt, first_w)
    first = engine_rows(rt.collect("O"))
    check_path(rt, "cf")
    snap = rt.snapshot()
    rt.shutdown()
    monkeypatch.setenv("CEP_NO_CF", "1")
    rt2 = fs.SiddhiAppRuntime(plan, ts_order=1)
    rt2.add_callback("O")
    rt2.restore(snap)
    send_all(rt2, second_w)
    second = engine_rows(rt2.collect("O"))
    check_path(rt2, "general")
    rt2.shutdown()
    assert_same_rows(first + second, want, "cf snapshot -> general restore")


def test_pending_lists_longer_than_pending_slots(path):
    """Siddhi's pending list is unbounded.  64 keys, B's rare (g: id % 25 ==
    0): runs of ~13 f-passing A's per key between g-passing B's, often more
    than pending_slots = 16 (SURVEY §7 "unbounded pending lists").  The
    closed-form path spills the tail to the pending pool and matches the
    oracle; the general path has per-key LDS lists and reports capacity."""
    w = workload.generate(0, 60000, 64, rate=1)
    plan = workload.PATTERN_PLAN.replace("id % 7 == 0", "id % 25 == 0")
    if path == "general":
        rt = fs.SiddhiAppRuntime(plan, ts_order=1, pending_slots=16)
        rt.add_callback("O")
        rt.send("A", w["ts"], [w["k"], w["ts"], w["id"], w["price"]], streams=w["stream"])
        with pytest.raises(fs.CepCapacityError):
            rt.flush()
        rt.shutdown()
        return
    assert case(plan, w, path, batches=3, chunk_events=16384, pending_slots=16) > 500


def test_pending_pool_exhausted_is_reported():
    w = workload.generate(0, 30000, 64, rate=1)
    plan = workload.PATTERN_PLAN.replace("id % 7 == 0", "id == 1000")   # no B: lists only grow
    rt = fs.SiddhiAppRuntime(plan, ts_order=1, pending_slots=4, pending_pool_log2=6)
    rt.add_callback("O")
    rt.send("A", w["ts"], [w["k"], w["ts"], w["id"], w["price"]], streams=w["stream"])
    with pytest.raises(fs.CepCapacityError, match="pool"):
        rt.flush()
    rt.shutdown()


def test_overflow_snapshot_restore():
    """Overflow runs survive snapshot / restore (snapshot v4 carries the
    pending count and every partial)."""
    w = workload.generate(0, 60000, 64, rate=1)
    plan = workload.PATTERN_PLAN.replace("id % 7 == 0", "id % 25 == 0")
    want = oracle_run(plan, workload_events(w)).get("O", [])
    h = 31000
    rt = fs.SiddhiAppRuntime(plan, ts_order=1, pending_slots=4)
    rt.add_callback("O")
    send_all(rt, {k: v[:h] for k, v in w.items()})
    first = engine_rows(rt.collect("O"))
    snap = rt.snapshot()
    rt.shutdown()
    rt2 = fs.SiddhiAppRuntime(plan, ts_order=1, pending_slots=4)
    rt2.add_callback("O")
    rt2.restore(snap)
    send_all(rt2, {k: v[h:] for k, v in w.items()})
    second = engine_rows(rt2.collect("O"))
    rt2.shutdown()
    assert_same_rows(first + second, want, "overflow snapshot/restore")


def test_fast_path_engaged_on_config3_device_batch():
    import torch
    os.environ.pop("CEP_NO_CF", None)
    d = workload.generate_device(0, 1 << 20, 1 << 14, rate=8)
    torch.cuda.synchronize()
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, ts_order=1)
    rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
    rt.flush()
    st = rt.stats()
    assert st.kernel_launches[L.K_CF_PARTITION] >= 1
    assert st.kernel_launches[L.K_CF_WALK] >= 1
    assert st.kernel_launches[L.K_WALK] == 0
    assert st.matches_out > 0
    rt.shutdown()
