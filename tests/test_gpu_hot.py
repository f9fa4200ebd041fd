"""Hot keys on the closed-form path (csrc/hot.hip) vs the C oracle.

Keys whose records would make their bucket a straggler are diverted by
k_cfpart into hot buckets and matched by grid-wide scans (k_hot_*), while
the walk keeps the rest; keys move between the two as the stream's skew
changes.  Every case compares the rows and their per-key order with
oracle/cep_oracle.c over the same events (BASELINE.md §3 Zipf variant and
harsher shapes: keys that go cold and hot again, hot keys whose B's are rare
so their pending lists spill to the overflow pool, sparse 64-bit key values).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cep_oracle as CO  # noqa: E402
import flink_siddhi as fs  # noqa: E402
from flink_siddhi import _lib as L  # noqa: E402
from flink_siddhi import workload  # noqa: E402
from test_gpu_geometry import F, assert_same_per_key  # noqa: E402


def run_batches(batches, keys, rate, plan, chunk, key_value=None, **opts):
    """batches: [(first, n, key remap table or None)] -> (device rows as numpy, stats)."""
    import torch
    rt = fs.SiddhiAppRuntime(plan, ts_order=1, chunk_events=chunk, ordered_output=0, key_capacity=keys, **opts)
    parts = []
    for first, n, table in batches:
        d = workload.generate_device(first, n, keys, rate=rate)
        if table is not None:
            d["k"] = torch.from_numpy(table).cuda()[d["k"].long()]
        k = d["k"] if key_value is None else key_value(d["k"])
        rt.send("A", d["ts"], [k, d["ts"], d["id"], d["price"]], streams=d["stream"])
        ts, seq, cols = rt.output_tensors("O")
        rt.flush()
        parts.append((ts, seq, cols))
    torch.cuda.synchronize()
    st = rt.stats()
    rt.shutdown()
    cat = lambda i: torch.cat([p[2][i] for p in parts]).cpu().numpy()  # noqa: E731
    out = {"k": cat(0), "p1": cat(1), "p2": cat(2), "t": cat(3),
           "ts": torch.cat([p[0] for p in parts]).cpu().numpy(),
           "seq": torch.cat([p[1] for p in parts]).cpu().numpy()}
    return out, st


def oracle_batches(batches, keys, rate, g, within):
    total = sum(n for _, n, _ in batches)
    w = CO.generate(0, total, keys, rate=rate, threads=16)
    for first, n, table in batches:
        if table is not None:
            w["k"][first:first + n] = table[w["k"][first:first + n]]
    po = CO.PatternOracle(keys, F, g, every=True, within=within)
    a, b, m = po.run(w)
    return {"k": w["k"][a], "p1": w["price"][a], "p2": w["price"][b], "t": w["ts"][b],
            "ts": w["ts"][b], "seq": b}, w


def plan_with(g_text, within_text):
    return (workload.PATTERN_PLAN.replace("id % 7 == 0", g_text)
            .replace("within 10 sec", within_text))


def test_hot_keys_come_and_go():
    # Zipf, then uniform (the hot keys go cold and are released), then Zipf
    # with other hot keys; 1 Mi-event chunks make keys with > 256 records per
    # chunk hot
    keys, rate, n = 1 << 16, 400, 1 << 21
    za = workload.zipf_map(keys, seed=7)
    zb = workload.zipf_map(keys, seed=99)
    tables = [za, za, za, None, None, zb, zb]
    batches = [(i * n, n, t) for i, t in enumerate(tables)]
    got, st = run_batches(batches, keys, rate, workload.PATTERN_PLAN, 1 << 20)
    want, _ = oracle_batches(batches, keys, rate, CO.cond(("id", 7, "==", 0)), 10000)
    assert st.kernel_launches[L.K_HOT] > 0, "hot-key path never engaged"
    assert st.kernel_launches[L.K_CF_WALK] > 0
    assert_same_per_key(got, want)
    assert len(want["k"]) > 300_000


def test_hot_keys_with_rare_b_spill_to_pool():
    # g true only for id == 0 (1 in 50 B's): a hot key's A's pile up for up to W, past the
    # 16 inline slots; the hot commit writes the overflow runs
    keys, rate, n = 1 << 14, 200, 1 << 21
    z = workload.zipf_map(keys, seed=3)
    batches = [(i * n, n, z) for i in range(4)]
    plan = plan_with("id % 97 == 0", "within 1 sec")
    got, st = run_batches(batches, keys, rate, plan, 1 << 20)
    want, _ = oracle_batches(batches, keys, rate, CO.cond(("id", 97, "==", 0)), 1000)
    assert st.kernel_launches[L.K_HOT] > 0
    assert_same_per_key(got, want)
    assert len(want["k"]) > 10_000


def test_hot_keys_sparse_long_values():
    # sparse_keys: 64-bit partition values through the device key map; the
    # hot rows output the original values
    keys, rate, n = 1 << 16, 400, 1 << 21
    z = workload.zipf_map(keys, seed=11)
    batches = [(i * n, n, z) for i in range(3)]
    base, mul = 1 << 40, 7919
    got, st = run_batches(batches, keys, rate, workload.PATTERN_PLAN.replace("k int", "k long"), 1 << 20,
                          key_value=lambda k: k.long() * mul + base, sparse_keys=1)
    want, _ = oracle_batches(batches, keys, rate, CO.cond(("id", 7, "==", 0)), 10000)
    assert st.kernel_launches[L.K_HOT] > 0
    got["k"] = ((got["k"].astype(np.int64) - base) // mul).astype(np.int32)
    assert_same_per_key(got, want)


def test_uniform_stream_never_diverts():
    # no key reaches the threshold: the hot kernels never run
    keys, rate, n = 1 << 16, 400, 1 << 21
    batches = [(i * n, n, None) for i in range(3)]
    got, st = run_batches(batches, keys, rate, workload.PATTERN_PLAN, 1 << 20)
    want, _ = oracle_batches(batches, keys, rate, CO.cond(("id", 7, "==", 0)), 10000)
    assert st.kernel_launches[L.K_HOT] == 0 and st.hot_keys == 0
    assert_same_per_key(got, want)


@pytest.mark.parametrize("world", [1, 2])
def test_hot_keys_on_shuffle_owners(world):
    # owners of the key shuffle (cep_send_records: k_cfpart from received
    # records) divert their hot keys too; the hot rows carry the global
    # arrival numbers of the received records
    import torch
    keys, rate, n_per, steps = 1 << 16, 400, 1 << 20, 4
    z = torch.from_numpy(workload.zipf_map(keys, seed=5)).cuda()
    plan = workload.PATTERN_PLAN
    rts = [fs.SiddhiAppRuntime(plan, ts_order=1, key_stride=world, key_offset=r, chunk_events=1 << 20,
                               key_capacity=keys, ordered_output=0) for r in range(world)]
    parts = [[] for _ in range(world)]
    for s in range(steps):
        segs = [[] for _ in range(world)]
        for src in range(world):
            first = (s * world + src) * n_per
            d = workload.generate_device(first, n_per, keys, rate=rate)
            d["k"] = z[d["k"].long()]
            recs, counts = rts[src].route("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], world,
                                          seq0=first, streams=d["stream"])
            off = np.concatenate([[0], np.cumsum(counts)])
            for r in range(world):
                segs[r].append(recs[off[r]:off[r + 1]].clone())
        for r in range(world):
            recv = torch.cat(segs[r], dim=0)
            rts[r].send_records(recv, recv.shape[0], n_per)
            ts, seq, cols = rts[r].output_tensors("O")
            rts[r].flush()
            parts[r].append((ts, seq, cols))
    torch.cuda.synchronize()
    hot = sum(rt.stats().kernel_launches[L.K_HOT] for rt in rts)
    got = {c: [] for c in ("k", "p1", "p2", "t", "ts", "seq")}
    for r in range(world):
        for ts, seq, cols in parts[r]:
            for c, v in zip(("k", "p1", "p2", "t"), cols):
                got[c].append(v.cpu().numpy())
            got["ts"].append(ts.cpu().numpy())
            got["seq"].append(seq.cpu().numpy())
    got = {c: np.concatenate(v) for c, v in got.items()}
    for rt in rts:
        rt.shutdown()
    total = steps * world * n_per
    w = CO.generate(0, total, keys, rate=rate, threads=16)
    w["k"] = z.cpu().numpy()[w["k"]]
    po = CO.PatternOracle(keys, F, CO.cond(("id", 7, "==", 0)), every=True, within=10000)
    a, b, m = po.run(w)
    want = {"k": w["k"][a], "p1": w["price"][a], "p2": w["price"][b], "t": w["ts"][b],
            "ts": w["ts"][b], "seq": b}
    assert hot > 0, "hot-key path never engaged on the owners"
    assert_same_per_key(got, want)


def test_low_threshold_fills_every_slot(monkeypatch):
    # threshold 16 at 1 Mi-event chunks: thousands of candidates per chunk, so
    # the candidate tiers overflow, all 1024 slots fill and busier keys
    # replace idle hot keys (k_hot_update's replacement pass); keys change hands
    # between the walk and the hot scans every chunk
    monkeypatch.setenv("CEP_HOT_THRESH", "16")
    keys, rate, n = 1 << 16, 400, 1 << 21
    za = workload.zipf_map(keys, seed=21)
    zb = workload.zipf_map(keys, seed=22)
    tables = [za, za, zb, zb, za]
    batches = [(i * n, n, t) for i, t in enumerate(tables)]
    got, st = run_batches(batches, keys, rate, workload.PATTERN_PLAN, 1 << 20)
    want, _ = oracle_batches(batches, keys, rate, CO.cond(("id", 7, "==", 0)), 10000)
    assert st.kernel_launches[L.K_HOT] > 0
    assert st.hot_keys > 512, st.hot_keys
    assert_same_per_key(got, want)


def test_hot_keys_come_and_go_with_overlap():
    # CEP_OVERLAP=1 runs each chunk's partition on the side stream beside the
    # previous chunk's walk; with hot keys the partition must also wait for
    # the previous hot update (it reads hot_id / hot_key).  The knob is read
    # once per process, so the case runs in one child process (the parent
    # keeps the GPU idle meanwhile) on the come-and-go stream above.
    import os
    import subprocess
    import sys
    from pathlib import Path
    here = Path(__file__).resolve().parent
    env = dict(os.environ, CEP_OVERLAP="1")
    code = ("import sys; sys.path[:0] = %r; import test_gpu_hot as t; "
            "t.test_hot_keys_come_and_go(); print('overlap ok')" % [str(here), str(here.parent / "oracle"),
                                                                     str(here.parent / "flink-siddhi_amd")])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "overlap ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
