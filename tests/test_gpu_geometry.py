"""GPU parity at the BENCHMARKED geometry (BASELINE config 3 exactly as
bench.py runs it): K = 2^20 partition keys, R = 400 events/ms, 32 Mi-event
chunks (4096 tiles of 8192 rows: the k_cfpart / k_cfwalk tile limit), device
batches, and 80 Mi events over three batches so per-key state carries across
chunk and batch borders (one batch ends 777 events into a chunk).

Checker: oracle/cep_oracle.c (the scalar restatement, one thread, full match
pairs) over the same events generated on the host by oracle_generate.  Every
output row (k, p1, p2, t, event ts, completing-event arrival number) must be
identical and each key's rows must come in the same order (Siddhi emission
order per key, AbstractSiddhiOperator.java:130 -> StreamOutputHandler.java:63);
the engine runs with ordered_output=0 as the bench does, so rows of different
keys may interleave differently.  Also checked: the order-sensitive row
digest (flink_siddhi.workload.rows_digest == oracle_pattern_mt's digest), the
digest bench.py compares on every run.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cep_oracle as CO  # noqa: E402
import flink_siddhi as fs  # noqa: E402
from flink_siddhi import _lib as L  # noqa: E402
from flink_siddhi import workload  # noqa: E402

K = 1 << 20
R = 400
CHUNK = 1 << 25
F = CO.cond(("price", 0, ">", 0.5))
G = CO.cond(("id", 7, "==", 0))


def run_engine(sizes, keys=K, rate=R, plan=workload.PATTERN_PLAN, key_of=None, **opts):
    """Device batches of the config-3 stream through the engine; returns the
    concatenated device output as numpy (emission order) and the stats."""
    import torch
    rt = fs.SiddhiAppRuntime(plan, ts_order=1, chunk_events=CHUNK, ordered_output=0, **opts)
    first, parts = 0, []
    for n in sizes:
        d = workload.generate_device(first, n, keys, rate=rate)
        if key_of is not None:
            d["k"] = key_of(d["k"])
        rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
        ts, seq, cols = rt.output_tensors("O")
        rt.flush()
        parts.append((ts, seq, cols))
        first += n
        del d
    torch.cuda.synchronize()
    st = rt.stats()
    assert st.kernel_launches[L.K_CF_WALK] > 0 and st.kernel_launches[L.K_WALK] == 0
    rt.shutdown()
    cat = lambda i: torch.cat([p[2][i] for p in parts])  # noqa: E731
    out = {"k": cat(0), "p1": cat(1), "p2": cat(2), "t": cat(3),
           "ts": torch.cat([p[0] for p in parts]), "seq": torch.cat([p[1] for p in parts])}
    return out, st


def oracle_rows(w, keys, within=10000):
    po = CO.PatternOracle(keys, F, G, every=True, within=within)
    a, b, m = po.run(w)
    assert m == len(a)
    return {"k": w["k"][a], "p1": w["price"][a], "p2": w["price"][b], "t": w["ts"][b],
            "ts": w["ts"][b], "seq": b}


def assert_same_per_key(got, want):
    """Identical rows, identical order inside every key."""
    n = len(want["k"])
    assert len(got["k"]) == n, (len(got["k"]), n)
    og = np.argsort(got["k"], kind="stable")
    ow = np.argsort(want["k"], kind="stable")
    for c in ("k", "p1", "p2", "t", "ts", "seq"):
        a, b = got[c][og], want[c][ow]
        if not np.array_equal(a, b):
            i = int(np.nonzero(a != b)[0][0])
            raise AssertionError("column %s differs at per-key position %d: engine %r oracle %r "
                                 "(key %d)" % (c, i, a[i], b[i], int(want["k"][ow][i])))


def test_config3_bench_geometry():
    sizes = [CHUNK + 777, CHUNK - 777, 1 << 24]
    out, st = run_engine(sizes)
    n = sum(sizes)
    assert st.events_in == n
    w = CO.generate(0, n, K, rate=R, threads=16)
    want = oracle_rows(w, K)
    got = {c: v.cpu().numpy() for c, v in out.items()}
    assert len(got["k"]) > 4_000_000          # ~0.066 matches per event
    assert st.matches_out == len(got["k"])
    assert_same_per_key(got, want)
    # the bench's order-sensitive digest agrees with the sharded oracle
    m, dig, _ = CO.pattern_mt(w, K, F, G, True, 10000, threads=16)
    assert m == len(want["k"])
    assert workload.rows_digest(out["k"], out["p1"], out["p2"], out["t"], out["seq"]) == dig


def test_vm_walk_16mi_chunks_vs_oracle():
    # the interpreter build of the walk (computed select items, sequences,
    # aggregates) takes 16 Mi-row chunks: a chunk spanning 8192 partition
    # tiles, plus a short second one, vs the C oracle
    import torch
    plan = workload.PATTERN_PLAN.replace("s1.price as p1", "s1.price * 2.0 as p1")
    n = (1 << 24) + 123457
    rt = fs.SiddhiAppRuntime(plan, ts_order=1, chunk_events=1 << 24, ordered_output=0)
    d = workload.generate_device(0, n, K, rate=R)
    rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
    ts, seq, cols = rt.output_tensors("O")
    rt.flush()
    st = rt.stats()
    assert st.kernel_launches[L.K_WALK] == 2 and st.kernel_launches[L.K_CF_WALK] == 0
    got = {"k": cols[0].cpu().numpy(), "p1": cols[1].cpu().numpy() / 2.0, "p2": cols[2].cpu().numpy(),
           "t": cols[3].cpu().numpy(), "ts": ts.cpu().numpy(), "seq": seq.cpu().numpy()}
    rt.shutdown()
    del d
    torch.cuda.empty_cache()
    w = CO.generate(0, n, K, rate=R, threads=16)
    assert_same_per_key(got, oracle_rows(w, K))


def test_config3_ordered_delivery_bench_geometry():
    # ordered_output = 1 (the drop-in default): the flush sorts each output's
    # rows by completing event on the device (stable on seq, so one event's
    # matches keep pending order) and delivers them to the host callback in
    # Siddhi's global emission order (StreamOutputHandler.java:63-92) — every
    # row identical to the oracle's, in the same position.
    import torch
    sizes = [CHUNK + 777, 1 << 23]
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, ts_order=1, chunk_events=CHUNK, ordered_output=1)
    rt.add_callback("O")
    first = 0
    for n in sizes:
        d = workload.generate_device(first, n, K, rate=R)
        rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
        rt.flush()
        first += n
        del d
    out = rt.collect("O")
    rt.shutdown()
    torch.cuda.empty_cache()
    w = CO.generate(0, first, K, rate=R, threads=16)
    po = CO.PatternOracle(K, F, G, every=True, within=10000)
    a, b, m = po.run(w)
    order = np.lexsort((a, b))     # completing event, then pending (arrival) order
    a, b = a[order], b[order]
    assert m > 2_000_000 and len(out.ts) == m, (len(out.ts), m)
    want = {"k": w["k"][a], "p1": w["price"][a], "p2": w["price"][b], "t": w["ts"][b], "ts": w["ts"][b], "seq": b}
    got = {"k": out.cols[0], "p1": out.cols[1], "p2": out.cols[2], "t": out.cols[3], "ts": out.ts, "seq": out.seq}
    for c in want:
        if not np.array_equal(got[c], want[c]):
            i = int(np.nonzero(got[c] != want[c])[0][0])
            raise AssertionError("column %s differs at row %d: engine %r oracle %r" % (c, i, got[c][i], want[c][i]))
