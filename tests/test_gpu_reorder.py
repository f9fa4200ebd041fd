"""Event-time reorder on the device vs the oracle.

The operator buffers event-time records in a PriorityQueue and hands those
with ts <= watermark to Siddhi in timestamp order
(AbstractSiddhiOperator.java:222-231, 238-247).  process_elements /
process_watermark do the same on the device; ties keep arrival order (the
reference PQ is not stable — SURVEY.md App. B a5 — so the oracle is fed the
stable (ts, arrival) order).  Bit-exact against the oracle run on that order.
"""
import numpy as np
import pytest

from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

pytestmark = pytest.mark.gpu

import flink_siddhi as fs  # noqa: E402
from flink_siddhi import workload  # noqa: E402

COLS = ("k", "ts", "id", "price", "stream")


def disordered(n, keys, rate, jitter, seed):
    """The generator stream, arriving out of order: row i arrives at rank of
    i + U[0, jitter) (bounded lateness)."""
    w = workload.generate(0, n, keys, rate=rate)
    rng = np.random.default_rng(seed)
    arrival = np.argsort(np.arange(n) + rng.integers(0, jitter, n), kind="stable")
    return {c: w[c][arrival] for c in COLS}


def sorted_by_ts(w):
    o = np.argsort(w["ts"], kind="stable")   # (ts, arrival)
    return {c: w[c][o] for c in COLS}


def run_reorder(plan, w, batches, out="O", perfect_watermarks=True, **opts):
    rt = fs.SiddhiAppRuntime(plan, **opts)
    rt.add_callback(out)
    n = len(w["ts"])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    # perfect watermark after batch b: every row not yet arrived is later
    suffix_min = np.minimum.accumulate(w["ts"][::-1])[::-1]
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        rt.process_elements("A", w["ts"][s:e], [w["k"][s:e], w["ts"][s:e], w["id"][s:e], w["price"][s:e]],
                            streams=w["stream"][s:e])
        if perfect_watermarks and e < n:
            rt.process_watermark(int(suffix_min[e]) - 1)
    rt.process_watermark(int(w["ts"].max()))
    assert rt.buffered() == 0
    rt.flush()
    got = engine_rows(rt.collect(out))
    rt.shutdown()
    return got


@pytest.mark.parametrize("rate,batches", [(1, 1), (4, 7), (16, 13)])
def test_reordered_pattern_matches_oracle_in_event_time_order(rate, batches):
    w = disordered(40000, 4096, rate, jitter=700, seed=rate)
    want = oracle_run(workload.PATTERN_PLAN, workload_events(sorted_by_ts(w))).get("O", [])
    got = run_reorder(workload.PATTERN_PLAN, w, batches)
    assert_same_rows(got, want, "reorder rate=%d batches=%d" % (rate, batches))
    assert len(want) > 100


def test_reordered_multi_chunk_buffers_across_watermarks():
    # several engine chunks per release, rows held back over many watermarks
    w = disordered(120000, 4096, 8, jitter=5000, seed=7)
    want = oracle_run(workload.PATTERN_PLAN, workload_events(sorted_by_ts(w))).get("O", [])
    got = run_reorder(workload.PATTERN_PLAN, w, 11, chunk_events=1 << 15)
    assert_same_rows(got, want, "reorder multi-chunk")


def test_watermark_releases_only_rows_at_or_before_it():
    w = sorted_by_ts(disordered(5000, 2048, 1, jitter=50, seed=3))
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt.add_callback("O")
    rt.process_elements("A", w["ts"], [w["k"], w["ts"], w["id"], w["price"]], streams=w["stream"])
    assert rt.buffered() == 5000
    mid = int(w["ts"][2499])
    rt.process_watermark(mid)
    assert rt.buffered() == int((w["ts"] > mid).sum())
    rt.process_watermark(int(w["ts"][0]) - 1)   # nothing new to release
    assert rt.buffered() == int((w["ts"] > mid).sum())
    rt.process_watermark(int(w["ts"].max()))
    assert rt.buffered() == 0
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    assert_same_rows(got, want, "watermark split")


def test_late_event_is_dropped():
    """late_policy=0: a row older than an earlier watermark's release is
    dropped and counted (it used to stay buffered and wedge every
    later watermark); the on-time rows of the same watermark still go
    through, the buffer drains, and later watermarks keep working.  (The
    default, late_policy=2, delivers it as the reference does:
    test_gpu_ooo.py.)"""
    plan = workload.PATTERN_PLAN.replace("within 10 sec", "within 1 sec")
    rt = fs.SiddhiAppRuntime(plan, late_policy=0)
    rt.add_callback("O")
    n = 100
    ts = np.arange(1000, 1000 + n, dtype=np.int64)
    z = np.zeros(n, dtype=np.int32)
    idv = np.where(np.arange(n) % 3 == 2, 7, 1).astype(np.int32)   # every 3rd row: a g-passing B
    p = np.full(n, 0.75)
    st = (np.arange(n) % 3 == 2).astype(np.uint8)
    rt.process_elements("A", ts, [z, ts, idv, p], streams=st)
    rt.process_watermark(1050)
    late = np.array([1020], dtype=np.int64)
    rt.process_elements("A", late, [z[:1], late, z[:1], p[:1]], streams=st[:1])
    more = np.arange(1100, 1110, dtype=np.int64)
    rt.process_elements("A", more, [z[:10], more, idv[:10], p[:10]], streams=st[:10])
    rt.process_watermark(1105)     # releases 1051..1105, drops the late 1020
    assert rt.stats().late_events == 1
    assert rt.buffered() == 4
    rt.process_watermark(2000)
    assert rt.buffered() == 0
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    allts = np.concatenate([ts, more])
    cols = [np.concatenate([z, z[:10]]), allts, np.concatenate([idv, idv[:10]]), np.concatenate([p, p[:10]])]
    stv = np.concatenate([st, st[:10]])
    ev = [("AB"[stv[i]], int(allts[i]), tuple(c[i].item() for c in cols)) for i in range(len(allts))]
    want = oracle_run(plan, ev).get("O", [])
    assert len(want) > 0
    assert_same_rows(got, want, "late row dropped")


def test_late_policy_reports_late_events():
    """late_policy=1: the on-time rows are still released, the late row is
    dropped, and the watermark call raises so a caller relying on the
    reference's hand-over of late rows (AbstractSiddhiOperator.java:238-245)
    notices."""
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, late_policy=1)
    n = 50
    ts = np.arange(1000, 1000 + n, dtype=np.int64)
    z = np.zeros(n, dtype=np.int32)
    p = np.full(n, 0.75)
    st = np.zeros(n, dtype=np.uint8)
    rt.process_elements("A", ts, [z, ts, z, p], streams=st)
    rt.process_watermark(1020)
    late = np.array([1005], dtype=np.int64)
    rt.process_elements("A", late, [z[:1], late, z[:1], p[:1]], streams=st[:1])
    with pytest.raises(ValueError, match="late"):
        rt.process_watermark(1030)
    assert rt.stats().late_events == 1
    assert rt.buffered() == n - 31
    rt.process_watermark(2000)     # no late rows: fine
    assert rt.buffered() == 0
    rt.shutdown()


def test_reordered_filter_matches_oracle():
    plan = workload.FILTER_PLAN
    n = 30000
    w = workload.generate(0, n, 1, single_stream=True, rate=4)
    rng = np.random.default_rng(11)
    arrival = np.argsort(np.arange(n) + rng.integers(0, 300, n), kind="stable")
    cols = {c: w[c][arrival] for c in ("id", "price", "ts")}
    rt = fs.SiddhiAppRuntime(plan)
    rt.add_callback("O")
    name = rt.intern("test_event")
    names = np.full(n, name, np.int32)
    for s in range(0, n, 7000):
        e = min(n, s + 7000)
        rt.process_elements("inputStream", cols["ts"][s:e],
                            [cols["id"][s:e], names[s:e], cols["price"][s:e], cols["ts"][s:e]])
    rt.process_watermark(int(cols["ts"].max()))
    rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    o = np.argsort(cols["ts"], kind="stable")
    ev = [("inputStream", t, (i, name, p, t)) for i, p, t in
          zip(cols["id"][o].tolist(), cols["price"][o].tolist(), cols["ts"][o].tolist())]
    want = oracle_run(plan, ev)["O"]
    assert_same_rows(got, want, "reordered filter")


def test_snapshot_keeps_rows_waiting_for_a_watermark():
    # the operator checkpoints its queue ("queuedRecordsState",
    # AbstractSiddhiOperator.java:98): buffered rows survive snapshot / restore
    w = disordered(40000, 4096, 2, jitter=900, seed=5)
    want = oracle_run(workload.PATTERN_PLAN, workload_events(sorted_by_ts(w))).get("O", [])
    half = 23000
    suffix_min = np.minimum.accumulate(w["ts"][::-1])[::-1]
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt.add_callback("O")
    rt.process_elements("A", w["ts"][:half], [w["k"][:half], w["ts"][:half], w["id"][:half], w["price"][:half]],
                        streams=w["stream"][:half])
    rt.process_watermark(int(suffix_min[half]) - 1)
    held = rt.buffered()
    assert held > 0
    rt.flush()
    first = engine_rows(rt.collect("O"))
    snap = rt.snapshot()
    rt.shutdown()
    rt2 = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt2.add_callback("O")
    rt2.restore(snap)
    assert rt2.buffered() == held
    rt2.process_elements("A", w["ts"][half:], [w["k"][half:], w["ts"][half:], w["id"][half:], w["price"][half:]],
                         streams=w["stream"][half:])
    rt2.process_watermark(int(w["ts"].max()))
    rt2.flush()
    second = engine_rows(rt2.collect("O"))
    rt2.shutdown()
    assert_same_rows(first + second, want, "reorder snapshot/restore")


def test_restore_rejects_truncated_snapshot_and_keeps_state():
    """A v3 snapshot cut inside the reorder-buffer rows is refused before
    anything on the device changes (restore used to commit while
    parsing); the untouched runtime keeps working."""
    w = disordered(20000, 1024, 2, jitter=600, seed=9)
    half = 12000
    suffix_min = np.minimum.accumulate(w["ts"][::-1])[::-1]
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt.process_elements("A", w["ts"][:half], [w["k"][:half], w["ts"][:half], w["id"][:half], w["price"][:half]],
                        streams=w["stream"][:half])
    rt.process_watermark(int(suffix_min[half]) - 1)
    held = rt.buffered()
    assert held > 0
    rt.flush()
    snap = rt.snapshot()
    rt.shutdown()
    rt2 = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    for cut in (len(snap) - 2, len(snap) - held * 5, 30):
        with pytest.raises(fs.CepStateError):
            rt2.restore(snap[:cut])
        assert rt2.buffered() == 0
    # a lying row count (n huge, bytes short) is refused too
    import struct
    body = bytearray(snap)
    # reorder rows (columns k ts id price + event ts + stream), then the
    # 1-byte key-map section of the one pattern and the (v5) u32 count of
    # multi-query groups
    tail = len(body) - 1 - 4 - held * (4 + 8 + 4 + 8 + 8 + 1)
    n_off = tail - 8 - 8                                   # i64 n, i64 released_max precede the rows
    assert struct.unpack_from("<q", body, n_off)[0] == held
    struct.pack_into("<q", body, n_off, (1 << 31) - 1)
    with pytest.raises(fs.CepStateError):
        rt2.restore(bytes(body))
    rt2.restore(snap)
    assert rt2.buffered() == held
    rt2.shutdown()


def test_restore_version2_snapshot():
    """Version-2 snapshots (per-key state only, no reorder section) still load."""
    import struct
    w = workload.generate(0, 30000, 2048, rate=1)
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    h = 17000
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt.add_callback("O")
    rt.send("A", w["ts"][:h], [w["k"][:h], w["ts"][:h], w["id"][:h], w["price"][:h]], streams=w["stream"][:h])
    rt.flush()
    first = engine_rows(rt.collect("O"))
    snap = bytearray(rt.snapshot())
    rt.shutdown()
    assert struct.unpack_from("<I", snap, 4)[0] == 5
    # version 2 layout: no per-key pending count, no reorder section (an
    # empty one is i32 input, u8 has_stream, i64 n, i64 released_max)
    v2 = bytearray(snap[:28])
    struct.pack_into("<I", v2, 4, 2)
    off = 28
    for _ in range(struct.unpack_from("<I", snap, 24)[0]):
        kc, S, sw, live = struct.unpack_from("<qIII", snap, off)
        v2 += snap[off:off + 20]
        off += 20
        for _ in range(live):
            key, hdr, n = struct.unpack_from("<IQI", snap, off)
            assert n == hdr & 0xff
            v2 += snap[off:off + 12]
            v2 += snap[off + 16:off + 16 + n * sw * 8]
            off += 16 + n * sw * 8
    assert len(snap) - off == 26   # empty reorder section + the key-map byte + no groups
    rt2 = fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
    rt2.add_callback("O")
    rt2.restore(bytes(v2))
    rt2.send("A", w["ts"][h:], [w["k"][h:], w["ts"][h:], w["id"][h:], w["price"][h:]], streams=w["stream"][h:])
    rt2.flush()
    second = engine_rows(rt2.collect("O"))
    rt2.shutdown()
    assert_same_rows(first + second, want, "v2 restore")
