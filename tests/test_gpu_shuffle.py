"""Key shuffle through the device path (one GPU, simulated world): every
source slice is routed by the engine (cep_route_batch: push-down + owner
grouping), owner r receives the slices' r-segments in source order and runs
them through cep_send_records on an engine that owns keys k % world == r.
The merged output must equal the CPU oracle over the whole stream."""
import numpy as np
import pytest
import torch

import flink_siddhi as fs
from flink_siddhi import _lib as L
from flink_siddhi import workload
from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

pytestmark = pytest.mark.gpu


def _dev(w):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in w.items()}


@pytest.mark.parametrize("path", ["cf", "general"])
@pytest.mark.parametrize("world", [2, 3])
def test_route_exchange_matches_oracle(world, path, monkeypatch):
    # owners run the received records through the closed-form fast path
    # (k_cfpart from records) or, with CEP_NO_CF=1, the general k_partition
    if path == "general":
        monkeypatch.setenv("CEP_NO_CF", "1")
    else:
        monkeypatch.delenv("CEP_NO_CF", raising=False)
    n_per, keys = 12000, 600
    plan = workload.PATTERN_PLAN
    sender = fs.SiddhiAppRuntime(plan, ts_order=1)
    owners = [fs.SiddhiAppRuntime(plan, ts_order=1, key_stride=world, key_offset=r, chunk_events=8192)
              for r in range(world)]
    for o in owners:
        o.add_callback("O")
    segs = [[] for _ in range(world)]
    for src in range(world):
        w = workload.generate(src * n_per, n_per, keys, rate=1)
        d = _dev(w)
        recs, counts = sender.route("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]],
                                    world, seq0=src * n_per, streams=d["stream"])
        off = np.concatenate([[0], np.cumsum(counts)])
        for r in range(world):
            segs[r].append(recs[off[r]:off[r + 1]].clone())
    got = []
    for r in range(world):
        recv = torch.cat(segs[r], dim=0)
        assert bool((recv[:, 1][1:] > recv[:, 1][:-1]).all()), "records not in arrival order"
        assert bool(((recv[:, 0] & 0xffffffff) % world == r).all())
        owners[r].send_records(recv, recv.shape[0], n_per)
        owners[r].flush()
        got += engine_rows(owners[r].collect("O"))
        st = owners[r].stats()
        if path == "cf":
            assert st.kernel_launches[L.K_CF_WALK] > 0 and st.kernel_launches[L.K_WALK] == 0
        else:
            assert st.kernel_launches[L.K_CF_WALK] == 0 and st.kernel_launches[L.K_WALK] > 0
    got.sort(key=lambda t: t[1])
    w = workload.generate(0, world * n_per, keys, rate=1)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    assert len(want) > 100
    assert_same_rows(got, want, "shuffle world=%d" % world)
    for rt in owners + [sender]:
        rt.shutdown()


@pytest.mark.parametrize("world", [4, 11])
def test_fast_route_equals_general_route(world, monkeypatch):
    # k_cfroute (8192-row tiles, scalar owner counters for world <= 8, LDS
    # counters above) and k_route (CEP_NO_CF=1) ship identical records
    n, keys = 50000, 4096
    w = workload.generate(0, n, keys, rate=1)
    d = _dev(w)
    got = {}
    for path in ("cf", "general"):
        if path == "general":
            monkeypatch.setenv("CEP_NO_CF", "1")
        else:
            monkeypatch.delenv("CEP_NO_CF", raising=False)
        rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, ts_order=1)
        recs, counts = rt.route("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], world,
                                seq0=7, streams=d["stream"])
        got[path] = (recs[:sum(counts)].cpu().numpy().copy(), counts)
        rt.shutdown()
    (ra, ca), (rb, cb) = got["cf"], got["general"]
    assert ca == cb and sum(ca) > 1000
    assert (ra[:, :4] == rb[:, :4]).all()
    is_b = ((ra[:, 0] >> 40) & 0xff) == 1
    assert (ra[is_b, 4] == rb[is_b, 4]).all()


@pytest.mark.parametrize("world", [1, 2])
def test_pipelined_route_overlaps_walk(world):
    # the bench's multi-GPU step loop (bench.py run_shuffle): rank r's engine
    # routes its slice of step s+1 on its route stream while the walk of step
    # s runs on its engine stream; send / receive buffers double-buffered,
    # reuse ordered by guard streams (send_records(signal=False) + signal)
    steps, n_per, keys = 4, 40000, 2000
    plan = workload.PATTERN_PLAN
    rts = [fs.SiddhiAppRuntime(plan, ts_order=1, key_stride=world, key_offset=r, chunk_events=16384)
           for r in range(world)]
    for rt in rts:
        rt.add_callback("O")
    guard = [[torch.cuda.Stream(), torch.cuda.Stream()] for _ in range(world)]
    bufs = {}
    data = [[_dev(workload.generate((s * world + r) * n_per, n_per, keys, rate=1))
             for r in range(world)] for s in range(steps)]

    def route(s, j):
        out = []
        for r in range(world):
            d = data[s][r]
            recs, counts = rts[r].route("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], world,
                                        seq0=(s * world + r) * n_per, streams=d["stream"],
                                        out=bufs.get(("send", r, j)))
            bufs[("send", r, j)] = recs
            out.append((recs, counts))
        return out

    cur = route(0, 0)
    for s in range(steps):
        j = s % 2
        offs = [np.concatenate([[0], np.cumsum(c)]) for _, c in cur]
        for r in range(world):
            torch.cuda.current_stream().wait_stream(guard[r][j])
            m = sum(int(cur[src][1][r]) for src in range(world))
            buf = bufs.get(("recv", r, j))
            if buf is None or buf.shape[0] < m:
                buf = torch.empty((max(m, 1), cur[0][0].shape[1]), dtype=torch.int64, device="cuda")
                bufs[("recv", r, j)] = buf
            o = 0
            for src in range(world):   # the all-to-all, in source-rank order
                a, b = offs[src][r], offs[src][r + 1]
                buf[o:o + b - a].copy_(cur[src][0][a:b])
                o += b - a
            rts[r].send_records(buf, m, n_per, signal=False)
            rts[r].signal(guard[r][j])
        if s + 1 < steps:
            cur = route(s + 1, 1 - j)
    got = []
    for rt in rts:
        rt.flush()
        got += engine_rows(rt.collect("O"))
    got.sort(key=lambda t: t[1])
    w = workload.generate(0, steps * world * n_per, keys, rate=1)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    assert len(want) > 1000
    assert_same_rows(got, want, "pipelined world=%d" % world)
    for rt in rts:
        rt.shutdown()


def _padded_round(world, n_per, keys, seg_cap, steps=1, cap_fn=None):
    """Sources route with cep_route_batch_padded; owner r receives segment r
    of every source in source order (the equal-split all-to-all) and feeds
    them to cep_send_records_padded.  No counts are read back anywhere."""
    plan = workload.PATTERN_PLAN
    senders = [fs.SiddhiAppRuntime(plan, ts_order=1) for _ in range(world)]
    owners = [fs.SiddhiAppRuntime(plan, ts_order=1, key_stride=world, key_offset=r, chunk_events=8192)
              for r in range(world)]
    for o in owners:
        o.add_callback("O")
    for s in range(steps):
        sent = []
        for src in range(world):
            g = s * world + src
            w = workload.generate(g * n_per, n_per, keys, rate=1)
            d = _dev(w)
            segs = senders[src].route_padded("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]],
                                             world, seq0=g * n_per, seg_cap=seg_cap, streams=d["stream"])
            sent.append(segs)
        torch.cuda.synchronize()
        S = 1 + seg_cap
        for r in range(world):
            recv = torch.cat([sent[src][r * S:(r + 1) * S] for src in range(world)], dim=0)
            owners[r].send_padded(recv, world, seg_cap, n_per)
    return senders, owners


@pytest.mark.parametrize("path", ["cf", "general"])
@pytest.mark.parametrize("world", [2, 3])
def test_padded_exchange_matches_oracle(world, path, monkeypatch):
    # fixed per-peer segments with in-band counts; the
    # null records (header + tail) must be invisible to both partitions
    if path == "general":
        monkeypatch.setenv("CEP_NO_CF", "1")
    else:
        monkeypatch.delenv("CEP_NO_CF", raising=False)
    from flink_siddhi import shuffle
    n_per, keys, steps = 12000, 600, 2
    cap = shuffle.padded_capacity(n_per, world)
    senders, owners = _padded_round(world, n_per, keys, cap, steps=steps)
    got = []
    for o in owners:
        o.flush()
        got += engine_rows(o.collect("O"))
    got.sort(key=lambda t: t[1])
    w = workload.generate(0, steps * world * n_per, keys, rate=1)
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    assert len(want) > 100
    assert_same_rows(got, want, "padded shuffle world=%d" % world)
    for rt in owners + senders:
        rt.shutdown()


def test_padded_segment_headers_carry_the_counts():
    world, n, keys = 4, 30000, 900
    w = workload.generate(0, n, keys, rate=1)
    d = _dev(w)
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, ts_order=1)
    recs, counts = rt.route("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], world, seq0=5,
                            streams=d["stream"])
    recs = recs[:sum(counts)].cpu().numpy().copy()
    cap = max(counts) + 3
    segs = rt.route_padded("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], world, seq0=5,
                           seg_cap=cap, streams=d["stream"])
    torch.cuda.synchronize()
    s = segs.cpu().numpy().reshape(world, 1 + cap, -1)
    off = np.concatenate([[0], np.cumsum(counts)])
    for r in range(world):
        h = s[r, 0]
        assert int(h[0]) & 0xffffffff == counts[r] and (int(h[0]) >> 32) & 0xff == 0
        assert int(h[1]) == 5 and int(h[2]) == int(w["ts"][0])
        assert (s[r, 1:1 + counts[r]] == recs[off[r]:off[r + 1]]).all()
        tail = s[r, 1 + counts[r]:]
        assert ((tail[:, 0] >> 32) & 0xff == 0).all()          # role 0: null records
        assert (tail[:, 1] == 5 + n - 1).all() and (tail[:, 2] == int(w["ts"][-1])).all()
    rt.shutdown()


def test_padded_overflow_fails_the_next_flush():
    world, n_per, keys = 2, 12000, 600
    senders, owners = _padded_round(world, n_per, keys, seg_cap=64)
    with pytest.raises(fs.CepCapacityError, match="seg_cap"):
        owners[0].flush()
    for rt in owners + senders:
        rt.shutdown()


def _spill_round(world, n_per, keys, seg_cap, steps, skew_step=None, rows=False):
    """As _padded_round with cep_route_*_padded_spill: every source's records
    past seg_cap go to its spill buffer; a step that spilled anywhere reaches
    the owners merged per source rank (shuffle.merge_padded), the others as
    padded segments.  skew_step: from that step on most keys map to owner 0
    (a key-distribution shift mid-stream)."""
    from flink_siddhi import shuffle
    plan = workload.PATTERN_PLAN
    senders = [fs.SiddhiAppRuntime(plan, ts_order=1) for _ in range(world)]
    owners = [fs.SiddhiAppRuntime(plan, ts_order=1, key_stride=world, key_offset=r, chunk_events=8192)
              for r in range(world)]
    for o in owners:
        o.add_callback("O")
    allw = []
    spilled_steps = 0
    for s in range(steps):
        sent, spills = [], []
        for src in range(world):
            g = s * world + src
            w = workload.generate(g * n_per, n_per, keys, rate=1)
            if skew_step is not None and s >= skew_step:
                w["k"] = np.where(w["k"] % 5 != 0, (w["k"] // world) * world, w["k"]).astype(np.int32)
            allw.append(w)
            d = _dev(w)
            words = senders[src].record_words()
            sbuf = torch.zeros((n_per, words), dtype=torch.int64, device="cuda")
            scnt = torch.zeros(world, dtype=torch.int64, device="cuda")
            segs = senders[src].route_padded("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]],
                                             world, seq0=g * n_per, seg_cap=seg_cap, streams=d["stream"],
                                             spill=(sbuf, scnt))
            sent.append(segs)
            spills.append((sbuf, scnt))
        torch.cuda.synchronize()
        S = 1 + seg_cap
        scounts = [[int(x) for x in sc.cpu().tolist()] for _, sc in spills]
        any_spill = sum(map(sum, scounts)) > 0
        spilled_steps += any_spill
        for r in range(world):
            recv = torch.cat([sent[src][r * S:(r + 1) * S] for src in range(world)], dim=0)
            if not any_spill:
                owners[r].send_padded(recv, world, seg_cap, n_per)
                continue
            # the exact spill exchange, simulated: source src's spill for
            # owner r is its r-th owner group
            parts, src_counts = [], []
            for src in range(world):
                off = sum(scounts[src][:r])
                c = scounts[src][r]
                parts.append(spills[src][0][off:off + c])
                src_counts.append(c)
            merged = shuffle.merge_padded(recv, world, seg_cap, torch.cat(parts, dim=0), src_counts)
            owners[r].send_records(merged, int(merged.shape[0]), n_per)
    return senders, owners, allw, spilled_steps


@pytest.mark.parametrize("world", [2, 3])
def test_padded_spill_survives_a_key_skew_shift(world):
    # a key-distribution shift that overflows seg_cap
    # mid-stream must not drop records or fail the job: every row vs the
    # oracle over the whole stream
    n_per, keys, steps = 12000, 600, 4
    from flink_siddhi import shuffle
    cap = shuffle.padded_capacity(n_per // 3, world, slack=0.25, floor=64)
    senders, owners, allw, spilled = _spill_round(world, n_per, keys, cap, steps, skew_step=2)
    assert spilled >= 2, "the skewed steps must overflow seg_cap"
    got = []
    for o in owners:
        o.flush()   # no CEP_E_CAPACITY: nothing was dropped
        got += engine_rows(o.collect("O"))
    got.sort(key=lambda t: t[1])
    w = {c: np.concatenate([x[c] for x in allw]) for c in allw[0]}
    want = oracle_run(workload.PATTERN_PLAN, workload_events(w)).get("O", [])
    assert len(want) > 100
    assert_same_rows(got, want, "padded spill world=%d" % world)
    for rt in owners + senders:
        rt.shutdown()
