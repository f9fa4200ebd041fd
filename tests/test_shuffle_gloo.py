"""Key shuffle protocol on CPU: world_size 2 over gloo (no GPU).

Each rank owns a contiguous slice of the global event sequence, pushes down
the pattern's state filters, groups the kept events by owner (key % world),
exchanges them with flink_siddhi.shuffle.exchange (the product's exchange
step; RCCL on GPUs, gloo here) and runs the CPU oracle on what it received,
in source-rank order.  The union of both shards' matches, merged on arrival
sequence, must equal the single-process oracle run over the whole stream
(keys are independent; source-rank concatenation preserves
global order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flink_siddhi import shuffle, workload
from helpers import oracle_run, workload_events

N_PER_RANK = 6000
KEYS = 96
PLAN = workload.PATTERN_PLAN


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q, side=False, padded=False):
    if side:   # counts over a separate gloo group, as beside RCCL on GPUs
        os.environ["CEP_COUNT_GROUP"] = "side"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = workload.generate(rank * N_PER_RANK, N_PER_RANK, KEYS, rate=1)
        seq = np.arange(rank * N_PER_RANK, (rank + 1) * N_PER_RANK, dtype=np.int64)
        # push-down: rows no state can use stay home (A[price > 0.5], B[id % 7 == 0])
        keep = np.where(w["stream"] == 0, w["price"] > 0.5, w["id"] % 7 == 0)
        owner = w["k"].astype(np.int64) % world
        rows = []
        counts = []
        for d in range(world):
            sel = keep & (owner == d)          # arrival order preserved
            counts.append(int(sel.sum()))
            rows.append(np.stack([seq[sel], w["k"][sel].astype(np.int64), w["ts"][sel],
                                  w["id"][sel].astype(np.int64), w["price"][sel].view(np.int64),
                                  w["stream"][sel].astype(np.int64)], axis=1))
        if padded:
            # cep_route_batch_padded's layout: per owner one header row (the
            # count in-band), the rows, null rows up to cap; equal-split
            # all-to-all, no count exchange (the step has no host round trip)
            cap = shuffle.padded_capacity(N_PER_RANK, world, floor=16)
            segs = np.zeros((world, 1 + cap, 6), dtype=np.int64)
            for d in range(world):
                segs[d, 0, 0] = counts[d]
                segs[d, 1:1 + counts[d]] = rows[d]
            got = shuffle.exchange_padded(torch.from_numpy(segs.reshape(world * (1 + cap), 6)), world)
            g = got.numpy().reshape(world, 1 + cap, 6)
            r = np.concatenate([g[s, 1:1 + int(g[s, 0, 0])] for s in range(world)], axis=0)
        else:
            recs = torch.from_numpy(np.concatenate(rows, axis=0).copy())
            got, m, src_counts = shuffle.exchange(recs, counts)
            r = got[:m].numpy()
        assert (np.diff(r[:, 0]) > 0).all(), "received records not in global arrival order"
        assert (r[:, 1] % world == rank).all(), "received a key this rank does not own"
        ev = {"k": r[:, 1].astype(np.int32), "ts": r[:, 2], "id": r[:, 3].astype(np.int32),
              "price": r[:, 4].view(np.float64), "stream": r[:, 5].astype(np.uint8)}
        out = oracle_run(PLAN, workload_events(ev)).get("O", [])
        # oracle seq = position in this shard's stream -> map back to global seq
        out = [(ts, int(r[s, 0]), data) for ts, s, data in out]
        allout = [None] * world
        dist.all_gather_object(allout, out)
        if rank == 0:
            q.put(allout)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("side,padded,world", [(False, False, 2), (True, False, 2), (False, True, 2),
                                               (False, True, 3)])
def test_key_shuffle_gloo_matches_single_process(side, padded, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, side, padded)) for r in range(world)]
    for p in procs:
        p.start()
    allout = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = sorted([row for shard in allout for row in shard], key=lambda t: t[1])
    w = workload.generate(0, world * N_PER_RANK, KEYS, rate=1)
    want = oracle_run(PLAN, workload_events(w)).get("O", [])
    assert len(want) > 50
    assert merged == want


def _reinit_main(rank, world, ports, q):
    # the side count group is cached per default group object; a
    # destroyed and re-initialised world must get a group of its own
    os.environ["CEP_COUNT_GROUP"] = "side"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    got = []
    try:
        for it, port in enumerate(ports):
            os.environ["MASTER_PORT"] = str(port)
            dist.init_process_group("gloo", rank=rank, world_size=world)
            counts = [rank * 10 + d + it for d in range(world)]
            got.append(shuffle.exchange_counts(counts))
            g = shuffle._count_group()
            assert g is not None and g != "device"
            dist.destroy_process_group()
        q.put((rank, got))
    except Exception as e:   # reported to the parent
        q.put((rank, repr(e)))


def test_count_group_survives_world_reinit():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ports = [_free_port(), _free_port()]
    procs = [ctx.Process(target=_reinit_main, args=(r, world, ports, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
        for it in range(2):
            assert res[r][it] == [s * 10 + r + it for s in range(world)]


def _calib_main(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # every rank learns the largest per-owner count of any rank
        counts = [100 * (rank + 1) + d for d in range(world)]
        q.put((rank, shuffle.calibrated_capacity(counts, slack=0.5, floor=7)))
    finally:
        dist.destroy_process_group()


def test_calibrated_capacity_is_the_global_max_plus_slack():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_calib_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    top = 100 * world + world - 1
    assert all(v == int(top + top * 0.5) + 7 for v in res.values()), res
