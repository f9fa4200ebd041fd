"""Key shuffle between GPU shards.

One process per GPU.  Every rank routes its contiguous slice of the global
event sequence (`SiddhiAppRuntime.route`: push-down filtering + owner =
key % world, owner-grouped records), exchanges the records with one
all-to-all (RCCL over xGMI with the "nccl" backend; gloo on CPU), and feeds
what it received, concatenated in source-rank order (hence in global arrival
order), to its own engine (`send_records`).  This mirrors Flink's keyBy
network shuffle in front of the operator (router/HashPartitioner.java:24-26,
router/DynamicPartitioner.java:43-60).
"""
from __future__ import annotations

import os
import weakref
from typing import List, Sequence

import torch
import torch.distributed as dist


def _host_staged() -> bool:
    # gloo moves host tensors only (CPU tests; rehearsal with ranks sharing a GPU)
    return dist.get_backend() != "nccl"


# default process group -> its count group.  Keyed weakly on the group
# object itself: a destroyed world's entry goes with it, and a re-initialised
# world (whose id() may repeat) gets a group of its own.
_COUNT_GROUP = weakref.WeakKeyDictionary()


def _count_group():
    """A gloo group beside the RCCL one for the per-owner counts: the counts
    are host integers already (the route returns them), and RCCL's alltoallv
    needs host split sizes, so exchanging them host to host keeps the step
    free of a device round trip (an all-to-all of a device tensor followed by
    a readback would wait for everything queued on torch's stream).

    `dist.new_group` is a collective: if it fails, it fails on the rank that
    raises and leaves the others blocked, so there is no per-rank fallback —
    the error propagates (CEP_COUNT_GROUP=device selects the RCCL counts on
    every rank instead, a choice all ranks make alike)."""
    world = dist.group.WORLD
    if world not in _COUNT_GROUP:
        mode = os.environ.get("CEP_COUNT_GROUP", "")
        if mode == "device":
            _COUNT_GROUP[world] = "device"
        elif _host_staged() and mode != "side":
            _COUNT_GROUP[world] = None          # the default group is gloo already
        else:
            _COUNT_GROUP[world] = dist.new_group(backend="gloo")
    return _COUNT_GROUP[world]


def exchange_counts(counts: Sequence[int], device=None) -> List[int]:
    """All-to-all of the per-owner record counts -> counts received from each
    source (host to host over the gloo side group: no GPU synchronisation;
    over RCCL with a readback only if that group could not be created)."""
    world = dist.get_world_size()
    g = _count_group()
    if g == "device":
        send = torch.tensor(list(counts), dtype=torch.int64, device=device)
        recv = torch.empty(world, dtype=torch.int64, device=device)
        dist.all_to_all_single(recv, send)
    else:
        send = torch.tensor(list(counts), dtype=torch.int64)
        recv = torch.empty(world, dtype=torch.int64)
        dist.all_to_all_single(recv, send, group=g)
    return [int(x) for x in recv.tolist()]


def exchange(records: torch.Tensor, counts: Sequence[int], out: torch.Tensor = None):
    """Send records[offsets[d] : offsets[d] + counts[d]] to rank d.

    `records` is [n, words] (int64 words).  Returns (received [m, words],
    m, per-source counts); received rows are in source-rank order."""
    words = records.shape[1]
    recv_counts = exchange_counts(counts, records.device)
    m = sum(recv_counts)
    if out is None or out.shape[0] < m:
        out = torch.empty((max(m, 1), words), dtype=records.dtype, device=records.device)
    n = sum(counts)
    osz = [c * words for c in recv_counts]
    isz = [c * words for c in counts]
    if _host_staged() and records.is_cuda:
        host_out = torch.empty(m * words, dtype=records.dtype)
        dist.all_to_all_single(host_out, records[:n].reshape(-1).cpu(),
                               output_split_sizes=osz, input_split_sizes=isz)
        out[:m].view(-1).copy_(host_out)
    else:
        dist.all_to_all_single(out[:m].view(-1), records[:n].reshape(-1),
                               output_split_sizes=osz, input_split_sizes=isz)
    return out, m, recv_counts


def padded_capacity(n: int, world: int, slack: float = 0.25, floor: int = 1024) -> int:
    """Records per owner segment for the padded exchange: the even share of
    a rank's n rows plus `slack` of it (owners are key % world, so for keys
    spread over many values the counts sit close to n / world) and a floor
    for small batches.  The caller may pass any larger value; an overflow is
    reported by the owner's next flush (cep_send_records_padded)."""
    share = -(-int(n) // int(world))
    return int(share + share * slack) + floor


def exchange_padded(segs: torch.Tensor, world: int, out: torch.Tensor = None) -> torch.Tensor:
    """Equal-split all-to-all of `world` fixed owner segments (rows [d * S,
    (d + 1) * S) go to rank d): no split sizes, so no count exchange and no
    host round trip.  Returns the world received segments in source-rank
    order (the layout cep_send_records_padded reads)."""
    if out is None or out.shape != segs.shape:
        out = torch.empty_like(segs)
    if _host_staged() and segs.is_cuda:
        host_out = torch.empty(segs.numel(), dtype=segs.dtype)
        dist.all_to_all_single(host_out, segs.reshape(-1).cpu())
        out.view(-1).copy_(host_out)
    else:
        dist.all_to_all_single(out.view(-1), segs.reshape(-1))
    return out


def calibrated_capacity(counts: Sequence[int], slack: float = 0.15, floor: int = 1024) -> int:
    """Segment capacity from one measured step (a two-phase route's host
    counts, e.g. during warm-up): the largest per-owner count over all ranks
    plus `slack` of it.  One host all-reduce, outside the step loop."""
    m = torch.tensor([max(counts) if len(counts) else 0], dtype=torch.int64)
    g = _count_group()
    if g == "device":
        m = m.cuda()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
    else:
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=g)
    top = int(m.item())
    return int(top + top * slack) + floor
