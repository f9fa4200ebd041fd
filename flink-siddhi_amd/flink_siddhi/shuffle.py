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


def segment_counts(segs: torch.Tensor, world: int, seg_cap: int, rows: bool = False) -> List[int]:
    """The true per-source record counts in the headers of `world` received
    padded segments (one small readback): records: header word 0 low 32 bits;
    rows: bits 32-62 (include/cep.h)."""
    h = segs.view(world, 1 + seg_cap, -1)[:, 0, 0].cpu()
    if rows:
        return [int((int(x) >> 32) & 0x7fffffff) for x in h.tolist()]
    return [int(int(x) & 0xffffffff) for x in h.tolist()]


def merge_padded(recv: torch.Tensor, world: int, seg_cap: int, spill_recv: torch.Tensor,
                 spill_src_counts: Sequence[int], rows: bool = False) -> torch.Tensor:
    """Owner input of a step whose padded exchange spilled: per source rank r
    (in rank order, i.e. global arrival order), the r-th segment's first
    min(count_r, seg_cap) records then the records r spilled for this owner
    (spill_recv holds them in source order, spill_src_counts[r] each).  Every
    record of the step arrives, in the order the owner would have seen them
    with a large enough seg_cap."""
    counts = segment_counts(recv, world, seg_cap, rows)
    segs = recv.view(world, 1 + seg_cap, -1)
    parts = []
    off = 0
    for r in range(world):
        kept = min(counts[r], seg_cap)
        if kept:
            parts.append(segs[r, 1:1 + kept])
        s = int(spill_src_counts[r])
        if s:
            parts.append(spill_recv[off:off + s])
        off += s
        if kept + s != counts[r]:
            raise RuntimeError("padded shuffle: source %d sent %d + %d spilled records for %d routed"
                               % (r, kept, s, counts[r]))
    if not parts:
        return recv[:0].reshape(0, segs.shape[2])
    return torch.cat(parts, dim=0)


class PaddedShuffle:
    """The padded key shuffle with a spill: no host round trip per step, and
    no record is ever dropped when an owner's share outgrows seg_cap (VERDICT
    r04 item 6: a key-distribution shift must not abort the job).

    Step s: route (cep_route_*_padded_spill: records past seg_cap go to a
    spill buffer, their per-owner counts to a device array copied to pinned
    memory without a sync), one equal-split all-to-all of the segments.  The
    owner's walk of step s is queued at step s + 1, after this rank has read
    its spill counts of step s (long done by then) and all ranks agreed on
    whether anyone spilled (one host all-reduce of an integer, beside the
    collectives).  Nobody spilled: the segments go to the engine as they are
    (cep_send_*_padded).  Someone spilled: one exact exchange of the spill
    buffers (counts first) and the owner's input is merged per source rank
    (merge_padded), so every record arrives in global arrival order."""

    def __init__(self, rt, world: int, seg_cap: int, spill_cap: int, rows: bool = False):
        self.rt, self.world, self.seg_cap, self.spill_cap, self.rows = rt, world, int(seg_cap), int(spill_cap), rows
        self.words = rt.row_words() if rows else rt.record_words()
        dev = torch.device("cuda", torch.cuda.current_device())
        self.segs = [None, None]
        self.recv = [None, None]
        self.merged = [None, None]
        self.sbuf = [torch.empty((max(1, self.spill_cap), self.words), dtype=torch.int64, device=dev)
                     for _ in range(2)]
        self.scnt = [torch.zeros(world, dtype=torch.int64, device=dev) for _ in range(2)]
        self.shost = [torch.zeros(world, dtype=torch.int64).pin_memory() for _ in range(2)]
        self.ev = [torch.cuda.Event(), torch.cuda.Event()]
        self.guard = [torch.cuda.Stream(), torch.cuda.Stream()]
        self.pending = None
        self.i = 0
        self.spilled_steps = 0
        self.spilled_records = 0

    def step(self, stream_id: str, ts, cols, seq0: int, events: int, streams=None):
        j = self.i % 2
        self.i += 1
        rt = self.rt
        self.segs[j] = rt.route_padded(stream_id, ts, cols, self.world, seq0=seq0, seg_cap=self.seg_cap,
                                       streams=streams, out=self.segs[j], rows=self.rows,
                                       spill=(self.sbuf[j], self.scnt[j]))
        # torch's stream is ordered after the route (route_padded signals it)
        self.shost[j].copy_(self.scnt[j], non_blocking=True)
        self.ev[j].record()
        torch.cuda.current_stream().wait_stream(self.guard[j])   # the walk that last read recv[j]
        self.recv[j] = exchange_padded(self.segs[j], self.world, out=self.recv[j])
        if self.pending is not None:
            self._finish(*self.pending)
        self.pending = (j, events)

    def finish(self):
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None

    def _finish(self, j: int, events: int):
        self.ev[j].synchronize()
        local = int(self.shost[j].sum().item())
        flag = torch.tensor([local], dtype=torch.int64)
        g = _count_group()
        if g == "device":
            flag = flag.cuda()
            dist.all_reduce(flag)
        else:
            dist.all_reduce(flag, group=g)
        rt = self.rt
        if int(flag.item()) == 0:
            rt.send_padded(self.recv[j], self.world, self.seg_cap, events, signal=False, rows=self.rows)
        else:
            self.spilled_steps += 1
            self.spilled_records += local
            counts = [int(x) for x in self.shost[j].tolist()]
            spill_recv, m, src = exchange(self.sbuf[j], counts)
            self.merged[j] = merge_padded(self.recv[j], self.world, self.seg_cap, spill_recv[:m], src, self.rows)
            n = int(self.merged[j].shape[0])
            if self.rows:
                rt.send_rows(self.merged[j], n, events, signal=False)
            else:
                rt.send_records(self.merged[j], n, events, signal=False)
        rt.signal(self.guard[j])
