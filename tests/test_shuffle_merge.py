"""CPU: the owner-side merge of the padded key shuffle with a spill
(flink_siddhi.shuffle.merge_padded).  A source's
records past seg_cap arrive in the second (exact) exchange; per source rank
the owner must see the segment's records then that source's spilled ones, so
its input is the source-rank concatenation it would have received with an
unbounded seg_cap (global arrival order).  Segments are laid out as
cep_route_batch_padded writes them (include/cep.h): header (count in the low
32 bits; rows: bits 32-62), records, null records."""
import pytest
import torch

from flink_siddhi import shuffle


def _segments(per_source, cap, words=4, rows=False):
    """per_source: one list of record ids per source rank -> (received
    segments, spill_recv, spill counts per source) as the exchange delivers
    them to one owner."""
    world = len(per_source)
    segs = torch.zeros((world * (1 + cap), words), dtype=torch.int64)
    spill = []
    counts = []
    for r, ids in enumerate(per_source):
        base = r * (1 + cap)
        n = len(ids)
        segs[base, 0] = ((n << 32) | 31) if rows else n
        kept = min(n, cap)
        for i in range(kept):
            segs[base + 1 + i] = torch.tensor([ids[i], 1000 + ids[i], r, 7])
        over = ids[kept:]
        counts.append(len(over))
        spill.extend(torch.tensor([x, 1000 + x, r, 7]) for x in over)
    spill_recv = torch.stack(spill) if spill else torch.zeros((0, words), dtype=torch.int64)
    return segs, spill_recv, counts


@pytest.mark.parametrize("rows", [False, True])
def test_merge_restores_source_rank_order(rows):
    per_source = [list(range(0, 9)), list(range(100, 102)), list(range(200, 215))]
    segs, spill, counts = _segments(per_source, cap=5, rows=rows)
    got = shuffle.merge_padded(segs, 3, 5, spill, counts, rows=rows)
    want = [x for ids in per_source for x in ids]
    assert got[:, 0].tolist() == want
    assert got[:, 1].tolist() == [1000 + x for x in want]


def test_merge_without_spill_is_the_segments():
    per_source = [[1, 2], [3], []]
    segs, spill, counts = _segments(per_source, cap=4)
    assert counts == [0, 0, 0]
    got = shuffle.merge_padded(segs, 3, 4, spill, counts)
    assert got[:, 0].tolist() == [1, 2, 3]


def test_merge_detects_a_lost_record():
    segs, spill, counts = _segments([list(range(8)), [50]], cap=3)
    counts[0] -= 1   # a spilled record went missing
    with pytest.raises(RuntimeError, match="spilled"):
        shuffle.merge_padded(segs, 2, 3, spill[1:], counts)
