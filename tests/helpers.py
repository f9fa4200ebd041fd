"""Shared test helpers: drive the oracle and the engine on the same events."""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

import siddhi_oracle as O


def oracle_run(plan: str, events: Sequence[Tuple[str, int, tuple]]):
    """events: [(stream_id, ts, row)] in arrival order -> {out: [(ts, seq, data)]}."""
    rt = O.OracleRuntime(plan)
    out: Dict[str, List] = {}
    for sid, ts, row in events:
        for ev in rt.send(sid, ts, row):
            out.setdefault(ev.stream, []).append((ev.ts, ev.seq, ev.data))
    return out


def workload_events(w: dict, names=("A", "B"), cols=("k", "ts", "id", "price")):
    """Generator columns -> oracle event list (rows in stream-definition order)."""
    n = len(w["ts"])
    colv = [w[c].tolist() for c in cols]
    st = w["stream"].tolist()
    ts = w["ts"].tolist()
    return [(names[st[i]], ts[i], tuple(c[i] for c in colv)) for i in range(n)]


def engine_rows(out) -> List[Tuple[int, int, tuple]]:
    """runtime.OutputRows -> [(ts, seq, data)] with Python scalars."""
    cols = [c.tolist() for c in out.cols]
    ts = out.ts.tolist()
    seq = out.seq.tolist()
    return [(ts[i], seq[i], tuple(c[i] for c in cols)) for i in range(len(ts))]


def assert_same_rows(got, want, ctx=""):
    if got == want:
        return
    n = min(len(got), len(want))
    for i in range(n):
        if got[i] != want[i]:
            raise AssertionError("%s: first difference at row %d: engine %r oracle %r "
                                 "(engine %d rows, oracle %d rows)"
                                 % (ctx, i, got[i], want[i], len(got), len(want)))
    raise AssertionError("%s: engine %d rows, oracle %d rows" % (ctx, len(got), len(want)))
