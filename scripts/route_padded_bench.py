"""Sender side of the padded key shuffle on one GPU:
cep_route_batch_padded over one 2^28-event config-3 batch for a simulated
world (no exchange), timed with HIP events on the route stream; then every
owner segment is checked against the route's own two-pass result (same
records, same order).  Prints one JSON line.  Run it under
`rocprofv3 --kernel-trace --stats` / `--pmc` for the per-kernel split.

usage: python scripts/route_padded_bench.py [world] [log2 events] [iters]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flink-siddhi_amd"))
import torch  # noqa: E402

import flink_siddhi as fs  # noqa: E402
from flink_siddhi import shuffle, workload  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 28)
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
keys = 1 << 20
rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, device=0, profile=1, ts_order=1)
d = workload.generate_device(0, n, keys, rate=400)
cols = [d["k"], d["ts"], d["id"], d["price"]]
torch.cuda.synchronize()
# ~1/3 of the rows are kept (push-down); 3 % slack as bench.py calibrates it
# (records past the cap spill, see shuffle.PaddedShuffle)
cap = shuffle.padded_capacity(n // 3, world, slack=0.03)
segs = None
times = []
for it in range(iters + 1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    segs = rt.route_padded("A", d["ts"], cols, world, seq0=0, seg_cap=cap, streams=d["stream"], out=segs)
    torch.cuda.synchronize()
    if it:
        times.append(time.perf_counter() - t0)
wrw = segs.shape[1]
# reference: the two-phase route of the same batch (owner-contiguous, counts)
recs, counts = rt.route("A", d["ts"], cols, world, seq0=0, streams=d["stream"])
torch.cuda.synchronize()
ok = True
off = 0
for o in range(world):
    seg = segs[o * (1 + cap):(o + 1) * (1 + cap)]
    c = int(seg[0, 0].item()) & 0xffffffff
    ok = ok and c == counts[o] and bool(torch.equal(seg[1:1 + c], recs[off:off + c]))
    off += counts[o]
st = rt.stats()
from flink_siddhi import _lib as L  # noqa: E402
k = L.K_ROUTE
route_us = 1e3 * st.kernel_ms[k] / max(1, st.kernel_timed[k])
rec_bytes = sum(counts) * wrw * 8
in_bytes = n * (4 + 8 + 1 + 4 + 8)
best = min(times)
print(json.dumps({"world": world, "events": n, "seg_cap": cap, "record_words": int(wrw),
                  "records": int(sum(counts)), "route_ms_wall_best": round(best * 1e3, 3),
                  "route_ms_wall_mean": round(1e3 * sum(times) / len(times), 3),
                  "k_route_avg_us_hip_events": round(route_us, 1),
                  "alg_bytes": in_bytes + rec_bytes, "achieved_GBs": round((in_bytes + rec_bytes) / best / 1e9, 1),
                  "matches_two_pass": ok,
                  "kernels": "k_cfroute (per-tile owner groups) + k_route_scan + k_route_gather + k_route_pad"}),
      flush=True)
