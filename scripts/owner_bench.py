"""Owner side of the padded key shuffle on one GPU: one 2^28-event config-3
batch routed at world 1 (every kept record in one padded segment), then fed
to an owner runtime with cep_send_records_padded, steps times; the owner's
k_cfpart (received-records build) and k_cfwalk launch times against the
same batch sent as local rows.  Prints one JSON line; the match counts of
the two paths must agree.

usage: python scripts/owner_bench.py [log2 events] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flink-siddhi_amd"))
import torch  # noqa: E402

import flink_siddhi as fs  # noqa: E402
from flink_siddhi import _lib as L  # noqa: E402
from flink_siddhi import shuffle, workload  # noqa: E402

n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 28)
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
keys = 1 << 20
opts = dict(ts_order=1, chunk_events=1 << 25, ordered_output=0, omit_seq=1, profile=1)


def kern(st0, st1, k):
    t = st1.kernel_timed[k] - st0.kernel_timed[k]
    return round(1e3 * (st1.kernel_ms[k] - st0.kernel_ms[k]) / t, 1) if t else None, \
        int(st1.kernel_launches[k] - st0.kernel_launches[k])


res = {"events_per_step": n, "steps": steps}
batches = []
for s in range(steps + 1):   # consecutive stream slices (ts ascending across steps)
    d = workload.generate_device(s * n, n, keys, rate=400)
    batches.append((d, [d["k"], d["ts"], d["id"], d["price"]]))
sender = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, **opts)
cap = shuffle.padded_capacity(n // 3, 1, slack=0.03)
segs = []
for s, (d, cols) in enumerate(batches):
    segs.append(sender.route_padded("A", d["ts"], cols, 1, seq0=s * n, seg_cap=cap, streams=d["stream"]))
torch.cuda.synchronize()
res["records"] = int(segs[0][0, 0].item()) & 0xffffffff
sender.shutdown()

for mode in ("local", "owner"):
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, **opts)
    for s in range(steps + 1):   # one warm-up step, then `steps` timed ones
        if s == 1:
            torch.cuda.synchronize()
            st0 = rt.stats()
            t0 = time.perf_counter()
        d, cols = batches[s]
        if mode == "local":
            rt.send("A", d["ts"], cols, streams=d["stream"])
        else:
            rt.send_padded(segs[s], 1, cap, events_represented=n)
        rt.flush()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    st1 = rt.stats()
    res[mode] = {"ms_per_step": round(dt * 1e3, 3), "events_per_s": round(n / dt, 1),
                 "k_cfpart_us": kern(st0, st1, L.K_CF_PARTITION), "k_cfwalk_us": kern(st0, st1, L.K_CF_WALK),
                 "matches_per_step": (st1.matches_out - st0.matches_out) // steps}
    rt.shutdown()
res["same_matches"] = res["local"]["matches_per_step"] == res["owner"]["matches_per_step"]
print(json.dumps(res))
