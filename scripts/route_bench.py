"""Sender-side shuffle timing on one GPU: route a 16 Mi-event config-3 batch
for a simulated world (no exchange), then feed owner 0's records to an owner
engine.  Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split."""
import sys
import time

import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flink-siddhi_amd"))
import torch  # noqa: E402

import flink_siddhi as fs  # noqa: E402
from flink_siddhi import workload  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = 1 << 24
rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, device=0, profile=1)
owner = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, device=0, key_capacity=(1 << 20) // world,
                            key_stride=world, key_offset=0, profile=1, ordered_output=0)
out = None
for it in range(6):
    d = workload.generate_device(it * n, n, 1 << 20, rate=400)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, counts = rt.route("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], world, seq0=it * n,
                           streams=d["stream"], out=out)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    owner.send_records(out, counts[0], n // world)
    owner.flush()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("route %.1f us  owner %.1f us  records %d (owner 0: %d)"
          % ((t1 - t0) * 1e6, (t2 - t1) * 1e6, sum(counts), counts[0]), flush=True)
