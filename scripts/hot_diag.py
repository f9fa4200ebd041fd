"""Diagnostics: does the hot-key path engage on the bench's Zipf stream?"""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flink-siddhi_amd"))
import torch
import flink_siddhi as fs
from flink_siddhi import _lib as L, workload

keys = 1 << 20
chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 25
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 26
table = torch.from_numpy(workload.zipf_map(keys)).cuda()
rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, chunk_events=chunk, ordered_output=0, profile=1)
for s in range(4):
    d = workload.generate_device(s * n, n, keys, rate=400)
    d["k"] = table[d["k"].long()]
    rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
    rt.flush()
    st = rt.stats()
    print("step", s, "hot_keys", st.hot_keys, "K_HOT", st.kernel_launches[L.K_HOT],
          "walk ms", round(st.kernel_ms[L.K_CF_WALK], 2), "hot ms", round(st.kernel_ms[L.K_HOT], 2),
          "part ms", round(st.kernel_ms[L.K_CF_PARTITION], 2), "matches", st.matches_out, flush=True)
