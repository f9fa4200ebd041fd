import sys, os
sys.path[:0] = ["flink-siddhi_amd", "oracle", "tests"]
import numpy as np
import flink_siddhi as fs
from flink_siddhi import workload
w = workload.generate(0, 100, 512, rate=1)
plan = workload.PATTERN_PLAN.replace("within 10 sec", "within 1 sec")
for i in range(100):
    print("ev", i, "k", w["k"][i], "s", w["stream"][i], "id", w["id"][i], "p>.5", w["price"][i] > 0.5)
rt = fs.SiddhiAppRuntime(plan, key_capacity=512, buckets_log2=0)
rt.add_callback("O")
rt.send("A", w["ts"], [w["k"], w["ts"], w["id"], w["price"]], streams=w["stream"])
rt.flush()
o = rt.collect("O")
ks = o.cols[0]; p1 = o.cols[1].view(np.uint64); p2 = o.cols[2].view(np.uint64); t = o.cols[3]
order = np.argsort(ks, kind="stable")
for j in order:
    meta = int(p1[j] >> 32); gts = int(p1[j] & 0xffffffff)
    print("w%d sp%d" % (ks[j] // 1000, ks[j] % 1000), "q", meta & 0xfff, "A", (meta >> 12) & 1, "B", (meta >> 13) & 1,
          "k6", (meta >> 14) & 63, "gts", gts, "ri", int(p2[j] >> 32), "snb", hex(int(p2[j] & 0xffff)),
          "kst", int(o.ts[j]) >> 32, "kc", int(o.ts[j]) & 0xffffffff, "hs", int(o.seq[j]) >> 16, "gs", int(o.seq[j]) & 0xffff,
          "kfb", hex(int(t[j]) >> 16), "klb", hex(int(t[j]) & 0xffff))
