import sys, os
sys.path[:0] = ["flink-siddhi_amd", "oracle", "tests"]
import numpy as np
import flink_siddhi as fs
from flink_siddhi import workload
from helpers import engine_rows, oracle_run, workload_events
from collections import defaultdict
def run(keys, n, lg, rate=1, plan=workload.PATTERN_PLAN, chunk=1<<22, verbose=True):
    w = workload.generate(0, n, keys, rate=rate)
    want = oracle_run(plan, workload_events(w)).get("O", [])
    rt = fs.SiddhiAppRuntime(plan, key_capacity=keys, buckets_log2=lg, chunk_events=chunk)
    rt.add_callback("O")
    rt.send("A", w["ts"], [w["k"], w["ts"], w["id"], w["price"]], streams=w["stream"])
    try:
        rt.flush()
    except Exception as e:
        print(keys, n, lg, "ERR", e); return None
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    gk = defaultdict(list); wk = defaultdict(list)
    for r in got: gk[r[2][0]].append(r)
    for r in want: wk[r[2][0]].append(r)
    bad = sorted(set([k for k in wk if gk.get(k) != wk[k]] + [k for k in gk if k not in wk]))
    if verbose:
        print(os.environ.get("CEP_WALK_V1", "v2"), keys, n, lg, "rows", len(got), len(want), "bad keys", len(bad), bad[:5], flush=True)
    return w, gk, wk, bad
plan1 = workload.PATTERN_PLAN.replace("within 10 sec", "within 1 sec")
for keys, n, lg in [(512, 20000, 0), (4096, 60000, 3)]:
    run(keys, n, lg, plan=plan1)
# smallest failing prefix for 512 keys, 1 bucket
lo, hi = 100, 20000
while lo < hi:
    mid = (lo + hi) // 2
    r = run(512, mid, 0, plan=plan1, verbose=False)
    if r is None or r[3]: hi = mid
    else: lo = mid + 1
print("first failing n", lo)
w, gk, wk, bad = run(512, lo, 0, plan=plan1)
k = bad[0]
print("key", k, "events of key:")
idx = np.nonzero(w["k"] == k)[0]
for i in idx:
    print("  i=%d s=%d id=%d price=%.4f ts=%d" % (i, w["stream"][i], w["id"][i], w["price"][i], w["ts"][i] - 1500000000000))
print(" got", [(r[1], round(r[2][1], 4)) for r in gk.get(k, [])])
print(" want", [(r[1], round(r[2][1], 4)) for r in wk.get(k, [])])
