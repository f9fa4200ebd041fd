"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace CSV."""
import csv
import glob
import sys

path = sys.argv[1] if len(sys.argv) > 1 else sorted(glob.glob("gpurun_out/trace/**/*kernel_trace.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows)
gaps = {}
for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
    g = s1 - e0
    key = (n0.split("(")[0][-22:], n1.split("(")[0][-22:])
    gaps.setdefault(key, []).append(g)
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print("%-24s -> %-24s n=%4d total=%8.1f us median=%7.1f us max=%8.1f us" %
          (k[0], k[1], len(v), sum(v) / 1e3, v[len(v) // 2] / 1e3, v[-1] / 1e3))
