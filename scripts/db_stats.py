"""Kernel stats CSV (the rocprofv3 --stats layout) from a rocprofv3 results
database: python scripts/db_stats.py <results.db> <out.csv>.  Adds the VGPR /
scratch / LDS columns of each kernel's dispatches."""
import csv
import sqlite3
import statistics
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = {}
for name, dur, vgpr, agpr, scratch, lds in c.execute(
        "select name, duration, vgpr_count, accum_vgpr_count, scratch_size, lds_size from kernels"):
    r = rows.setdefault(name, {"d": [], "vgpr": vgpr, "agpr": agpr, "scratch": scratch, "lds": lds})
    r["d"].append(dur)
total = sum(sum(r["d"]) for r in rows.values()) or 1
with open(out, "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev",
                "VGPR", "AGPR", "ScratchBytes", "LDSBytes"])
    for name, r in sorted(rows.items(), key=lambda kv: -sum(kv[1]["d"])):
        d = r["d"]
        w.writerow([name, len(d), sum(d), round(sum(d) / len(d), 3), round(100.0 * sum(d) / total, 2), min(d), max(d),
                    round(statistics.pstdev(d), 3), r["vgpr"], r["agpr"], r["scratch"], r["lds"]])
