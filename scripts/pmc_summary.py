"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) per kernel.

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md
(HBM/rocprofv3 section): FETCH_SIZE and WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports half the bytes of wide streaming reads, so it is doubled.
Writes the JSON that bench.py reports as roofline.traffic.
usage: python scripts/pmc_summary.py gpurun_out/pmc profiles/r01_pmc.json
"""
import collections
import csv
import glob
import json
import sys


def short(name):
    for k in ("k_cfpart", "k_cfwalk", "k_mqpart", "k_mqwalk", "k_partition", "k_walk", "k_filter", "k_generate",
              "k_cfroute", "k_route_gather", "k_route_pad", "k_route_scan", "k_route"):
        if k in name:
            return k
    return None


def main(src, dst):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(src + "/pass*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in vals.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"counters_mean_per_launch": m}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            rd = 2.0 * m["FETCH_SIZE"] * 1024.0
            wr = m["WRITE_SIZE"] * 1024.0
            e["hbm_read_bytes"] = rd
            e["hbm_write_bytes"] = wr
            e["hbm_bytes_per_launch"] = rd + wr
        if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
            e["wait_fraction"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        out[k] = e
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k, e in out.items():
        print(k, {x: round(y, 3) if isinstance(y, float) else None for x, y in e.items()
                  if x != "counters_mean_per_launch"})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
