"""Config-5 cost split (diagnostics): times the 32 sequence queries and the 32
group-by / having queries of BASELINE config 5 separately, on the same
device-resident batches as `bench.py --workload config5`, so DESIGN.md can say
which half bounds the 64-query app.  Prints one JSON line per variant."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "flink-siddhi_amd"))

import torch  # noqa: E402
import flink_siddhi as fs  # noqa: E402
from flink_siddhi import workload  # noqa: E402


def plan_parts():
    full = workload.config5_plan()
    head = full[:full.index("partition with")]
    seq_end = full.index(" end;") + len(" end;")
    return {"sequences": full[:seq_end], "aggregations": head + full[seq_end:], "all": full}


def main(n=1 << 24, keys=1 << 20, steps=3):
    batches = []
    for s in range(steps + 1):
        d = workload.generate_device(s * n, n, keys, rate=400, single_stream=False, device="cuda")
        d["stream"] = workload.config5_streams(d["price"]).to(torch.uint8)
        batches.append(d)
    torch.cuda.synchronize()
    for name, plan in plan_parts().items():
        rt = fs.SiddhiAppRuntime(plan, device=0, key_capacity=keys, pending_slots=4, profile=4,
                                 ordered_output=0, chunk_events=n)
        for i, d in enumerate(batches):
            if i == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
            rt.flush()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        st = rt.stats()
        rt.shutdown()
        print(json.dumps({"variant": name, "ms_per_step": round(dt * 1e3, 2), "events_per_s": round(n / dt),
                          "rows_out": int(st.matches_out)}), flush=True)


if __name__ == "__main__":
    main()
