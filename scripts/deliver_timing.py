"""Host-delivery timing split (diagnostics): per step, the time to enqueue a
config-3 batch (send), the flush (device sort / gathers / D2H / callback) and
the callback itself, with ordered_output 0 and 1.  Prints one JSON line per
variant."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "flink-siddhi_amd"))

import torch  # noqa: E402
import flink_siddhi as fs  # noqa: E402
from flink_siddhi import workload  # noqa: E402


def main(n=1 << 28, keys=1 << 20, steps=3):
    batches = [workload.generate_device(s * n, n, keys, rate=400, device="cuda") for s in range(steps + 1)]
    torch.cuda.synchronize()
    for ordered in (1, 0):
        rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, device=0, key_capacity=keys, chunk_events=1 << 25,
                                 ordered_output=ordered)
        cb_t = [0.0]
        rows = [0]

        def cb(r):
            t = time.perf_counter()
            rows[0] += len(r)
            cb_t[0] += time.perf_counter() - t
        rt.add_callback("O", cb, copy=False)
        tl = []
        for i, d in enumerate(batches):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
            t1 = time.perf_counter()
            rt.flush()
            t2 = time.perf_counter()
            if i:
                tl.append((t1 - t0, t2 - t1))
        rt.shutdown()
        print(json.dumps({"ordered": ordered, "send_ms": [round(a * 1e3, 2) for a, _ in tl],
                          "flush_ms": [round(b * 1e3, 2) for _, b in tl], "rows": rows[0],
                          "callback_ms_total": round(cb_t[0] * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
