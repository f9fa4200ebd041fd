"""Benchmark: matched-pattern events/s (BASELINE.json metric) on MI355X.

Default workload = BASELINE.json configs[2] (config 3): keyed
`partition with (k of A, k of B) begin from every s1=A[price > 0.5] ->
s2=B[id % 7 == 0] within 10 sec select s1.k, s1.price, s2.price, s2.ts ...`,
K = 2^20 partition keys, N = 2^28 events per step, R = 400 events/ms.
A step = one pass of the hot path (predicate + key-bucket partition + per-key
NFA walk + match emission) over one batch of N events already resident in
HBM; the per-key pattern state carries from step to step (each step is the
next N events of one stream).  With --gpus N > 1 (torchrun), each rank owns
the keys k % N == rank and processes N events per step (weak scaling).

`--workload filter` runs configs[1] (config 2): `inputStream[price > 0.5 and
id % 7 == 0] select *` over 10^8 events.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "flink-siddhi_amd"))

# per-kernel HIP events around every PROFILE_EVERY-th launch of each kernel
# (every event between two kernels widens the gap between them by ~5 us:
# timing every launch costs ~4 % of the throughput; CEP_PROFILE=0: none)
PROFILE_EVERY = int(os.environ.get("CEP_PROFILE", "4"))
HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
PATTERN_IN_BYTES = 4 + 8 + 1 + 4 + 8     # k, ts, stream, id, price per event
PATTERN_OUT_BYTES = 4 + 8 + 8 + 8 + 8    # k, p1, p2, t + event ts per match
FILTER_IN_BYTES = 4 + 8                   # id, price per event
FILTER_OUT_BYTES = 4 + 4 + 8 + 8 + 8      # id, name, price, timestamp + event ts


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["pattern", "filter"], default="pattern")
    ap.add_argument("--events", type=int, default=0, help="events per step per GPU")
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--rate", type=int, default=400, help="events per ms")
    ap.add_argument("--chunk", type=int, default=1 << 25)
    ap.add_argument("--buckets-log2", type=int, default=0,
                    help="key buckets = 2^n (0: engine default, <= 512 keys per bucket)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--ingest", choices=["shuffle", "prepartitioned"], default="shuffle",
                    help="multi-GPU pattern input: engine key shuffle over RCCL, or keyed upstream")
    return ap.parse_args()


def dist_init(args):
    """One process per GPU.  CEP_DIST_BACKEND=gloo (rehearsal on a box with
    fewer GPUs than ranks: ranks share devices, exchanges staged via host)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    backend = os.environ.get("CEP_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def _coll_device():
    import torch.distributed as dist
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(world, v: float) -> float:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(world, v: float) -> float:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (scripts/gpu_pmc.sh -> scripts/pmc_summary.py -> profiles/r01_pmc.json;
    FETCH_SIZE doubled per the gfx950 caveat).  Measured in separate
    rocprofv3 --pmc passes of this same bench command; null if absent."""
    import glob
    import json as _json
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                          "profiles", "*pmc*.json")))
    for f in reversed(files):
        try:
            d = _json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in d and "hbm_bytes_per_launch" in d[kernel]:
            return {"bytes_per_launch": round(d[kernel]["hbm_bytes_per_launch"]),
                    "read": round(d[kernel]["hbm_read_bytes"]),
                    "write": round(d[kernel]["hbm_write_bytes"]),
                    "source": os.path.relpath(f, os.path.dirname(os.path.abspath(__file__)))}
    return None


def cpu_baseline_pattern(args, budget_s):
    """Oracle C restatement (kind "port") on the host cores: one thread over a
    bounded prefix of the stream (~0.8 x budget_s of CPU time), then the same
    restatement sharded by key (key % T, arrival order kept per shard) over T
    threads (ctypes releases the GIL), timed over one pre-split sample of up
    to 2^27 events.  Reported value = the T-thread rate; the 1-thread rate is
    kept beside it."""
    import threading
    import numpy as np
    sys.path.insert(0, str(ROOT / "oracle"))
    import cep_oracle as CO
    from flink_siddhi import workload
    f, g = CO.cond(("price", 0, ">", 0.5)), CO.cond(("id", 7, "==", 0))
    # one thread
    po = CO.PatternOracle(args.keys, f, g, every=True, within=10000)
    chunk = 1 << 22
    done, spent, matches = 0, 0.0, 0
    while spent < budget_s * 0.8 and done < (1 << 28):
        w = workload.generate(done, chunk, args.keys, rate=args.rate)
        t0 = time.perf_counter()
        _, _, m = po.run(w, out_cap=chunk)
        spent += time.perf_counter() - t0
        matches += m
        done += chunk
    one = done / spent
    # T threads, key-sharded
    T = max(1, min(16, os.cpu_count() or 1))
    n = min(1 << 27, int(one * budget_s / 2 * T))
    n = max(chunk, (n // chunk) * chunk)
    w = workload.generate(0, n, args.keys, rate=args.rate)
    shard = w["k"] % T
    order = np.argsort(shard, kind="stable")
    bounds = np.searchsorted(shard[order], np.arange(T + 1))
    parts = []
    for t in range(T):
        idx = order[bounds[t]:bounds[t + 1]]
        part = {c: np.ascontiguousarray(w[c][idx]) for c in ("k", "stream", "id", "price", "ts")}
        part["k"] = (part["k"] // T).astype(np.int32)   # shard-local dense keys
        parts.append(part)
    del w, shard, order
    oracles = [CO.PatternOracle((args.keys + T - 1) // T, f, g, every=True, within=10000)
               for _ in range(T)]
    res = [0] * T

    def work(t):
        _, _, m = oracles[t].run(parts[t], out_cap=len(parts[t]["ts"]))
        res[t] = m

    threads = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    t0 = time.perf_counter()
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "events/s", "cores": T, "kind": "port",
            "sample": "first %d events of the config-3 stream (K=%d, R=%d/ms) sharded by key "
                      "over %d threads, oracle/cep_oracle.c, %d matches, %.2f s; 1 thread: "
                      "%.0f events/s over the first %d events"
                      % (n, args.keys, args.rate, T, sum(res), dt, one, done),
            "value_1core": one}


def cpu_baseline_filter(args, n_total, budget_s):
    sys.path.insert(0, str(ROOT / "oracle"))
    import cep_oracle as CO
    from flink_siddhi import workload
    f = CO.cond(("price", 0, ">", 0.5), ("id", 7, "==", 0))
    chunk = 1 << 23
    done, spent = 0, 0.0
    while spent < budget_s and done < n_total:
        w = workload.generate(done, chunk, 1, single_stream=True)
        t0 = time.perf_counter()
        CO.filter_indices(w["id"], w["price"], f)
        spent += time.perf_counter() - t0
        done += chunk
    return {"value": done / spent, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": "first %d events of the config-2 stream, oracle/cep_oracle.c "
                      "single-threaded, %.1f s" % (done, spent)}


def main():
    args = parse()
    import numpy as np
    import torch
    import flink_siddhi as fs
    from flink_siddhi import _lib as L
    from flink_siddhi import workload

    world, rank, local = dist_init(args)
    pattern = args.workload == "pattern"
    n = args.events or ((1 << 28) if pattern else 100_000_000)
    steps, warm = args.steps, args.warmup

    if pattern:
        plan = workload.PATTERN_PLAN
        opts = dict(device=local, key_capacity=(args.keys + world - 1) // world,
                    key_stride=world, key_offset=rank, chunk_events=args.chunk,
                    profile=PROFILE_EVERY, ordered_output=0)
        if args.buckets_log2:
            opts["buckets_log2"] = args.buckets_log2
    else:
        plan = workload.FILTER_PLAN
        opts = dict(device=local, profile=PROFILE_EVERY, ordered_output=0)
    rt = fs.SiddhiAppRuntime(plan, **opts)

    # Inputs for every step, generated on the device before the timed region.
    # Multi-GPU: rank r's events are the ones whose key it owns (the result of
    # the keyBy shuffle), drawn from its own contiguous index ranges.
    # Multi-GPU ingest: "shuffle" (default) — rank r holds global index range
    # r of each step and the engine routes it (push-down + owner = k % world),
    # RCCL all-to-all moves the records, each owner walks what it received;
    # "prepartitioned" — the input is already keyed upstream (Flink keyBy):
    # rank r draws only keys it owns, no exchange.
    shuffle_mode = pattern and world > 1 and args.ingest == "shuffle"
    batches = []
    for s in range(warm + steps):
        first = (s * world + rank) * n
        d = workload.generate_device(first, n, args.keys, rate=args.rate,
                                     single_stream=not pattern, device="cuda")
        d["first"] = first
        if pattern and world > 1 and not shuffle_mode:
            d["k"] = (d["k"] // world) * world + rank     # owned keys, same distribution
        if not pattern:
            d["name"] = torch.zeros(n, dtype=torch.int32, device="cuda")
        batches.append(d)
    torch.cuda.synchronize()

    bufs = {}

    def step(d):
        if shuffle_mode:
            from flink_siddhi import shuffle
            recs, counts = rt.route("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]],
                                    world, seq0=d["first"], streams=d["stream"],
                                    out=bufs.get("send"))
            bufs["send"] = recs
            recv, m, _ = shuffle.exchange(recs, counts, out=bufs.get("recv"))
            bufs["recv"] = recv
            rt.send_records(recv, m, n)
        elif pattern:
            rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
        else:
            rt.send("inputStream", d["ts"], [d["id"], d["name"], d["price"], d["ts"]])
        rt.flush()

    for s in range(warm):
        step(batches[s])
    st0 = rt.stats()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        step(batches[warm + s])
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    st1 = rt.stats()
    dt_max = max_over_ranks(world, dt)
    events_total = sum_over_ranks(world, float(n * steps))
    matches_total = sum_over_ranks(world, float(st1.matches_out - st0.matches_out))
    value = events_total / dt_max

    # per-kernel HIP-event times on the engine's stream over the timed region
    kern = {}
    for k, name in ((L.K_PARTITION, "k_partition"), (L.K_WALK, "k_walk"), (L.K_FILTER, "k_filter"),
                    (L.K_ROUTE, "k_route"), (L.K_CF_PARTITION, "k_cfpart"), (L.K_CF_WALK, "k_cfwalk")):
        launches = st1.kernel_launches[k] - st0.kernel_launches[k]
        timed = st1.kernel_timed[k] - st0.kernel_timed[k]
        ms = st1.kernel_ms[k] - st0.kernel_ms[k]
        if launches and timed and ms > 0:
            kern[name] = {"launches": int(launches), "timed_launches": int(timed),
                          "avg_us": 1e3 * ms / timed, "total_ms": ms / timed * launches}
    m_per_event = (st1.matches_out - st0.matches_out) / float(n * steps)
    if pattern:
        # a launch of either pattern kernel processes one chunk of events: its
        # algorithmic bytes are SURVEY §8(d)'s per-event figure x the chunk
        alg_per_event = PATTERN_IN_BYTES + PATTERN_OUT_BYTES * m_per_event
        per_launch = {}
        for kname in ("k_partition", "k_walk", "k_cfpart", "k_cfwalk"):
            if kname in kern:
                per_launch[kname] = alg_per_event * n * steps / kern[kname]["launches"]
        if shuffle_mode:
            # route reads the whole step batch once; the owner's partition pass
            # then reads records, not events (its bytes are not attributed here)
            per_launch["k_route"] = PATTERN_IN_BYTES * n
    else:
        per_launch = {"k_filter": (FILTER_IN_BYTES + FILTER_OUT_BYTES * m_per_event) * n}
        alg_per_event = FILTER_IN_BYTES + FILTER_OUT_BYTES * m_per_event
    roofline = None
    timed_k = [k for k in kern if k in per_launch]
    if timed_k:   # CEP_PROFILE=0 (no per-kernel timer events): no kernel roofline
        dom = max(timed_k, key=lambda k: kern[k]["total_ms"])
        achieved = per_launch[dom] / (kern[dom]["avg_us"] * 1e-6) / 1e9
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": pmc_traffic(dom) if world == 1 else None,
                    "bytes_per_launch": per_launch[dom], "avg_launch_us": round(kern[dom]["avg_us"], 2)}
    per_gpu_events = value / world
    pipeline = {"alg_bytes_per_event": round(alg_per_event, 3),
                "achieved": round(per_gpu_events * alg_per_event / 1e9, 1), "unit": "GB/s",
                "frac": round(per_gpu_events * alg_per_event / 1e9 / HBM_PEAK_GBS, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline_pattern(args, args.cpu_seconds) if pattern else \
            cpu_baseline_filter(args, n, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": "matched-pattern events/sec (whole node) at 1/2/4/8 MI355X + % HBM roofline",
            "value": round(value, 1), "unit": "events/s", "n_gpus": world,
            "steps": steps, "warmup": warm, "ms_per_step": round(1e3 * dt_max / steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64+int32+int64", "data": "synthetic (splitmix64 counter stream, BASELINE.md §3)",
            "config": ({"workload": "config3: keyed every A -> B within 10 sec, partition with k",
                        "keys": args.keys, "events_per_step_per_gpu": n, "rate_per_ms": args.rate,
                        "chunk_events": args.chunk, "parallelism": "key-sharded x%d" % world,
                        "ingest": (("%s all-to-all key shuffle" % ("rccl" if _coll_device() == "cuda"
                                                                    else "gloo host-staged"))
                                    if shuffle_mode else
                                   "pre-partitioned (keyed upstream)") if world > 1 else "local"}
                       if pattern else
                       {"workload": "config2: inputStream[price > 0.5 and id % 7 == 0] select *",
                        "events_per_step_per_gpu": n, "parallelism": "replicas x%d" % world}),
            "matches_per_s": round(matches_total / dt_max, 1),
            "matches_per_event": round(m_per_event, 5),
            "roofline": roofline,
            "pipeline_roofline": pipeline,
            "kernels": kern,
            "cpu_baseline": cpu,
            "speedup_vs_cpu_baseline": round(value / cpu["value"], 1) if cpu else None,
        }
        print(json.dumps(out), flush=True)
    rt.shutdown()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
