"""Benchmark: matched-pattern events/s (BASELINE.json metric) on MI355X.

Default workload = BASELINE.json configs[2] (config 3): keyed
`partition with (k of A, k of B) begin from every s1=A[price > 0.5] ->
s2=B[id % 7 == 0] within 10 sec select s1.k, s1.price, s2.price, s2.ts ...`,
K = 2^20 partition keys, N = 2^28 events per step, R = 400 events/ms.
A step = one pass of the hot path (predicate + key-bucket partition + per-key
NFA walk + match emission) over one batch of N events already resident in
HBM; the per-key pattern state carries from step to step (each step is the
next N events of one stream).  With --gpus N > 1 each rank owns the keys
k % N == rank and processes N events per step (weak scaling); without
WORLD_SIZE in the environment bench.py starts the N rank processes itself
(launch_ranks), under torchrun it uses the ranks it is given.

`--workload filter` runs configs[1] (config 2): `inputStream[price > 0.5 and
id % 7 == 0] select *` over 10^8 events.

`--workload config5` runs configs[4] (config 5) on the GPUs given: one app of
64 queries — 32 `every s1=A[price > q/32], s2=B[id == q%50]+, s3=C[id ==
(q+1)%50] within 10 sec` sequences under `partition with (k ...)` and 32
`group by k having` aggregations — over three keyed streams, K = 2^20 keys,
2^24 events per step.

Before the timed region (N=1): a parity check — a fresh runtime processes the
first step's events and the order-sensitive digest of its device output is
compared with oracle/cep_oracle.c's digest over the same events ("parity" in
the JSON line) — and the CPU baseline (the same restatement sharded by key
over the host's cores).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import math
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
PATTERN_SEL_BYTES = 4 + 8 + 8 + 8         # k, p1, p2, t per match (28 B)
PATTERN_OUT_BYTES = PATTERN_SEL_BYTES + 8 + 8   # + event ts + arrival seq the engine writes
CF_REC_BYTES = 16                         # closed-form record (w0 + one carried word)
CF_STATE_BYTES = 2 * (4 + 16)             # per key per walk launch: header + slot 0 (ts, p1), read + write
FILTER_IN_BYTES = 4 + 8                   # id, price per event
FILTER_OUT_BYTES = 4 + 4 + 8 + 8 + 8 + 8  # id, name, price, timestamp + event ts + seq (design)
FILTER_SEL_BYTES = 4 + 4 + 8 + 8          # id, name, price, timestamp (24 B per selected row)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["pattern", "filter", "config5"], default="pattern")
    ap.add_argument("--events", type=int, default=0, help="events per step per GPU")
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--keys-dist", choices=["uniform", "zipf"], default="uniform",
                    help="zipf: the BASELINE.md §3 Zipf s=1.1 variant (workload.zipf_map remap)")
    ap.add_argument("--rate", type=int, default=400, help="events per ms")
    ap.add_argument("--chunk", type=int, default=1 << 25)
    ap.add_argument("--buckets-log2", type=int, default=0,
                    help="key buckets = 2^n (0: engine default, <= 512 keys per bucket)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle parity check")
    ap.add_argument("--exchange", choices=["padded", "twophase"], default="padded",
                    help="key shuffle (pattern records / config-5 rows): fixed owner segments with in-band "
                         "counts (no host round trip per step) or counts first, then an exact alltoallv")
    ap.add_argument("--ingest", choices=["shuffle", "prepartitioned", "host", "host-pageable"],
                    default="shuffle",
                    help="multi-GPU pattern input: engine key shuffle over RCCL, or keyed upstream; "
                         "1 GPU: host = batches in pinned host memory fed over PCIe (host-pageable: "
                         "ordinary host memory) instead of device-resident inputs")
    ap.add_argument("--deliver", action="store_true",
                    help="deliver every match to a host callback at each flush (pinned D2H)")
    ap.add_argument("--ordered", action="store_true",
                    help="with --deliver: ordered_output=1, rows sorted into Siddhi's global emission "
                         "order on the device before the D2H (the drop-in default)")
    ap.add_argument("--with-seq", action="store_true",
                    help="with --deliver: also deliver each row's arrival number (omitted by default, as the "
                         "reference's output handler does not read it)")
    ap.add_argument("--ts-order", type=int, choices=[0, 1], default=1,
                    help="cep_options.ts_order: 1 (default here) declares the input in event-time order -- the "
                         "BASELINE generator's ts = T0 + i / R never decrease -- and runs the event-time fast "
                         "paths; 0 runs the order-tolerant path (exact for timestamps in any order, the engine "
                         "default)")
    ap.add_argument("--parity-steps", type=int, default=4,
                    help="config 5: steps of the stream the parity check covers (fresh state)")
    return ap.parse_args()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nranks, argv=None, script=None, env=None, poll_s=0.2):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes of
    this same command (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT in their environment) and wait for them.  The
    parent never imports torch or touches the GPU, so nothing is exec'd from a
    GPU-initialised process.  Rank 0 prints the JSON line on the inherited
    stdout.  If any rank exits non-zero the others are terminated (by their
    own PIDs) and the parent returns that rank's exit code.  Reference
    parallelism: one Siddhi runtime per Flink subtask
    (core/.../operator/AbstractSiddhiOperator.java:308-312), events routed by
    router/DynamicPartitioner.java:43-60 / HashPartitioner.java:24-26."""
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    script = str(Path(__file__).resolve()) if script is None else script
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base["MASTER_PORT"] = base.get("MASTER_PORT") or str(_free_port())
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(nranks):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                 LOCAL_WORLD_SIZE=str(nranks), GROUP_RANK="0", CEP_LAUNCHED_BY="bench.py")
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=e,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print("bench.py launcher: rank %d exited with %d; stopping the other ranks"
                          % (procs.index(p), c), file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def dist_init(args):
    """One process per GPU.  CEP_DIST_BACKEND=gloo (rehearsal on a box with
    fewer GPUs than ranks: ranks share devices, exchanges staged via host)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    import torch
    backend = os.environ.get("CEP_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one node by contract: gloo (the shuffle's host-to-host count group,
        # or the rehearsal backend) binds the loopback interface
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    return world, rank, local


def _coll_device():
    import torch.distributed as dist
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def _backend_name(world):
    if world == 1:
        return None
    import torch.distributed as dist
    return str(dist.get_backend())


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def reduce_over_ranks(world, v: float, op: str) -> float:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def host_cores():
    """Host cores this process may use: the CPU affinity set, capped by the
    cgroup CPU quota when one is set (a GPU box's share of a larger machine)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    for f in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, p = open(f).read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            quota = q / p
    except (OSError, ValueError):
        pass
    use = n if quota is None else max(1, min(n, int(math.ceil(quota))))
    return use, n, quota


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    of this workload (scripts/gpu_pmc.sh -> scripts/pmc_summary.py ->
    profiles/rNN_pmc_<workload>.json; FETCH_SIZE doubled per the gfx950
    caveat), measured in separate rocprofv3 --pmc passes of the same bench
    command; null if no summary of this workload exists (a Zipf run is never
    credited with the uniform run's counters)."""
    import glob
    files = sorted(glob.glob(str(ROOT / "profiles" / ("r*_pmc_%s.json" % workload))))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in d and "hbm_bytes_per_launch" in d[kernel]:
            return {"bytes_per_launch": round(d[kernel]["hbm_bytes_per_launch"]),
                    "read": round(d[kernel]["hbm_read_bytes"]),
                    "write": round(d[kernel]["hbm_write_bytes"]),
                    "source": os.path.relpath(f, str(ROOT))}
    return None


_ZIPF = {}


def remap_keys(args, k):
    """--keys-dist zipf: key -> workload.zipf_map(keys)[key] (numpy or torch)."""
    if args.keys_dist != "zipf":
        return k
    from flink_siddhi import workload
    if "np" not in _ZIPF:
        _ZIPF["np"] = workload.zipf_map(args.keys)
    if isinstance(k, __import__("numpy").ndarray):
        return _ZIPF["np"][k]
    import torch
    if "dev" not in _ZIPF:
        _ZIPF["dev"] = torch.from_numpy(_ZIPF["np"]).to(k.device)
    return _ZIPF["dev"][k.long()]


# ---------------------------------------------------------------- pattern --
def pattern_conds():
    sys.path.insert(0, str(ROOT / "oracle"))
    import cep_oracle as CO
    return CO, CO.cond(("price", 0, ">", 0.5)), CO.cond(("id", 7, "==", 0))


def pattern_parity(args, n, opts):
    """Fresh runtime over the first step's events (events [0, n), the bench
    geometry): the order-sensitive digest of its device output vs the C
    restatement's digest over the same events, sharded by key over the host
    threads.  Returns (result dict, host columns for the CPU baseline)."""
    import torch
    import flink_siddhi as fs
    from flink_siddhi import workload
    CO, f, g = pattern_conds()
    rt = fs.SiddhiAppRuntime(workload.PATTERN_PLAN, **dict(opts, profile=0))
    d = workload.generate_device(0, n, args.keys, rate=args.rate)
    d["k"] = remap_keys(args, d["k"])
    rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
    _, seq, cols = rt.output_tensors("O", copy=False)
    got_m = int(seq.shape[0])
    got_d = workload.rows_digest(cols[0], cols[1], cols[2], cols[3], seq)
    rt.flush()
    rt.shutdown()
    del d, seq, cols
    torch.cuda.empty_cache()
    T, _, _ = host_cores()
    w = CO.generate(0, n, args.keys, rate=args.rate, threads=T)
    w["k"] = remap_keys(args, w["k"])
    want_m, want_d, _ = CO.pattern_mt(w, args.keys, f, g, True, 10000, threads=T)
    kept = float(((w["stream"] == 0) & (w["price"] > 0.5)).sum() +
                 ((w["stream"] == 1) & (w["id"] % 7 == 0)).sum()) / n
    res = {"parity": "ok" if (got_m, got_d) == (want_m, want_d) else "MISMATCH",
           "events": n, "matches": got_m, "digest": "%016x" % got_d,
           "oracle_matches": want_m, "oracle_digest": "%016x" % want_d,
           "checker": "oracle/cep_oracle.c oracle_pattern_mt (fresh state, events [0, n))"}
    return res, w, kept


def cpu_baseline_pattern(args, w):
    """The C restatement (kind "port": the Java reference cannot run in this
    image) on the host cores: one thread, then sharded by key
    (k % T) over T threads, over the same 2^28 events of the parity check."""
    CO, f, g = pattern_conds()
    n = len(w["ts"])
    T, naff, quota = host_cores()
    m1, _, s1 = CO.pattern_mt(w, args.keys, f, g, True, 10000, threads=1)
    mT, _, sT = CO.pattern_mt(w, args.keys, f, g, True, 10000, threads=T)
    return {"value": round(n / sT, 1), "unit": "events/s", "cores": T, "kind": "port",
            "sample": "events [0, %d) of the config-3 stream (K=%d, R=%d/ms), oracle/cep_oracle.c "
                      "sharded by key over %d threads (affinity %d CPUs, cgroup quota %s), %d matches, "
                      "%.2f s; 1 thread: %.0f events/s (%.2f s)"
                      % (n, args.keys, args.rate, T, naff, "none" if quota is None else "%.1f" % quota,
                         mT, sT, n / s1, s1),
            "value_1core": round(n / s1, 1)}


# ----------------------------------------------------------------- filter --
def filter_parity(args, n):
    import numpy as np
    import torch
    import flink_siddhi as fs
    from flink_siddhi import workload
    CO, _, _ = pattern_conds()
    rt = fs.SiddhiAppRuntime(workload.FILTER_PLAN, ordered_output=0)
    d = workload.generate_device(0, n, 1, single_stream=True)
    name = torch.zeros(n, dtype=torch.int32, device="cuda")
    rt.send("inputStream", d["ts"], [d["id"], name, d["price"], d["ts"]])
    _, seq, cols = rt.output_tensors("O", copy=False)
    got_m = int(seq.shape[0])
    got_d = workload.rows_digest(cols[0], cols[2], cols[2], cols[3], seq)
    ordered = bool((seq[1:] > seq[:-1]).all().item()) if got_m > 1 else True
    rt.flush()
    rt.shutdown()
    del d, name, seq, cols
    T, _, _ = host_cores()
    w = CO.generate(0, n, 1, single_stream=True, threads=T)
    sel = CO.filter_indices(w["id"], w["price"], CO.cond(("price", 0, ">", 0.5), ("id", 7, "==", 0)))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    want_d = workload.rows_digest(t(w["id"][sel]), t(w["price"][sel]), t(w["price"][sel]),
                                  t(w["ts"][sel]), t(sel))
    ok = ordered and (got_m, got_d) == (len(sel), want_d)
    return {"parity": "ok" if ok else "MISMATCH", "events": n, "matches": got_m,
            "digest": "%016x" % got_d, "oracle_matches": int(len(sel)), "oracle_digest": "%016x" % want_d,
            "checker": "oracle/cep_oracle.c oracle_filter (arrival order)"}, w


def cpu_baseline_filter(w):
    CO, _, _ = pattern_conds()
    f = CO.cond(("price", 0, ">", 0.5), ("id", 7, "==", 0))
    n = len(w["id"])
    t0 = time.perf_counter()
    CO.filter_indices(w["id"], w["price"], f)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "events/s", "cores": 1, "kind": "port",
            "sample": "events [0, %d) of the config-2 stream, oracle/cep_oracle.c single-threaded, "
                      "%.2f s" % (n, dt)}


# ---------------------------------------------------------------- config 5 --
C5_SEQ_SEL_BYTES = 4 + 8 + 8 + 8    # Seq<q>: k, p1, p2, t3
C5_AGG_SEL_BYTES = 4 + 8 + 8        # Agg<q>: k, total, n


def config5_parity(args, opts, n, steps):
    """A fresh runtime over the bench stream's first `steps` steps (n events
    each, output read per step as the bench flushes it) vs oracle/mq_oracle.c
    sharded by key over the host cores on the same events: every one of the
    64 outputs by row count and order-sensitive digest (per-key order, every
    select word, ts, seq).  The oracle's processing time is the CPU baseline
    (kind "port": the Java reference cannot run in this image)."""
    import numpy as np
    import torch
    import flink_siddhi as fs
    from flink_siddhi import workload
    sys.path.insert(0, str(ROOT / "oracle"))
    import cep_oracle as CO
    outs = workload.CONFIG5_OUTPUTS
    rt = fs.SiddhiAppRuntime(workload.config5_plan(), **dict(opts, profile=0))
    base = {o: torch.zeros(args.keys, dtype=torch.int64, device="cuda") for o in outs}
    cnt = {o: 0 for o in outs}
    dig = {o: 0 for o in outs}
    for s in range(steps):
        d = workload.generate_device(s * n, n, args.keys, rate=args.rate)
        d["k"] = remap_keys(args, d["k"])
        d["stream"] = workload.config5_streams(d["price"]).to(torch.uint8)
        rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
        for o in outs:
            ts, seq, cols = rt.output_tensors(o, copy=False)
            cnt[o] += int(ts.shape[0])
            try:
                dig[o] = (dig[o] + workload.rows_digest_words(cols[0], cols, ts, seq, base[o])) & ((1 << 64) - 1)
            except ValueError:   # keys outside the key space: a mismatch, reported as such
                dig[o] = -1
        rt.reset_output()
        del d
    rt.shutdown()
    del base
    torch.cuda.empty_cache()
    T, naff, quota = host_cores()
    w = CO.generate(0, steps * n, args.keys, rate=args.rate, threads=T)
    w["k"] = remap_keys(args, w["k"])
    w["stream"] = workload.config5_streams(w["price"]).astype(np.uint8)
    wc, wd, sec = CO.mq_mt(CO.config5_queries(), w, args.keys, threads=T)
    bad = [o for i, o in enumerate(outs) if (cnt[o], dig[o]) != (wc[i], wd[i])]
    seq_rows = sum(wc[:32])
    agg_rows = sum(wc[32:])
    res = {"parity": "ok" if not bad else "MISMATCH", "events": steps * n, "steps": steps,
           "rows": sum(cnt.values()), "seq_rows": seq_rows, "agg_rows": agg_rows,
           "mismatched_outputs": bad[:8],
           "checker": "oracle/mq_oracle.c mq_run_mt (fresh state, events [0, %d)): every output's row count "
                      "and order-sensitive digest" % (steps * n)}
    cpu = {"value": round(steps * n / sec, 1), "unit": "events/s", "cores": T, "kind": "port",
           "sample": "events [0, %d) of the config-5 stream (K=%d, R=%d/ms), oracle/mq_oracle.c sharded by key "
                     "over %d threads (affinity %d CPUs, cgroup quota %s), %d rows, %.2f s"
                     % (steps * n, args.keys, args.rate, T, naff, "none" if quota is None else "%.1f" % quota,
                        seq_rows + agg_rows, sec)}
    sel = (C5_SEQ_SEL_BYTES * seq_rows + C5_AGG_SEL_BYTES * agg_rows) / max(1, seq_rows + agg_rows)
    return res, cpu, sel


# ------------------------------------------------------------------- main --
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun around us: start the ranks ourselves (before any torch import)
        sys.exit(launch_ranks(args.gpus))
    import torch
    import flink_siddhi as fs
    from flink_siddhi import _lib as L
    from flink_siddhi import workload

    world, rank, local = dist_init(args)
    pattern = args.workload == "pattern"
    config5 = args.workload == "config5"
    n = args.events or ((1 << 28) if pattern else (1 << 24) if config5 else 100_000_000)
    steps, warm = args.steps, args.warmup

    if pattern:
        plan = workload.PATTERN_PLAN
        opts = dict(device=local, key_capacity=(args.keys + world - 1) // world,
                    key_stride=world, key_offset=rank, chunk_events=args.chunk,
                    profile=PROFILE_EVERY, ordered_output=0, ts_order=args.ts_order)
        if args.buckets_log2:
            opts["buckets_log2"] = args.buckets_log2
    elif config5:
        plan = workload.config5_plan()
        opts = dict(device=local, key_capacity=(args.keys + world - 1) // world, key_stride=world,
                    key_offset=rank, pending_slots=4, profile=PROFILE_EVERY, ordered_output=0,
                    chunk_events=min(args.chunk, 1 << 24), ts_order=args.ts_order)
    else:
        plan = workload.FILTER_PLAN
        opts = dict(device=local, profile=PROFILE_EVERY, ordered_output=0)

    # parity + CPU baseline first (N=1): the host leg needs the same events
    parity, cpu, kept = None, None, None
    c5_sel = C5_AGG_SEL_BYTES
    if config5:
        if world == 1 and not (args.no_parity and args.no_cpu):
            parity, cpu, c5_sel = config5_parity(args, opts, n, args.parity_steps)
            if args.no_parity:
                parity = None
            if args.no_cpu:
                cpu = None
    elif world == 1 and not (args.no_parity and args.no_cpu):
        if pattern:
            parity, w, kept = pattern_parity(args, n, opts)
            if not args.no_cpu:
                cpu = cpu_baseline_pattern(args, w)
        else:
            parity, w = filter_parity(args, n)
            if not args.no_cpu:
                cpu = cpu_baseline_filter(w)
        if args.no_parity:
            parity = None
        del w
    if args.ordered:
        opts["ordered_output"] = 1
    if not args.with_seq:
        # the reference's StreamOutputHandler never reads the arrival number:
        # with unordered output it is not even stored, and it is not gathered
        # or copied to the host (cep_options.omit_seq); the parity runs above
        # keep it (their digests cover it)
        opts["omit_seq"] = 1
    rt = fs.SiddhiAppRuntime(plan, **opts)

    # Inputs for every step, generated on the device before the timed region.
    # Multi-GPU ingest: "shuffle" (default) — rank r holds global index range
    # r of each step and the engine routes it (push-down + owner = k % world),
    # RCCL all-to-all moves the records, each owner walks what it received;
    # "prepartitioned" — the input is already keyed upstream (Flink keyBy):
    # rank r draws only keys it owns, no exchange.
    shuffle_mode = (pattern or config5) and world > 1 and args.ingest == "shuffle"
    host_ingest = args.ingest in ("host", "host-pageable") and world == 1
    batches = []
    for s in range(warm + steps):
        first = (s * world + rank) * n
        d = workload.generate_device(first, n, args.keys, rate=args.rate,
                                     single_stream=not pattern, device="cuda")
        d["first"] = first
        if pattern or config5:
            d["k"] = remap_keys(args, d["k"])
        if (pattern or config5) and world > 1 and not shuffle_mode:
            d["k"] = (d["k"] // world) * world + rank     # owned keys, same distribution
        if config5:
            d["stream"] = workload.config5_streams(d["price"]).to(torch.uint8)
        elif not pattern:
            d["name"] = torch.zeros(n, dtype=torch.int32, device="cuda")
        if host_ingest:   # the batch lives in host memory; the engine stages it over PCIe
            d = {c: (v.cpu().pin_memory() if args.ingest == "host" else v.cpu()).numpy()
                 if hasattr(v, "cpu") else v for c, v in d.items()}
        batches.append(d)
    torch.cuda.synchronize()

    bufs = {}
    delivered = [0]
    if args.deliver:
        outs = workload.CONFIG5_OUTPUTS if config5 else ["O"]
        for o in outs:
            rt.add_callback(o, lambda rows: delivered.__setitem__(0, delivered[0] + len(rows)), copy=False)

    guard = [torch.cuda.Stream(), torch.cuda.Stream()] if shuffle_mode else None

    # pattern: k_cfroute with predicate push-down; config 5 (64 queries,
    # sequences): whole rows (cep_route_rows)
    route_fn = rt.route if pattern else rt.route_rows
    send_fn = rt.send_records if pattern else rt.send_rows

    def route(d, j):
        # inputs were generated before the timed region (synchronized): the
        # route of step s+1 need not queue behind the exchange on torch's stream
        recs, counts = route_fn("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]],
                                world, seq0=d["first"], streams=d["stream"],
                                out=bufs.get(("send", j)), wait=False)
        bufs[("send", j)] = recs
        return recs, counts

    seg_cap = [0]

    pshuf = [None]

    def run_padded(blist):
        # Padded exchange with a spill (flink_siddhi.shuffle.PaddedShuffle):
        # fixed owner segments with in-band counts, one equal-split
        # all-to-all, nothing read back on the step's critical path; an
        # owner's records past seg_cap go to a spill buffer and, when any
        # rank spilled (one host all-reduce of an integer, one step late),
        # through a second exact exchange -- a key-distribution shift never
        # drops a record.  The owner's walk of step s is queued at step s+1.
        from flink_siddhi import shuffle
        if pshuf[0] is None:
            pshuf[0] = shuffle.PaddedShuffle(rt, world, seg_cap[0], spill_cap=n // 2, rows=not pattern)
        ps = pshuf[0]
        for d in blist:
            ps.step("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], seq0=d["first"], events=n,
                    streams=d["stream"])
        ps.finish()
        rt.flush()

    def run_shuffle(blist):
        # Software pipeline over steps, double-buffered send / receive: the
        # route of step s+1 (engine route stream) and the record all-to-all of
        # step s+1 (RCCL) run while the walk of step s runs on the engine stream.
        from flink_siddhi import shuffle
        if not blist:
            return
        if args.exchange == "padded" and seg_cap[0] == 0:
            # calibrate the segment capacity on the first warm-up step
            # (two-phase: host counts), then every later step is padded
            recs, counts = route(blist[0], 0)
            # 3 % over the largest owner: records past it spill (PaddedShuffle),
            # so the slack only sizes the common case, and every padding
            # record is bytes on xGMI and a null record for the owner
            seg_cap[0] = shuffle.calibrated_capacity(counts, slack=0.03)
            recv, m, _ = shuffle.exchange(recs, counts, out=bufs.get(("recv", 0)))
            bufs[("recv", 0)] = recv
            send_fn(recv, m, n, signal=False)
            rt.signal(guard[0])
            blist = blist[1:]
            if not blist:
                rt.flush()
                return
        if args.exchange == "padded":
            run_padded(blist)
            return
        cur = route(blist[0], 0)
        for i in range(len(blist)):
            j = i % 2
            recs, counts = cur
            torch.cuda.current_stream().wait_stream(guard[j])   # the walk that last read recv[j]
            recv, m, _ = shuffle.exchange(recs, counts, out=bufs.get(("recv", j)))
            bufs[("recv", j)] = recv
            send_fn(recv, m, n, signal=False)
            rt.signal(guard[j])
            if i + 1 < len(blist):
                cur = route(blist[i + 1], 1 - j)
        rt.flush()

    def step(d):
        if pattern or config5:
            rt.send("A", d["ts"], [d["k"], d["ts"], d["id"], d["price"]], streams=d["stream"])
        else:
            rt.send("inputStream", d["ts"], [d["id"], d["name"], d["price"], d["ts"]])
        rt.flush()

    if shuffle_mode:
        run_shuffle(batches[:warm])
    else:
        for s in range(warm):
            step(batches[s])
    st0 = rt.stats()
    d0 = delivered[0]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if shuffle_mode:
        run_shuffle(batches[warm:])
    else:
        for s in range(steps):
            step(batches[warm + s])
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    st1 = rt.stats()
    dt_max = reduce_over_ranks(world, dt, "max")
    events_total = reduce_over_ranks(world, float(n * steps), "sum")
    matches_total = reduce_over_ranks(world, float(st1.matches_out - st0.matches_out), "sum")
    value = events_total / dt_max

    # per-kernel HIP-event times on the engine's stream over the timed region
    kern = {}
    for k, name in ((L.K_PARTITION, "k_partition"), (L.K_WALK, "k_walk"), (L.K_FILTER, "k_filter"),
                    (L.K_ROUTE, "k_route"), (L.K_CF_PARTITION, "k_cfpart"), (L.K_CF_WALK, "k_cfwalk"),
                    (L.K_MQ_PARTITION, "k_mqpart"), (L.K_MQ_WALK, "k_mqwalk")):
        launches = st1.kernel_launches[k] - st0.kernel_launches[k]
        timed = st1.kernel_timed[k] - st0.kernel_timed[k]
        ms = st1.kernel_ms[k] - st0.kernel_ms[k]
        if launches and timed and ms > 0:
            kern[name] = {"launches": int(launches), "timed_launches": int(timed),
                          "avg_us": round(1e3 * ms / timed, 2), "total_ms": round(ms / timed * launches, 3)}
    m_per_event = (st1.matches_out - st0.matches_out) / float(n * steps)
    ev_total = float(n * steps)
    keys_local = (args.keys + world - 1) // world
    # SURVEY §8(d) algorithmic bytes per event: the columns the workload reads
    # once + the selected attributes of every output row
    if pattern:
        alg_per_event = PATTERN_IN_BYTES + PATTERN_SEL_BYTES * m_per_event
    elif config5:
        alg_per_event = PATTERN_IN_BYTES + c5_sel * m_per_event
    else:
        alg_per_event = FILTER_IN_BYTES + FILTER_SEL_BYTES * m_per_event   # 13.92 B at 8 % selectivity
    # Design bytes (diagnostic): what each kernel of this implementation must
    # move per launch — its inputs, records it writes / reads, output rows
    # with their ts / seq, per-key state.
    kept = kept if kept is not None else 0.33
    design = {}
    if pattern:
        design = {
            "k_cfpart": ev_total * (PATTERN_IN_BYTES + CF_REC_BYTES * kept),
            "k_cfwalk": ev_total * (CF_REC_BYTES * kept + PATTERN_OUT_BYTES * m_per_event),
            "k_partition": ev_total * PATTERN_IN_BYTES,
            "k_walk": ev_total * PATTERN_OUT_BYTES * m_per_event,
        }
        for k in ("k_cfwalk", "k_walk"):
            if k in kern:
                design[k] += kern[k]["launches"] * keys_local * CF_STATE_BYTES
        if shuffle_mode:
            design["k_route"] = ev_total * PATTERN_IN_BYTES
    elif config5:
        rec = 8 * (2 + 1)   # k_mqpart record: w0, w1, price (the ts column aliases the event ts)
        st_words = 32 * 4 + 32 * 3
        design = {"k_mqpart": ev_total * (PATTERN_IN_BYTES + rec),
                  "k_mqwalk": ev_total * (rec + (c5_sel + 16) * m_per_event)}
        if "k_mqwalk" in kern:
            design["k_mqwalk"] += kern["k_mqwalk"]["launches"] * keys_local * st_words * 8 * 2
    else:
        design = {"k_filter": ev_total * (FILTER_IN_BYTES + FILTER_OUT_BYTES * m_per_event)}
    # PMC summaries are per workload (scripts/gpu_pmc.sh runs of the default
    # config-3 / filter / config-5 commands)
    pmc_tag = ("config3" if args.keys_dist == "uniform" else "zipf") if pattern else \
        ("config5" if config5 else "filter")
    per_kernel = {}
    for kname, b in design.items():
        if kname not in kern:
            continue
        per_launch = b / kern[kname]["launches"]
        ach = per_launch / (kern[kname]["avg_us"] * 1e-6) / 1e9
        per_kernel[kname] = {"design_bytes_per_launch": round(per_launch), "avg_launch_us": kern[kname]["avg_us"],
                             "design_achieved": round(ach, 1), "design_frac": round(ach / HBM_PEAK_GBS, 4),
                             "traffic": pmc_traffic(kname, pmc_tag) if world == 1 else None}
    roofline = None
    if kern:   # CEP_PROFILE=0 (no per-kernel timer events): no kernel roofline
        # the dominant kernel (largest share of the step's kernel time),
        # credited with the §8(d) bytes of the events one launch covers
        dom = max(kern, key=lambda k: kern[k]["total_ms"])
        ev_launch = ev_total / kern[dom]["launches"]
        alg_launch = alg_per_event * ev_launch
        ach = alg_launch / (kern[dom]["avg_us"] * 1e-6) / 1e9
        tr = pmc_traffic(dom, pmc_tag) if world == 1 else None
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": tr["bytes_per_launch"] if tr else None,
                    "alg_bytes_per_event": round(alg_per_event, 3), "events_per_launch": round(ev_launch),
                    "alg_bytes_per_launch": round(alg_launch), "avg_launch_us": kern[dom]["avg_us"],
                    "formula": "alg_bytes_per_event * events_per_launch / avg_launch_us"}
    per_gpu_events = value / world
    pipeline = {"alg_bytes_per_event": round(alg_per_event, 3),
                "achieved": round(per_gpu_events * alg_per_event / 1e9, 1), "unit": "GB/s",
                "peak": HBM_PEAK_GBS,
                "frac": round(per_gpu_events * alg_per_event / 1e9 / HBM_PEAK_GBS, 4)}

    in_b = PATTERN_IN_BYTES if (pattern or config5) else 4 + 4 + 8 + 8 + 8   # bytes per host event
    if rank == 0:
        out = {
            "metric": "matched-pattern events/sec (whole node) at 1/2/4/8 MI355X + % HBM roofline",
            "value": round(value, 1), "unit": "events/s", "n_gpus": world,
            "backend": _backend_name(world),
            "rccl_world": world if _backend_name(world) == "nccl" else 0,
            "launcher": os.environ.get("CEP_LAUNCHED_BY", "torchrun" if world > 1 else "none"),
            "steps": steps, "warmup": warm, "ms_per_step": round(1e3 * dt_max / steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64+int32+int64", "data": "synthetic (splitmix64 counter stream, BASELINE.md §3)",
            "config": ({"workload": "config3: keyed every A -> B within 10 sec, partition with k",
                        "keys": args.keys, "keys_dist": args.keys_dist if args.keys_dist == "uniform" else "zipf(s=1.1)",
                        "events_per_step_per_gpu": n, "rate_per_ms": args.rate,
                        "chunk_events": args.chunk, "parallelism": "key-sharded x%d" % world,
                        "ts_order": ("event-time order (ts_order=1: event-time fast paths)" if args.ts_order
                                     else "any order (ts_order=0: order-tolerant path)"),
                        "ingest": (("%s all-to-all key shuffle (%s)" % ("rccl" if _coll_device() == "cuda"
                                                                         else "gloo host-staged",
                                                                         "padded segments, in-band counts, "
                                                                         "spill exchange on overflow"
                                                                         if args.exchange == "padded"
                                                                         else "two-phase"))
                                    if shuffle_mode else
                                   "pre-partitioned (keyed upstream)") if world > 1 else
                                  ("host (%s memory over PCIe)" % ("pinned" if args.ingest == "host" else "pageable")
                                   if host_ingest else "device-resident")}
                       if pattern else
                       {"workload": "config5: 64 queries (32 every A, B+, C within 10 sec sequences with "
                                    "id == q%50, 32 group-by/having aggregations), 3 keyed streams",
                        "keys": args.keys, "keys_dist": args.keys_dist if args.keys_dist == "uniform" else "zipf(s=1.1)",
                        "events_per_step_per_gpu": n, "rate_per_ms": args.rate,
                        "parallelism": "key-sharded x%d" % world,
                        "ingest": (("%s all-to-all row shuffle (%s)" % ("rccl" if _coll_device() == "cuda"
                                                                        else "gloo host-staged",
                                                                        "padded segments, in-band counts"
                                                                        if args.exchange == "padded"
                                                                        else "two-phase"))
                                   if shuffle_mode else "pre-partitioned (keyed upstream)")
                        if world > 1 else "local"}
                       if config5 else
                       {"workload": "config2: inputStream[price > 0.5 and id % 7 == 0] select *",
                        "events_per_step_per_gpu": n, "parallelism": "replicas x%d" % world}),
            "shuffle_spilled_steps": pshuf[0].spilled_steps if pshuf[0] is not None else None,
            "matches_per_s": round(matches_total / dt_max, 1),
            "matches_per_event": round(m_per_event, 5),
            "pipeline_roofline": pipeline,
            "roofline": roofline,
            "roofline_kernels": per_kernel,
            "kernels": kern,
            "parity": parity,
            "host_io": ({"ingest": args.ingest if host_ingest else "device-resident", "bytes_in_per_event": in_b,
                         "pcie_in_GBs": round(value * in_b / 1e9, 2) if host_ingest else 0.0,
                         "delivered_rows": delivered[0] - d0 if args.deliver else None,
                         "delivered_rows_per_s": round((delivered[0] - d0) / dt_max, 1) if args.deliver else None,
                         "ordered_output": bool(args.ordered)}
                        if host_ingest or args.deliver else None),
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
