"""Synthetic keyed event streams.

Counter-based, so host (numpy), device (libcep `cep_generate`) and any rank
of a multi-GPU job produce the identical stream for any index range:

    r(i, j) = splitmix64(seed ^ (i * 0x9E3779B97F4A7C15) ^ j),  seed = 0x5EEDC0DE
    key    = r(i,0) mod K
    stream = r(i,1) >> 63          (0 = A, 1 = B)
    id     = r(i,2) mod 50         (RandomEventSource.java:60 id range)
    price  = (r(i,3) >> 11) * 2^-53  in [0, 1)  (Random.nextDouble, :61)
    ts     = T0 + floor(i / R) ms
"""
from __future__ import annotations

import numpy as np

SEED = 0x5EEDC0DE
GOLDEN = 0x9E3779B97F4A7C15
T0 = 1_500_000_000_000

PATTERN_PLAN = (
    "define stream A (k int, ts long, id int, price double);"
    "define stream B (k int, ts long, id int, price double);"
    "partition with (k of A, k of B) begin "
    "from every s1=A[price > 0.5] -> s2=B[id % 7 == 0] within 10 sec "
    "select s1.k as k, s1.price as p1, s2.price as p2, s2.ts as t "
    "insert into O; end;")

FILTER_PLAN = (
    "define stream inputStream (id int, name string, price double, timestamp long);"
    "from inputStream[price > 0.5 and id % 7 == 0] select * insert into O;")


def config5_plan() -> str:
    """BASELINE config 5 exactly as SURVEY §8(d) states it, one app of 64
    queries over three keyed streams: q = 0..31 `every s1=A[price > q/32],
    s2=B[id == q%50]+, s3=C[id == (q+1)%50] within 10 sec` (outputs Seq<q>),
    q = 32..63 `from A[price > (q-32)/32] select k, sum(price) as total,
    count() as n group by k having total > 1.0` (outputs Agg<q>)."""
    ev = "".join("define stream %s (k int, ts long, id int, price double);" % s for s in "ABC")
    seq = ["partition with (k of A, k of B, k of C) begin "]
    for q in range(32):
        seq.append("from every s1=A[price > %s], s2=B[id == %d]+, s3=C[id == %d] within 10 sec "
                   "select s1.k as k, s1.price as p1, s2[last].price as p2, s3.ts as t3 insert into Seq%d;"
                   % (repr(q / 32.0), q % 50, (q + 1) % 50, q))
    seq.append(" end;")
    agg = ["from A[price > %s] select k, sum(price) as total, count() as n "
           "group by k having total > 1.0 insert into Agg%d;" % (repr((q - 32) / 32.0), q)
           for q in range(32, 64)]
    return ev + "".join(seq) + "".join(agg)


CONFIG5_OUTPUTS = ["Seq%d" % q for q in range(32)] + ["Agg%d" % q for q in range(32, 64)]


def config5_streams(price):
    """Stream handle (0 = A, 1 = B, 2 = C) of each event for config 5: a
    function of the generated price (numpy or torch), as the tests do."""
    return (price * 1000).astype(np.int64) % 3 if isinstance(price, np.ndarray) else \
        ((price * 1000).long() % 3)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def generate(first: int, n: int, keys: int, rate: int = 400, seed: int = SEED,
             t0: int = T0, single_stream: bool = False):
    """Columns for events [first, first+n): dict of numpy arrays."""
    i = np.arange(first, first + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        b = np.uint64(seed) ^ (i * np.uint64(GOLDEN))
    key = (splitmix64(b ^ np.uint64(0)) % np.uint64(keys)).astype(np.int32)
    stream = np.zeros(n, np.uint8) if single_stream else \
        (splitmix64(b ^ np.uint64(1)) >> np.uint64(63)).astype(np.uint8)
    idv = (splitmix64(b ^ np.uint64(2)) % np.uint64(50)).astype(np.int32)
    price = (splitmix64(b ^ np.uint64(3)) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    ts = (t0 + (i // np.uint64(rate)).astype(np.int64)).astype(np.int64)
    return {"k": key, "stream": stream, "id": idv, "price": price, "ts": ts}


def zipf_map(keys: int, s: float = 1.1, seed: int = 7):
    """Zipf(s) over `keys` ranks as a key -> key remap of the uniform
    generator's keys (BASELINE.md §3 "Zipf s=1.1 variant"): key k (uniform in
    [0, keys)) becomes perm[rank], rank = the Zipf inverse CDF at (k + 0.5) /
    keys; perm scatters the hot ranks over the key space (and so over
    buckets).  Returns the int32 lookup table (numpy): zipf_key = table[k]."""
    r = np.arange(1, keys + 1, dtype=np.float64)
    w = r ** -s
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    u = (np.arange(keys, dtype=np.float64) + 0.5) / keys
    rank = np.minimum(np.searchsorted(cdf, u, side="left"), keys - 1)
    perm = np.random.default_rng(seed).permutation(keys).astype(np.int32)
    return perm[rank]


def _lsr(x, s: int):
    """Logical right shift of int64 tensors (torch's >> is arithmetic)."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def _smix_t(z):
    z = z + (GOLDEN - (1 << 64))
    z = (z ^ _lsr(z, 30)) * (0xBF58476D1CE4E5B9 - (1 << 64))
    z = (z ^ _lsr(z, 27)) * (0x94D049BB133111EB - (1 << 64))
    return z ^ _lsr(z, 31)


def rows_digest(k, p1, p2, t, seq) -> int:
    """Order-sensitive digest of config-3 output rows (torch tensors on any
    device, rows in emission order): sum over rows of
    oracle_row_digest(k, rank of the row among its key's rows, p1, p2, t,
    seq) mod 2^64 — the same function as oracle/cep_oracle.c, so a bench or
    test can compare the engine's device output with the oracle without
    moving rows to the host.  Independent of how keys interleave, sensitive
    to the order inside each key."""
    import torch
    n = int(k.shape[0])
    if n == 0:
        return 0
    k64 = k.to(torch.int64)
    order = torch.argsort(k64, stable=True)
    ks = k64[order]
    idx = torch.arange(n, device=k.device, dtype=torch.int64)
    start = torch.zeros(n, dtype=torch.bool, device=k.device)
    start[0] = True
    start[1:] = ks[1:] != ks[:-1]
    first = torch.cummax(torch.where(start, idx, torch.zeros_like(idx)), 0).values
    rank = torch.empty_like(idx)
    rank[order] = idx - first
    x = _smix_t((k64 & 0xFFFFFFFF) | (rank << 32))
    x = _smix_t(x ^ p1.contiguous().view(torch.int64))
    x = _smix_t(x ^ p2.contiguous().view(torch.int64))
    x = _smix_t(x ^ t.to(torch.int64))
    x = _smix_t(x ^ seq.to(torch.int64))
    return int(x.sum().item()) & ((1 << 64) - 1)


def _key_ranks(k64):
    """Rank of every row among the rows of its key, in row order."""
    import torch
    n = int(k64.shape[0])
    order = torch.argsort(k64, stable=True)
    ks = k64[order]
    idx = torch.arange(n, device=k64.device, dtype=torch.int64)
    start = torch.zeros(n, dtype=torch.bool, device=k64.device)
    start[0] = True
    start[1:] = ks[1:] != ks[:-1]
    first = torch.cummax(torch.where(start, idx, torch.zeros_like(idx)), 0).values
    rank = torch.empty_like(idx)
    rank[order] = idx - first
    return rank


def rows_digest_words(key, cols, ts, seq, rank_base=None) -> int:
    """Order-sensitive digest of any output stream's rows (torch tensors,
    rows in emission order): sum over rows of oracle/mq_oracle.c
    mq_row_digest(key, rank among the key's rows, every select column as a
    64-bit word — ints sign-extended, doubles as their bits — , ts, seq).
    rank_base (int64 tensor indexed by key, optional): rows each key had in
    earlier parts of the same output; it is advanced by this part's rows, so
    a stream flushed in parts digests like the whole."""
    import torch
    n = int(ts.shape[0])
    if n == 0:
        return 0
    k64 = key.to(torch.int64)
    rank = _key_ranks(k64)
    if rank_base is not None:
        lo, hi = int(k64.min().item()), int(k64.max().item())
        if lo < 0 or hi >= rank_base.shape[0]:   # (a wrong key must not index out of bounds)
            raise ValueError("output key %d..%d outside [0, %d)" % (lo, hi, rank_base.shape[0]))
        rank = rank + rank_base[k64]
        rank_base.index_add_(0, k64, torch.ones_like(k64))
    x = _smix_t((k64 & 0xFFFFFFFF) | (rank << 32))
    for c in cols:
        c = c.contiguous()
        w = c.view(torch.int64) if c.dtype == torch.float64 else \
            c.view(torch.int32).to(torch.int64) if c.dtype == torch.float32 else c.to(torch.int64)
        x = _smix_t(x ^ w)
    x = _smix_t(x ^ ts.to(torch.int64))
    x = _smix_t(x ^ seq.to(torch.int64))
    return int(x.sum().item()) & ((1 << 64) - 1)


def generate_device(first: int, n: int, keys: int, rate: int = 400, seed: int = SEED,
                    t0: int = T0, single_stream: bool = False, device="cuda"):
    """Same stream, generated on the GPU into torch tensors (bench inputs)."""
    import ctypes as C
    import torch
    from . import _lib as L
    key = torch.empty(n, dtype=torch.int32, device=device)
    ts = torch.empty(n, dtype=torch.int64, device=device)
    stream = torch.empty(n, dtype=torch.uint8, device=device)
    idv = torch.empty(n, dtype=torch.int32, device=device)
    price = torch.empty(n, dtype=torch.float64, device=device)
    s = torch.cuda.current_stream(device).cuda_stream
    rc = L.lib().cep_generate(first, n, seed, keys, rate, t0, 1 if single_stream else 0,
                              C.c_void_p(key.data_ptr()), C.c_void_p(ts.data_ptr()),
                              C.c_void_p(stream.data_ptr()), C.c_void_p(idv.data_ptr()),
                              C.c_void_p(price.data_ptr()), C.c_void_p(s))
    L.raise_for(rc, "cep_generate failed")
    return {"k": key, "stream": stream, "id": idv, "price": price, "ts": ts}
