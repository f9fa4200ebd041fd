"""Config-5 family plans (SiddhiQL text for the engine and the Python oracle)
and their oracle/mq_oracle.c query descriptors, shared by the CPU oracle
cross-checks and the GPU parity tests.

* `workload.config5_plan()` — BASELINE config 5 exactly (CO.config5_queries);
* `variant_plan()` — the same shape with `id % 10` sequence conditions (they
  complete often on short streams) and aggregations over all three streams
  with `id >= q` filters and `having total > 1 + q/8`.
"""
import numpy as np

import cep_oracle as CO

EV3 = ("define stream A (k int, ts long, id int, price double);"
       "define stream B (k int, ts long, id int, price double);"
       "define stream C (k int, ts long, id int, price double);")
NAMES = ("A", "B", "C")
NQ = 32


def variant_plan():
    seq = ["partition with (k of A, k of B, k of C) begin "]
    for q in range(NQ):
        seq.append("from every s1=A[price > %s], s2=B[id %% 10 == %d]+, s3=C[id %% 10 == %d] "
                   "within 10 sec select s1.k as k, s1.price as p1, s2[last].price as p2, "
                   "s3.ts as t3 insert into Seq%d;" % (repr(q / 64.0), q % 10, (q + 1) % 10, q))
    seq.append(" end;")
    agg = []
    for q in range(NQ):
        agg.append("from %s[id >= %d] select k, sum(price) as total, count() as n "
                   "group by k having total > %s insert into Agg%d;"
                   % (NAMES[q % 3], q, repr(1.0 + q / 8.0), q))
    return EV3 + "".join(seq) + "".join(agg)


def variant_queries(within=10000):
    qs = []
    for q in range(NQ):
        qs.append(CO.nfa_query([(0, 1, 1, [("price", 0, ">", q / 64.0)]),
                                (1, 1, -1, [("id", 10, "==", q % 10)]),
                                (2, 1, 1, [("id", 10, "==", (q + 1) % 10)])],
                               [(0, 0, "k"), (0, 0, "price"), (1, -1, "price"), (2, 0, "ts")], within=within))
    for q in range(NQ):
        qs.append(CO.agg_query(q % 3, [("id", 0, ">=", q)], [("sum", "price"), ("count", None)],
                               ["k", ("agg", 0), ("agg", 1)], having=(1, ">", 1.0 + q / 8.0)))
    return qs


def variant_outputs():
    return ["Seq%d" % q for q in range(NQ)] + ["Agg%d" % q for q in range(NQ)]


def three_streams(n, keys, rate=1, first=0):
    """The BASELINE stream with config 5's stream split (0 = A, 1 = B, 2 = C)."""
    from flink_siddhi import workload
    w = workload.generate(first, n, keys, rate=rate)
    w["stream"] = workload.config5_streams(w["price"]).astype(np.uint8)
    return w


def events(w):
    k, ts, i, p, st = (w[c].tolist() for c in ("k", "ts", "id", "price", "stream"))
    return [(NAMES[st[j]], ts[j], (k[j], ts[j], i[j], p[j])) for j in range(len(ts))]


def word(v) -> int:
    """A Python-oracle output value as the C oracle's raw 64-bit word."""
    if isinstance(v, float):
        return int(np.array([v], np.float64).view(np.uint64)[0])
    return int(v) & ((1 << 64) - 1)


def as_words(rows):
    return [(ts, seq, tuple(word(v) for v in data)) for ts, seq, data in rows]
