"""N-state patterns and sequences with count states on the device (SURVEY.md
§8 row a3: `every s1=A, s2=B+, s3=C within` and friends) vs the CPU oracle,
bit-exact, on seeded three-stream workloads."""
import numpy as np
import pytest

import flink_siddhi as fs
from flink_siddhi import workload
from helpers import assert_same_rows, engine_rows, oracle_run

pytestmark = pytest.mark.gpu

EV3 = ("define stream A (k int, ts long, id int, price double);"
       "define stream B (k int, ts long, id int, price double);"
       "define stream C (k int, ts long, id int, price double);")
NAMES = ("A", "B", "C")


def three_streams(n, keys, seed_shift=0):
    w = workload.generate(seed_shift, n, keys, rate=1)
    w["stream"] = ((w["price"] * 1000).astype(np.int64) % 3).astype(np.uint8)
    return w


def events(w):
    k, ts, i, p, st = (w[c].tolist() for c in ("k", "ts", "id", "price", "stream"))
    return [(NAMES[st[j]], ts[j], (k[j], ts[j], i[j], p[j])) for j in range(len(ts))]


def run(plan, w, batches=1, **opts):
    rt = fs.SiddhiAppRuntime(plan, **opts)
    rt.add_callback("O")
    n = len(w["ts"])
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        rt.send("A", w["ts"][s:e], [w["k"][s:e], w["ts"][s:e], w["id"][s:e], w["price"][s:e]],
                streams=w["stream"][s:e])
        rt.flush()
    got = engine_rows(rt.collect("O"))
    rt.shutdown()
    return got


def case(query, n=20000, keys=256, batches=1, **opts):
    plan = EV3 + query
    w = three_streams(n, keys)
    want = oracle_run(plan, events(w)).get("O", [])
    got = run(plan, w, batches=batches, **opts)
    assert_same_rows(got, want, query)
    return len(want)


P3 = "partition with (k of A, k of B, k of C) begin "


def test_config5_sequence_kleene():
    m = case(P3 + "from every s1=A[price > 0.25], s2=B[id < 30]+, s3=C[id > 20] within 10 sec "
             "select s1.k as k, s1.price as p1, s2[last].price as p2, s3.price as p3 "
             "insert into O; end;", n=60000, keys=64)
    assert m > 10


def test_sequence_two_states_strict_contiguity():
    m = case(P3 + "from every s1=A[id < 25], s2=B[id >= 25] "
             "select s1.id as i1, s2.id as i2, s2.ts as t insert into O; end;")
    assert m > 100


def test_sequence_kleene_first_last_and_optional():
    m = case(P3 + "from every s1=A, s2=B[price > 0.2]+, s3=C? , s4=A[id > 40] within 5 sec "
             "select s1.id as a, s2.id as b0, s2[last].id as bl, s4.id as d "
             "insert into O; end;", n=40000, keys=32)
    assert m > 10


def test_three_state_pattern_with_captures():
    m = case(P3 + "from every s1=A[price > 0.5] -> s2=B[id == s1.id % 7] -> s3=C[price < s1.price] "
             "within 3 sec select s1.k as k, s1.id as i1, s2.id as i2, s3.price as p3 "
             "insert into O; end;", n=30000, keys=128)
    assert m > 50


def test_non_every_three_state_pattern_unpartitioned():
    m = case("from s1=A[id == 3] -> s2=B[id == 4] -> s3=C[id == 5] "
             "select s1.ts as t1, s2.ts as t2, s3.ts as t3 insert into O;", n=20000, keys=16)
    assert m == 1


def test_sequence_multi_chunk_multi_batch():
    m = case(P3 + "from every s1=A[price > 0.6], s2=B+, s3=C within 2 sec "
             "select s1.price as p1, s2[last].price as p2, s3.price as p3 insert into O; end;",
             n=40000, keys=512, batches=3, chunk_events=4096)
    assert m > 100


def _max_recent_starts(w, stream=0, within_ms=10000, cond=None):
    """Largest number of state-1 starts of one key inside one `within`
    span: a lower bound on that key's live partials when completions are
    rare (VERDICT r03 item 5 asks for >= 40)."""
    best = 0
    sel = w["stream"] == stream
    if cond is not None:
        sel &= cond
    for k in np.unique(w["k"]):
        ts = np.sort(w["ts"][sel & (w["k"] == k)])
        if len(ts):
            j = np.searchsorted(ts, ts - within_ms, side="left")
            best = max(best, int((np.arange(len(ts)) - j + 1).max()))
    return best


PLONG = (P3 + "from every s1=A[price > 0.1] -> s2=B[id % 4 == 0] -> s3=C[id % 211 == 0] within 10 sec "
         "select s1.k as k, s1.price as p1, s2.id as i2, s3.ts as t3 insert into O; end;")


@pytest.mark.parametrize("batches,chunk", [(1, 1 << 22), (4, 4096)])
def test_three_state_pattern_pending_lists_beyond_slots(batches, chunk):
    # 16 keys at 1 event/ms: every key keeps far more live partials than its
    # 16 inline slots; the rest live in the pending pool (nfa_key) across
    # windows, chunks and batches, and every match equals the oracle's
    w = three_streams(40000, 16)
    assert _max_recent_starts(w, cond=w["price"] > 0.1) >= 40
    plan = EV3 + PLONG
    want = oracle_run(plan, events(w)).get("O", [])
    got = run(plan, w, batches=batches, pending_slots=16, chunk_events=chunk)
    assert len(want) > 1000
    assert_same_rows(got, want, "3-state, long pending lists")


def test_three_state_pool_lists_survive_snapshot():
    w = three_streams(30000, 16)
    plan = EV3 + PLONG
    want = oracle_run(plan, events(w)).get("O", [])
    half = 17000
    rt = fs.SiddhiAppRuntime(plan, pending_slots=16, chunk_events=4096)
    rt.add_callback("O")
    rt.send("A", w["ts"][:half], [w["k"][:half], w["ts"][:half], w["id"][:half], w["price"][:half]],
            streams=w["stream"][:half])
    rt.flush()
    first = engine_rows(rt.collect("O"))
    snap = rt.snapshot()
    rt.shutdown()
    rt2 = fs.SiddhiAppRuntime(plan, pending_slots=16, chunk_events=4096)
    rt2.add_callback("O")
    rt2.restore(snap)
    rt2.send("A", w["ts"][half:], [w["k"][half:], w["ts"][half:], w["id"][half:], w["price"][half:]],
             streams=w["stream"][half:])
    rt2.flush()
    second = engine_rows(rt2.collect("O"))
    rt2.shutdown()
    assert_same_rows(first + second, want, "3-state snapshot with pool lists")


def test_short_lists_in_large_chunks_book_no_pool():
    # a key whose window holds more records than free
    # slots used to book 2 x (n + records) pool slots up front, so a large
    # chunk with few keys exhausted a small pool even though every list stays
    # within its inline slots.  Lists here stay short (each C completes the
    # advanced partials); 8 keys x ~37 k records per chunk would book ~600 k
    # slots against a pool of 2^12: the flush must succeed, rows bit-exact.
    plan = EV3 + (P3 + "from every s1=A[price > 0.5] -> s2=B -> s3=C within 1 sec "
                  "select s1.k as k, s1.price as p1, s2.id as i2, s3.ts as t3 insert into O; end;")
    w = three_streams(300000, 8)
    want = oracle_run(plan, events(w)).get("O", [])
    got = run(plan, w, pending_slots=16, chunk_events=1 << 22, pending_pool_log2=12)
    assert len(want) > 10000
    assert_same_rows(got, want, "short lists, large chunk, small pool")
