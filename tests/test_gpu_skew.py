"""Skewed and sparse partition keys vs the C oracle (oracle/cep_oracle.c).

Zipf s = 1.1 over 2^20 keys (BASELINE.md §3's variant of config 3): the
hottest key carries ~9 % of the events, so its bucket's walk spans hundreds
of LDS windows, and runs of more than pending_slots A's between two of its
B's are routine — the tail of such a list lives in the pending pool.  Rows
and per-key order must equal the oracle's.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cep_oracle as CO  # noqa: E402
from flink_siddhi import workload  # noqa: E402
from test_gpu_geometry import CHUNK, F, G, assert_same_per_key, oracle_rows, run_engine  # noqa: E402


def zipf_case(n, keys, rate, within_plan="within 10 sec", within=10000):
    import torch
    table = workload.zipf_map(keys)
    tdev = torch.from_numpy(table).cuda()
    plan = workload.PATTERN_PLAN.replace("within 10 sec", within_plan)
    out, st = run_engine([n // 2, n - n // 2], keys=keys, rate=rate, plan=plan,
                         key_of=lambda k: tdev[k.long()])
    w = CO.generate(0, n, keys, rate=rate, threads=16)
    w["k"] = table[w["k"]]
    want = oracle_rows(w, keys, within=within)
    got = {c: v.cpu().numpy() for c, v in out.items()}
    assert_same_per_key(got, want)
    return len(want["k"]), w


def test_zipf_keys_config3():
    m, w = zipf_case(1 << 24, 1 << 20, 400)
    counts = np.bincount(w["k"], minlength=1 << 20)
    assert counts.max() > 0.05 * len(w["k"])      # a real heavy hitter
    assert m > 500_000


def test_zipf_keys_dense_rate_long_lists():
    # 64 ms of events per key per W at rate 20/ms: the hot keys keep long lists
    m, _ = zipf_case(1 << 22, 1 << 16, 20, within_plan="within 2 sec", within=2000)
    assert m > 100_000
