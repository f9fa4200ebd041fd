"""The owner-wave walk (csrc/cf_walk.hip, k_cfwalk2), selected per process
with CEP_CF_WALK=2, against the oracle: one child process (the selection is
read once per process) running the closed-form path over several windows,
chunks and batches, with long pending lists (the overflow pool) included."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]

SCRIPT = r'''
import sys
sys.path[:0] = [r"%(root)s/flink-siddhi_amd", r"%(root)s/tests", r"%(root)s/oracle"]
import numpy as np
import flink_siddhi as fs
from flink_siddhi import _lib as L, workload
from helpers import assert_same_rows, engine_rows, oracle_run, workload_events

def case(plan, n, keys, batches, **opts):
    w = workload.generate(0, n, keys, rate=1)
    rt = fs.SiddhiAppRuntime(plan, **opts)
    rt.add_callback("O")
    cuts = np.linspace(0, n, batches + 1).astype(int)
    for b in range(batches):
        s, e = cuts[b], cuts[b + 1]
        rt.send("A", w["ts"][s:e], [w["k"][s:e], w["ts"][s:e], w["id"][s:e], w["price"][s:e]],
                streams=w["stream"][s:e])
    rt.flush()
    got = engine_rows(rt.collect("O"))
    assert rt.stats().kernel_launches[L.K_CF_WALK] > 0
    rt.shutdown()
    want = oracle_run(plan, workload_events(w)).get("O", [])
    assert_same_rows(got, want, plan)
    return len(want)

m = case(workload.PATTERN_PLAN, 40000, 2048, 3, chunk_events=8192)
assert m > 50
# g never holds for most partials: ~39 live partials per key at 16 slots
long_plan = workload.PATTERN_PLAN.replace("id %% 7 == 0", "id == 49")
case(long_plan, 30000, 64, 2, pending_slots=16)
print("walk2 ok", m)
'''


def test_owner_wave_walk_matches_oracle():
    env = dict(os.environ, CEP_CF_WALK="2")
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": str(ROOT)}], env=env, capture_output=True,
                       text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "walk2 ok" in r.stdout
