"""Regenerates config1_itcase.json: the input of SiddhiCEPITCase
testUnboundedPojoStreamSimplePatternMatch (SiddhiCEPITCase.java:332-357).

Two RandomEventSource(50) sources (RandomEventSource.java:56-66): id = n % 50,
name = "test_event", price = Random.nextDouble() (seeded here: it is not in
the output), ts = T0 + 1000 n for both sources, merged in event-time order as
AbstractSiddhiOperator.processWatermark drains its priority queue (ties:
inputStream1 first).  Expected output: the single golden line asserted at
SiddhiCEPITCase.java:354-356.
"""
import json
import random
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "oracle"))
from test_oracle_golden import ITCASE_GOLDEN, ITCASE_PLAN  # noqa: E402

T0 = 1_500_000_000_000
rnd = random.Random(42)
events = []
for n in range(50):
    for sid in ("inputStream1", "inputStream2"):
        ts = T0 + 1000 * n
        events.append([sid, ts, [n % 50, "test_event", rnd.random(), ts]])
out = {"plan": ITCASE_PLAN, "events": events, "expected": [ITCASE_GOLDEN],
       "source": "SiddhiCEPITCase.java:332-357"}
(Path(__file__).parent / "config1_itcase.json").write_text(json.dumps(out, indent=1))
