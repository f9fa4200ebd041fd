"""Dynamic plans on the GPU: a control-event script (plans added, paused,
resumed, updated, removed, added mid-stream) replayed through one
`SiddhiOperator`, each plan's output compared row for row with the oracle fed
exactly the events that plan received (AbstractSiddhiOperator.onEventReceived
:400-467, AddRouteOperator.processElement :54-98; the scenario extends
SiddhiCEPITCase.testDynamicalStreamSimplePatternMatch :466-533, whose four
plans are p1-p4 here).  Routing keys vs Java hashCode semantics
(AddRouteOperator.java:83-92, HashPartitioner.java:24-26)."""
import math
import struct

import numpy as np
import pytest
import torch

import flink_siddhi as fs
from flink_siddhi.operator import MetadataControlEvent, OperationControlEvent, SiddhiOperator
from helpers import assert_same_rows, oracle_run

pytestmark = pytest.mark.gpu

SCHEMA = [("id", "int"), ("name", "string"), ("price", "double"), ("timestamp", "long")]
SCHEMAS = {"inputStream1": SCHEMA, "inputStream2": SCHEMA}
NAMES = ["nm%d" % i for i in range(6)]

PLANS = {
    "p1": "from inputStream1 select timestamp, id, name, price insert into outputStream1;",
    "p2": "from inputStream1 select id, timestamp, name, price group by id insert into outputStream2;",
    "p3": "from inputStream1 select name, timestamp, id, price group by name insert into outputStream3;",
    "p4": "from inputStream2 select timestamp, id, name, price group by name insert into outputStream4;",
    "p5": ("partition with (id of inputStream1, id of inputStream2) begin "
           "from every s1=inputStream1[price > 0.5] -> s2=inputStream2[price < 0.3] within 1 sec "
           "select s1.id as id, s1.price as p1, s2.price as p2, s2.timestamp as t "
           "insert into outputStream5; end;"),
    "p6": ("from inputStream1[price > 0.3] select name, sum(price) as total, count() as n "
           "group by name having total > 2.0 insert into outputStream6;"),
    "p7": "from inputStream2[name == 'nm3' or name == 'zz'] select id, name insert into outputStream7;",
}
P6_UPDATED = ("from inputStream1[price > 0.6] select name, sum(price) as total, count() as n "
              "group by name having total > 1.5 insert into outputStream6;")
P8 = "from inputStream2[id < 10] select id, price, name insert into outputStream8;"
OUTS = {"p1": "outputStream1", "p2": "outputStream2", "p3": "outputStream3", "p4": "outputStream4",
        "p5": "outputStream5", "p6": "outputStream6", "p7": "outputStream7", "p8": "outputStream8"}


def batch(rng, n, t0):
    ids = rng.integers(0, 50, n).astype(np.int32)
    names = rng.integers(0, len(NAMES), n)
    price = rng.random(n)
    ts = (t0 + np.cumsum(rng.integers(0, 4, n))).astype(np.int64)
    return ids, names, price, ts


class Script:
    """Drives the operator and records, per plan generation, the events it
    received, for the oracle."""

    def __init__(self, op):
        self.op = op
        self.gen = {}        # plan id -> [(plan text, [events])] (one entry per runtime)
        self.enabled = {}

    def add(self, pid, plan):
        self.op.on_event_received(MetadataControlEvent.builder().add_execution_plan(pid, plan).build())
        self.op.add_callback(pid, OUTS[pid])
        self.gen.setdefault(pid, []).append((plan, []))
        self.enabled[pid] = True

    def update(self, pid, plan):
        self.op.on_event_received(MetadataControlEvent.builder().update_execution_plan(pid, plan).build())
        self.gen[pid].append((plan, []))

    def remove(self, pid):
        self.op.on_event_received(MetadataControlEvent.builder().remove_execution_plan(pid).build())
        self.enabled.pop(pid)

    def able(self, pid, on):
        ev = OperationControlEvent.enable_query(pid) if on else OperationControlEvent.disable_query(pid)
        self.op.on_event_received(ev)
        self.enabled[pid] = on

    def send(self, sid, b, device):
        ids, names, price, ts = b
        nid = np.array([self.op.intern(NAMES[i]) for i in range(len(NAMES))], np.int32)[names]
        cols = [ids, nid, price, ts]
        if device:
            cols = [torch.from_numpy(c).cuda() for c in cols]
            reached = self.op.process(sid, cols[3], cols)
        else:
            reached = self.op.process(sid, ts, cols)
        rows = [(sid, int(ts[i]), (int(ids[i]), NAMES[names[i]], float(price[i]), int(ts[i])))
                for i in range(len(ts))]
        want = 0
        for pid, on in self.enabled.items():
            plan = self.gen[pid][-1][0]
            if on and sid in plan:
                self.gen[pid][-1][1].extend(rows)
                want += 1
        assert reached == want, (sid, reached, want)


def test_control_event_script_matches_oracle():
    rng = np.random.default_rng(11)
    op = SiddhiOperator(SCHEMAS)
    sc = Script(op)
    for pid in ("p1", "p2", "p3", "p4", "p5", "p6", "p7"):
        sc.add(pid, PLANS[pid])
    assert sorted(op.plan_ids()) == sorted(PLANS)
    t = 1_500_000_000_000
    for step in range(4):
        if step == 1:
            sc.able("p2", False)
        if step == 2:
            sc.able("p2", True)
            sc.update("p6", P6_UPDATED)
            sc.remove("p3")
        if step == 3:
            sc.add("p8", P8)
        b1 = batch(rng, 3000, t)
        b2 = batch(rng, 3000, int(b1[3][-1]))   # p5 reads both: non-decreasing time
        t = int(b2[3][-1])
        sc.send("inputStream1", b1, device=(step % 2 == 0))
        sc.send("inputStream2", b2, device=(step % 2 == 1))
    op.flush()
    total = 0
    for pid, gens in sc.gen.items():
        if pid == "p3":
            continue   # removed: its runtime (and rows) are gone, as in the reference
        want = []
        for plan, events in gens:
            want += oracle_run(op.enriched_plan(plan), events).get(OUTS[pid], [])
        out = op.collect(pid, OUTS[pid])
        defs = op.plan(pid).stream_definition(OUTS[pid])
        cols = []
        for (name, ty), c in zip(defs, out.cols):
            cols.append([op.lookup(int(v)) for v in c] if ty == fs._lib.STRING else c.tolist())
        got = [(int(out.ts[i]), int(out.seq[i]), tuple(c[i] for c in cols)) for i in range(len(out.ts))]
        assert_same_rows(got, want, pid)
        total += len(want)
        if pid in ("p1", "p4", "p5", "p6", "p7", "p8"):
            assert len(want) > 0, pid
    assert total > 10000
    op.shutdown()


def test_update_of_unknown_plan_and_duplicate_add_fail():
    op = SiddhiOperator(SCHEMAS)
    op.add_plan("a", PLANS["p1"])
    with pytest.raises(ValueError, match="already exists"):
        op.add_plan("a", PLANS["p1"])
    with pytest.raises(ValueError, match="does not exist"):
        op.update_plan("b", PLANS["p1"])
    with pytest.raises(fs.UndefinedStreamException):
        op.add_plan("c", "from nowhere select x insert into O;")
    op.remove_plan("zzz")   # unknown ids are ignored
    assert op.plan_ids() == ["a"]
    op.shutdown()


# ---------------------------------------------------------------- routing keys --
def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def java_hash(v, ty):
    if ty == "int":
        return _i32(v)
    if ty == "long":
        u = v & 0xFFFFFFFFFFFFFFFF
        return _i32(u ^ (u >> 32))
    if ty == "double":
        u = 0x7ff8000000000000 if math.isnan(v) else struct.unpack("<Q", struct.pack("<d", v))[0]
        return _i32(u ^ (u >> 32))
    if ty == "float":
        return _i32(0x7fc00000 if math.isnan(v) else struct.unpack("<I", struct.pack("<f", v))[0])
    if ty == "bool":
        return 1231 if v else 1237
    h = 0
    b = v.encode("utf-16-be")
    for i in range(0, len(b), 2):
        h = (h * 31 + ((b[i] << 8) | b[i + 1])) & 0xFFFFFFFF
    return _i32(h)


def test_partition_channels_follow_java_hashcode():
    plan = ("define stream S (i int, l long, d double, f float, b bool, s string);"
            "from S select i insert into O;")
    rt = fs.SiddhiAppRuntime(plan)
    strs = ["", "a", "abc", "Aa", "BB", "polygenelubricants", "été", "\U0001D11E clef", "nm3"]
    n = 4096
    rng = np.random.default_rng(5)
    iv = rng.integers(-2**31, 2**31, n).astype(np.int32)
    iv[:4] = [0, -1, -2**31, 2**31 - 1]
    lv = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    lv[:4] = [0, -1, -2**63, 1 << 32]
    dv = rng.standard_normal(n) * 1e6
    dv[:5] = [0.0, -0.0, float("nan"), float("inf"), 1.0]
    fv = (rng.standard_normal(n) * 1e3).astype(np.float32)
    fv[:3] = [0.0, float("nan"), -1.5]
    bv = (rng.random(n) < 0.5).astype(np.uint8)
    sid = np.array([rt.intern(s) for s in strs], np.int32)[rng.integers(0, len(strs), n)]
    ts = np.arange(n, dtype=np.int64)
    host = {"i": iv, "l": lv, "d": dv, "f": fv, "b": bv, "s": sid}
    cols = [torch.from_numpy(host[c]).cuda() for c in "ildfbs"]
    tsd = torch.from_numpy(ts).cuda()
    types = dict(zip("ildfbs", ["int", "long", "double", "float", "bool", "string"]))
    for nchan in (1, 3, 8):
        for f in "ildfbs":
            ch, keys = rt.partition_channels("S", tsd, cols, f, nchan, keys=True)
            torch.cuda.synchronize()
            vals = host[f].tolist()
            if f == "s":
                vals = [rt.lookup(v) for v in vals]
            elif f == "b":
                vals = [bool(v) for v in vals]
            want = np.array([abs(java_hash(v, types[f])) for v in vals], np.int64)
            np.testing.assert_array_equal(keys.cpu().numpy(), want, err_msg=f)
            np.testing.assert_array_equal(ch.cpu().numpy(), want % nchan, err_msg=f)
        # no group-by key: -1 and a channel in range; a key the stream lacks: 0
        ch, keys = rt.partition_channels("S", tsd, cols, None, nchan, seq0=7, keys=True)
        torch.cuda.synchronize()
        assert (keys.cpu().numpy() == -1).all()
        c = ch.cpu().numpy()
        assert c.min() >= 0 and c.max() < nchan
        if nchan == 8:
            assert len(set(c.tolist())) == 8
        ch, keys = rt.partition_channels("S", tsd, cols, "absent", nchan, keys=True)
        torch.cuda.synchronize()
        assert (keys.cpu().numpy() == 0).all() and (ch.cpu().numpy() == 0).all()
    assert java_hash("abc", "string") == 96354 and java_hash(1.0, "double") == 1072693248
    rt.shutdown()


def test_operator_route_uses_each_plans_last_partition_key():
    op = SiddhiOperator(SCHEMAS)
    for pid in ("p1", "p2", "p3", "p5"):
        op.add_plan(pid, PLANS[pid])
    rng = np.random.default_rng(3)
    ids, names, price, ts = batch(rng, 2000, 0)
    nid = np.array([op.intern(s) for s in NAMES], np.int32)[names]
    cols = [torch.from_numpy(c).cuda() for c in (ids, nid, price, ts)]
    r = op.route("inputStream1", cols[3], cols, 4, keys=True)
    torch.cuda.synchronize()
    assert sorted(r) == ["p1", "p2", "p3", "p5"]
    np.testing.assert_array_equal(r["p2"][1].cpu().numpy(), np.abs(ids.astype(np.int64)))
    want3 = np.array([abs(java_hash(NAMES[i], "string")) for i in names], np.int64)
    np.testing.assert_array_equal(r["p3"][1].cpu().numpy(), want3)
    np.testing.assert_array_equal(r["p3"][0].cpu().numpy(), want3 % 4)
    assert (r["p1"][1].cpu().numpy() == -1).all()
    op.enable("p2", False)
    assert "p2" not in op.route("inputStream1", cols[3], cols, 4)
    assert op.partition_keys("p2") == ["id"] and op.partition_keys("p5") == ["id", "id"]
    op.shutdown()


def test_route_plan_over_streams_with_different_group_by_attributes():
    # A plan reading two streams partitioned on differently named attributes:
    # the router's key list is the concatenation of every stream's group-by
    # list (AddRouteOperator.java:159-175), and each row takes the LAST key of
    # that list (:83-92 overwrites setPartitionKey per key).  A stream without
    # a field of that name sums no hashCode: partition key 0, channel 0.  An
    # update appends the new plan's keys to the old list (:166-171).
    schemas = {"s1": [("id", "int"), ("price", "double"), ("timestamp", "long")],
               "s2": [("uid", "int"), ("price", "double"), ("timestamp", "long")]}
    plan = ("partition with (id of s1, uid of s2) begin "
            "from every a=s1[price > 0.5] -> b=s2[price < 0.3] within 1 sec "
            "select a.id as id, b.uid as u insert into O; end;")
    op = SiddhiOperator(schemas)
    op.add_plan("px", plan)
    assert op.partition_keys("px") == ["id", "uid"]
    rng = np.random.default_rng(11)
    n = 3000
    ids = rng.integers(-1000, 1000, n).astype(np.int32)
    price = rng.random(n)
    ts = np.arange(n, dtype=np.int64)
    cols = [torch.from_numpy(c).cuda() for c in (ids, price, ts)]
    r1 = op.route("s1", cols[2], cols, 5, keys=True)
    r2 = op.route("s2", cols[2], cols, 5, keys=True)
    torch.cuda.synchronize()
    assert (r1["px"][1].cpu().numpy() == 0).all() and (r1["px"][0].cpu().numpy() == 0).all()
    want = np.abs(ids.astype(np.int64))
    np.testing.assert_array_equal(r2["px"][1].cpu().numpy(), want)
    np.testing.assert_array_equal(r2["px"][0].cpu().numpy(), want % 5)
    # update to a plan keyed on price of s2 only: the list grows, the last key
    # is now s1's (id): s1 rows route by id, s2 rows (no id field) to key 0
    plan2 = ("partition with (uid of s2, id of s1) begin "
             "from every a=s2[price > 0.5] -> b=s1[price < 0.3] within 1 sec "
             "select a.uid as u, b.id as id insert into O; end;")
    op.update_plan("px", plan2)
    assert op.partition_keys("px") == ["id", "uid", "id", "uid"] or \
        op.partition_keys("px") == ["id", "uid", "uid", "id"]
    last = op.partition_keys("px")[-1]
    r1 = op.route("s1", cols[2], cols, 5, keys=True)
    r2 = op.route("s2", cols[2], cols, 5, keys=True)
    torch.cuda.synchronize()
    k1, k2 = r1["px"][1].cpu().numpy(), r2["px"][1].cpu().numpy()
    if last == "id":
        np.testing.assert_array_equal(k1, want)
        assert (k2 == 0).all()
    else:
        assert (k1 == 0).all()
        np.testing.assert_array_equal(k2, want)
    op.shutdown()
