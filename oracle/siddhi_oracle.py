"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

Independent pure-Python restatement of the Siddhi 4.2.40 semantics that
flink-siddhi delegates to (`AbstractSiddhiOperator.java:130`
`inputStreamHandlers.get(streamId).send(timestamp, data)`), for the SiddhiQL
subset on the hot path: filters, projections, `every A -> B ... within`
patterns, sequences with count states, `partition with (...)`, and
`group by ... having` running aggregates.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import this module, and only as the checker.  The product path
(flink-siddhi_amd/, libcep.so) never imports or links anything under oracle/.

Parity pinning: Siddhi itself (Java, 3rd-party, not vendored)
cannot run in this image — no JDK, no jars.  The oracle is
pinned by the reference's own test fixtures:
  * SiddhiCEPITCase.java:332-357 (config-1 golden row, exact content),
  * SiddhiSyntaxTest.java:47-82 (order-preserving pass-through),
  * SiddhiExecutionPlanSchemaTest.java:47 (DDL string format),
  * SiddhiCEPITCase.java pass-through line counts (5/6/30).
Everything else (within boundary, multiple pendings, Kleene, aggregates,
div-by-zero) follows SURVEY.md Appendix A and is "parity unpinned"; each KAT in
tests/ names the App. A item it depends on.

This parser is written independently of the C++ front end in
flink-siddhi_amd/csrc so that a front-end bug is not shared with the checker.
"""
from __future__ import annotations

import math
import re
import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

# --------------------------------------------------------------------------
# Types (SiddhiTypeFactory.java:42-54 maps Java <-> Siddhi attribute types)
# --------------------------------------------------------------------------
INT, LONG, FLOAT, DOUBLE, BOOL, STRING, OBJECT = ("int", "long", "float",
                                                  "double", "bool", "string",
                                                  "object")
NUMERIC_RANK = {INT: 0, LONG: 1, FLOAT: 2, DOUBLE: 3}
TYPE_NAMES = {"int": INT, "long": LONG, "float": FLOAT, "double": DOUBLE,
              "bool": BOOL, "boolean": BOOL, "string": STRING,
              "object": OBJECT}


class SiddhiError(Exception):
    """Plan parse/validation error (SiddhiAppCreationException analogue)."""


def _wrap32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def _wrap64(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v & (1 << 63) else v


def _f32(x: float) -> float:
    try:
        return struct.unpack("<f", struct.pack("<f", x))[0]
    except OverflowError:
        return math.copysign(math.inf, x)


def _java_idiv(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _java_irem(a: int, b: int) -> int:
    return a - b * _java_idiv(a, b)


def _fdiv(a: float, b: float) -> float:
    if b == 0.0:
        if a != a or a == 0.0:
            return math.nan
        neg = (math.copysign(1.0, a) < 0) != (math.copysign(1.0, b) < 0)
        return -math.inf if neg else math.inf
    return a / b


def _fmod(a: float, b: float) -> float:
    if b == 0.0 or math.isinf(a) or a != a or b != b:
        return math.nan
    if math.isinf(b):
        return a
    return math.fmod(a, b)


def java_double_str(d: float) -> str:
    """Double.toString for the Map/Row text form (StreamOutputHandler.java:103-109).

    Shortest round-trip digits (Python repr), laid out with Java's rules:
    plain decimal for 1e-3 <= |d| < 1e7, otherwise d.dddE<exp>.
    """
    from decimal import Decimal
    if d != d:
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    sign = "-" if d < 0 else ""
    a = abs(d)
    t = Decimal(repr(a)).as_tuple()
    digits = "".join(map(str, t.digits)).lstrip("0")
    exp10 = t.exponent + len(t.digits) - 1 - (len(t.digits) - len(
        "".join(map(str, t.digits)).lstrip("0")))
    digits = digits.rstrip("0") or "0"
    if 1e-3 <= a < 1e7:
        if exp10 >= 0:
            ip = (digits[:exp10 + 1]).ljust(exp10 + 1, "0")
            fp = digits[exp10 + 1:] or "0"
            return sign + ip + "." + fp
        return sign + "0." + "0" * (-exp10 - 1) + digits
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(exp10)


def java_value_str(v: Any, t: str) -> str:
    if v is None:
        return "null"
    if t in (DOUBLE, FLOAT):
        return java_double_str(float(v))
    if t == BOOL:
        return "true" if v else "false"
    return str(v)


# --------------------------------------------------------------------------
# Lexer
# --------------------------------------------------------------------------
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*")
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[lLfFdD]?)
  | (?P<op>->|==|!=|<=|>=|<|>|\+|-|\*|/|%|\(|\)|\[|\]|,|;|=|\.|\#|:|@|\?)
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
""", re.X | re.S)

KEYWORDS = {"define", "stream", "from", "select", "insert", "into", "every",
            "within", "and", "or", "not", "as", "partition", "with", "of",
            "begin", "end", "group", "by", "having", "true", "false", "last",
            "all", "events", "current", "expired", "is", "null"}

TIME_UNITS = {
    "millisec": 1, "millisecond": 1, "milliseconds": 1, "millisecs": 1,
    "ms": 1, "sec": 1000, "secs": 1000, "second": 1000, "seconds": 1000,
    "min": 60000, "mins": 60000, "minute": 60000, "minutes": 60000,
    "hour": 3600000, "hours": 3600000, "day": 86400000, "days": 86400000,
    "week": 604800000, "weeks": 604800000,
    "month": 2630000000, "months": 2630000000,
    "year": 31556900000, "years": 31556900000,
}


@dataclass
class Tok:
    kind: str   # 'id' 'kw' 'num' 'str' 'op' 'eof'
    val: str
    pos: int


def tokenize(text: str) -> List[Tok]:
    out: List[Tok] = []
    i = 0
    while i < len(text):
        m = _TOKEN_RE.match(text, i)
        if not m:
            raise SiddhiError("unexpected character %r at %d" % (text[i], i))
        k = m.lastgroup
        v = m.group(k)
        if k == "id" and v.lower() in KEYWORDS:
            out.append(Tok("kw", v.lower(), i))
        elif k != "ws":
            out.append(Tok(k, v, i))
        i = m.end()
    out.append(Tok("eof", "", len(text)))
    return out


# --------------------------------------------------------------------------
# AST
# --------------------------------------------------------------------------
@dataclass
class Attr:
    name: str
    type: str


@dataclass
class StreamDef:
    id: str
    attrs: List[Attr]

    def index(self, name: str) -> int:
        for i, a in enumerate(self.attrs):
            if a.name == name:
                return i
        raise SiddhiError("attribute %s not in stream %s" % (name, self.id))


@dataclass
class Expr:
    kind: str                    # const attr bin not neg call
    op: str = ""
    args: List["Expr"] = field(default_factory=list)
    value: Any = None
    vtype: str = ""              # for const
    ref: Optional[str] = None    # stream ref / alias for attr
    idx: Any = None              # s1[0] / s1[last] index for count states
    name: str = ""               # attribute / function name
    # filled by binder:
    t: str = ""
    slot: Any = None


@dataclass
class PState:
    alias: Optional[str]
    stream: str
    cond: Optional[Expr]
    every: bool = False
    min_count: int = 1
    max_count: int = 1            # -1 = unbounded


@dataclass
class SelectItem:
    expr: Expr
    name: str


@dataclass
class Query:
    kind: str                    # 'single' | 'pattern' | 'sequence'
    stream: Optional[str] = None             # single
    alias: Optional[str] = None
    filters: List[Expr] = field(default_factory=list)
    states: List[PState] = field(default_factory=list)
    within: Optional[int] = None
    select: Optional[List[SelectItem]] = None   # None => select *
    group_by: List[Expr] = field(default_factory=list)
    having: Optional[Expr] = None
    out: str = ""
    partition: Optional[Dict[str, str]] = None  # stream -> key attr
    out_attrs: List[Attr] = field(default_factory=list)


@dataclass
class App:
    streams: Dict[str, StreamDef]
    queries: List[Query]
    out_streams: Dict[str, StreamDef]


class Parser:
    def __init__(self, text: str):
        self.toks = tokenize(text)
        self.i = 0

    # helpers
    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind: str, val: Optional[str] = None) -> Optional[Tok]:
        t = self.peek()
        if t.kind == kind and (val is None or t.val == val):
            self.i += 1
            return t
        return None

    def expect(self, kind: str, val: Optional[str] = None) -> Tok:
        t = self.accept(kind, val)
        if t is None:
            p = self.peek()
            raise SiddhiError("expected %s %s at %d, got %r" %
                              (kind, val or "", p.pos, p.val))
        return t

    def ident(self) -> str:
        t = self.peek()
        if t.kind == "id":
            self.i += 1
            return t.val
        raise SiddhiError("expected identifier at %d, got %r" % (t.pos, t.val))

    # app
    def parse_app(self):
        streams: Dict[str, StreamDef] = {}
        queries: List[Query] = []
        while self.peek().kind != "eof":
            if self.accept("op", ";"):
                continue
            while self.peek().kind == "op" and self.peek().val == "@":
                self._skip_annotation()
            t = self.peek()
            if t.kind == "kw" and t.val == "define":
                sd = self.parse_define()
                if sd.id in streams:
                    raise SiddhiError("duplicate stream " + sd.id)
                streams[sd.id] = sd
            elif t.kind == "kw" and t.val == "from":
                queries.append(self.parse_query())
            elif t.kind == "kw" and t.val == "partition":
                queries.extend(self.parse_partition())
            else:
                raise SiddhiError("unexpected %r at %d" % (t.val, t.pos))
        return streams, queries

    def _skip_annotation(self):
        self.expect("op", "@")
        self.ident()
        if self.accept("op", ":"):
            self.ident()
        if self.accept("op", "("):
            depth = 1
            while depth:
                t = self.next()
                if t.kind == "eof":
                    raise SiddhiError("unterminated annotation")
                if t.kind == "op" and t.val == "(":
                    depth += 1
                elif t.kind == "op" and t.val == ")":
                    depth -= 1

    def parse_define(self) -> StreamDef:
        self.expect("kw", "define")
        self.expect("kw", "stream")
        sid = self.ident()
        self.expect("op", "(")
        attrs = []
        while True:
            name = self.ident() if self.peek().kind == "id" else self.next().val
            tt = self.next()
            tname = tt.val.lower()
            if tname not in TYPE_NAMES:
                raise SiddhiError("unknown type " + tt.val)
            attrs.append(Attr(name, TYPE_NAMES[tname]))
            if self.accept("op", ")"):
                break
            self.expect("op", ",")
        return StreamDef(sid, attrs)

    def parse_partition(self) -> List[Query]:
        self.expect("kw", "partition")
        self.expect("kw", "with")
        self.expect("op", "(")
        keys: Dict[str, str] = {}
        while True:
            attr = self.ident()
            self.expect("kw", "of")
            sid = self.ident()
            keys[sid] = attr
            if self.accept("op", ")"):
                break
            self.expect("op", ",")
        self.expect("kw", "begin")
        qs = []
        while not self.accept("kw", "end"):
            if self.accept("op", ";"):
                continue
            q = self.parse_query()
            q.partition = dict(keys)
            qs.append(q)
        return qs

    def parse_query(self) -> Query:
        self.expect("kw", "from")
        q = self.parse_input()
        if self.accept("kw", "select"):
            if self.accept("op", "*"):
                q.select = None
            else:
                items = []
                while True:
                    e = self.parse_expr()
                    name = None
                    if self.accept("kw", "as"):
                        name = self.ident()
                    if name is None:
                        if e.kind == "attr":
                            name = e.name
                        else:
                            raise SiddhiError("select expression needs 'as'")
                    items.append(SelectItem(e, name))
                    if not self.accept("op", ","):
                        break
                q.select = items
        if self.accept("kw", "group"):
            self.expect("kw", "by")
            while True:
                q.group_by.append(self.parse_primary())
                if not self.accept("op", ","):
                    break
        if self.accept("kw", "having"):
            q.having = self.parse_expr()
        self.expect("kw", "insert")
        if self.peek().kind == "kw" and self.peek().val in ("all", "current",
                                                            "expired"):
            self.next()
            self.expect("kw", "events")
        self.expect("kw", "into")
        q.out = self.ident()
        return q

    def _is_state_elem(self) -> bool:
        # `every`? alias '=' stream  |  stream '[' ...
        j = 0
        if self.peek(j).kind == "kw" and self.peek(j).val == "every":
            return True
        return (self.peek(j).kind == "id" and self.peek(j + 1).kind == "op"
                and self.peek(j + 1).val == "=")

    def parse_input(self) -> Query:
        if not self._is_state_elem():
            sid = self.ident()
            q = Query(kind="single", stream=sid)
            while True:
                if self.accept("op", "["):
                    q.filters.append(self.parse_expr())
                    self.expect("op", "]")
                elif self.peek().kind == "op" and self.peek().val == "#":
                    raise SiddhiError("unsupported: stream handlers/windows")
                else:
                    break
            if self.accept("kw", "as"):
                q.alias = self.ident()
            if self.peek().kind == "kw" and self.peek().val in ("join",):
                raise SiddhiError("unsupported: join")
            if self.peek().kind == "id" and self.peek().val.lower() in (
                    "join", "left", "right", "full", "inner", "unidirectional"):
                raise SiddhiError("unsupported: join")
            return q
        states = [self.parse_state()]
        sep = None
        while True:
            t = self.peek()
            if t.kind == "op" and t.val in ("->", ","):
                if sep is None:
                    sep = t.val
                elif sep != t.val:
                    raise SiddhiError("mixing -> and , is unsupported")
                self.next()
                states.append(self.parse_state())
            else:
                break
        q = Query(kind="pattern" if sep in (None, "->") else "sequence",
                  states=states)
        if self.accept("kw", "within"):
            q.within = self.parse_time()
        for k, s in enumerate(states):
            if s.every and k != 0:
                raise SiddhiError("unsupported: every on a non-start state")
        return q

    def parse_time(self) -> int:
        total = 0
        got = False
        while self.peek().kind == "num":
            n = self.next().val.rstrip("lL")
            unit = self.ident() if self.peek().kind == "id" else None
            if unit is None or unit.lower() not in TIME_UNITS:
                raise SiddhiError("bad time unit %r" % unit)
            total += int(float(n) * TIME_UNITS[unit.lower()])
            got = True
        if not got:
            raise SiddhiError("expected time constant")
        return total

    def parse_state(self) -> PState:
        every = bool(self.accept("kw", "every"))
        alias = self.ident()
        self.expect("op", "=")
        sid = self.ident()
        cond = None
        if self.accept("op", "["):
            cond = self.parse_expr()
            self.expect("op", "]")
        st = PState(alias=alias, stream=sid, cond=cond, every=every)
        t = self.peek()
        if t.kind == "op" and t.val == "+":
            self.next()
            st.min_count, st.max_count = 1, -1
        elif t.kind == "op" and t.val == "*":
            self.next()
            st.min_count, st.max_count = 0, -1
        elif t.kind == "op" and t.val == "?":
            self.next()
            st.min_count, st.max_count = 0, 1
        elif t.kind == "op" and t.val == "<":
            self.next()
            lo = int(self.expect("num").val)
            hi = lo
            if self.accept("op", ":"):
                hi = -1
                if self.peek().kind == "num":
                    hi = int(self.next().val)
            self.expect("op", ">")
            st.min_count, st.max_count = lo, hi
        return st

    # expressions: or > and > not > compare > additive > multiplicative > unary
    def parse_expr(self) -> Expr:
        e = self.parse_and()
        while self.accept("kw", "or"):
            e = Expr("bin", op="or", args=[e, self.parse_and()])
        return e

    def parse_and(self) -> Expr:
        e = self.parse_not()
        while self.accept("kw", "and"):
            e = Expr("bin", op="and", args=[e, self.parse_not()])
        return e

    def parse_not(self) -> Expr:
        if self.accept("kw", "not"):
            return Expr("not", args=[self.parse_not()])
        return self.parse_cmp()

    def parse_cmp(self) -> Expr:
        e = self.parse_add()
        t = self.peek()
        if t.kind == "op" and t.val in ("==", "!=", "<", "<=", ">", ">="):
            self.next()
            e = Expr("bin", op=t.val, args=[e, self.parse_add()])
        return e

    def parse_add(self) -> Expr:
        e = self.parse_mul()
        while self.peek().kind == "op" and self.peek().val in ("+", "-"):
            op = self.next().val
            e = Expr("bin", op=op, args=[e, self.parse_mul()])
        return e

    def parse_mul(self) -> Expr:
        e = self.parse_unary()
        while self.peek().kind == "op" and self.peek().val in ("*", "/", "%"):
            op = self.next().val
            e = Expr("bin", op=op, args=[e, self.parse_unary()])
        return e

    def parse_unary(self) -> Expr:
        if self.accept("op", "-"):
            inner = self.parse_unary()
            if inner.kind == "const" and inner.vtype in NUMERIC_RANK:
                v = -inner.value
                if inner.vtype == INT:
                    v = _wrap32(v)
                elif inner.vtype == LONG:
                    v = _wrap64(v)
                return Expr("const", value=v, vtype=inner.vtype)
            return Expr("neg", args=[inner])
        return self.parse_primary()

    def parse_primary(self) -> Expr:
        t = self.peek()
        if self.accept("op", "("):
            e = self.parse_expr()
            self.expect("op", ")")
            return e
        if t.kind == "num":
            self.next()
            return _num_const(t.val)
        if t.kind == "str":
            self.next()
            s = t.val[1:-1].encode().decode("unicode_escape")
            return Expr("const", value=s, vtype=STRING)
        if t.kind == "kw" and t.val in ("true", "false"):
            self.next()
            return Expr("const", value=(t.val == "true"), vtype=BOOL)
        if t.kind == "id":
            name = self.next().val
            if self.accept("op", "("):
                args = []
                if not self.accept("op", ")"):
                    while True:
                        args.append(self.parse_expr())
                        if self.accept("op", ")"):
                            break
                        self.expect("op", ",")
                return Expr("call", name=name.lower(), args=args)
            if self.peek().kind == "op" and self.peek().val == ":":
                raise SiddhiError("unsupported: extension function " + name)
            idx = None
            if self.peek().kind == "op" and self.peek().val == "[":
                self.next()
                if self.accept("kw", "last"):
                    idx = "last"
                else:
                    idx = int(self.expect("num").val)
                self.expect("op", "]")
            if self.accept("op", "."):
                attr = self.ident() if self.peek().kind == "id" else self.next().val
                return Expr("attr", ref=name, idx=idx, name=attr)
            if idx is not None:
                raise SiddhiError("indexed reference needs an attribute")
            return Expr("attr", ref=None, name=name)
        raise SiddhiError("unexpected %r at %d" % (t.val, t.pos))


def _num_const(s: str) -> Expr:
    suf = s[-1].lower()
    if suf == "l":
        return Expr("const", value=_wrap64(int(s[:-1])), vtype=LONG)
    if suf == "f":
        return Expr("const", value=_f32(float(s[:-1])), vtype=FLOAT)
    if suf == "d":
        return Expr("const", value=float(s[:-1]), vtype=DOUBLE)
    if any(c in s for c in ".eE"):
        return Expr("const", value=float(s), vtype=DOUBLE)
    v = int(s)
    if v > 0x7FFFFFFF:
        raise SiddhiError("int literal out of range: " + s)
    return Expr("const", value=v, vtype=INT)


# --------------------------------------------------------------------------
# Binding / typing
# --------------------------------------------------------------------------
AGGS = {"sum", "count", "avg", "min", "max"}


def _arith_type(a: str, b: str) -> str:
    if a not in NUMERIC_RANK or b not in NUMERIC_RANK:
        raise SiddhiError("arithmetic on non-numeric types %s, %s" % (a, b))
    return a if NUMERIC_RANK[a] >= NUMERIC_RANK[b] else b


class Binder:
    """Resolves attribute references to slots and computes expression types.

    Slot forms: ('cur', attr_index) for the current event of a single-stream
    query; ('st', state_index, count_index, attr_index) for pattern states;
    ('out', out_index) for `having` over output attributes.
    """

    def __init__(self, app_streams: Dict[str, StreamDef], q: Query):
        self.streams = app_streams
        self.q = q

    def bind(self, e: Expr, ctx: str, cur_state: Optional[int] = None) -> str:
        if e.kind == "const":
            e.t = e.vtype
            return e.t
        if e.kind == "attr":
            e.slot, e.t = self._resolve(e, ctx, cur_state)
            return e.t
        if e.kind == "not":
            t = self.bind(e.args[0], ctx, cur_state)
            if t != BOOL:
                raise SiddhiError("not requires bool")
            e.t = BOOL
            return BOOL
        if e.kind == "neg":
            t = self.bind(e.args[0], ctx, cur_state)
            if t not in NUMERIC_RANK:
                raise SiddhiError("negation of non-numeric")
            e.t = t
            return t
        if e.kind == "bin":
            a = self.bind(e.args[0], ctx, cur_state)
            b = self.bind(e.args[1], ctx, cur_state)
            op = e.op
            if op in ("and", "or"):
                if a != BOOL or b != BOOL:
                    raise SiddhiError("%s requires bool operands" % op)
                e.t = BOOL
            elif op in ("==", "!="):
                if a in NUMERIC_RANK and b in NUMERIC_RANK:
                    pass
                elif a != b:
                    raise SiddhiError("cannot compare %s with %s" % (a, b))
                e.t = BOOL
            elif op in ("<", "<=", ">", ">="):
                if a not in NUMERIC_RANK or b not in NUMERIC_RANK:
                    raise SiddhiError("ordering compare on non-numeric")
                e.t = BOOL
            else:
                e.t = _arith_type(a, b)
            return e.t
        if e.kind == "call":
            if e.name not in AGGS:
                raise SiddhiError("unsupported function " + e.name)
            if ctx != "select":
                raise SiddhiError("aggregate outside select")
            if e.name == "count":
                if e.args:
                    self.bind(e.args[0], ctx, cur_state)
                e.t = LONG
                return LONG
            if len(e.args) != 1:
                raise SiddhiError(e.name + " takes one argument")
            t = self.bind(e.args[0], ctx, cur_state)
            if t not in NUMERIC_RANK:
                raise SiddhiError(e.name + " of non-numeric")
            if e.name == "sum":
                e.t = LONG if t in (INT, LONG) else DOUBLE
            elif e.name == "avg":
                e.t = DOUBLE
            else:
                e.t = t
            return e.t
        raise SiddhiError("bad expression")

    def _resolve(self, e: Expr, ctx: str, cur_state: Optional[int]):
        q = self.q
        if ctx == "having":
            for i, a in enumerate(q.out_attrs):
                if e.ref is None and a.name == e.name:
                    return ("out", i), a.type
            # fallthrough: Siddhi also allows input attributes in having
        if q.kind == "single":
            sd = self.streams[q.stream]
            if e.ref is not None and e.ref not in (q.stream, q.alias):
                raise SiddhiError("unknown stream reference " + e.ref)
            i = sd.index(e.name)
            return ("cur", i), sd.attrs[i].type
        # pattern / sequence
        if e.ref is None:
            if cur_state is None:
                raise SiddhiError("unqualified attribute %s in pattern select"
                                  % e.name)
            sd = self.streams[q.states[cur_state].stream]
            i = sd.index(e.name)
            return ("st", cur_state, "cur", i), sd.attrs[i].type
        for k, st in enumerate(q.states):
            if st.alias == e.ref:
                if cur_state is not None and k > cur_state:
                    raise SiddhiError("reference to later state " + e.ref)
                sd = self.streams[st.stream]
                i = sd.index(e.name)
                idx = e.idx
                if k == cur_state:
                    idx = "cur"
                elif idx is None:
                    idx = 0
                return ("st", k, idx, i), sd.attrs[i].type
        raise SiddhiError("unknown reference " + e.ref)


def parse_app(text: str) -> App:
    streams, queries = Parser(text).parse_app()
    out_streams: Dict[str, StreamDef] = {}
    for q in queries:
        if q.kind == "single":
            if q.stream not in streams:
                raise SiddhiError("undefined stream " + q.stream)
            b = Binder(streams, q)
            for f in q.filters:
                if b.bind(f, "filter") != BOOL:
                    raise SiddhiError("filter must be bool")
            if q.select is None:
                q.select = [SelectItem(Expr("attr", name=a.name), a.name)
                            for a in streams[q.stream].attrs]
        else:
            for st in q.states:
                if st.stream not in streams:
                    raise SiddhiError("undefined stream " + st.stream)
            b = Binder(streams, q)
            for k, st in enumerate(q.states):
                if st.cond is not None:
                    if b.bind(st.cond, "filter", cur_state=k) != BOOL:
                        raise SiddhiError("condition must be bool")
            if q.select is None:
                raise SiddhiError("pattern query needs a select clause")
        if q.partition is not None:
            used = ([q.stream] if q.kind == "single"
                    else [s.stream for s in q.states])
            for s in used:
                if s not in q.partition:
                    raise SiddhiError("stream %s not partitioned" % s)
                streams[s].index(q.partition[s])
        names = set()
        q.out_attrs = []
        for it in q.select:
            t = b.bind(it.expr, "select")
            if it.name in names:
                raise SiddhiError("duplicate output attribute " + it.name)
            names.add(it.name)
            q.out_attrs.append(Attr(it.name, t))
        for g in q.group_by:
            b.bind(g, "group")
        if q.having is not None:
            if b.bind(q.having, "having") != BOOL:
                raise SiddhiError("having must be bool")
        od = StreamDef(q.out, list(q.out_attrs))
        if q.out in streams:
            raise SiddhiError("insert into an input stream is unsupported")
        if q.out in out_streams:
            prev = out_streams[q.out]
            if [(a.name, a.type) for a in prev.attrs] != \
                    [(a.name, a.type) for a in od.attrs]:
                raise SiddhiError("incompatible output definitions for "
                                  + q.out)
        out_streams[q.out] = od
    return App(streams, queries, out_streams)


# --------------------------------------------------------------------------
# Evaluation (Java / Siddhi value semantics)
# --------------------------------------------------------------------------
def _convert(v, frm: str, to: str):
    if v is None or frm == to:
        return v
    if to == LONG:
        return int(v)
    if to == FLOAT:
        return _f32(float(v))
    if to == DOUBLE:
        return float(v)
    return v


def evaluate(e: Expr, env) -> Any:
    k = e.kind
    if k == "const":
        return e.value
    if k == "attr":
        return env(e.slot)
    if k == "not":
        v = evaluate(e.args[0], env)
        return not bool(v)
    if k == "neg":
        v = evaluate(e.args[0], env)
        if v is None:
            return None
        if e.t == INT:
            return _wrap32(-v)
        if e.t == LONG:
            return _wrap64(-v)
        return -v
    if k == "bin":
        op = e.op
        if op == "and":
            return bool(evaluate(e.args[0], env)) and bool(
                evaluate(e.args[1], env))
        if op == "or":
            return bool(evaluate(e.args[0], env)) or bool(
                evaluate(e.args[1], env))
        a = evaluate(e.args[0], env)
        b = evaluate(e.args[1], env)
        ta, tb = e.args[0].t, e.args[1].t
        if op in ("==", "!=", "<", "<=", ">", ">="):
            if a is None or b is None:
                return False
            if ta in NUMERIC_RANK and tb in NUMERIC_RANK:
                ct = _arith_type(ta, tb)
                a = _convert(a, ta, ct)
                b = _convert(b, tb, ct)
            if op == "==":
                return a == b
            if op == "!=":
                return a != b
            if op == "<":
                return a < b
            if op == "<=":
                return a <= b
            if op == ">":
                return a > b
            return a >= b
        if a is None or b is None:
            return None
        t = e.t
        a = _convert(a, ta, t)
        b = _convert(b, tb, t)
        if t in (INT, LONG):
            w = _wrap32 if t == INT else _wrap64
            if op == "+":
                return w(a + b)
            if op == "-":
                return w(a - b)
            if op == "*":
                return w(a * b)
            if b == 0:
                return None          # App. A.2: int div/mod by zero -> null
            if op == "/":
                return w(_java_idiv(a, b))
            return w(_java_irem(a, b))
        if op == "+":
            r = a + b
        elif op == "-":
            r = a - b
        elif op == "*":
            r = a * b
        elif op == "/":
            r = _fdiv(a, b)
        else:
            r = _fmod(a, b)
        return _f32(r) if t == FLOAT else r
    raise SiddhiError("cannot evaluate " + k)


# --------------------------------------------------------------------------
# Runtime
# --------------------------------------------------------------------------
@dataclass
class OutEvent:
    stream: str
    ts: int
    data: Tuple
    seq: int = -1      # input sequence number of the completing event


class _Agg:
    def __init__(self, name: str, t: str):
        self.name = name
        self.t = t
        self.n = 0
        self.s = 0 if t == LONG else 0.0
        self.m = None

    def add(self, v):
        if self.name == "count":
            self.n += 1
            return
        if v is None:
            return
        self.n += 1
        if self.name == "sum":
            self.s = _wrap64(self.s + v) if self.t == LONG else self.s + float(v)
        elif self.name == "avg":
            self.s += float(v)
        elif self.name == "min":
            self.m = v if self.m is None or v < self.m else self.m
        elif self.name == "max":
            self.m = v if self.m is None or v > self.m else self.m

    def value(self):
        if self.name == "count":
            return self.n
        if self.name == "sum":
            return self.s if self.n else None
        if self.name == "avg":
            return self.s / self.n if self.n else None
        return self.m


def _agg_walk(e: Expr, out: list):
    if e.kind == "call" and e.name in AGGS:
        out.append(e)
        return
    for a in e.args:
        _agg_walk(a, out)


class _Partial:
    __slots__ = ("j", "events", "count", "start_ts")

    def __init__(self, j, events, count, start_ts):
        self.j = j                 # state currently collecting / next to match
        self.events = events       # per state: list of (ts, row)
        self.count = count         # events collected at state j
        self.start_ts = start_ts


class _SingleInstance:
    def __init__(self, q: Query):
        self.q = q
        self.aggs: Dict[Tuple, List[_Agg]] = {}

    def on_event(self, ts, row, stream, seq, out):
        q = self.q
        if stream != q.stream:
            return
        env = lambda slot: row[slot[1]]  # noqa: E731
        for f in q.filters:
            if not evaluate(f, env):
                return
        aggs_in_select: List[Expr] = []
        for it in q.select:
            _agg_walk(it.expr, aggs_in_select)
        if aggs_in_select:
            gkey = tuple(evaluate(g, env) for g in q.group_by)
            st = self.aggs.get(gkey)
            if st is None:
                st = [_Agg(a.name, a.t) for a in aggs_in_select]
                self.aggs[gkey] = st
            for a, ae in zip(st, aggs_in_select):
                a.add(evaluate(ae.args[0], env) if ae.args else None)
            vals = {id(ae): a.value() for a, ae in zip(st, aggs_in_select)}

            def env2(slot):
                return row[slot[1]]

            data = tuple(_eval_with_aggs(it.expr, env2, vals)
                         for it in q.select)
        else:
            data = tuple(evaluate(it.expr, env) for it in q.select)
        if q.having is not None:
            def envh(slot):
                if slot[0] == "out":
                    return data[slot[1]]
                return row[slot[1]]
            if not evaluate(q.having, envh):
                return
        out.append(OutEvent(q.out, ts, data, seq))


def _eval_with_aggs(e: Expr, env, vals):
    if e.kind == "call" and e.name in AGGS:
        return vals[id(e)]
    if e.kind in ("const", "attr"):
        return evaluate(e, env)
    # rebuild evaluation with aggregate leaves substituted
    sub = Expr(e.kind, op=e.op, value=e.value, vtype=e.vtype, t=e.t,
               args=[Expr("const", value=_eval_with_aggs(a, env, vals),
                          vtype=a.t, t=a.t) for a in e.args])
    return evaluate(sub, env)


class _PatternInstance:
    """Pending partial matches of one pattern/sequence instance.

    Pattern (`->`) semantics, SURVEY.md App. A.3: partials advance in creation
    order; an event never advances a partial it created; `within` is checked
    against the start event when an event of the partial's awaited stream
    arrives (strict `>` expires); states after the start are not `every`, so a
    matched partial is consumed.  Sequence (`,`) semantics, App. A.5: every
    event on any of the sequence's streams that does not advance a partial
    discards it; count states collect consecutive matches.
    """

    def __init__(self, q: Query):
        self.q = q
        self.partials: List[_Partial] = []
        self.started = False
        self.streams = {s.stream for s in q.states}

    def _cond(self, k, ts, row, p: Optional[_Partial]):
        st = self.q.states[k]
        if st.cond is None:
            return True

        def env(slot):
            _, si, idx, ai = slot
            if si == k and idx == "cur":
                return row[ai]
            evs = p.events[si] if p is not None else []
            if not evs:
                return None
            if idx == "last":
                return evs[-1][1][ai]
            if idx == "cur":
                idx = 0
            if idx >= len(evs):
                return None
            return evs[idx][1][ai]
        return bool(evaluate(st.cond, env))

    def _emit(self, p: _Partial, ts, seq, out):
        q = self.q

        def env(slot):
            _, si, idx, ai = slot
            evs = p.events[si]
            if not evs:
                return None
            if idx == "last":
                return evs[-1][1][ai]
            if idx == "cur":
                idx = 0
            if idx >= len(evs):
                return None
            return evs[idx][1][ai]
        data = tuple(evaluate(it.expr, env) for it in q.select)
        if q.having is not None:
            def envh(slot):
                if slot[0] == "out":
                    return data[slot[1]]
                return env(slot)
            if not evaluate(q.having, envh):
                return
        out.append(OutEvent(q.out, ts, data, seq))

    def on_event(self, ts, row, stream, seq, out):
        if stream not in self.streams:
            return
        if self.q.kind == "pattern":
            self._pattern_event(ts, row, stream, seq, out)
        else:
            self._sequence_event(ts, row, stream, seq, out)

    # ---- patterns (->) --------------------------------------------------
    def _pattern_event(self, ts, row, stream, seq, out):
        q = self.q
        n = len(q.states)
        keep: List[_Partial] = []
        fresh: List[_Partial] = []
        for p in self.partials:
            st = q.states[p.j]
            if st.stream != stream:
                keep.append(p)
                continue
            if q.within is not None and abs(ts - p.start_ts) > q.within:
                continue                      # expired -> dropped
            if not self._cond(p.j, ts, row, p):
                keep.append(p)
                continue
            evs = [list(x) for x in p.events]
            evs[p.j].append((ts, row))
            if p.j + 1 == n:
                self._emit(_Partial(p.j + 1, evs, 0, p.start_ts), ts, seq, out)
            else:
                fresh.append(_Partial(p.j + 1, evs, 0, p.start_ts))
        s0 = q.states[0]
        if s0.stream == stream and (s0.every or not self.started):
            if self._cond(0, ts, row, None):
                self.started = True
                evs = [[] for _ in range(n)]
                evs[0].append((ts, row))
                if n == 1:
                    self._emit(_Partial(1, evs, 0, ts), ts, seq, out)
                else:
                    fresh.append(_Partial(1, evs, 0, ts))
        self.partials = keep + fresh

    # ---- sequences (,) ---------------------------------------------------
    def _sequence_event(self, ts, row, stream, seq, out):
        q = self.q
        n = len(q.states)
        survivors: List[_Partial] = []
        for p in self.partials:
            if q.within is not None and abs(ts - p.start_ts) > q.within:
                continue
            adv = self._seq_advance(p, ts, row, stream, seq, out)
            survivors.extend(adv)
        s0 = q.states[0]
        if s0.stream == stream and (s0.every or not self.started):
            if self._cond(0, ts, row, None):
                self.started = True
                evs = [[] for _ in range(n)]
                evs[0].append((ts, row))
                p = _Partial(0, evs, 1, ts)
                survivors.extend(self._settle(p, ts, seq, out))
        self.partials = survivors

    def _settle(self, p: _Partial, ts, seq, out) -> List[_Partial]:
        """State p.j has collected p.count events.  Emit when the count is
        satisfied and every later state is optional; a partial whose last
        state is a still-growing Kleene state stays to collect more."""
        q = self.q
        n = len(q.states)
        st = q.states[p.j]
        done = p.count >= st.min_count and all(
            q.states[k].min_count == 0 for k in range(p.j + 1, n))
        if not done:
            return [p]
        self._emit(p, ts, seq, out)
        if p.j == n - 1 and (st.max_count == -1 or p.count < st.max_count):
            return [p]
        return []

    def _seq_advance(self, p: _Partial, ts, row, stream, seq, out):
        q = self.q
        n = len(q.states)
        st = q.states[p.j]
        # option 1: stay in the current count state
        if st.stream == stream and (st.max_count == -1 or
                                    p.count < st.max_count):
            if self._cond(p.j, ts, row, p):
                evs = [list(x) for x in p.events]
                evs[p.j].append((ts, row))
                p2 = _Partial(p.j, evs, p.count + 1, p.start_ts)
                return self._settle(p2, ts, seq, out)
        # option 2: move to a later state (skipping optional ones)
        if p.count >= st.min_count:
            j = p.j + 1
            while j < n:
                sj = q.states[j]
                if sj.stream == stream and self._cond(j, ts, row, p):
                    evs = [list(x) for x in p.events]
                    evs[j].append((ts, row))
                    p2 = _Partial(j, evs, 1, p.start_ts)
                    return self._settle(p2, ts, seq, out)
                if sj.min_count > 0:
                    break
                j += 1
        return []          # strict contiguity: not advanced -> discarded


class OracleRuntime:
    """Siddhi-semantics runtime: send(stream, ts, row) -> list[OutEvent].

    Mirrors SiddhiAppRuntime.getInputHandler(id).send(ts, Object[]) plus a
    StreamCallback.  Partitioned queries keep one instance per
    partition-key value (Siddhi `partition with`).
    """

    def __init__(self, plan: str):
        self.app = parse_app(plan)
        self.instances: List[Dict[Any, Any]] = [dict() for _ in self.app.queries]
        self.seq = 0

    def stream_def(self, sid: str) -> StreamDef:
        if sid in self.app.streams:
            return self.app.streams[sid]
        if sid in self.app.out_streams:
            return self.app.out_streams[sid]
        raise SiddhiError("undefined stream " + sid)

    def send(self, stream: str, ts: int, row) -> List[OutEvent]:
        if stream not in self.app.streams:
            raise SiddhiError("undefined stream " + stream)
        row = tuple(row)
        out: List[OutEvent] = []
        seq = self.seq
        self.seq += 1
        for qi, q in enumerate(self.app.queries):
            if q.partition is not None:
                if stream not in q.partition:
                    continue
                kv = row[self.app.streams[stream].index(q.partition[stream])]
            else:
                kv = None
            inst = self.instances[qi].get(kv)
            if inst is None:
                inst = (_SingleInstance(q) if q.kind == "single"
                        else _PatternInstance(q))
                self.instances[qi][kv] = inst
            inst.on_event(ts, row, stream, seq, out)
        return out


def format_map(out_def: StreamDef, data: Tuple) -> str:
    """returnAsMap text form: TreeMap (keys sorted) -> '{a=1, b=x}'.

    StreamOutputHandler.java:103-109 builds a TreeMap; GenericRecord.getMap
    returns it and Flink writeAsText calls toString().
    """
    items = sorted(zip([a.name for a in out_def.attrs],
                       [a.type for a in out_def.attrs], data),
                   key=lambda x: x[0])
    return "{" + ", ".join("%s=%s" % (k, java_value_str(v, t))
                           for k, t, v in items) + "}"


def stream_definition_expression(stream_id: str,
                                 attrs: List[Tuple[str, str]]) -> str:
    """SiddhiStreamSchema.getStreamDefinitionExpression (SiddhiStreamSchema.java:63-71)."""
    return "define stream %s (%s);" % (
        stream_id, ",".join("%s %s" % (n, t) for n, t in attrs))
