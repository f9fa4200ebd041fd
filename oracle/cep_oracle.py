"""ctypes wrapper of oracle/cep_oracle.c — TEST INFRASTRUCTURE ONLY.

Used by tests/ (large-size parity) and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

_LIB = Path(__file__).resolve().parent / "libcep_oracle.so"
OP = {"==": 0, "!=": 1, "<": 2, "<=": 3, ">": 4, ">=": 5}
COL = {"id": 0, "price": 1, "k": 2}


class Term(C.Structure):
    _fields_ = [("col", C.c_int32), ("mod", C.c_int32), ("op", C.c_int32), ("k", C.c_double)]


class Cond(C.Structure):
    _fields_ = [("nterms", C.c_int32), ("t", Term * 4)]


def cond(*terms) -> Cond:
    """terms: (col, mod, op, const), e.g. ("id", 7, "==", 0) for id % 7 == 0."""
    c = Cond()
    c.nterms = len(terms)
    for i, (col, mod, op, k) in enumerate(terms):
        c.t[i] = Term(COL[col], mod, OP[op], float(k))
    return c


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(str(_LIB))
        L.oracle_filter.restype = C.c_int64
        L.oracle_filter.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.POINTER(Cond), C.c_void_p]
        L.oracle_pattern_state.restype = C.c_void_p
        L.oracle_pattern_state.argtypes = [C.c_int64]
        L.oracle_pattern_state_free.argtypes = [C.c_void_p]
        L.oracle_pattern.restype = C.c_int64
        L.oracle_pattern.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(Cond),
                                     C.POINTER(Cond), C.c_int, C.c_int64, C.c_void_p,
                                     C.c_void_p, C.c_int64]
        _lib = L
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def filter_indices(idv, price, f: Cond) -> np.ndarray:
    idv = np.ascontiguousarray(idv, np.int32)
    price = np.ascontiguousarray(price, np.float64)
    sel = np.empty(len(idv), np.int64)
    m = lib().oracle_filter(len(idv), _p(idv), _p(price), C.byref(f), _p(sel))
    return sel[:m]


class PatternOracle:
    """Stateful keyed `[every] s1=A[f] -> s2=B[g] within W` (config 3 shape)."""

    def __init__(self, nkeys: int, f: Cond, g: Cond, every=True, within=-1):
        self.st = lib().oracle_pattern_state(nkeys)
        self.f, self.g, self.every, self.within = f, g, every, within
        self.idx = 0

    def __del__(self):
        if getattr(self, "st", None):
            lib().oracle_pattern_state_free(self.st)
            self.st = None

    def run(self, w: dict, out_cap=None):
        n = len(w["ts"])
        cap = n if out_cap is None else out_cap
        oa = np.empty(cap, np.int64)
        ob = np.empty(cap, np.int64)
        cols = [np.ascontiguousarray(w["k"], np.int32), np.ascontiguousarray(w["stream"], np.uint8),
                np.ascontiguousarray(w["id"], np.int32), np.ascontiguousarray(w["price"], np.float64),
                np.ascontiguousarray(w["ts"], np.int64)]
        m = lib().oracle_pattern(self.st, n, self.idx, *[_p(c) for c in cols], C.byref(self.f),
                                 C.byref(self.g), 1 if self.every else 0, self.within,
                                 _p(oa), _p(ob), cap)
        self.idx += n
        k = min(m, cap)
        return oa[:k], ob[:k], m
