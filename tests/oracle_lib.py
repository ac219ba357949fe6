"""ctypes access to the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
this module; it is the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, Optional, Tuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
REF_HARNESS = os.path.join(ORACLE_DIR, "_ref", "ref_harness")

SEM_CPU, SEM_JIT = 0, 1
_DT = {np.dtype(np.int32): 0, np.dtype(np.int64): 1, np.dtype(np.float32): 2, np.dtype(np.float64): 3}


class _Col(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("dtype", ctypes.c_int32), ("data", ctypes.c_void_p)]


class _Table(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("n_cols", ctypes.c_int32), ("cols", ctypes.POINTER(_Col))]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
        _lib = ctypes.CDLL(LIB)
        P, E, S, I64, I32 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int32
        T = ctypes.POINTER(_Table)
        _lib.ora_lower.argtypes = [E, E, S, E, S]
        _lib.ora_split_where.argtypes = [E, E, S, E, S]
        _lib.ora_split_where.restype = None
        _lib.ora_project_filter.argtypes = [T, E, E, I32, P, P, P, P, E, S]
        _lib.ora_sum.argtypes = [T, E, E, I32, P, P, E, S]
        _lib.ora_group_sum.argtypes = [T, E, E, E, I32, I64, P, P, P, P, E, S]
        _lib.ora_stats.argtypes = [T, E, E, I32, P, P, P, P, E, S]
        _lib.ora_group_agg.argtypes = [T, E, E, E, I32, I64, P, P, P, P, P, P, E, S]
        _lib.ora_topk.argtypes = [T, E, E, E, I64, I32, I32, P, P, P, P, E, S]
        _lib.ora_scan_baseline.argtypes = [T, E, P, P]
        _lib.ora_scan_baseline.restype = I64
    return _lib


class OracleError(RuntimeError):
    pass


class HostTable:
    """Host columns (numpy) in the oracle's table layout."""

    def __init__(self, cols: Dict[str, np.ndarray]):
        self.arrays = {k: np.ascontiguousarray(v) for k, v in cols.items()}
        lens = {len(v) for v in self.arrays.values()}
        assert len(lens) <= 1, "ragged columns"
        self.n = lens.pop() if lens else 0
        self._names = [k.encode() for k in self.arrays]
        self._cols = (_Col * max(1, len(self.arrays)))()
        for i, (k, v) in enumerate(self.arrays.items()):
            self._cols[i] = _Col(self._names[i], _DT[v.dtype], v.ctypes.data)
        self.c = _Table(self.n, len(self.arrays), self._cols)


def _err():
    return ctypes.create_string_buffer(1024)


def _chk(rc, err):
    if rc != 0:
        raise OracleError(err.value.decode())


def lower(expr: str) -> str:
    out, err = ctypes.create_string_buffer(4096), _err()
    _chk(lib().ora_lower(expr.encode(), out, len(out), err, len(err)), err)
    return out.value.decode()


def split_where(query: str) -> Tuple[str, str]:
    e, c = ctypes.create_string_buffer(4096), ctypes.create_string_buffer(4096)
    lib().ora_split_where(query.encode(), e, len(e), c, len(c))
    return e.value.decode(), c.value.decode()


def project_filter(t: HostTable, expr: str, cond: Optional[str], sem: int = SEM_JIT):
    vals = np.empty(max(1, t.n), np.float32)
    idx = np.empty(max(1, t.n), np.int64)
    cnt = ctypes.c_int64(0)
    err = _err()
    _chk(lib().ora_project_filter(ctypes.byref(t.c), expr.encode(), cond.encode() if cond else None, sem,
                                  vals.ctypes.data, idx.ctypes.data, ctypes.addressof(cnt), None, err,
                                  len(err)), err)
    return vals[: cnt.value], idx[: cnt.value]


def dense(t: HostTable, expr: str, cond: Optional[str], fill: np.ndarray, sem: int = SEM_JIT) -> np.ndarray:
    out = fill.astype(np.float32).copy()
    cnt = ctypes.c_int64(0)
    err = _err()
    _chk(lib().ora_project_filter(ctypes.byref(t.c), expr.encode(), cond.encode() if cond else None, sem, None,
                                  None, ctypes.addressof(cnt), out.ctypes.data, err, len(err)), err)
    return out


def reduce_sum(t: HostTable, expr: str, cond: Optional[str], sem: int = SEM_JIT):
    s, c = ctypes.c_double(0), ctypes.c_int64(0)
    err = _err()
    _chk(lib().ora_sum(ctypes.byref(t.c), expr.encode(), cond.encode() if cond else None, sem,
                       ctypes.addressof(s), ctypes.addressof(c), err, len(err)), err)
    return s.value, c.value


def group_sum(t: HostTable, val_expr: str, key_expr: str, cond: Optional[str] = None, sem: int = SEM_JIT,
              capacity: int = 1 << 20):
    keys = np.empty(capacity, np.int32)
    sums = np.empty(capacity, np.float64)
    cnts = np.empty(capacity, np.int64)
    g = ctypes.c_int64(0)
    err = _err()
    _chk(lib().ora_group_sum(ctypes.byref(t.c), val_expr.encode(), key_expr.encode(),
                             cond.encode() if cond else None, sem, capacity, keys.ctypes.data, sums.ctypes.data,
                             cnts.ctypes.data, ctypes.addressof(g), err, len(err)), err)
    n = g.value
    return keys[:n], sums[:n], cnts[:n]


def stats(t: HostTable, expr: str, cond: Optional[str] = None, sem: int = SEM_JIT):
    s, c = ctypes.c_double(0), ctypes.c_int64(0)
    mn, mx = ctypes.c_float(0), ctypes.c_float(0)
    err = _err()
    _chk(lib().ora_stats(ctypes.byref(t.c), expr.encode(), cond.encode() if cond else None, sem,
                         ctypes.addressof(s), ctypes.addressof(c), ctypes.addressof(mn), ctypes.addressof(mx),
                         err, len(err)), err)
    return s.value, c.value, np.float32(mn.value), np.float32(mx.value)


def group_agg(t: HostTable, val_expr: str, key_expr: str, cond: Optional[str] = None, sem: int = SEM_JIT,
              capacity: int = 1 << 20):
    keys = np.empty(capacity, np.int32)
    sums = np.empty(capacity, np.float64)
    cnts = np.empty(capacity, np.int64)
    mins = np.empty(capacity, np.float32)
    maxs = np.empty(capacity, np.float32)
    g = ctypes.c_int64(0)
    err = _err()
    _chk(lib().ora_group_agg(ctypes.byref(t.c), val_expr.encode(), key_expr.encode(),
                             cond.encode() if cond else None, sem, capacity, keys.ctypes.data, sums.ctypes.data,
                             cnts.ctypes.data, mins.ctypes.data, maxs.ctypes.data, ctypes.addressof(g), err,
                             len(err)), err)
    n = g.value
    return keys[:n], sums[:n], cnts[:n], mins[:n], maxs[:n]


def topk(t: HostTable, order_expr: str, k: int, descending: bool = True, cond: Optional[str] = None,
         select_expr: Optional[str] = None, sem: int = SEM_JIT):
    keys = np.empty(k, np.float32)
    idx = np.empty(k, np.int64)
    vals = np.empty(k, np.float32)
    n = ctypes.c_int64(0)
    err = _err()
    _chk(lib().ora_topk(ctypes.byref(t.c), order_expr.encode(), cond.encode() if cond else None,
                        select_expr.encode() if select_expr else None, k, 1 if descending else 0, sem,
                        keys.ctypes.data, idx.ctypes.data, vals.ctypes.data, ctypes.addressof(n), err, len(err)),
         err)
    m = n.value
    return keys[:m], idx[:m], vals[:m]


def scan_baseline(t: HostTable, query: str) -> int:
    vals = np.empty(max(1, t.n), np.float32)
    idx = np.empty(max(1, t.n), np.int64)
    return int(lib().ora_scan_baseline(ctypes.byref(t.c), query.encode(), vals.ctypes.data, idx.ctypes.data))
