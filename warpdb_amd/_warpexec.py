"""ctypes binding of the C ABI in include/warpexec.h (libwarpexec.so).

This is the Python side of the drop-in boundary: every function here is a
thin call into the native library with raw device pointers.  Device memory
comes from torch tensors (``tensor.data_ptr()``) and the stream from
``torch.cuda.current_stream().cuda_stream``; torch is plumbing only.

The library is loaded from the package directory (built in-tree by
``make -C warpdb_amd``).  There is no fallback: if the library is missing,
``load()`` raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libwarpexec.so")

WX_OK = 0
WX_ERR_INVALID = 1
WX_ERR_COMPILE = 2
WX_ERR_DEVICE = 3
WX_ERR_CAPACITY = 4
WX_ERR_UNSUPPORTED = 5
WX_ERR_INTERNAL = 6

INT32, INT64, FLOAT32, FLOAT64, STRING = 0, 1, 2, 3, 4

F_SYNC = 1
F_NO_CUSTOM = 2
F_TIME = 4
F_F64_COUNTS = 8  # reduce_sum: count written as a double (one f64 all-reduce combines shards)
F_ROW_ORDER = 16  # group_sum / group_agg: sums folded in row order (bit-identical to the reference's fold)

GROUP_WINDOW_BINS = 2048
GROUP_EXCHANGE_DOUBLES = 2 * GROUP_WINDOW_BINS + 1  # [sums | counts as f64 | out-of-window groups]
GROUP_EXCHANGE_MAX_SLOTS = 1024
GROUP_SLOT_MAX = 4096  # n_slots * slot_groups bound
GROUP_NEEDS_MERGE = -2  # wx_group_combine_slots: some shard's out-of-window groups did not fit its slot
TOPK_MAX = 32
TOPK_RECORD_BYTES = TOPK_MAX * 16 + 8  # wx_topk_record: keys f32[32] | vals f32[32] | rows i64[32] | count i64
TOPK_MERGE_MAX = 4096  # n_records * k bound


def group_slots_doubles(n_slots: int, slot_groups: int) -> int:
    """WX_GROUP_SLOTS_DOUBLES: the one-collective GROUP BY exchange buffer."""
    return GROUP_EXCHANGE_DOUBLES + n_slots * (1 + 3 * slot_groups)


def group_list_layout(cap: int):
    """WX_GROUP_LIST_*: (record bytes, sums offset, counts offset) of one
    shard's group list record (int64 count | int32 keys[cap] padded to 8 B |
    f64 sums[cap] | int64 counts[cap])."""
    sums_off = 8 + 8 * ((cap + 1) // 2)
    counts_off = sums_off + 8 * cap
    return counts_off + 8 * cap, sums_off, counts_off

MODE_DENSE = 0
MODE_DENSE_FILL = 1
MODE_COMPACT = 2

OP_DENSE, OP_COMPACT, OP_SUM, OP_GROUP, OP_TOPK, OP_UTIL = 0, 1, 2, 3, 4, 5

EXPORTED_SYMBOLS = (
    "wx_project_filter",
    "wx_reduce_sum",
    "wx_reduce_stats",
    "wx_group_sum",
    "wx_group_agg",
    "wx_group_partials",
    "wx_group_combine",
    "wx_group_partials_slots",
    "wx_group_combine_slots",
    "wx_group_merge_lists",
    "wx_topk_merge",
    "wx_order_head",
    "wx_head_merge",
    "wx_cast",
    "wx_topk",
    "wx_sort_pairs",
    "wx_sort_float",
    "wx_sort_float_from",
    "wx_sort_by_key",
    "wx_sort_float_limit",
    "wx_sort_by_key_limit",
    "wx_fill_synthetic",
    "wx_prepare",
    "wx_check",
    "wx_timing_read",
    "wx_timing_read_device",
    "wx_cache_stats",
    "wx_shutdown",
    "wx_abi_version",
)


class WxCol(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("dtype", ctypes.c_int32), ("d_ptr", ctypes.c_void_p)]


class WxTable(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("n_cols", ctypes.c_int32), ("cols", ctypes.POINTER(WxCol))]


class WxStats(ctypes.Structure):
    _fields_ = [("sum", ctypes.c_double), ("count", ctypes.c_int64), ("min", ctypes.c_float),
                ("max", ctypes.c_float)]


class WxLaunch(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("stream", ctypes.c_void_p),
        ("custom_src", ctypes.c_char_p),
        ("flags", ctypes.c_uint32),
    ]


class WarpExecError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


_lib = None


def load() -> ctypes.CDLL:
    """Load libwarpexec.so (after torch, so both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(
            f"{LIB_PATH} is missing: build it with `make -C warpdb_amd` (no CPU fallback exists)"
        )
    try:  # share torch's libamdhip64/libhiprtc when torch is present
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    P, I32, I64, U64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
    S, E = ctypes.c_size_t, ctypes.c_char_p
    T, L = ctypes.POINTER(WxTable), ctypes.POINTER(WxLaunch)
    pI64, pD = ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)
    sig = {
        "wx_project_filter": [T, E, E, L, I32, P, P, I32, I64, P, pI64, E, S],
        "wx_reduce_sum": [T, E, E, L, P, pD, pI64, E, S],
        "wx_reduce_stats": [T, E, E, L, P, ctypes.POINTER(WxStats), E, S],
        "wx_group_sum": [T, E, E, E, L, I32, I64, P, P, P, P, pI64, E, S],
        "wx_group_agg": [T, E, E, E, L, I32, I64, P, P, P, P, P, P, pI64, E, S],
        "wx_group_partials": [T, E, E, E, L, I32, P, I64, P, P, P, P, pI64, E, S],
        "wx_group_combine": [P, I32, P, P, P, I64, L, I64, P, P, P, P, pI64, E, S],
        "wx_group_partials_slots": [T, E, E, E, L, I32, P, I32, I32, I32, I64, P, P, P, P, pI64, E, S],
        "wx_group_combine_slots": [P, I32, I32, I32, L, I64, P, P, P, P, pI64, E, S],
        "wx_topk_merge": [P, I32, I32, I32, L, P, P, P, P, pI64, E, S],
        "wx_order_head": [T, E, E, E, I64, I32, L, I64, P, I64, E, S],
        "wx_head_merge": [P, I32, I64, I64, I32, L, P, P, P, P, pI64, E, S],
        "wx_group_merge_lists": [P, I32, I64, P, I32, L, I64, P, P, P, P, pI64, E, S],
        "wx_cast": [P, I32, P, I32, I64, L, E, S],
        "wx_topk": [T, E, E, E, I32, I32, L, I64, P, P, P, P, pI64, E, S],
        "wx_sort_pairs": [P, P, I64, I32, L, E, S],
        "wx_sort_float": [P, I64, I32, L, E, S],
        "wx_sort_float_from": [P, P, I64, I32, L, E, S],
        "wx_sort_by_key": [P, P, I64, I32, L, E, S],
        "wx_sort_float_limit": [P, I64, I64, I32, L, E, S],
        "wx_sort_by_key_limit": [P, P, I64, I64, I32, L, E, S],
        "wx_fill_synthetic": [P, I32, I64, U64, I32, D, D, I64, L, E, S],
        "wx_prepare": [T, I32, E, E, E, I32, L, E, S, E, S],
        "wx_check": [L, E, S],
        "wx_timing_read": [pD, pI64, E, S],
        "wx_timing_read_device": [I32, pD, pI64, E, S],
    }
    for name, argtypes in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    lib.wx_cache_stats.argtypes = [pI64, pI64]
    lib.wx_cache_stats.restype = None
    lib.wx_shutdown.argtypes = []
    lib.wx_shutdown.restype = None
    lib.wx_abi_version.argtypes = []
    lib.wx_abi_version.restype = ctypes.c_int32
    _lib = lib
    return lib


def _enc(s: Optional[str]) -> Optional[bytes]:
    return None if s is None else s.encode()


def _check(status: int, err) -> None:
    if status != WX_OK:
        raise WarpExecError(status, err.value.decode(errors="replace"))


@dataclass
class Column:
    name: str
    dtype: int
    ptr: int  # device address


class Table:
    """A wx_table over caller-owned device columns (kept alive by `owners`)."""

    def __init__(self, n_rows: int, columns: Sequence[Column], owners: Sequence[object] = ()):
        self.n_rows = int(n_rows)
        self.columns = list(columns)
        self._owners = list(owners)
        self._names = [c.name.encode() for c in self.columns]
        self._cols = (WxCol * max(1, len(self.columns)))()
        for i, c in enumerate(self.columns):
            self._cols[i] = WxCol(self._names[i], c.dtype, c.ptr)
        self.c = WxTable(self.n_rows, len(self.columns), self._cols)

    @classmethod
    def from_tensors(cls, **cols) -> "Table":
        import torch

        dmap = {torch.int32: INT32, torch.int64: INT64, torch.float32: FLOAT32, torch.float64: FLOAT64}
        n = None
        out = []
        for name, t in cols.items():
            if n is None:
                n = t.numel()
            if t.numel() != n:
                raise ValueError("columns differ in length")
            if not t.is_contiguous():
                raise ValueError(f"column {name} is not contiguous")
            out.append(Column(name, dmap[t.dtype], t.data_ptr()))
        return cls(n or 0, out, owners=list(cols.values()))


def make_launch(device: int = 0, stream: int = 0, custom_src: Optional[str] = None, flags: int = 0) -> WxLaunch:
    L = WxLaunch(device, stream or None, _enc(custom_src), flags)
    L._keep = custom_src  # noqa: SLF001 - keep the bytes object alive
    return L


def _err():
    return ctypes.create_string_buffer(8192)


def project_filter(table: Table, expr: str, cond: Optional[str], launch: WxLaunch, mode: int,
                   out_vals: int = 0, out_idx: int = 0, idx_bytes: int = 8, row_base: int = 0,
                   d_count: int = 0, want_count: bool = False) -> Optional[int]:
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_project_filter(ctypes.byref(table.c), _enc(expr), _enc(cond), ctypes.byref(launch), mode,
                               out_vals or None, out_idx or None, idx_bytes, row_base, d_count or None,
                               ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def reduce_sum(table: Table, expr: str, cond: Optional[str], launch: WxLaunch, d_out: int = 0,
               want_host: bool = True):
    lib = load()
    err = _err()
    s, c = ctypes.c_double(0), ctypes.c_int64(0)
    st = lib.wx_reduce_sum(ctypes.byref(table.c), _enc(expr), _enc(cond), ctypes.byref(launch), d_out or None,
                           ctypes.byref(s) if want_host else None, ctypes.byref(c) if want_host else None,
                           err, len(err))
    _check(st, err)
    return (s.value, c.value) if want_host else None


def group_sum(table: Table, val_expr: str, key_expr: str, cond: Optional[str], launch: WxLaunch,
              key_window_lo: int, capacity: int, d_keys: int, d_sums: int, d_counts: int,
              d_n_groups: int = 0, want_count: bool = True) -> Optional[int]:
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_group_sum(ctypes.byref(table.c), _enc(val_expr), _enc(key_expr), _enc(cond),
                          ctypes.byref(launch), key_window_lo, capacity, d_keys or None, d_sums or None,
                          d_counts or None, d_n_groups or None, ctypes.byref(h) if want_count else None,
                          err, len(err))
    _check(st, err)
    return h.value if want_count else None


def reduce_stats(table: Table, expr: str, cond: Optional[str], launch: WxLaunch, d_out: int = 0,
                 want_host: bool = True):
    """(sum, count, min, max) of (float)expr WHERE cond; MIN / MAX skip NaN, NaN when empty."""
    lib = load()
    err = _err()
    h = WxStats()
    st = lib.wx_reduce_stats(ctypes.byref(table.c), _enc(expr), _enc(cond), ctypes.byref(launch), d_out or None,
                             ctypes.byref(h) if want_host else None, err, len(err))
    _check(st, err)
    return (h.sum, h.count, h.min, h.max) if want_host else None


def group_agg(table: Table, val_expr: str, key_expr: str, cond: Optional[str], launch: WxLaunch,
              key_window_lo: int, capacity: int, d_keys: int, d_sums: int, d_counts: int, d_mins: int = 0,
              d_maxs: int = 0, d_n_groups: int = 0, want_count: bool = True) -> Optional[int]:
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_group_agg(ctypes.byref(table.c), _enc(val_expr), _enc(key_expr), _enc(cond),
                          ctypes.byref(launch), key_window_lo, capacity, d_keys or None, d_sums or None,
                          d_counts or None, d_mins or None, d_maxs or None, d_n_groups or None,
                          ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def group_partials(table: Table, val_expr: str, key_expr: str, cond: Optional[str], launch: WxLaunch,
                   key_window_lo: int, d_window: int, capacity: int, d_keys: int, d_sums: int, d_counts: int,
                   d_n_extra: int = 0, want_count: bool = False) -> Optional[int]:
    """Per-shard GROUP BY partials in the exchange layout (include/warpexec.h)."""
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_group_partials(ctypes.byref(table.c), _enc(val_expr), _enc(key_expr), _enc(cond),
                               ctypes.byref(launch), key_window_lo, d_window, capacity, d_keys or None,
                               d_sums or None, d_counts or None, d_n_extra or None,
                               ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def group_combine(d_window: int, key_window_lo: int, d_x_keys: int, d_x_sums: int, d_x_counts: int, n_extra: int,
                  launch: WxLaunch, capacity: int, d_keys: int, d_sums: int, d_counts: int, d_n_groups: int = 0,
                  want_count: bool = False) -> Optional[int]:
    """Final groups from a combined exchange window + combined out-of-window groups."""
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_group_combine(d_window, key_window_lo, d_x_keys or None, d_x_sums or None, d_x_counts or None,
                              n_extra, ctypes.byref(launch), capacity, d_keys or None, d_sums or None,
                              d_counts or None, d_n_groups or None, ctypes.byref(h) if want_count else None,
                              err, len(err))
    _check(st, err)
    return h.value if want_count else None


def group_partials_slots(table: Table, val_expr: str, key_expr: str, cond: Optional[str], launch: WxLaunch,
                         key_window_lo: int, d_exchange: int, n_slots: int, slot: int, slot_groups: int,
                         capacity: int, d_keys: int, d_sums: int, d_counts: int, d_n_extra: int = 0,
                         want_count: bool = False) -> Optional[int]:
    """Per-shard GROUP BY partials in the one-collective exchange layout
    (window + this shard's slot, zeros in the others; include/warpexec.h)."""
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_group_partials_slots(ctypes.byref(table.c), _enc(val_expr), _enc(key_expr), _enc(cond),
                                     ctypes.byref(launch), key_window_lo, d_exchange, n_slots, slot, slot_groups,
                                     capacity, d_keys or None, d_sums or None, d_counts or None, d_n_extra or None,
                                     ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def group_combine_slots(d_exchange: int, n_slots: int, slot_groups: int, key_window_lo: int, launch: WxLaunch,
                        capacity: int, d_keys: int, d_sums: int, d_counts: int, d_n_groups: int = 0,
                        want_count: bool = False) -> Optional[int]:
    """Final groups from a combined one-collective exchange buffer; the count
    is GROUP_NEEDS_MERGE (-2) when a shard's slot overflowed, -1 when a
    shard's general-key table did."""
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_group_combine_slots(d_exchange, n_slots, slot_groups, key_window_lo, ctypes.byref(launch), capacity,
                                    d_keys or None, d_sums or None, d_counts or None, d_n_groups or None,
                                    ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def group_merge_lists(d_lists: int, n_lists: int, list_capacity: int, d_window: int, key_window_lo: int,
                      launch: WxLaunch, capacity: int, d_keys: int, d_sums: int, d_counts: int, d_n_groups: int = 0,
                      want_count: bool = False) -> Optional[int]:
    """Final groups from n_lists gathered group list records (device; see
    group_list_layout), merged with the combined window d_window (0: none).
    The count is -1 when a list's count was negative or above list_capacity."""
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_group_merge_lists(d_lists or None, n_lists, list_capacity, d_window or None, key_window_lo,
                                  ctypes.byref(launch), capacity, d_keys or None, d_sums or None, d_counts or None,
                                  d_n_groups or None, ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def topk_merge(d_records: int, n_records: int, k: int, descending: bool, launch: WxLaunch, d_keys: int = 0,
               d_idx: int = 0, d_vals: int = 0, d_count: int = 0, want_count: bool = False) -> Optional[int]:
    """Global top-K from n_records wx_topk_record candidate records (device)."""
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_topk_merge(d_records or None, n_records, k, 1 if descending else 0, ctypes.byref(launch),
                           d_keys or None, d_idx or None, d_vals or None, d_count or None,
                           ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def head_record_bytes(cap: int) -> int:
    """WX_HEAD_RECORD_BYTES: count i64 | keys f32[cap] | vals f32[cap] | rows i64[cap]."""
    return 8 + 16 * cap


def order_head(table: Table, order_expr: str, cond: Optional[str], select_expr: Optional[str], limit: int,
               descending: bool, launch: WxLaunch, d_record: int, cap: int, row_base: int = 0) -> None:
    """This shard's ORDER BY .. LIMIT head of any length into a head record (synchronous)."""
    lib = load()
    err = _err()
    _check(lib.wx_order_head(ctypes.byref(table.c), _enc(order_expr), _enc(cond), _enc(select_expr), limit,
                             1 if descending else 0, ctypes.byref(launch), row_base, d_record or None, cap, err,
                             len(err)), err)


def head_merge(d_records: int, n_records: int, cap: int, limit: int, descending: bool, launch: WxLaunch,
               d_keys: int = 0, d_rows: int = 0, d_vals: int = 0, d_count: int = 0) -> int:
    """The global head of n_records head records (device); returns its length."""
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    _check(lib.wx_head_merge(d_records or None, n_records, cap, limit, 1 if descending else 0, ctypes.byref(launch),
                             d_keys or None, d_rows or None, d_vals or None, d_count or None, ctypes.byref(h), err,
                             len(err)), err)
    return h.value


def cast(d_src: int, src_dtype: int, d_dst: int, dst_dtype: int, n: int, launch: WxLaunch) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_cast(d_src or None, src_dtype, d_dst or None, dst_dtype, n, ctypes.byref(launch), err, len(err)),
           err)


def topk(table: Table, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int, descending: bool,
         launch: WxLaunch, d_keys: int = 0, d_idx: int = 0, d_vals: int = 0, row_base: int = 0,
         d_count: int = 0, want_count: bool = True) -> Optional[int]:
    lib = load()
    err = _err()
    h = ctypes.c_int64(-1)
    st = lib.wx_topk(ctypes.byref(table.c), _enc(order_expr), _enc(cond), _enc(select_expr), k,
                     1 if descending else 0, ctypes.byref(launch), row_base, d_keys or None, d_idx or None,
                     d_vals or None, d_count or None, ctypes.byref(h) if want_count else None, err, len(err))
    _check(st, err)
    return h.value if want_count else None


def sort_pairs(d_keys: int, d_vals: int, count: int, ascending: bool, launch: WxLaunch) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_sort_pairs(d_keys, d_vals, count, 1 if ascending else 0, ctypes.byref(launch), err, len(err)), err)


def sort_float(d_vals: int, count: int, ascending: bool, launch: WxLaunch) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_sort_float(d_vals, count, 1 if ascending else 0, ctypes.byref(launch), err, len(err)), err)


def sort_by_key(d_keys: int, d_vals: int, count: int, ascending: bool, launch: WxLaunch) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_sort_by_key(d_keys, d_vals, count, 1 if ascending else 0, ctypes.byref(launch), err, len(err)), err)


def sort_float_from(d_src: int, d_dst: int, count: int, ascending: bool, launch: WxLaunch) -> None:
    """Sorted copy of d_src's float keys into d_dst (d_src is not written)."""
    lib = load()
    err = _err()
    _check(lib.wx_sort_float_from(d_src, d_dst, count, 1 if ascending else 0, ctypes.byref(launch), err, len(err)),
           err)


def sort_float_limit(d_vals: int, count: int, limit: int, ascending: bool, launch: WxLaunch) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_sort_float_limit(d_vals, count, limit, 1 if ascending else 0, ctypes.byref(launch), err, len(err)),
           err)


def sort_by_key_limit(d_keys: int, d_vals: int, count: int, limit: int, ascending: bool, launch: WxLaunch) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_sort_by_key_limit(d_keys, d_vals, count, limit, 1 if ascending else 0, ctypes.byref(launch), err,
                                    len(err)), err)


def fill_synthetic(d_ptr: int, dtype: int, n: int, seed: int, kind: int, lo: float, hi: float,
                   launch: WxLaunch, row_base: int = 0) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_fill_synthetic(d_ptr, dtype, n, seed, kind, lo, hi, row_base, ctypes.byref(launch), err,
                                 len(err)), err)


def prepare(table: Optional[Table], op: int, expr: Optional[str] = None, cond: Optional[str] = None,
            aux: Optional[str] = None, k: int = 0, launch: Optional[WxLaunch] = None,
            want_source: bool = False) -> Optional[str]:
    lib = load()
    err = _err()
    src = ctypes.create_string_buffer(1 << 20) if want_source else None
    L = launch or make_launch()
    st = lib.wx_prepare(ctypes.byref(table.c) if table is not None else None, op, _enc(expr), _enc(cond),
                        _enc(aux), k, ctypes.byref(L), src, len(src) if src is not None else 0, err, len(err))
    _check(st, err)
    return src.value.decode() if want_source else None


def check(launch: WxLaunch) -> None:
    lib = load()
    err = _err()
    _check(lib.wx_check(ctypes.byref(launch), err, len(err)), err)


def timing_read(device: Optional[int] = None):
    """(total ms, launches) of the unread WX_F_TIME launches of the process
    (of `device` only, when given)."""
    lib = load()
    err = _err()
    ms, n = ctypes.c_double(0), ctypes.c_int64(0)
    if device is None:
        _check(lib.wx_timing_read(ctypes.byref(ms), ctypes.byref(n), err, len(err)), err)
    else:
        _check(lib.wx_timing_read_device(device, ctypes.byref(ms), ctypes.byref(n), err, len(err)), err)
    return ms.value, n.value


def cache_stats():
    lib = load()
    c, h = ctypes.c_int64(0), ctypes.c_int64(0)
    lib.wx_cache_stats(ctypes.byref(c), ctypes.byref(h))
    return c.value, h.value
