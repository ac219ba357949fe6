"""One process per GPU: row-sharded queries over torch.distributed (RCCL).

Each rank owns a contiguous shard of the table resident in its GPU's HBM
(rows [row_base, row_base + n) with the reference's ceil(N / devices)
partition, src/multi_gpu_utils.cpp:24-32) and runs the query locally through
the C ABI.  The exchanges are the ones the result needs, one collective each
(SURVEY.md 8(e)):

  compaction   all-gather of the per-shard passing counts (int64) -> global
               offsets (the reference concatenates shard results in device
               order)
  SUM          all-reduce of {sum, count} as two doubles (the count is exact
               below 2^53; WX_F_F64_COUNTS writes it that way)
  GROUP BY     ONE all-reduce of the exchange buffer: the dense key window
               (2048 sums, 2048 counts, 1 out-of-window group count) and one
               slot per shard holding its first 64 out-of-window groups, zero
               elsewhere, so the same SUM both reduces the window and gathers
               the slots; wx_group_combine_slots merges them on the device.
               Only when a shard had more out-of-window groups than its slot
               holds (every rank sees it in the same combined buffer) does an
               all-gather of every shard's fixed-size group list record
               follow, merged by wx_group_merge_lists on the device; with
               many keys (group_sum_lists) that all-gather is the exchange
  top-K        all-gather of one 520-byte wx_topk_record per shard (K keys,
               values, global rows, count), merged by wx_topk_merge on the
               device (better key, NaN last, then the smaller row)

With the "nccl" backend these run on RCCL over xGMI on device tensors; with
"gloo" (CPU tests, or several ranks sharing one GPU) the same code stages
through host tensors.  Without an initialised process group (one GPU, one
process) every exchange is the identity.  bench.py times exactly these
functions.

Test hook: WARPDB_EXCHANGE_ONE_RANK=1 runs the multi-rank exchanges even
with one rank, so a one-GPU box executes the RCCL collectives (a one-rank
communicator) and the exchange kernels end to end.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

GROUP_WINDOW_BINS = 2048
GROUP_EXCHANGE_DOUBLES = 2 * GROUP_WINDOW_BINS + 1


def shard_range(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """[begin, end) rows of `rank` under ceil(n / world) contiguous chunks."""
    chunk = (n_rows + world - 1) // world if world > 0 else n_rows
    b = min(n_rows, rank * chunk)
    return b, min(n_rows, b + chunk)


def exchange_one_rank() -> bool:
    """Test hook: the exchanges run even with one rank (WARPDB_EXCHANGE_ONE_RANK=1)."""
    return os.environ.get("WARPDB_EXCHANGE_ONE_RANK") == "1"


def _single(group=None) -> bool:
    """True when there is nothing to exchange (no process group, or one rank)."""
    if not (dist.is_available() and dist.is_initialized()):
        return True
    return dist.get_world_size(group) == 1 and not exchange_one_rank()


def _world(group=None) -> int:
    return 1 if not (dist.is_available() and dist.is_initialized()) else dist.get_world_size(group)


def _rank(group=None) -> int:
    return 0 if not (dist.is_available() and dist.is_initialized()) else dist.get_rank(group)


def _host_staged(group=None) -> bool:
    return not _single(group) and dist.get_backend(group) != "nccl"


def _dev(group=None) -> torch.device:
    if _host_staged(group) or (_single(group) and not torch.cuda.is_available()):
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


# ----------------------------------------------- the exchange's own stream
# One RCCL communicator per rank (include/warpcomm.h, libwarpdb) whose
# collectives are enqueued on the caller's current stream -- the stream the
# partials and merge kernels run on -- instead of torch.distributed's
# internal one (two cross-stream event waits per exchange, ~14 us of a
# 160-us C3-strong step, profiles/r04/c3_step_probe.txt).  Built once per
# process group by enable_stream_comm (a collective: ShardedQuery calls it on
# every rank); WARPDB_STREAM_COMM=0 keeps torch.distributed's collectives.
# process-group key -> (the group object, world size, rank, _warpcomm.Comm or
# None = torch.distributed's collectives).  The group object is held, so a
# later process group of the same name (torch reuses names, and the default
# group is always "WORLD") is a different object: the entry is then stale and
# dropped on lookup instead of handing out a communicator with other peers.
_COMMS = {}
_COMM_DT = {torch.float64: 3, torch.int64: 1, torch.float32: 2, torch.int32: 0}  # wx_dtype


def _gkey(group):
    """Registry key of a process group: its name (stable for the group's
    lifetime, unlike id(), which a new object may reuse)."""
    if group is None:
        return "WORLD"
    name = getattr(group, "group_name", None)
    return ("name", name) if name else ("id", id(group))


def _gobj(group):
    return dist.distributed_c10d._get_default_group() if group is None else group


def _entry(group):
    """The registry entry of `group` if it was built for this very process
    group (same object, size and rank); a stale entry is dropped.  Its
    communicator is not destroyed here: its peers may be gone, and a
    destroy could wait on them (release_stream_comms before
    dist.destroy_process_group is the clean path)."""
    key = _gkey(group)
    e = _COMMS.get(key)
    if e is None:
        return None
    g, n, r, _ = e
    if g is not _gobj(group) or n != dist.get_world_size(group) or r != dist.get_rank(group):
        del _COMMS[key]
        return None
    return e


def stream_comm(group=None):
    """This rank's own communicator for `group`, or None."""
    e = _entry(group)
    return e[3] if e else None


def enable_stream_comm(group=None) -> bool:
    """Collective over `group` (every rank calls it, once per group): build
    this rank's RCCL communicator on the device of the current stream.  Only
    when the exchanges would run on RCCL anyway (a device process group with
    something to exchange).  Ranks agree before and after the build, so
    either every rank uses its own communicator or none does (then the
    exchanges stay on torch.distributed, with a warning)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False  # no process group: nothing to exchange over
    key = _gkey(group)
    e = _entry(group)
    if e is not None:
        return e[3] is not None
    _COMMS[key] = (_gobj(group), dist.get_world_size(group), dist.get_rank(group), None)
    if _single(group) or _host_staged(group) or os.environ.get("WARPDB_STREAM_COMM", "1") == "0":
        return False
    from . import _warpcomm as wc

    def agree(ok: bool) -> bool:
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        return float(t.item()) == 1.0

    why = None
    cid = bytes(wc.ID_BYTES)
    try:
        wc.load()
        if dist.get_rank(group) == 0:
            cid = wc.unique_id()
    except Exception as e:  # noqa: BLE001 - reported below, every rank falls back together
        why = e
    if not agree(why is None):
        import warnings

        warnings.warn(f"own RCCL communicator unavailable ({why or 'on another rank'}): "
                      "exchanges use torch.distributed", RuntimeWarning)
        return False
    idt = torch.tensor(list(cid), dtype=torch.uint8, device="cuda")
    dist.broadcast(idt, src=0 if group is None else dist.get_global_rank(group, 0), group=group)
    comm = None
    try:
        comm = wc.Comm(bytes(idt.cpu().tolist()), dist.get_world_size(group), dist.get_rank(group),
                       torch.cuda.current_device())
    except Exception as e:  # noqa: BLE001
        why = e
    if not agree(comm is not None):
        if comm is not None:
            comm.close()
        import warnings

        warnings.warn(f"own RCCL communicator failed ({why or 'on another rank'}): exchanges use torch.distributed",
                      RuntimeWarning)
        return False
    _COMMS[key] = (_gobj(group), dist.get_world_size(group), dist.get_rank(group), comm)
    return True


def release_stream_comms() -> None:
    """Destroy the communicators enable_stream_comm built.  Call it before
    dist.destroy_process_group (the device work using them must be done); an
    entry left behind is never reused by a later process group (see _entry)."""
    for key, e in list(_COMMS.items()):
        if e[3] is not None:
            e[3].close()
    _COMMS.clear()


def _comm_op(op):
    from . import _warpcomm as wc

    return {dist.ReduceOp.SUM: wc.SUM, dist.ReduceOp.MAX: wc.MAX, dist.ReduceOp.MIN: wc.MIN}.get(op)


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    """In-place all-reduce of t wherever it lives (gloo stages a device tensor
    on the host; with this rank's own communicator, RCCL on the current stream)."""
    if _single(group):
        return t
    c = stream_comm(group)
    if c is not None and t.is_cuda and t.is_contiguous() and t.dtype in _COMM_DT and _comm_op(op) is not None:
        c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _COMM_DT[t.dtype], _comm_op(op),
                     torch.cuda.current_stream().cuda_stream)
        return t
    if _host_staged(group) and t.device.type != "cpu":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


def all_gather(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenation over ranks of equally sized tensors (one collective)."""
    if _single(group):
        return t.reshape(-1)
    world = dist.get_world_size(group)
    c = stream_comm(group)
    if c is not None and t.is_cuda:
        src = t.reshape(-1).contiguous()
        out = torch.empty(world * src.numel(), dtype=src.dtype, device=src.device)
        c.all_gather(src.data_ptr(), out.data_ptr(), src.numel() * src.element_size(),
                     torch.cuda.current_stream().cuda_stream)
        return out
    if _host_staged(group):
        parts = [torch.empty_like(t, device="cpu") for _ in range(world)]
        dist.all_gather(parts, t.cpu(), group=group)
        return torch.cat(parts).to(t.device)
    out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.reshape(-1), group=group)
    return out


# ------------------------------------------------------------- compaction
def exchange_counts_device(count: torch.Tensor, group=None) -> torch.Tensor:
    """All shards' passing counts (int64[world]) from this shard's count (int64[1])."""
    return all_gather(count.reshape(1).to(torch.int64), group)


def exchange_counts(local_count: int, group=None) -> Tuple[int, int, List[int]]:
    """Global offset of this shard's compacted rows, the total, and all counts."""
    rank = _rank(group)
    counts = exchange_counts_device(torch.tensor([local_count], dtype=torch.int64, device=_dev(group)),
                                    group).cpu().tolist()
    return sum(counts[:rank]), sum(counts), counts


# ------------------------------------------------------------------- SUM
def exchange_sum_device(out: torch.Tensor, group=None) -> torch.Tensor:
    """{sum, count} as float64[2] (WX_F_F64_COUNTS layout), summed in place."""
    return all_reduce_(out, group=group)


def allreduce_sum(local_sum: float, local_count: int, group=None) -> Tuple[float, int]:
    t = torch.tensor([local_sum, float(local_count)], dtype=torch.float64, device=_dev(group))
    exchange_sum_device(t, group)
    return float(t[0].item()), int(t[1].item())


# -------------------------------------------------------------- GROUP BY
def exchange_group_window(window: torch.Tensor, group=None) -> torch.Tensor:
    """Sum the shards' exchange windows (wx_group_partials layout) in place."""
    if window.numel() != GROUP_EXCHANGE_DOUBLES or window.dtype != torch.float64:
        raise ValueError("window must be float64[2 * 2048 + 1]")
    return all_reduce_(window, group=group)


GROUP_SLOT_MAX = 4096  # n_slots * slot_groups bound of wx_group_combine_slots


def group_slot_groups(world: int) -> int:
    """Out-of-window groups each shard's exchange slot carries (64, fewer
    above 64 ranks so that world * slot_groups stays <= 4096)."""
    return max(1, min(64, GROUP_SLOT_MAX // max(1, world)))


def group_slot_counts(exchange: torch.Tensor, world: int, slot_groups: int) -> List[int]:
    """Every shard's out-of-window group count from a combined exchange buffer
    (-1: that shard's general-key table overflowed)."""
    sl = 1 + 3 * slot_groups
    slots = exchange.reshape(-1)[GROUP_EXCHANGE_DOUBLES:GROUP_EXCHANGE_DOUBLES + world * sl]
    return [int(x) for x in slots.view(world, sl)[:, 0].tolist()]


def group_exchange_error(counts: List[int], capacity: int) -> Optional[str]:
    """The error every rank raises after the exchange, or None.  It depends
    only on the combined buffer, which is the same on every rank, so no rank
    raises alone while the others wait in the next collective."""
    for r, c in enumerate(counts):
        if c < 0:
            return f"shard {r}: general-key group table overflowed"
        if c > capacity:
            return f"shard {r}: {c} groups outside the key window exceed capacity {capacity}"
    return None


# ------------------------------------------------------------------ top-K
TOPK_MAX = 32
TOPK_RECORD_BYTES = TOPK_MAX * 16 + 8  # wx_topk_record (include/warpexec.h)


def topk_record_views(rec: torch.Tensor):
    """(keys f32[32], vals f32[32], rows i64[32], count i64[1]) views of one
    wx_topk_record held in a uint8 tensor of TOPK_RECORD_BYTES."""
    if rec.dtype != torch.uint8 or rec.numel() != TOPK_RECORD_BYTES:
        raise ValueError("a top-K record is uint8[520]")
    return (rec[0:128].view(torch.float32), rec[128:256].view(torch.float32), rec[256:512].view(torch.int64),
            rec[512:520].view(torch.int64))


def exchange_topk_records(rec: torch.Tensor, group=None) -> torch.Tensor:
    """Every shard's candidate record, concatenated in rank order: ONE
    all-gather of 520 bytes per shard (RCCL on device tensors)."""
    return all_gather(rec, group)


def merge_topk_device(rec: torch.Tensor, k: int, descending: bool, launch, out_k: torch.Tensor,
                      out_i: torch.Tensor, out_v: torch.Tensor, out_n: torch.Tensor, group=None):
    """Global top-K left in HBM with no host round trip: the all-gather of the
    shards' records, then wx_topk_merge (one HIP kernel: better key first, NaN
    last, ties by the smaller row).  Returns (keys, rows, vals, count)."""
    from . import _warpexec as wx

    if rec.device.type != "cuda":
        raise RuntimeError("merge_topk_device runs on the GPU (wx_topk_merge); no CPU path exists")
    allr = exchange_topk_records(rec, group)
    n_rec = allr.numel() // TOPK_RECORD_BYTES
    wx.topk_merge(allr.data_ptr(), n_rec, k, descending, launch, out_k.data_ptr(), out_i.data_ptr(),
                  out_v.data_ptr(), out_n.data_ptr())
    return out_k[:k], out_i[:k], out_v[:k], out_n


@dataclass
class Shard:
    """This rank's slice of a row-sharded table, resident on its GPU."""

    columns: dict  # name -> device tensor
    row_base: int
    n_rows: int

    def table(self):
        from . import _warpexec as wx

        return wx.Table.from_tensors(**self.columns)


class ShardedQuery:
    """Run the C-ABI operations on the local shard and exchange results.

    The *_device methods are asynchronous (results stay in HBM, on the
    current stream); the others return host values.  `flags` is OR-ed into
    every launch (e.g. WX_F_TIME for the bench)."""

    def __init__(self, shard: Shard, custom_src: Optional[str] = None, group=None, flags: int = 0):
        from . import _warpexec as wx

        self.wx = wx
        self.shard = shard
        self.group = group
        self.table = shard.table()
        self.world = _world(group)
        self.exchange = not _single(group)  # the multi-rank exchanges run
        dev = torch.cuda.current_device()
        stream = torch.cuda.current_stream().cuda_stream
        self.launch = wx.make_launch(device=dev, stream=stream, custom_src=custom_src, flags=flags)
        self.launch_sum = wx.make_launch(device=dev, stream=stream, custom_src=custom_src,
                                         flags=flags | wx.F_F64_COUNTS)
        self.launch_sync = wx.make_launch(device=dev, stream=stream, custom_src=custom_src, flags=flags | wx.F_SYNC)
        # secondary kernels (combines, finalizes) stay out of WX_F_TIME timing
        self.launch_aux = wx.make_launch(device=dev, stream=stream, custom_src=custom_src, flags=0)
        self._bufs = {}
        self._gbufs = {}  # capacity -> _group_bufs views
        self._grecs = {}  # capacity -> group list record and its views
        self._ex_pool = None  # exchange timing (time_exchanges): preallocated HIP events
        self._ex_next = 0
        # the exchanges' collectives: RCCL on this stream through the rank's
        # own communicator (a collective call: every rank builds its
        # ShardedQuery), else torch.distributed's
        self.stream_comm = self.exchange and enable_stream_comm(group)

    # --- exchange timing (bench) -------------------------------------------
    def time_exchanges(self, steps: int) -> None:
        """Record a HIP event pair around the exchange part (collective + the
        device merge after it) of the next `steps` multi-rank *_device calls,
        on the stream the launches use; read with exchange_ms()."""
        self._ex_pool = [torch.cuda.Event(enable_timing=True) for _ in range(2 * steps)]
        self._ex_next = 0

    def _ex_mark(self) -> None:
        if self._ex_pool is not None and self.exchange and self._ex_next < len(self._ex_pool):
            self._ex_pool[self._ex_next].record()
            self._ex_next += 1

    def exchange_ms(self) -> Optional[float]:
        """Average exchange time (ms) of the calls since time_exchanges; None
        when nothing was exchanged (one shard).  Synchronises."""
        pool, n = self._ex_pool, self._ex_next // 2
        self._ex_pool = None
        if not pool or n == 0:
            return None
        pool[2 * n - 1].synchronize()
        return sum(pool[2 * i].elapsed_time(pool[2 * i + 1]) for i in range(n)) / n

    def _buf(self, name: str, n: int, dtype) -> torch.Tensor:
        b = self._bufs.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            b = torch.empty(max(1, n), dtype=dtype, device="cuda")
            self._bufs[name] = b
        return b

    # --- compaction -------------------------------------------------------
    def compact_device(self, expr: str, cond: Optional[str], vals: torch.Tensor, idx: Optional[torch.Tensor],
                       idx_bytes: int, count: torch.Tensor) -> torch.Tensor:
        """Local ordered compaction (shard-global row ids with 8-byte indices)
        + the count all-gather; returns all shards' counts (device int64[world])."""
        self.wx.project_filter(self.table, expr, cond, self.launch, self.wx.MODE_COMPACT, vals.data_ptr(),
                               idx.data_ptr() if idx is not None else 0, idx_bytes,
                               self.shard.row_base if idx_bytes == 8 else 0, d_count=count.data_ptr())
        self._ex_mark()
        out = exchange_counts_device(count, self.group)
        self._ex_mark()
        return out

    def compact(self, expr: str, cond: Optional[str], idx_bytes: int = 8):
        n = self.shard.n_rows
        vals = torch.empty(max(1, n), dtype=torch.float32, device="cuda")
        idx = torch.empty(max(1, n), dtype=torch.int64 if idx_bytes == 8 else torch.int32, device="cuda")
        count = torch.zeros(1, dtype=torch.int64, device="cuda")
        counts = self.compact_device(expr, cond, vals, idx, idx_bytes, count).cpu().tolist()
        self.wx.check(self.launch)
        rank = _rank(self.group)
        c = counts[rank]
        return vals[:c], idx[:c], sum(counts[:rank]), sum(counts)

    # --- SUM --------------------------------------------------------------
    def sum_device(self, expr: str, cond: Optional[str], out: torch.Tensor) -> torch.Tensor:
        """out (float64[2]) <- global {SUM(expr), COUNT} over every shard."""
        self.wx.reduce_sum(self.table, expr, cond, self.launch_sum, d_out=out.data_ptr(), want_host=False)
        self._ex_mark()
        exchange_sum_device(out, self.group)
        self._ex_mark()
        return out

    def sum(self, expr: str, cond: Optional[str]) -> Tuple[float, int]:
        out = self._buf("sum", 2, torch.float64)[:2]
        self.sum_device(expr, cond, out)
        self.wx.check(self.launch)
        h = out.cpu()
        return float(h[0]), int(h[1])

    # --- GROUP BY ---------------------------------------------------------
    def _group_record(self, capacity: int):
        """This shard's group list record (wx_group_merge_lists layout) and
        its (keys, sums, counts, count) views."""
        got = self._grecs.get(capacity)
        if got is None:  # one record per capacity: cached views never outlive a reallocation
            nbytes, so, co = self.wx.group_list_layout(capacity)
            rec = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            got = (rec, rec[8:8 + 4 * capacity].view(torch.int32), rec[so:so + 8 * capacity].view(torch.float64),
                   rec[co:co + 8 * capacity].view(torch.int64), rec[0:8].view(torch.int64))
            self._grecs[capacity] = got
        return got

    def _group_bufs(self, capacity: int):
        """Exchange buffer and the out-of-window groups, written straight into
        this shard's list record (the many-key fallback gathers it as is).
        Built once per capacity: the views hold their storage, and a timed
        multi-rank step pays no tensor slicing on the host."""
        got = self._gbufs.get(capacity)
        if got is not None:
            return got
        wx = self.wx
        S = group_slot_groups(self.world)
        nd = wx.group_slots_doubles(self.world, S)
        _, xk, xs, xc, nx = self._group_record(capacity)
        got = (S, self._buf("gex", nd, torch.float64)[:nd], xk, xs, xc, nx, self._buf("gok", capacity, torch.int32),
               self._buf("gos", capacity, torch.float64), self._buf("goc", capacity, torch.int64),
               self._buf("gng", 1, torch.int64))
        self._gbufs[capacity] = got
        return got

    def group_sum_device(self, val_expr: str, key_expr: str, cond: Optional[str], key_lo: int = 0,
                         capacity: int = 1 << 16):
        """GROUP BY over every shard with no host synchronisation: per-shard
        partials written straight into the one-collective exchange layout
        (window + this shard's slot of out-of-window groups), ONE all-reduce,
        the final merge on the device (wx_group_combine_slots).  Returns
        (keys, sums, counts, n_groups) device tensors of `capacity` entries.
        n_groups reads GROUP_NEEDS_MERGE (-2) when some shard had more
        out-of-window groups than its slot holds -- the same value on every
        rank -- and group_sum then takes the variable-size merge; -1 when a
        shard's general-key table overflowed.  One shard: wx_group_sum alone."""
        wx = self.wx
        S, ex, xk, xs, xc, nx, ok, osm, oc, ng = self._group_bufs(capacity)
        if not self.exchange:  # one shard: the single-GPU kernel + finalize, nothing to exchange or read back
            wx.group_sum(self.table, val_expr, key_expr, cond, self.launch, key_lo, capacity, ok.data_ptr(),
                         osm.data_ptr(), oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            return ok, osm, oc, ng
        wx.group_partials_slots(self.table, val_expr, key_expr, cond, self.launch, key_lo, ex.data_ptr(), self.world,
                                _rank(self.group), S, capacity, xk.data_ptr(), xs.data_ptr(), xc.data_ptr(),
                                d_n_extra=nx.data_ptr())
        self._ex_mark()
        all_reduce_(ex, group=self.group)
        wx.group_combine_slots(ex.data_ptr(), self.world, S, key_lo, self.launch_aux, capacity, ok.data_ptr(),
                               osm.data_ptr(), oc.data_ptr(), d_n_groups=ng.data_ptr())
        self._ex_mark()
        return ok, osm, oc, ng

    def group_sum_lists_device(self, val_expr: str, key_expr: str, cond: Optional[str], capacity: int = 1 << 20):
        """GROUP BY with many distinct keys per shard: every shard's groups
        (wx_group_sum -- the range-partitioned kernels for a wide key range)
        written straight into its list record, ONE all-gather of the records,
        and wx_group_merge_lists on the device.  No window and no slots; the
        only host reads are the local key-range probe of wx_group_sum.
        Returns (keys, sums, counts, n_groups) device tensors of `capacity`
        entries; n_groups is -1 on every rank when some shard had more than
        `capacity` groups."""
        wx = self.wx
        rec, xk, xs, xc, nx = self._group_record(capacity)
        ok, osm, oc = (self._buf("gok", capacity, torch.int32), self._buf("gos", capacity, torch.float64),
                       self._buf("goc", capacity, torch.int64))
        ng = self._buf("gng", 1, torch.int64)
        wx.group_sum(self.table, val_expr, key_expr, cond, self.launch, 0, capacity, xk.data_ptr(), xs.data_ptr(),
                     xc.data_ptr(), d_n_groups=nx.data_ptr(), want_count=False)
        self._ex_mark()
        lists = all_gather(rec, self.group) if self.exchange else rec
        wx.group_merge_lists(lists.data_ptr(), self.world if self.exchange else 1, capacity, 0, 0, self.launch_aux,
                             capacity, ok.data_ptr(), osm.data_ptr(), oc.data_ptr(), d_n_groups=ng.data_ptr())
        self._ex_mark()
        return ok, osm, oc, ng

    def group_sum_lists(self, val_expr: str, key_expr: str, cond: Optional[str], capacity: int = 1 << 20):
        """group_sum_lists_device with the groups returned (ascending keys)."""
        ok, osm, oc, ng = self.group_sum_lists_device(val_expr, key_expr, cond, capacity)
        n = int(ng.item())
        try:
            self.wx.check(self.launch)
        except self.wx.WarpExecError:
            if n >= 0:
                raise
        if n < 0 or n > capacity:
            raise self.wx.WarpExecError(self.wx.WX_ERR_CAPACITY, f"groups exceed capacity {capacity} on some shard")
        return ok[:n].clone(), osm[:n].clone(), oc[:n].clone()

    def group_sum(self, val_expr: str, key_expr: str, cond: Optional[str], key_lo: int = 0,
                  capacity: int = 1 << 16):
        """GROUP BY over every shard as device tensors of the final groups.
        Every decision after the exchange is taken from the all-reduced
        buffer, which is identical on every rank, so the ranks raise or take
        the fallback merge together (never one rank alone)."""
        wx = self.wx
        ok, osm, oc, ng = self.group_sum_device(val_expr, key_expr, cond, key_lo, capacity)
        n = int(ng.item())  # synchronises
        if self.exchange:
            S, ex, xk, xs, xc, nx = self._group_bufs(capacity)[:6]
            counts = group_slot_counts(ex.cpu(), self.world, S)
            err = group_exchange_error(counts, capacity)
            if err is not None:
                try:
                    wx.check(self.launch)  # clear this shard's own flag (the same condition)
                except wx.WarpExecError:
                    pass
                raise wx.WarpExecError(wx.WX_ERR_CAPACITY, err)
            if n == wx.GROUP_NEEDS_MERGE:  # some shard's out-of-window groups outgrew its slot
                # every shard's whole out-of-window list (already in its record):
                # one all-gather, merged with the combined window on the device
                rec = self._group_record(capacity)[0]
                lists = all_gather(rec, self.group)
                # identical records on every rank: a capacity error is raised by all of them
                n = wx.group_merge_lists(lists.data_ptr(), self.world, capacity, ex.data_ptr(), key_lo,
                                         self.launch_aux, capacity, ok.data_ptr(), osm.data_ptr(), oc.data_ptr(),
                                         d_n_groups=ng.data_ptr(), want_count=True)
        self.wx.check(self.launch)
        if n > capacity or n < 0:
            raise self.wx.WarpExecError(self.wx.WX_ERR_CAPACITY, f"{n} groups exceed capacity {capacity}")
        return ok[:n].clone(), osm[:n].clone(), oc[:n].clone()

    # --- top-K ------------------------------------------------------------
    def topk_device(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int,
                    descending: bool):
        """This shard's top-K written straight into its wx_topk_record
        (keys, global rows, SELECT values, count), asynchronous; ties by
        ascending row index, NaN last.  Returns the record (uint8[520])."""
        rec = self._buf("trec", TOPK_RECORD_BYTES, torch.uint8)[:TOPK_RECORD_BYTES]
        rk, rv, ri, rn = topk_record_views(rec)
        self.wx.topk(self.table, order_expr, cond, select_expr, k, descending, self.launch, rk.data_ptr(),
                     ri.data_ptr(), rv.data_ptr(), row_base=self.shard.row_base, d_count=rn.data_ptr(),
                     want_count=False)
        return rec

    def topk_merged_device(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int,
                           descending: bool):
        """Global top-K left in HBM, no host synchronisation: this shard's
        record, one all-gather, wx_topk_merge.  Returns (keys, rows, vals, count)."""
        rec = self.topk_device(order_expr, cond, select_expr, k, descending)
        if not self.exchange:  # one shard's list is final (its count is already <= k)
            rk, rv, ri, rn = topk_record_views(rec)
            return rk[:k], ri[:k], rv[:k], rn
        self._ex_mark()
        out = merge_topk_device(rec, k, descending, self.launch_aux, self._buf("tmk", k, torch.float32),
                                self._buf("tmi", k, torch.int64), self._buf("tmv", k, torch.float32),
                                self._buf("tmn", 1, torch.int64), self.group)
        self._ex_mark()
        return out

    def topk_heads(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int,
                   descending: bool):
        """ORDER BY .. LIMIT k for any k (beyond the 32-candidate records):
        this shard's first k rows in ORDER BY order (wx_order_head, global
        rows, synchronous), ONE all-gather of the head records, wx_head_merge
        on the device (ties by ascending row).  Returns host tensors (keys,
        rows, vals) of the global head."""
        wx = self.wx
        nb = wx.head_record_bytes(k)
        rec = self._buf("hrec", nb, torch.uint8)[:nb]
        wx.order_head(self.table, order_expr, cond, select_expr, k, descending, self.launch_aux, rec.data_ptr(), k,
                      row_base=self.shard.row_base)
        allr = all_gather(rec, self.group) if self.exchange else rec
        ok, oi, ov = (self._buf("hk", k, torch.float32), self._buf("hi", k, torch.int64),
                      self._buf("hv", k, torch.float32))
        m = wx.head_merge(allr.data_ptr(), allr.numel() // nb, k, k, descending, self.launch_aux, ok.data_ptr(),
                          oi.data_ptr(), ov.data_ptr())
        self.wx.check(self.launch)
        return ok[:m].cpu(), oi[:m].cpu(), ov[:m].cpu()

    def topk(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int, descending: bool):
        """Global top-K as host tensors (topk_merged_device + one read-back;
        k > 32: topk_heads)."""
        if k > TOPK_MAX:
            return self.topk_heads(order_expr, cond, select_expr, k, descending)
        tk, ti, tv, tn = self.topk_merged_device(order_expr, cond, select_expr, k, descending)
        m = int(tn.reshape(-1)[0].item())  # synchronises
        self.wx.check(self.launch)
        return tk[:m].cpu(), ti[:m].cpu(), tv[:m].cpu()
