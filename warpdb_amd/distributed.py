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
  GROUP BY     all-reduce of the dense key window (2048 sums, 2048 counts,
               1 out-of-window group count: 4097 doubles); only when some
               shard saw keys outside the window, an all-gather merge of
               those groups follows
  top-K        all-gather of K packed candidates (key, value, row) + count
               per shard, merged by (key, row) -- on the host (merge_topk) or,
               without a host round trip, on the device (merge_topk_device)

With the "nccl" backend these run on RCCL over xGMI on device tensors; with
"gloo" (CPU tests, or several ranks sharing one GPU) the same code stages
through host tensors.  Without an initialised process group (one GPU, one
process) every exchange is the identity.  bench.py times exactly these
functions.
"""
from __future__ import annotations

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


def _single(group=None) -> bool:
    return not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1


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


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    """In-place all-reduce of t wherever it lives (gloo stages a device tensor on the host)."""
    if _single(group):
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


def _gather_padded(t: torch.Tensor, n: int, group=None) -> Tuple[torch.Tensor, List[int]]:
    """All-gather the first n entries of t from every rank (variable n)."""
    world = _world(group)
    dev = _dev(group)
    sizes = all_gather(torch.tensor([n], dtype=torch.int64, device=dev), group).cpu().tolist()
    m = max(1, max(sizes))
    buf = torch.zeros(m, dtype=t.dtype, device=dev)
    if n:
        buf[:n] = t[:n].to(dev)
    out = all_gather(buf, group)
    parts = [out[r * m: r * m + sizes[r]] for r in range(world)]
    return torch.cat(parts), sizes


def merge_groups(keys: torch.Tensor, sums: torch.Tensor, counts: torch.Tensor, n: int, group=None):
    """Combine per-shard (key, sum, count) groups by key; ascending keys, float64 sums.

    The fallback for keys outside the dense window (and the general merge)."""
    k, _ = _gather_padded(keys.to(torch.int64), n, group)
    s, _ = _gather_padded(sums.to(torch.float64), n, group)
    c, _ = _gather_padded(counts.to(torch.int64), n, group)
    uk, inv = torch.unique(k, sorted=True, return_inverse=True)
    ss = torch.zeros(uk.numel(), dtype=torch.float64, device=k.device).index_add_(0, inv, s)
    cc = torch.zeros(uk.numel(), dtype=torch.int64, device=k.device).index_add_(0, inv, c)
    return uk.to(torch.int32), ss, cc


# ------------------------------------------------------------------ top-K
def _f32_bits(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.float32).contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF


def exchange_topk(keys: torch.Tensor, idx: torch.Tensor, vals: torch.Tensor, n: int, k: int, group=None):
    """All shards' candidates from one all-gather: per shard an int64[2k + 1]
    record (count, then k x (key bits << 32 | value bits, row))."""
    dev = keys.device if not _host_staged(group) else torch.device("cpu")
    rec = torch.zeros(2 * k + 1, dtype=torch.int64, device=dev)
    rec[0] = n
    if n:
        kv = (_f32_bits(keys[:n]) << 32) | _f32_bits(vals[:n])
        rec[1: 1 + 2 * n: 2] = kv.to(dev)
        rec[2: 2 + 2 * n: 2] = idx[:n].to(torch.int64).to(dev)
    allr = all_gather(rec, group).cpu().view(-1, 2 * k + 1)
    ks, vs, rs = [], [], []
    for r in range(allr.shape[0]):
        m = int(allr[r, 0])
        body = allr[r, 1: 1 + 2 * m].view(-1, 2)
        kv = body[:, 0]
        ks.append(((kv >> 32) & 0xFFFFFFFF).to(torch.int32).view(torch.float32))
        vs.append((kv & 0xFFFFFFFF).to(torch.int32).view(torch.float32))
        rs.append(body[:, 1])
    return torch.cat(ks), torch.cat(rs), torch.cat(vs)


def merge_topk_candidates(gk: torch.Tensor, gi: torch.Tensor, gv: torch.Tensor, k: int, descending: bool):
    """Global top-K of gathered candidates; ties by ascending row index, NaN last."""
    order = torch.argsort(gi, stable=True)
    gk, gi, gv = gk[order], gi[order], gv[order]
    key = torch.where(torch.isnan(gk), torch.full_like(gk, float("inf") if not descending else -float("inf")), gk)
    order = torch.argsort(key, descending=descending, stable=True)
    nan_last = torch.isnan(gk[order])
    order = torch.cat([order[~nan_last], order[nan_last]])[:k]
    return gk[order], gi[order], gv[order]


def merge_topk(keys: torch.Tensor, idx: torch.Tensor, vals: torch.Tensor, n: int, k: int, descending: bool,
               group=None):
    """Global top-K from per-shard candidates (one all-gather, then the merge)."""
    gk, gi, gv = exchange_topk(keys, idx, vals, n, k, group)
    return merge_topk_candidates(gk, gi, gv, k, descending)


def merge_topk_device(keys: torch.Tensor, idx: torch.Tensor, vals: torch.Tensor, count: torch.Tensor, k: int,
                      descending: bool, group=None):
    """merge_topk without a host round trip: one all-gather of every shard's
    k candidate slots (unused slots masked by the shard's device-side count),
    then stable sorts on the device -- by row, by key, by class (number,
    NaN, unused slot) -- so ties keep the smallest row and NaN sorts last.
    Returns (keys, rows, vals) of k slots and the global count min(k, total),
    all on the device of `keys` (gloo stages through the host)."""
    dev = keys.device
    if _single(group):  # one shard's list is final (its count is already <= k)
        return keys[:k], idx[:k], vals[:k], count.reshape(1)
    rec = torch.zeros(2 * k + 1, dtype=torch.int64, device=dev)
    rec[0:1] = count.reshape(1).to(torch.int64)
    rec[1: 1 + 2 * k: 2] = (_f32_bits(keys[:k]) << 32) | _f32_bits(vals[:k])
    rec[2: 2 + 2 * k: 2] = idx[:k].to(torch.int64)
    allr = all_gather(rec, group).view(-1, 2 * k + 1)
    n = allr[:, 0:1]
    body = allr[:, 1:].reshape(-1, k, 2)
    kv, gi = body[:, :, 0].reshape(-1), body[:, :, 1].reshape(-1)
    gk = ((kv >> 32) & 0xFFFFFFFF).to(torch.int32).view(torch.float32)
    gv = (kv & 0xFFFFFFFF).to(torch.int32).view(torch.float32)
    used = (torch.arange(k, device=dev).reshape(1, k) < n).reshape(-1)
    cls = torch.where(used, torch.isnan(gk).to(torch.int64), torch.full_like(gi, 2))
    fill = float("-inf") if descending else float("inf")
    key = torch.where(cls == 0, gk, torch.full_like(gk, fill))
    order = torch.argsort(gi, stable=True)
    order = order[torch.argsort(key[order], descending=descending, stable=True)]
    order = order[torch.argsort(cls[order], stable=True)][:k]
    total = torch.clamp(n.sum().reshape(1), max=k)
    return gk[order], gi[order], gv[order], total


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
        dev = torch.cuda.current_device()
        stream = torch.cuda.current_stream().cuda_stream
        self.launch = wx.make_launch(device=dev, stream=stream, custom_src=custom_src, flags=flags)
        self.launch_sum = wx.make_launch(device=dev, stream=stream, custom_src=custom_src,
                                         flags=flags | wx.F_F64_COUNTS)
        self.launch_sync = wx.make_launch(device=dev, stream=stream, custom_src=custom_src, flags=flags | wx.F_SYNC)
        # secondary kernels (combines, finalizes) stay out of WX_F_TIME timing
        self.launch_aux = wx.make_launch(device=dev, stream=stream, custom_src=custom_src, flags=0)
        self._bufs = {}

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
        return exchange_counts_device(count, self.group)

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
        return exchange_sum_device(out, self.group)

    def sum(self, expr: str, cond: Optional[str]) -> Tuple[float, int]:
        out = self._buf("sum", 2, torch.float64)[:2]
        self.sum_device(expr, cond, out)
        self.wx.check(self.launch)
        h = out.cpu()
        return float(h[0]), int(h[1])

    # --- GROUP BY ---------------------------------------------------------
    def group_sum_device(self, val_expr: str, key_expr: str, cond: Optional[str], key_lo: int = 0,
                         capacity: int = 1 << 16):
        """GROUP BY over every shard: per-shard partials, ONE all-reduce of
        the 4097-double window, the final merge on the device.  Returns
        (keys, sums, counts, n_groups) device tensors of `capacity` entries;
        reads one double back to learn whether any shard saw keys outside
        the window (then their groups are all-gathered and merged).  With a
        single shard it is wx_group_sum alone (asynchronous)."""
        wx = self.wx
        window = self._buf("gwin", GROUP_EXCHANGE_DOUBLES, torch.float64)[:GROUP_EXCHANGE_DOUBLES]
        xk = self._buf("gxk", capacity, torch.int32)
        xs = self._buf("gxs", capacity, torch.float64)
        xc = self._buf("gxc", capacity, torch.int64)
        nx = self._buf("gnx", 1, torch.int64)
        ok = self._buf("gok", capacity, torch.int32)
        osm = self._buf("gos", capacity, torch.float64)
        oc = self._buf("goc", capacity, torch.int64)
        ng = self._buf("gng", 1, torch.int64)
        if self.world == 1:  # one shard: the single-GPU kernel + finalize, nothing to exchange or read back
            wx.group_sum(self.table, val_expr, key_expr, cond, self.launch, key_lo, capacity, ok.data_ptr(),
                         osm.data_ptr(), oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            return ok, osm, oc, ng
        wx.group_partials(self.table, val_expr, key_expr, cond, self.launch, key_lo, window.data_ptr(), capacity,
                          xk.data_ptr(), xs.data_ptr(), xc.data_ptr(), d_n_extra=nx.data_ptr())
        exchange_group_window(window, self.group)
        wx.group_combine(window.data_ptr(), key_lo, 0, 0, 0, 0, self.launch_aux, capacity, ok.data_ptr(),
                         osm.data_ptr(), oc.data_ptr(), d_n_groups=ng.data_ptr())
        if window[2 * GROUP_WINDOW_BINS].item() != 0.0:  # keys outside the window on some shard
            mk, ms, mc = merge_groups(xk, xs, xc, int(nx.item()), self.group)
            mk, ms, mc = mk.cuda(), ms.cuda(), mc.cuda()
            wx.group_combine(window.data_ptr(), key_lo, mk.data_ptr(), ms.data_ptr(), mc.data_ptr(), mk.numel(),
                             self.launch_aux, capacity, ok.data_ptr(), osm.data_ptr(), oc.data_ptr(),
                             d_n_groups=ng.data_ptr())
            self._keep = (mk, ms, mc)  # alive until the stream has consumed them
        return ok, osm, oc, ng

    def group_sum(self, val_expr: str, key_expr: str, cond: Optional[str], key_lo: int = 0,
                  capacity: int = 1 << 16):
        ok, osm, oc, ng = self.group_sum_device(val_expr, key_expr, cond, key_lo, capacity)
        self.wx.check(self.launch)
        n = int(ng.item())
        if n > capacity:
            raise self.wx.WarpExecError(self.wx.WX_ERR_CAPACITY, f"{n} groups exceed capacity {capacity}")
        return ok[:n].clone(), osm[:n].clone(), oc[:n].clone()

    # --- top-K ------------------------------------------------------------
    def topk_device(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int,
                    descending: bool):
        """This shard's top-K (keys, global rows, SELECT values, count) on the
        device, asynchronous; ties by ascending row index, NaN last."""
        tk = self._buf("tk", k, torch.float32)
        ti = self._buf("ti", k, torch.int64)
        tv = self._buf("tv", k, torch.float32)
        tn = self._buf("tn", 1, torch.int64)
        self.wx.topk(self.table, order_expr, cond, select_expr, k, descending, self.launch, tk.data_ptr(),
                     ti.data_ptr(), tv.data_ptr(), row_base=self.shard.row_base, d_count=tn.data_ptr(),
                     want_count=False)
        return tk, ti, tv, tn

    def topk_merged_device(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int,
                           descending: bool):
        """Global top-K left in HBM, no host synchronisation: this shard's
        candidates, then merge_topk_device.  Returns (keys, rows, vals, count)."""
        tk, ti, tv, tn = self.topk_device(order_expr, cond, select_expr, k, descending)
        return merge_topk_device(tk, ti, tv, tn, k, descending, self.group)

    def topk(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int, descending: bool):
        """Global top-K as host tensors: one all-gather of every shard's K
        candidates, then the (key, row) merge; a single shard is already final."""
        tk, ti, tv, tn = self.topk_device(order_expr, cond, select_expr, k, descending)
        if self.world == 1:
            m = int(tn.item())  # synchronises
            self.wx.check(self.launch)
            return tk[:m].cpu(), ti[:m].cpu(), tv[:m].cpu()
        m = int(tn.item())
        self.wx.check(self.launch)
        return merge_topk(tk, ti, tv, m, k, descending, self.group)
