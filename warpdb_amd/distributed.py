"""One process per GPU: row-sharded queries over torch.distributed (RCCL).

Each rank owns a contiguous shard of the table resident in its GPU's HBM
(rows [row_base, row_base + n) with the reference's ceil(N / devices)
partition, src/multi_gpu_utils.cpp:24-32) and runs the query locally through
the C ABI.  The exchanges are the ones the result needs and nothing else:

  compaction   all-gather of per-shard passing counts -> global offsets
               (the reference concatenates shard results in device order)
  SUM          all-reduce of one float64 sum and one int64 count
  GROUP BY     all-gather of the per-shard (key, sum, count) groups, merged
               in ascending key order
  top-K        all-gather of K candidates per shard, merged by (key, row)

With the "nccl" backend these run on RCCL over xGMI; with "gloo" (CPU tests)
the same code runs on host tensors.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """[begin, end) rows of `rank` under ceil(n / world) contiguous chunks."""
    chunk = (n_rows + world - 1) // world if world > 0 else n_rows
    b = min(n_rows, rank * chunk)
    return b, min(n_rows, b + chunk)


def _dev(group=None) -> torch.device:
    backend = dist.get_backend(group)
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def exchange_counts(local_count: int, group=None) -> Tuple[int, int, List[int]]:
    """Global offset of this shard's compacted rows, the total, and all counts."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _dev(group)
    mine = torch.tensor([local_count], dtype=torch.int64, device=dev)
    allc = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allc, mine, group=group)
    counts = allc.cpu().tolist()
    return sum(counts[:rank]), sum(counts), counts


def allreduce_sum(local_sum: float, local_count: int, group=None) -> Tuple[float, int]:
    dev = _dev(group)
    s = torch.tensor([local_sum], dtype=torch.float64, device=dev)
    c = torch.tensor([local_count], dtype=torch.int64, device=dev)
    dist.all_reduce(s, group=group)
    dist.all_reduce(c, group=group)
    return float(s.item()), int(c.item())


def _gather_padded(t: torch.Tensor, n: int, group=None) -> Tuple[torch.Tensor, List[int]]:
    """All-gather the first n entries of t from every rank (variable n)."""
    world = dist.get_world_size(group)
    dev = _dev(group)
    ns = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(ns, torch.tensor([n], dtype=torch.int64, device=dev), group=group)
    sizes = ns.cpu().tolist()
    m = max(1, max(sizes))
    buf = torch.zeros(m, dtype=t.dtype, device=dev)
    if n:
        buf[:n] = t[:n].to(dev)
    out = torch.zeros(world * m, dtype=t.dtype, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    parts = [out[r * m: r * m + sizes[r]] for r in range(world)]
    return torch.cat(parts), sizes


def merge_groups(keys: torch.Tensor, sums: torch.Tensor, counts: torch.Tensor, n: int, group=None):
    """Combine per-shard GROUP BY results; ascending keys, float64 sums."""
    k, _ = _gather_padded(keys.to(torch.int64), n, group)
    s, _ = _gather_padded(sums.to(torch.float64), n, group)
    c, _ = _gather_padded(counts.to(torch.int64), n, group)
    uk, inv = torch.unique(k, sorted=True, return_inverse=True)
    ss = torch.zeros(uk.numel(), dtype=torch.float64, device=k.device).index_add_(0, inv, s)
    cc = torch.zeros(uk.numel(), dtype=torch.int64, device=k.device).index_add_(0, inv, c)
    return uk.to(torch.int32), ss, cc


def merge_topk(keys: torch.Tensor, idx: torch.Tensor, vals: torch.Tensor, n: int, k: int, descending: bool,
               group=None):
    """Global top-K from per-shard candidates; ties by ascending row index."""
    gk, _ = _gather_padded(keys.to(torch.float32), n, group)
    gi, _ = _gather_padded(idx.to(torch.int64), n, group)
    gv, _ = _gather_padded(vals.to(torch.float32), n, group)
    # stable sorts: by row index, then by key (NaN last in either direction)
    order = torch.argsort(gi, stable=True)
    gk, gi, gv = gk[order], gi[order], gv[order]
    key = torch.where(torch.isnan(gk), torch.full_like(gk, float("inf") if not descending else -float("inf")), gk)
    order = torch.argsort(key, descending=descending, stable=True)
    nan_last = torch.isnan(gk[order])
    order = torch.cat([order[~nan_last], order[nan_last]])[:k]
    return gk[order], gi[order], gv[order]


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
    """Run the C-ABI operations on the local shard and exchange results."""

    def __init__(self, shard: Shard, custom_src: Optional[str] = None, group=None):
        from . import _warpexec as wx

        self.wx = wx
        self.shard = shard
        self.group = group
        self.table = shard.table()
        self.launch = wx.make_launch(device=torch.cuda.current_device(),
                                     stream=torch.cuda.current_stream().cuda_stream, custom_src=custom_src,
                                     flags=wx.F_SYNC)

    def compact(self, expr: str, cond: Optional[str], idx_bytes: int = 8):
        n = self.shard.n_rows
        vals = torch.empty(max(1, n), dtype=torch.float32, device="cuda")
        idx = torch.empty(max(1, n), dtype=torch.int64 if idx_bytes == 8 else torch.int32, device="cuda")
        c = self.wx.project_filter(self.table, expr, cond, self.launch, self.wx.MODE_COMPACT, vals.data_ptr(),
                                   idx.data_ptr(), idx_bytes, self.shard.row_base if idx_bytes == 8 else 0,
                                   want_count=True)
        offset, total, _ = exchange_counts(c, self.group)
        return vals[:c], idx[:c], offset, total

    def sum(self, expr: str, cond: Optional[str]):
        s, c = self.wx.reduce_sum(self.table, expr, cond, self.launch)
        return allreduce_sum(s, c, self.group)

    def group_sum(self, val_expr: str, key_expr: str, cond: Optional[str], capacity: int = 1 << 16):
        keys = torch.empty(capacity, dtype=torch.int32, device="cuda")
        sums = torch.empty(capacity, dtype=torch.float64, device="cuda")
        cnts = torch.empty(capacity, dtype=torch.int64, device="cuda")
        g = self.wx.group_sum(self.table, val_expr, key_expr, cond, self.launch, 0, capacity, keys.data_ptr(),
                              sums.data_ptr(), cnts.data_ptr())
        return merge_groups(keys, sums, cnts, g, self.group)

    def topk(self, order_expr: str, cond: Optional[str], select_expr: Optional[str], k: int, descending: bool):
        tk = torch.empty(k, dtype=torch.float32, device="cuda")
        ti = torch.empty(k, dtype=torch.int64, device="cuda")
        tv = torch.empty(k, dtype=torch.float32, device="cuda")
        m = self.wx.topk(self.table, order_expr, cond, select_expr, k, descending, self.launch, tk.data_ptr(),
                         ti.data_ptr(), tv.data_ptr(), row_base=self.shard.row_base)
        return merge_topk(tk, ti, tv, m, k, descending, self.group)
