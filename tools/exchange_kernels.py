#!/usr/bin/env python3
"""Timing of the multi-GPU GROUP BY / top-K exchange kernels on one GPU (the
collective itself is not run): one C3 shard of the strong-scaled 8-GPU run
(1.25e8 rows, 1K int32 keys) through wx_group_partials_slots with 8 slots,
then wx_group_combine_slots on that buffer; wx_topk + wx_topk_merge over 8
records.  Per kernel: median of 50 launches with HIP events (run under
rocprofv3 for the per-kernel split)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402
from warpdb_amd import distributed as wd  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
s = torch.cuda.current_stream()
L = wx.make_launch(stream=s.cuda_stream, flags=0)
p = torch.empty(n, dtype=torch.float32, device="cuda")
k = torch.empty(n, dtype=torch.int32, device="cuda")
wx.fill_synthetic(p.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
wx.fill_synthetic(k.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
t = wx.Table.from_tensors(price=p, quantity=k)
S = wd.group_slot_groups(world)
ex = torch.zeros(wx.group_slots_doubles(world, S), dtype=torch.float64, device="cuda")
cap = 4096
xk = torch.empty(cap, dtype=torch.int32, device="cuda")
xs = torch.empty(cap, dtype=torch.float64, device="cuda")
xc = torch.empty(cap, dtype=torch.int64, device="cuda")
nx = torch.empty(1, dtype=torch.int64, device="cuda")
ok = torch.empty(cap, dtype=torch.int32, device="cuda")
osm = torch.empty(cap, dtype=torch.float64, device="cuda")
oc = torch.empty(cap, dtype=torch.int64, device="cuda")
ng = torch.empty(1, dtype=torch.int64, device="cuda")


def timed(fn, reps=50):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(5):
        fn()
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2] * 1e3


part = lambda: wx.group_partials_slots(t, "price[idx]", "quantity[idx]", None, L, 0, ex.data_ptr(), world, 0, S, cap,
                                       xk.data_ptr(), xs.data_ptr(), xc.data_ptr(), d_n_extra=nx.data_ptr())
comb = lambda: wx.group_combine_slots(ex.data_ptr(), world, S, 0, L, cap, ok.data_ptr(), osm.data_ptr(),
                                      oc.data_ptr(), d_n_groups=ng.data_ptr())
print(f"group partials (sum + finalize, {n} rows, {world} slots): {timed(part):.1f} us", flush=True)
print(f"group combine_slots (empty slots): {timed(comb):.1f} us  groups={int(ng.item())}", flush=True)
single = lambda: wx.group_sum(t, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), osm.data_ptr(),
                              oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
print(f"single-GPU group_sum (sum + finalize): {timed(single):.1f} us", flush=True)
rec = torch.zeros(world * wx.TOPK_RECORD_BYTES, dtype=torch.uint8, device="cuda")
r0 = rec[:wx.TOPK_RECORD_BYTES]
tk = lambda: wx.topk(t, "price[idx]", None, None, 5, True, L, r0[:128].data_ptr(), r0[256:512].data_ptr(),
                     r0[128:256].data_ptr(), row_base=0, d_count=r0[512:520].data_ptr(), want_count=False)
print(f"topk scan + finalize ({n} rows): {timed(tk):.1f} us", flush=True)
for r in range(1, world):
    rec[r * wx.TOPK_RECORD_BYTES:(r + 1) * wx.TOPK_RECORD_BYTES].copy_(r0)
mk = torch.empty(5, dtype=torch.float32, device="cuda")
mi = torch.empty(5, dtype=torch.int64, device="cuda")
mv = torch.empty(5, dtype=torch.float32, device="cuda")
mn = torch.empty(1, dtype=torch.int64, device="cuda")
mg = lambda: wx.topk_merge(rec.data_ptr(), world, 5, True, L, mk.data_ptr(), mi.data_ptr(), mv.data_ptr(),
                           mn.data_ptr())
print(f"topk_merge ({world} records): {timed(mg):.1f} us", flush=True)
