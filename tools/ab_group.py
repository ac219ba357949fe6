#!/usr/bin/env python3
"""A/B (GPU, diagnostic): wx_group_sum with its finalize vs wx_group_partials
(the multi-shard export) on the C3 table, interleaved, HIP-event kernel time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream)
Lt = wx.make_launch(stream=stream, flags=wx.F_TIME)
price = torch.empty(n, dtype=torch.float32, device="cuda")
key = torch.empty(n, dtype=torch.int32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
t = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()), wx.Column("quantity", wx.INT32, key.data_ptr())])
cap = 4096
ok = torch.empty(cap, dtype=torch.int32, device="cuda")
os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
oc = torch.empty(cap, dtype=torch.int64, device="cuda")
ng = torch.zeros(1, dtype=torch.int64, device="cuda")
win = torch.zeros(4097, dtype=torch.float64, device="cuda")
nx = torch.zeros(1, dtype=torch.int64, device="cuda")


def a(Lx):
    wx.group_sum(t, "price[idx]", "quantity[idx]", None, Lx, 0, cap, ok.data_ptr(), os_.data_ptr(), oc.data_ptr(),
                 d_n_groups=ng.data_ptr(), want_count=False)


def b(Lx):
    wx.group_partials(t, "price[idx]", "quantity[idx]", None, Lx, 0, win.data_ptr(), cap, ok.data_ptr(),
                      os_.data_ptr(), oc.data_ptr(), d_n_extra=nx.data_ptr())


res = {"group_sum": [], "group_partials": []}
for f in (a, b):
    f(L)
    f(L)
wx.check(L)
wx.timing_read()
for _ in range(15):
    for name, f in (("group_sum", a), ("group_partials", b)):
        f(Lt)
        ms, k = wx.timing_read()
        res[name].append(ms / k)
for name, ts in res.items():
    ts.sort()
    print(f"{name:16s} median {ts[len(ts) // 2]:.4f} ms  min {ts[0]:.4f}  {n * 8 / ts[len(ts) // 2] / 1e6:.1f} GB/s")
