#!/usr/bin/env python3
"""A/B of the dense projection's masked mode (GPU, diagnostic only).

`jit_compile_and_launch`'s contract (src/jit.cpp:55-61) leaves rows failing
the WHERE untouched (WX_MODE_DENSE).  Variants, interleaved in one process,
HIP events around the kernel: masked writes (WX_DENSE_BLEND=0), read + blend
+ whole-quad writes (WX_DENSE_BLEND=1, default), and fill mode for scale.
Each variant's output is checked against torch.

usage: python tools/ab_dense_masked.py [n=1e9] [rounds=7]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream, flags=0)
Lt = wx.make_launch(stream=stream, flags=wx.F_TIME)
price = torch.empty(n, dtype=torch.float32, device="cuda")
qty = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 2, 1, 1, 100, L)
table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()), wx.Column("quantity", wx.FLOAT32, qty.data_ptr())])
out = torch.empty(n, dtype=torch.float32, device="cuda")
E, C = "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)"
VARIANTS = {"masked_writes": ("WX_DENSE_BLEND=0", wx.MODE_DENSE), "blend": ("", wx.MODE_DENSE),
            "blend_unpipelined": ("WX_DENSE_BLEND_PIPE=0", wx.MODE_DENSE),
            "fill": ("", wx.MODE_DENSE_FILL)}
res = {k: [] for k in VARIANTS}
def setenv(v):
    os.environ["WARPDB_EXTRA_DEFINES"] = v[0]


for name, v in VARIANTS.items():
    setenv(v)
    mode = v[1]
    out.fill_(-7.0)
    wx.project_filter(table, E, C, L, mode, out.data_ptr(), 0, 4, 0)
    wx.check(L)
    m = price > 15.0
    want = torch.where(m, price * qty, torch.full_like(price, -7.0 if mode == wx.MODE_DENSE else 0.0))
    ok = torch.equal(out.view(torch.int32), want.view(torch.int32))
    del m, want
    print(f"{name:16s} check {'ok' if ok else 'BAD'}", flush=True)
wx.timing_read()
for r in range(rounds):
    for name, v in VARIANTS.items():
        setenv(v)
        wx.project_filter(table, E, C, Lt, v[1], out.data_ptr(), 0, 4, 0)
        ms, k = wx.timing_read()
        res[name].append(ms / k)
for name, ts in res.items():
    ts.sort()
    med = ts[len(ts) // 2]
    print(f"{name:16s} median {med:7.3f} ms  min {ts[0]:7.3f}  {n / med / 1e6:8.1f} G rows/s")
