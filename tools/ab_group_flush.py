#!/usr/bin/env python3
"""Diagnostic (GPU): what the GROUP BY window's global flush costs -- the C3
kernel with and without it (WX_DIAG_NO_FLUSH, results invalid) at the
strong-scaled 8-GPU shard size and at 1e9 rows; interleaved rounds, HIP-event
time of the main kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

s = torch.cuda.current_stream()
L = wx.make_launch(stream=s.cuda_stream)
Lt = wx.make_launch(stream=s.cuda_stream, flags=wx.F_TIME)
cap = 4096
ok = torch.empty(cap, dtype=torch.int32, device="cuda")
os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
oc = torch.empty(cap, dtype=torch.int64, device="cuda")
ng = torch.zeros(1, dtype=torch.int64, device="cuda")
for n in (125_000_000, 1_000_000_000):
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    key = torch.empty(n, dtype=torch.int32, device="cuda")
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
    t = wx.Table.from_tensors(price=price, quantity=key)
    for rnd in range(3):
        for v in ("", "WX_DIAG_NO_FLUSH"):
            os.environ["WARPDB_EXTRA_DEFINES"] = v
            for _ in range(3):
                wx.group_sum(t, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), os_.data_ptr(),
                             oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            wx.timing_read()
            for _ in range(20):
                wx.group_sum(t, "price[idx]", "quantity[idx]", None, Lt, 0, cap, ok.data_ptr(), os_.data_ptr(),
                             oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            torch.cuda.synchronize()
            kms, nl = wx.timing_read()
            print(f"n={n:>11d} round {rnd} [{v or 'full'}] kernel {kms / nl * 1e3:.1f} us", flush=True)
    del price, key, t
