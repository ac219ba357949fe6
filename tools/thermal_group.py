#!/usr/bin/env python3
"""Diagnostic (GPU): the C3 GROUP BY kernel's time before and after ~20 s of
the compaction streaming at full power, and after 10 s idle -- why the
default bench's secondary GROUP BY line (run after the headline) reads
slower than a standalone run of the same kernel."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

s = torch.cuda.current_stream()
L = wx.make_launch(stream=s.cuda_stream)
Lt = wx.make_launch(stream=s.cuda_stream, flags=wx.F_TIME)
n = 10**9
price = torch.empty(n, dtype=torch.float32, device="cuda")
key = torch.empty(n, dtype=torch.int32, device="cuda")
qty = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 2, 1, 1, 100, L)
tg = wx.Table.from_tensors(price=price, quantity=key)
tp = wx.Table.from_tensors(price=price, quantity=qty)
cap = 4096
ok = torch.empty(cap, dtype=torch.int32, device="cuda")
os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
oc = torch.empty(cap, dtype=torch.int64, device="cuda")
ng = torch.zeros(1, dtype=torch.int64, device="cuda")
vals = torch.empty(n, dtype=torch.float32, device="cuda")
idx = torch.empty(n, dtype=torch.int32, device="cuda")


def group_ms():
    wx.timing_read()
    for _ in range(20):
        wx.group_sum(tg, "price[idx]", "quantity[idx]", None, Lt, 0, cap, ok.data_ptr(), os_.data_ptr(),
                     oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
    torch.cuda.synchronize()
    k, nl = wx.timing_read()
    return k / nl


def project(seconds):
    t0 = time.time()
    while time.time() - t0 < seconds:
        for _ in range(50):
            wx.project_filter(tp, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", L, wx.MODE_COMPACT,
                              vals.data_ptr(), idx.data_ptr(), 4, 0)
        torch.cuda.synchronize()


group_ms()
print(f"cold: group {group_ms():.4f} ms", flush=True)
project(20)
print(f"after 20 s of compaction: group {group_ms():.4f} ms, then {group_ms():.4f}", flush=True)
time.sleep(10)
print(f"after 10 s idle: group {group_ms():.4f} ms", flush=True)
project(20)
print(f"after 20 s of compaction: group {group_ms():.4f} ms", flush=True)
# how fast the clocks come back: 20-launch windows (~23 ms each) after idle gaps
for gap in (0.2, 1.0, 3.0, 10.0):
    project(3)
    time.sleep(gap)
    print(f"after {gap} s idle, consecutive 20-launch windows: " +
          " ".join(f"{group_ms():.4f}" for _ in range(12)), flush=True)
# the same after a busy-wait on the host with the GPU idle (what a host-side self-check looks like)
project(3)
t0 = time.time()
while time.time() - t0 < 1.0:
    pass
print("after 1 s host busy: " + " ".join(f"{group_ms():.4f}" for _ in range(12)), flush=True)
