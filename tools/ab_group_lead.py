#!/usr/bin/env python3
"""A/B (GPU): wx_group_sum with and without the wave-combined adds of a
shared window bin (WX_GROUP_LEAD), on the C3 table (1e9 rows, 1024 uniform
int32 keys) and on a skewed one (SKEW of the rows on key 7), interleaved in
one process, HIP-event kernel time per launch.

usage: python tools/ab_group_lead.py [rows] [skew,skew,...] [variant;variant;...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
skews = [float(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,0.9").split(",")]
variants = sys.argv[3].split(";") if len(sys.argv) > 3 else ["", "WX_GROUP_LEAD=0"]
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream)
Lt = wx.make_launch(stream=stream, flags=wx.F_TIME)
price = torch.empty(n, dtype=torch.float32, device="cuda")
key0 = torch.empty(n, dtype=torch.int32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
wx.fill_synthetic(key0.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
cap = 4096
ok = torch.empty(cap, dtype=torch.int32, device="cuda")
os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
oc = torch.empty(cap, dtype=torch.int64, device="cuda")
ng = torch.zeros(1, dtype=torch.int64, device="cuda")
for skew in skews:
    key = key0.clone()
    if skew > 0:
        key.masked_fill_(torch.rand(n, device="cuda") < skew, 7)
    t = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()), wx.Column("quantity", wx.INT32, key.data_ptr())])
    res = {v: [] for v in variants}
    sums = {}
    for v in variants:  # compile + warm
        os.environ["WARPDB_EXTRA_DEFINES"] = v
        for _ in range(2):
            wx.group_sum(t, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), os_.data_ptr(),
                         oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
        wx.check(L)
        sums[v] = (os_[:1024].clone(), oc[:1024].clone())
    wx.timing_read()
    for rnd in range(15):
        for v in variants[rnd % len(variants):] + variants[:rnd % len(variants)]:
            os.environ["WARPDB_EXTRA_DEFINES"] = v
            wx.group_sum(t, "price[idx]", "quantity[idx]", None, Lt, 0, cap, ok.data_ptr(), os_.data_ptr(),
                         oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            ms, k = wx.timing_read()
            res[v].append(ms / k)
    base = sums[variants[0]]
    for v, ts in res.items():
        ts.sort()
        same_counts = bool(torch.equal(sums[v][1], base[1]))
        rel = float(((sums[v][0] - base[0]).abs() / base[0].abs().clamp_min(1e-300)).max())
        print(f"skew {skew:4.2f} [{v or 'default'}] wx_group_sum median {ts[len(ts) // 2]:.4f} ms  min {ts[0]:.4f}  "
              f"{n * 8 / ts[len(ts) // 2] / 1e9:.2f} TB/s  counts equal {same_counts}, max rel sum gap {rel:.1e}",
              flush=True)
