#!/usr/bin/env python3
"""A/B (GPU, tuning): wx_group_sum (C3 shape, 1K int32 keys) across grid
densities (WARPDB_GRID_PER_CU) and row quads per thread (WX_UNROLL), at the
strong-scaled 8-GPU shard size and at 1e9 rows; interleaved rounds, HIP-event
time of the main kernel (WX_F_TIME) and of the whole call with its finalize."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

sizes = [int(float(x)) for x in (sys.argv[1] if len(sys.argv) > 1 else "1.25e8,1e9").split(",")]
# per_cu:unroll[:gblock]
cfgs = [(c.split(":") + ["256"])[:3] for c in (sys.argv[2] if len(sys.argv) > 2 else "4:2,2:2,2:4,1:4,1:8,4:4").split(",")]
s = torch.cuda.current_stream()
L = wx.make_launch(stream=s.cuda_stream)
Lt = wx.make_launch(stream=s.cuda_stream, flags=wx.F_TIME)
cap = 4096
ok = torch.empty(cap, dtype=torch.int32, device="cuda")
os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
oc = torch.empty(cap, dtype=torch.int64, device="cuda")
ng = torch.zeros(1, dtype=torch.int64, device="cuda")
for n in sizes:
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    key = torch.empty(n, dtype=torch.int32, device="cuda")
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
    t = wx.Table.from_tensors(price=price, quantity=key)
    res = {}
    for rnd in range(3):
        for per_cu, unroll, gblock in cfgs:
            os.environ["WARPDB_GRID_PER_CU"] = per_cu
            os.environ["WARPDB_GBLOCK"] = gblock
            os.environ["WARPDB_EXTRA_DEFINES"] = "" if unroll == "4" else f"WX_UNROLL={unroll}"
            for _ in range(3):
                wx.group_sum(t, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), os_.data_ptr(),
                             oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            wx.timing_read()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                wx.group_sum(t, "price[idx]", "quantity[idx]", None, Lt, 0, cap, ok.data_ptr(), os_.data_ptr(),
                             oc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            e1.record(s)
            torch.cuda.synchronize()
            kms, nl = wx.timing_read()
            res.setdefault((per_cu, unroll, gblock), []).append((kms / nl * 1e3, e0.elapsed_time(e1) / 20 * 1e3))
            assert int(ng.item()) == 1024
    for (per_cu, unroll, gblock), v in res.items():
        print(f"n={n:>11d} gblock={gblock} per_cu={per_cu} unroll={unroll}: kernel " +
              " ".join(f"{a:.1f}" for a, _ in v) + " us | call " + " ".join(f"{b:.1f}" for _, b in v) + " us",
              flush=True)
    del price, key, t
os.environ.pop("WARPDB_GRID_PER_CU")
os.environ.pop("WARPDB_GBLOCK")
