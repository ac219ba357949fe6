#!/usr/bin/env python3
"""Per-workgroup timeline of wx_project_compact_deep (WX_DIAG_TIMELINE):
entry, first tickets, first evaluation and end times relative to the first
workgroup's entry, and tiles per workgroup -- where C2's fixed cost at 1e8
rows goes.  usage: python tools/timeline_compact.py [rows ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

L = wx.make_launch(stream=torch.cuda.current_stream().cuda_stream, flags=0)
for n in [int(float(x)) for x in (sys.argv[1:] or ["1e8", "1e9"])]:
    p = torch.empty(n, dtype=torch.float32, device="cuda")
    q = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(p.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    wx.fill_synthetic(q.data_ptr(), wx.FLOAT32, n, 2, 1, 1, 100, L)
    t = wx.Table.from_tensors(price=p, quantity=q)
    vals = torch.empty(n, dtype=torch.float32, device="cuda")
    idx = torch.empty(n, dtype=torch.int32, device="cuda")
    for diag in ("", "WX_DIAG_TIMELINE"):
        os.environ["WARPDB_EXTRA_DEFINES"] = diag
        ts = []
        for r in range(8):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            wx.project_filter(t, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", L, wx.MODE_COMPACT,
                              vals.data_ptr(), idx.data_ptr(), 4, 0)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print(f"n={n} [{diag or 'plain'}] call median {ts[4]*1e3:.3f} ms", flush=True)
    del p, q, vals, idx, t
