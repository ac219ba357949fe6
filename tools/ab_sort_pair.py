#!/usr/bin/env python3
"""A/B of the radix key tiles' paired look-back (WX_RS_LB_PAIR) in one
process: alternating builds, 1e9 uniform float keys, median of 5 sorts each
(fresh copy outside the timed region), plus the sort's own order check."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
variants = sys.argv[2].split(";") if len(sys.argv) > 2 else ["", "WX_RS_LB_PAIR=0"]
L = wx.make_launch(stream=torch.cuda.current_stream().cuda_stream, flags=0)
src = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(src.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
buf = torch.empty_like(src)
for rnd in range(3):
    for v in variants:
        os.environ["WARPDB_EXTRA_DEFINES"] = v
        ts = []
        for r in range(6):
            buf.copy_(src)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            wx.sort_float(buf.data_ptr(), n, True, L)
            torch.cuda.synchronize()
            if r:
                ts.append(time.perf_counter() - t0)
        ok = bool((buf[1:] >= buf[:-1]).all().item())
        ts.sort()
        print(f"round {rnd} [{v or 'default'}] median {ts[len(ts)//2]*1e3:.3f} ms  min {ts[0]*1e3:.3f}  sorted={ok}",
              flush=True)
