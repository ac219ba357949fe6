#!/usr/bin/env python3
"""A/B of the radix sorts in one process: the three-pass reduce-then-scan sort
(wx_radix.hip, the default) against the four-pass onesweep
(WARPDB_RS_ALGO=onesweep), rounds alternating.  Float keys (uniform 0..40, as
the bench) and int keys + float payload; every result is checked bit for bit
against torch's stable sort.

usage: python tools/ab_sort3.py [sizes, default 1e6,1e8,1e9] [rounds, default 3] [algos, default onesweep,rts]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

sizes = [int(float(x)) for x in (sys.argv[1] if len(sys.argv) > 1 else "1e6,1e8,1e9").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
algos = (sys.argv[3] if len(sys.argv) > 3 else "onesweep,rts").split(",")
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream, flags=0)
for n in sizes:
    src = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(src.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    wx.fill_synthetic(keys.data_ptr(), wx.INT32, n, 3, 1, -(1 << 30), (1 << 30), L)
    pay = torch.arange(n, dtype=torch.int32, device="cuda").view(torch.float32)
    ref_f = torch.sort(src).values
    rk, ri = torch.sort(keys, stable=True)
    ref_v = pay.view(torch.int32)[ri]
    del ri
    buf = torch.empty_like(src)
    kb = torch.empty_like(keys)
    vb = torch.empty_like(pay)
    res = {}
    for r in range(rounds + 1):
        for algo in algos:
            os.environ["WARPDB_RS_ALGO"] = algo
            for what in ("float", "pairs"):
                buf.copy_(src)
                kb.copy_(keys)
                vb.copy_(pay)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if what == "float":
                    wx.sort_float(buf.data_ptr(), n, True, L)
                else:
                    wx.sort_pairs(kb.data_ptr(), vb.data_ptr(), n, True, L)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                if what == "float":
                    ok = bool(torch.equal(buf.view(torch.int32), ref_f.view(torch.int32)))
                else:
                    ok = bool(torch.equal(kb, rk)) and bool(torch.equal(vb.view(torch.int32), ref_v))
                if not ok:
                    print(f"MISMATCH {algo} {what} n={n}", flush=True)
                if r:
                    res.setdefault((algo, what), []).append(dt)
    for (algo, what), ts in sorted(res.items()):
        ts.sort()
        print(f"n={n:>11d} {what:6s} {algo:9s} median {ts[len(ts) // 2] * 1e3:8.3f} ms  min {ts[0] * 1e3:8.3f} ms  "
              f"{n / ts[len(ts) // 2] / 1e9:6.1f} G keys/s", flush=True)
    del src, keys, pay, ref_f, rk, ref_v, buf, kb, vb
    torch.cuda.empty_cache()
