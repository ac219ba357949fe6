#!/usr/bin/env python3
"""Time wx_sort_float / wx_sort_pairs (jit_sort_float / jit_sort_pairs) on the
GPU: LSD radix sort against the bitonic network, uniform float32 keys.

usage: python tools/bench_sort.py [sizes, default 1e6,1e7,1e8,1e9] [bitonic max size]
Each call sorts a fresh copy (the copy is outside the timed region); the time
is the whole synchronous call (histogram read-back included).  GB/s counts
4 B read for the histogram + 8 B (float) or 16 B (pairs) per executed pass.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

sizes = [int(float(x)) for x in (sys.argv[1] if len(sys.argv) > 1 else "1e6,1e7,1e8,1e9").split(",")]
bitonic_max = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1e8
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream, flags=0)
for n in sizes:
    src = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(src.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    wx.fill_synthetic(keys.data_ptr(), wx.INT32, n, 3, 1, -(1 << 30), (1 << 30), L)
    buf = torch.empty_like(src)
    kb = torch.empty_like(keys)
    for algo in ("radix", "bitonic"):
        if algo == "bitonic" and n > bitonic_max:
            continue
        os.environ["WARPDB_SORT"] = algo
        for what in ("float", "pairs"):
            ts = []
            reps = 5 if algo == "radix" else 2
            for r in range(reps + 1):
                buf.copy_(src)
                kb.copy_(keys)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if what == "float":
                    wx.sort_float(buf.data_ptr(), n, True, L)
                else:
                    wx.sort_pairs(kb.data_ptr(), buf.data_ptr(), n, True, L)
                torch.cuda.synchronize()
                if r:
                    ts.append(time.perf_counter() - t0)
            ts.sort()
            med = ts[len(ts) // 2]
            if what == "float":
                ok = bool((buf[1:] >= buf[:-1]).all().item())
                gb = n * (4 + 4 * 8)
            else:
                ok = bool((kb[1:] >= kb[:-1]).all().item())
                gb = n * (4 + 4 * 16)
            print(f"{algo:8s} {what:6s} n={n:>11d}  {med * 1e3:9.3f} ms  {n / med / 1e9:7.2f} G keys/s  "
                  f"{gb / med / 1e9:7.1f} GB/s (4 passes)  sorted={ok}", flush=True)
    del src, keys, buf, kb
    torch.cuda.empty_cache()

# ORDER BY .. LIMIT k: the partial sort (top-digit head + full sort of it)
n = sizes[-1]
src = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(src.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
buf = torch.empty_like(src)
os.environ["WARPDB_SORT"] = "radix"
for k, asc in ((100, True), (100, False), (1_000_000, True), (1_000_000, False)):
    ts = []
    for r in range(4):
        buf.copy_(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wx.sort_float_limit(buf.data_ptr(), n, k, asc, L)
        torch.cuda.synchronize()
        if r:
            ts.append(time.perf_counter() - t0)
    ts.sort()
    ref = torch.sort(src, descending=not asc).values[:k]
    ok = bool(torch.equal(buf[:k], ref))
    print(f"limit    float  n={n:>11d}  k={k:>8d} {'asc ' if asc else 'desc'} {ts[len(ts) // 2] * 1e3:9.3f} ms  "
          f"head correct={ok}", flush=True)
