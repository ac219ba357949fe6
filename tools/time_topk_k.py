#!/usr/bin/env python3
"""Time ORDER BY price DESC LIMIT k (wx_topk: scan + finalize) for several k
on the bench's C5 column (1e9 uniform f32 prices by default), HIP events
around the kernels (WX_F_TIME), and check the keys against torch.topk.

usage: python tools/time_topk_k.py [rows] [k,k,...] [reps] [variant;variant;...]
(variants: WARPDB_EXTRA_DEFINES lists, e.g. "WX_TOPK_SEED=0;" -- "" is the
default build; each line also reports the whole query per call, seed pass and
finalize included, from torch events around the calls)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
ks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,5,8,16,32").split(",")]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream)
Lt = wx.make_launch(stream=stream, flags=wx.F_TIME)
price = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
table = wx.Table.from_tensors(price=price)
ref = torch.topk(price, max(ks)).values
variants = sys.argv[4].split(";") if len(sys.argv) > 4 else [os.environ.get("WARPDB_EXTRA_DEFINES", "")]
for rnd in range(int(os.environ.get("AB_ROUNDS", "1"))):
    for var in variants[rnd % len(variants):] + variants[:rnd % len(variants)]:
        os.environ["WARPDB_EXTRA_DEFINES"] = var
        for k in ks:
            keys = torch.empty(k, device="cuda")
            for _ in range(3):
                wx.topk(table, "price[idx]", None, None, k, True, L, keys.data_ptr())
            torch.cuda.synchronize()
            wx.timing_read()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                wx.topk(table, "price[idx]", None, None, k, True, Lt, keys.data_ptr())
            e1.record()
            torch.cuda.synchronize()
            ms, launches = wx.timing_read()
            ok = bool(torch.equal(keys, ref[:k]))
            print(f"[{var or 'default'}] k={k:3d}  scan {ms / max(1, launches):.4f} ms per launch ({launches} launches)  "
                  f"{4 * n / (ms / max(1, launches)) / 1e9:.2f} TB/s of the column  "
                  f"query {e0.elapsed_time(e1) / reps:.4f} ms  keys ok={ok}", flush=True)
