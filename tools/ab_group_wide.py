#!/usr/bin/env python3
"""A/B of the range-partitioned GROUP BY's build variants in one process
(WARPDB_EXTRA_DEFINES per variant, rotating order each round): 1e9 rows x
10^6 uniform int32 keys (bench.py's --workload group --keys 1000000 table),
the per-kernel times of one query summed from the WX_F_TIME events.  Every
variant but diagnostic ones must return the first variant's groups.

usage: python tools/ab_group_wide.py [rows] [rounds] 'DEFINES_A' 'DEFINES_B' ...
       ('' = the default build; diagnostic variants contain DIAG)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
variants = sys.argv[3:] or [""]
stream = torch.cuda.current_stream().cuda_stream
L0 = wx.make_launch(stream=stream, flags=0)
price = torch.empty(n, dtype=torch.float32, device="cuda")
key = torch.empty(n, dtype=torch.int32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L0)
wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 999_999, L0)
table = wx.Table.from_tensors(price=price, quantity=key)
cap = 1 << 20
ok = torch.empty(cap, dtype=torch.int32, device="cuda")
os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
oc = torch.empty(cap, dtype=torch.int64, device="cuda")
L = wx.make_launch(stream=stream, flags=wx.F_TIME)
ref = None
res = {v: [] for v in variants}
for r in range(rounds):
    order = variants[r % len(variants):] + variants[:r % len(variants)]
    for v in order:
        os.environ["WARPDB_EXTRA_DEFINES"] = v
        for _ in range(2):  # compile / warm
            wx.group_sum(table, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), os_.data_ptr(),
                         oc.data_ptr())
        wx.timing_read()
        reps = 5
        for _ in range(reps):
            g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), os_.data_ptr(),
                             oc.data_ptr())
        ms, launches = wx.timing_read()
        res[v].append(ms / reps)
        if "DIAG" not in v:
            got = (ok[:g].clone(), oc[:g].clone(), os_[:g].clone())
            if ref is None:
                ref = got
            elif not (torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
                      and torch.allclose(got[2], ref[2], rtol=1e-12, atol=0)):
                raise SystemExit(f"variant {v!r}: groups differ from the first variant's")
    print(f"round {r}: " + "  ".join(f"[{v or 'default'}] {res[v][-1]:.3f} ms" for v in variants), flush=True)
for v in variants:
    x = sorted(res[v])
    print(f"[{v or 'default'}] kernels per query: median {x[len(x) // 2]:.3f} ms, min {x[0]:.3f} ms ({g} groups)")
