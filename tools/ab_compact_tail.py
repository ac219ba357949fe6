#!/usr/bin/env python3
"""A/B of the deep compaction's tail variants in one process, variants
rotating each round: C2's query over `rows` synthetic rows, kernel time from
the WX_F_TIME events.  A variant is a number (WARPDB_COMPACT_HALF_TAIL: half
tiles per workgroup at the end of a launch, 0 = every tile full) or
`defines` (WARPDB_EXTRA_DEFINES, e.g. WX_DEEP_EARLY_LAST=0) or `N:defines`.
Every variant must return the first variant's rows and values bit for bit.

usage: python tools/ab_compact_tail.py [rows] [rounds] [reps] VARIANT ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
variants = sys.argv[4:] or ["0", "2"]
stream = torch.cuda.current_stream().cuda_stream
L0 = wx.make_launch(stream=stream)
price = torch.empty(n, dtype=torch.float32, device="cuda")
qty = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 11, 0, 0.0, 40.0, L0)
wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 12, 1, 1, 100, L0)
table = wx.Table.from_tensors(price=price, quantity=qty)
vals = torch.empty(n, dtype=torch.float32, device="cuda")
idx = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
L = wx.make_launch(stream=stream, flags=wx.F_TIME)
E, C = "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)"


def q(launch):
    wx.project_filter(table, E, C, launch, wx.MODE_COMPACT, vals.data_ptr(), idx.data_ptr(), 4, 0,
                      d_count=cnt.data_ptr())


ref = None
res = {v: [] for v in variants}
for r in range(rounds):
    order = variants[r % len(variants):] + variants[:r % len(variants)]
    for v in order:
        ht, _, defs = v.partition(":") if (v[:1].isdigit() or ":" in v) else ("0", "", v)
        os.environ["WARPDB_COMPACT_HALF_TAIL"] = ht or "0"
        os.environ["WARPDB_EXTRA_DEFINES"] = defs
        for _ in range(10):
            q(L)
        wx.timing_read()
        for _ in range(reps):
            q(L)
        ms, launches = wx.timing_read()
        res[v].append(ms / launches)
        m = int(cnt.item())
        got = (m, vals[:m].clone(), idx[:m].clone())
        if ref is None:
            ref = got
        elif not (got[0] == ref[0] and torch.equal(got[1].view(torch.int32), ref[1].view(torch.int32))
                  and torch.equal(got[2], ref[2])):
            raise SystemExit(f"variant {v}: result differs from variant {variants[0]}")
    print(f"round {r}: " + "  ".join(f"[{v}] {res[v][-1] * 1e3:.1f} us" for v in variants), flush=True)
for v in variants:
    x = sorted(res[v])
    print(f"[{v}] kernel median {x[len(x) // 2] * 1e3:.1f} us, min {x[0] * 1e3:.1f} us "
          f"({ref[0]} of {n} rows pass, bit-equal)")
