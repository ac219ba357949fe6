#!/usr/bin/env python3
"""Wall time of GROUP BY with and without WX_F_ROW_ORDER on bench.py's C3
table (price f32 U[0, 40), quantity int32 U{0..keys-1}), per call, and the
row-order sums' distance from the ordinary ones.  Row order runs twice: the
key-span path (counting scatter + fold, keys spanning <= 2048; straight
from the table, then after an ordinary call, WARPDB_GROUP_ROWS=ordinary) and the
general path (compactions + radix pair sort + fold, WARPDB_GROUP_ROWS=general);
their sums must agree bit for bit.

usage: python tools/time_group_row_order.py [rows] [keys] [reps] [variant;variant;...]
(variants: WARPDB_EXTRA_DEFINES lists for the row-order runs, e.g.
";WX_FOLD_EXACT=0" -- every variant's sums must equal the first's bit for bit;
ROW_SKEW=0.9 puts 90 % of the rows on one key)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
nk = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1024
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
stream = torch.cuda.current_stream().cuda_stream
L0 = wx.make_launch(stream=stream)
price = torch.empty(n, dtype=torch.float32, device="cuda")
key = torch.empty(n, dtype=torch.int32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L0)
wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, nk - 1, L0)
skew = float(os.environ.get("ROW_SKEW", "0"))  # this share of the rows on key 7 (a big group)
if skew > 0:
    key.masked_fill_(torch.rand(n, device="cuda") < skew, 7)
table = wx.Table.from_tensors(price=price, quantity=key)
cap = max(4096, 2 * nk)
out = {}
variants = sys.argv[4].split(";") if len(sys.argv) > 4 else [os.environ.get("WARPDB_EXTRA_DEFINES", "")]
runs = [("plain", wx.F_SYNC, "")]
for var in variants:
    tag = f" [{var}]" if var else ""
    runs += [("row-order" + tag, wx.F_ROW_ORDER | wx.F_SYNC, var),
             ("row-order ordinary-first" + tag, wx.F_ROW_ORDER | wx.F_SYNC, var),
             ("row-order general" + tag, wx.F_ROW_ORDER | wx.F_SYNC, var)]
for label, flags, var in runs:
    os.environ["WARPDB_EXTRA_DEFINES"] = var
    if label.startswith("row-order general"):
        os.environ["WARPDB_GROUP_ROWS"] = "general"
    elif label.startswith("row-order ordinary-first"):
        os.environ["WARPDB_GROUP_ROWS"] = "ordinary"  # the span path after an ordinary call
    ok = torch.empty(cap, dtype=torch.int32, device="cuda")
    os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
    oc = torch.empty(cap, dtype=torch.int64, device="cuda")
    L = wx.make_launch(stream=stream, flags=flags)
    g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), os_.data_ptr(),
                     oc.data_ptr())
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, L, 0, cap, ok.data_ptr(), os_.data_ptr(),
                         oc.data_ptr())
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    out[label] = (ok[:g].clone(), os_[:g].clone(), oc[:g].clone())
    os.environ.pop("WARPDB_GROUP_ROWS", None)
    print(f"{label:40s} {n} rows x {nk} keys: median {ts[len(ts) // 2] * 1e3:.2f} ms, min {ts[0] * 1e3:.2f} ms "
          f"({g} groups)", flush=True)
(k0, s0, c0) = out["plain"]
first = [lab for lab, _, _ in runs if lab != "plain"]
(k1, s1, c1) = out[first[0]]
for lab in first[1:]:
    (k2, s2, c2) = out[lab]
    assert torch.equal(k1, k2) and torch.equal(c1, c2)
    assert torch.equal(s1.view(torch.int64), s2.view(torch.int64)), f"{lab} differs from {first[0]}"
print(f"row-order sums equal bit for bit across {len(first)} runs (key-span and general paths, every variant)")
assert torch.equal(k0, k1) and torch.equal(c0, c1)
rel = ((s1 - s0).abs() / s1.abs().clamp_min(1e-300)).max().item()
diff = int((s1.view(torch.int64) != s0.view(torch.int64)).sum().item())
print(f"row-order vs plain sums: {diff} of {len(s0)} groups differ in their bits, max relative gap {rel:.3e}")
