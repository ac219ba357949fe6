#!/usr/bin/env python3
"""A/B grid size and unroll of the grid-stride kernels (SUM, GROUP BY, top-K, dense projection)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
rounds = 5
stream = torch.cuda.current_stream().cuda_stream
DISC = "__device__ float discount(float price, float rate) { return price * rate; }\n"
L = wx.make_launch(stream=stream, custom_src=DISC)
Lt = wx.make_launch(stream=stream, custom_src=DISC, flags=wx.F_TIME)
price = torch.empty(n, dtype=torch.float32, device="cuda")
key = torch.empty(n, dtype=torch.int32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()), wx.Column("quantity", wx.INT32, key.data_ptr())])
res = torch.zeros(2, dtype=torch.float64, device="cuda")
cap = 4096
gk = torch.empty(cap, dtype=torch.int32, device="cuda")
gs = torch.empty(cap, dtype=torch.float64, device="cuda")
gc = torch.empty(cap, dtype=torch.int64, device="cuda")
ng = torch.zeros(1, dtype=torch.int64, device="cuda")
tk = torch.empty(5, device="cuda")
ti = torch.empty(5, dtype=torch.int64, device="cuda")
tv = torch.empty(5, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
dense = torch.empty(n, dtype=torch.float32, device="cuda")

OPS = {
    "sum": (4, lambda Lx: wx.reduce_sum(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", Lx, d_out=res.data_ptr(), want_host=False)),
    "group": (8, lambda Lx: wx.group_sum(table, "price[idx]", "quantity[idx]", None, Lx, 0, cap, gk.data_ptr(), gs.data_ptr(), gc.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)),
    "dense": (12, lambda Lx: wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", Lx, wx.MODE_DENSE_FILL, dense.data_ptr())),
    "dense_masked": (10.5, lambda Lx: wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", Lx, wx.MODE_DENSE, dense.data_ptr())),
    "topk": (4, lambda Lx: wx.topk(table, "price[idx]", None, "discount(price[idx], 0.9f)", 5, True, Lx, tk.data_ptr(), ti.data_ptr(), tv.data_ptr(), d_count=cnt.data_ptr(), want_count=False)),
}
EXTRA = os.environ.get("ABL_EXTRA", "")
VARIANTS = [(g, u) for g in tuple(int(x) for x in os.environ.get("ABL_GRIDS", "2,4,8").split(",")) for u in tuple(int(x) for x in os.environ.get("ABL_UNROLLS", "2,4,8").split(","))]
for name, (bpr, fn) in OPS.items():
    if len(sys.argv) > 2 and name not in sys.argv[2].split(","):
        continue
    out = []
    for g, u in VARIANTS:
        os.environ["WARPDB_GRID_PER_CU"] = str(g)
        os.environ["WARPDB_EXTRA_DEFINES"] = f"WX_UNROLL={u}" + ("," + EXTRA if EXTRA else "")
        fn(L)
        fn(L)
        wx.check(L)
        wx.timing_read()
        ts = []
        for _ in range(rounds):
            fn(Lt)
            ms, k = wx.timing_read()
            ts.append(ms / k)
        ts.sort()
        out.append((ts[len(ts) // 2], g, u))
    if os.environ.get("ABL_SIMPLE"):
        os.environ["WARPDB_GRID_PER_CU"] = "8"
        os.environ["WARPDB_EXTRA_DEFINES"] = "WX_UNROLL=4,WX_STRIDE_SIMPLE=1"
        fn(L)
        wx.timing_read()
        ts = []
        for _ in range(rounds):
            fn(Lt)
            ms, k = wx.timing_read()
            ts.append(ms / k)
        ts.sort()
        out.append((ts[len(ts) // 2], 8, "4-simple"))
    for med, g, u in sorted(out):
        print(f"{name:6s} grid/CU {g} unroll {u}: {med:7.3f} ms  {n * bpr / med / 1e6:7.1f} GB/s", flush=True)

e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
tmp = torch.empty_like(price)
ts = []
for _ in range(rounds + 1):
    e0.record()
    tmp.copy_(price)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
ts = sorted(ts[1:])
print(f"torch copy 4 GB: {ts[len(ts)//2]:.3f} ms  {n * 8 / ts[len(ts)//2] / 1e6:.1f} GB/s (r+w)")
