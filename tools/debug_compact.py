"""Diagnostic: run the compaction at several sizes / residencies and report."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from warpdb_amd import _warpexec as wx
os.environ["WARPDB_DEBUG"] = "1"
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream, flags=wx.F_SYNC)
for n_log in [22, 24, 26, 28]:
    n = 1 << n_log
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr())])
    out_v = torch.empty(n, dtype=torch.float32, device="cuda")
    out_i = torch.empty(n, dtype=torch.int32, device="cuda")
    for env in [{}, {"WARPDB_COMPACT_BPC_FORCE": "1"}, {"WARPDB_COMPACT_BPC_FORCE": "2"}, {"WARPDB_COMPACT_SCHED": "ticket"}]:
        for k in ("WARPDB_COMPACT_BPC_FORCE", "WARPDB_COMPACT_SCHED"):
            os.environ.pop(k, None)
        os.environ.update(env)
        try:
            c = wx.project_filter(table, "price[idx]", "(price[idx] > 15.0f)", L, wx.MODE_COMPACT, out_v.data_ptr(), out_i.data_ptr(), 4, 0, want_count=True)
            ref = int((price > 15).sum().item())
            ok = c == ref and torch.equal(out_i[:c], torch.nonzero(price > 15).flatten().int())
            print(n_log, env, "count", c, "ok" if ok else "MISMATCH", flush=True)
        except wx.WarpExecError as e:
            print(n_log, env, "ERROR", e, flush=True)
