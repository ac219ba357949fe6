#!/usr/bin/env python3
"""Where a radix pass spends its time (GPU, diagnostic only).

Sorts 1e9 uniform float32 keys with diagnostic builds of the pass kernel
(WARPDB_EXTRA_DEFINES, see wx_template.hip): without the look-back, without
the in-wave ranking, without the global key stores, and combinations.  The
diagnostic builds produce wrong orders; only their times mean anything.

usage: python tools/ablate_sort.py [n=1e9] [variant,...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

D = "WARPDB_EXTRA_DEFINES"
VARIANTS = {
    "full": {},
    "no_lookback": {D: "WX_RS_DIAG_NO_LOOKBACK=1"},
    "no_rank": {D: "WX_RS_DIAG_NO_RANK=1"},
    "no_store": {D: "WX_RS_DIAG_NO_STORE=1"},
    "no_rank_no_lookback": {D: "WX_RS_DIAG_NO_RANK=1,WX_RS_DIAG_NO_LOOKBACK=1"},
    "no_rank_no_store": {D: "WX_RS_DIAG_NO_RANK=1,WX_RS_DIAG_NO_STORE=1"},
    "load_lds_only": {D: "WX_RS_DIAG_NO_RANK=1,WX_RS_DIAG_NO_STORE=1,WX_RS_DIAG_NO_LOOKBACK=1"},
    "rank_g1": {D: "WX_RS_RANK_G=1"},
    "minw6": {D: "WX_RS_MINW=6"},
    "items16_minw6": {D: "WX_RS_MINW=6", "WARPDB_RS_ITEMS": "16"},
    "items16": {"WARPDB_RS_ITEMS": "16"},
    "items24": {"WARPDB_RS_ITEMS": "24"},
    "rank_g4": {D: "WX_RS_RANK_G=4"},
    "rank_lead0": {D: "WX_RS_RANK_LEAD=0"},
    "lb_first": {D: "WX_RS_LB_FIRST=1"},
    "lbw2": {"WARPDB_RS_LBW": "2"},
    "lbw2_first": {"WARPDB_RS_LBW": "2", D: "WX_RS_LB_FIRST=1"},
    "hcopies4": {D: "WX_RS_HCOPIES=4"},
    "hcopies16": {D: "WX_RS_HCOPIES=16"},
    "hcopies32": {D: "WX_RS_HCOPIES=32"},
    "hunroll2": {D: "WX_RS_HUNROLL=2"},
    "hunroll8": {D: "WX_RS_HUNROLL=8"},
}
KNOBS = (D, "WARPDB_RS_ITEMS", "WARPDB_RS_BLOCK", "WARPDB_RS_LBW")
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
if len(sys.argv) > 2:
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in sys.argv[2].split(",")}
L = wx.make_launch(stream=torch.cuda.current_stream().cuda_stream, flags=0)
src = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(src.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
buf = torch.empty_like(src)
for name, env in VARIANTS.items():
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(env)
    ts = []
    for r in range(6):
        buf.copy_(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wx.sort_float(buf.data_ptr(), n, True, L)
        torch.cuda.synchronize()
        if r:
            ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2]
    ok = bool((buf[1:] >= buf[:-1]).all().item())
    print(f"{name:22s} {med * 1e3:8.3f} ms  {n / med / 1e9:6.2f} G keys/s  sorted={ok}", flush=True)
for k in KNOBS:
    os.environ.pop(k, None)
