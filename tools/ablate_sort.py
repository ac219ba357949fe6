#!/usr/bin/env python3
"""Where a radix pass spends its time (GPU, diagnostic only).

Sorts 1e9 uniform float32 keys with diagnostic builds of the pass kernel
(WARPDB_EXTRA_DEFINES, see warpdb_amd/csrc/kernels/wx_radix.hip): without the look-back, without
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
    "lbstats": {D: "WX_RS_DIAG_LBSTATS=1"},
    "full_b": {},
    "lb_first_b": {D: "WX_RS_LB_FIRST=1"},
    "full_c": {},
    "lb_first_c": {D: "WX_RS_LB_FIRST=1"},
    "skip": {D: "WX_RS_SKIP=1"},
    "skip_m2g2": {D: "WX_RS_SKIP=1,WX_RS_SKIP_MIN=2,WX_RS_SKIP_GROW=2"},
    "skip_m8g4": {D: "WX_RS_SKIP=1,WX_RS_SKIP_MIN=8,WX_RS_SKIP_GROW=4"},
    "skip_lbw4": {D: "WX_RS_SKIP=1", "WARPDB_RS_LBW": "4"},
    "skip_lbstats": {D: "WX_RS_SKIP=1,WX_RS_DIAG_LBSTATS=1"},
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
    "lbw1": {"WARPDB_RS_LBW": "1"},
    "lbw2": {"WARPDB_RS_LBW": "2"},
    "lbw3": {"WARPDB_RS_LBW": "3"},
    "lbw2_first": {"WARPDB_RS_LBW": "2", D: "WX_RS_LB_FIRST=1"},
    "hcopies4": {D: "WX_RS_HCOPIES=4"},
    "hcopies16": {D: "WX_RS_HCOPIES=16"},
    "hcopies32": {D: "WX_RS_HCOPIES=32"},
    "hunroll2": {D: "WX_RS_HUNROLL=2"},
    "hunroll8": {D: "WX_RS_HUNROLL=8"},
    "rank_base0": {D: "WX_RS_RANK_BASE=0"},
    "items24_minw6": {D: "WX_RS_MINW=6", "WARPDB_RS_ITEMS": "24"},
    "items28": {"WARPDB_RS_ITEMS": "28"},
    "items32": {"WARPDB_RS_ITEMS": "32"},
    "items12_minw6": {D: "WX_RS_MINW=6", "WARPDB_RS_ITEMS": "12"},
    "items20": {"WARPDB_RS_ITEMS": "20"},
    "items34": {"WARPDB_RS_ITEMS": "34"},
    "items36": {"WARPDB_RS_ITEMS": "36"},
    "items40": {"WARPDB_RS_ITEMS": "40"},
    "items48": {"WARPDB_RS_ITEMS": "48"},
    "b1024_i16": {"WARPDB_RS_BLOCK": "1024", "WARPDB_RS_ITEMS": "16"},
    "b1024_i20": {"WARPDB_RS_BLOCK": "1024", "WARPDB_RS_ITEMS": "20"},
    "b768_i20": {"WARPDB_RS_BLOCK": "768", "WARPDB_RS_ITEMS": "20"},
    "b384_i40": {"WARPDB_RS_BLOCK": "384", "WARPDB_RS_ITEMS": "40"},
    "b256_i48": {"WARPDB_RS_BLOCK": "256", "WARPDB_RS_ITEMS": "48"},
    "items32_lbw2": {"WARPDB_RS_ITEMS": "32", "WARPDB_RS_LBW": "2"},
    "lbw4": {"WARPDB_RS_LBW": "4"},
    "nosplit": {D: "WX_RS_SPLIT=0"},
    "b256_i32": {"WARPDB_RS_BLOCK": "256", "WARPDB_RS_ITEMS": "32", D: "WX_RS_SPLIT=0"},
    "b256_i32_split": {"WARPDB_RS_BLOCK": "256", "WARPDB_RS_ITEMS": "32"},
    "b256_i28": {"WARPDB_RS_BLOCK": "256", "WARPDB_RS_ITEMS": "28", D: "WX_RS_SPLIT=0"},
    "b320_i32": {"WARPDB_RS_BLOCK": "320", "WARPDB_RS_ITEMS": "32", D: "WX_RS_SPLIT=0"},
    "b384_i28": {"WARPDB_RS_BLOCK": "384", "WARPDB_RS_ITEMS": "28", D: "WX_RS_SPLIT=0"},
    "b448_i24": {"WARPDB_RS_BLOCK": "448", "WARPDB_RS_ITEMS": "24", D: "WX_RS_SPLIT=0"},
    "nosplit_lbw2": {D: "WX_RS_SPLIT=0", "WARPDB_RS_LBW": "2"},
    "lbw8": {"WARPDB_RS_LBW": "8"},
    "lbw4_first": {"WARPDB_RS_LBW": "4", D: "WX_RS_LB_FIRST=1"},
    "lbw4_i28": {"WARPDB_RS_LBW": "4", "WARPDB_RS_ITEMS": "28"},
    "items32_g1": {"WARPDB_RS_ITEMS": "32", D: "WX_RS_RANK_G=1"},
    "hwide": {"WARPDB_RS_HWIDE": "1"},
    "hnarrow": {"WARPDB_RS_HWIDE": "0"},
    "hwide_u2": {"WARPDB_RS_HWIDE": "1", D: "WX_RS_HUNROLL=2"},
    "hwide_u8": {"WARPDB_RS_HWIDE": "1", D: "WX_RS_HUNROLL=8"},
    "hwide_nopipe": {"WARPDB_RS_HWIDE": "1", D: "WX_RS_HPIPE=0"},
    "nt_store": {D: "WX_RS_NT_STORE=1"},
    "hwide_u2_nopipe": {"WARPDB_RS_HWIDE": "1", D: "WX_RS_HUNROLL=2,WX_RS_HPIPE=0"},
}
KNOBS = (D, "WARPDB_RS_ITEMS", "WARPDB_RS_BLOCK", "WARPDB_RS_LBW", "WARPDB_RS_HWIDE")
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
