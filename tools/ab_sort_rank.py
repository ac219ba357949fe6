#!/usr/bin/env python3
"""A/B of radix-sort builds (WARPDB_EXTRA_DEFINES variants) in one process,
float keys or int key + payload pairs, with full checks: keys ordered, and
for pairs every payload (the input row, as bits) on its own key with equal
keys in input order -- the stability the LSD passes depend on.

usage: ab_sort_rank.py N {keys,pairs} [KEY_SPAN] "variant;variant;..."
(KEY_SPAN: int keys drawn from [0, KEY_SPAN), 0 = full 32-bit range)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1]))
kind = sys.argv[2]
span = int(float(sys.argv[3]))
variants = sys.argv[4].split(";")
L = wx.make_launch(stream=torch.cuda.current_stream().cuda_stream, flags=0)
if kind == "keys":
    src = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(src.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
else:
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    if span:
        src = torch.randint(0, span, (n,), dtype=torch.int32, device="cuda", generator=g)
    else:
        src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
    rows = torch.arange(n, dtype=torch.int32, device="cuda")
buf = torch.empty_like(src)
pay = torch.empty(n, dtype=torch.int32, device="cuda") if kind == "pairs" else None


def check():
    a = buf
    if not bool((a[1:] >= a[:-1]).all()):
        return "NOT ORDERED"
    if kind == "pairs":
        eq = a[1:] == a[:-1]
        if not bool((pay[1:][eq] > pay[:-1][eq]).all()):
            return "UNSTABLE"
        if not torch.equal(src[pay.long()], a):
            return "PAYLOAD MISPLACED"
    return "ok"


ENV_KNOBS = ("WARPDB_RS_PLAIN", "WARPDB_RS_LEAD", "WARPDB_RS_RANK_ATOMIC")


def apply(v):
    """'WX_RS_ITEMS=16,WARPDB_RS_LEAD=0': WARPDB_* items are environment test
    hooks, the rest kernel defines (WX_RS_BLOCK / WX_RS_ITEMS among them: the
    host reads the tile geometry back from the define list)."""
    for k in ENV_KNOBS:
        os.environ.pop(k, None)
    defs = []
    for item in filter(None, v.split(",")):
        if item.startswith("WARPDB_"):
            k, val = item.split("=", 1)
            os.environ[k] = val
        else:
            defs.append(item)
    os.environ["WARPDB_EXTRA_DEFINES"] = ",".join(defs)


ROUNDS = int(os.environ.get("AB_ROUNDS", "3"))
for rnd in range(ROUNDS):
    for v in variants[rnd % len(variants):] + variants[:rnd % len(variants)]:  # rotating order
        apply(v)
        ts = []
        for r in range(6):
            buf.copy_(src)
            if pay is not None:
                pay.copy_(rows)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if kind == "keys":
                wx.sort_float(buf.data_ptr(), n, True, L)
            else:
                wx.sort_pairs(buf.data_ptr(), pay.data_ptr(), n, True, L)
            torch.cuda.synchronize()
            if r:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        print(f"round {rnd} [{v or 'default'}] {kind} span={span} median {ts[len(ts)//2]*1e3:.3f} ms  "
              f"min {ts[0]*1e3:.3f}  check={check()}", flush=True)
