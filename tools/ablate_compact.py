#!/usr/bin/env python3
"""A/B the compaction kernel variants in one process (GPU).  Diagnostic only.

Each variant is selected through the environment knobs read per call by
libwarpexec (WARPDB_COMPACT_GROUPS / _SCHED / _BPC, WARPDB_EXTRA_DEFINES);
timings are HIP events around the kernel (WX_F_TIME), interleaved rounds.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
torch.cuda.set_device(0)
stream = torch.cuda.current_stream().cuda_stream
L = wx.make_launch(stream=stream, flags=0)
Lt = wx.make_launch(stream=stream, flags=wx.F_TIME)
price = torch.empty(n, dtype=torch.float32, device="cuda")
qty = torch.empty(n, dtype=torch.float32, device="cuda")
wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 2, 1, 1, 100, L)
table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()), wx.Column("quantity", wx.FLOAT32, qty.data_ptr())])
out_v = torch.empty(n, dtype=torch.float32, device="cuda")
out_i = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
ref_count = int((price > 15.0).sum().item())

VARIANTS = {
    "dw8_g4": {"WARPDB_COMPACT_SCHED": "static"},
    "dw12_g4": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "12"},
    "dw15_g4": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "15"},
    "dw12_g6": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "12", "WARPDB_COMPACT_GROUPS": "6"},
    "dw15_g4_lb2": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "15", "WARPDB_EXTRA_DEFINES": "WX_LB_PER_LANE=2"},
    "dw15_nolookback": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "15",
                        "WARPDB_EXTRA_DEFINES": "WX_DIAG_NO_LOOKBACK"},
    "dw15_nostore": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "15",
                     "WARPDB_EXTRA_DEFINES": "WX_DIAG_NO_STORE"},
    "dw15_plainld": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_NT_LOAD=0"},
    "dw15_ntst": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_NT_STORE=1"},
    "dw15_plainld_ntst": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_NT_LOAD=0,WX_NT_STORE=1"},
    "dw12_ntst": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "12", "WARPDB_EXTRA_DEFINES": "WX_NT_STORE=1"},
    "v0_w0": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_COMPACT_VSTORE=0,WX_COMPACT_WHOLE_LOADS=0"},
    "v1_w0": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_COMPACT_VSTORE=1,WX_COMPACT_WHOLE_LOADS=0"},
    "v0_w1": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_COMPACT_VSTORE=0,WX_COMPACT_WHOLE_LOADS=1"},
    "v1_w1": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_COMPACT_VSTORE=1,WX_COMPACT_WHOLE_LOADS=1"},
    "v1_w0_dw12": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "12", "WARPDB_EXTRA_DEFINES": "WX_COMPACT_VSTORE=1,WX_COMPACT_WHOLE_LOADS=0"},
    "dw7_2pc": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "7", "WARPDB_COMPACT_BPC_FORCE": "2",
                "WARPDB_EXTRA_DEFINES": "WX_COMPACT_MINBLOCKS=2"},
    "dw7_1pc": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "7", "WARPDB_COMPACT_BPC_FORCE": "1"},
    "dw7_g8_2pc": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "7", "WARPDB_COMPACT_GROUPS": "8", "WARPDB_COMPACT_BPC_FORCE": "2",
                   "WARPDB_EXTRA_DEFINES": "WX_COMPACT_MINBLOCKS=2"},
    "dw15": {"WARPDB_COMPACT_SCHED": "static"},
    "deep": {},
    "deep_ntst": {"WARPDB_EXTRA_DEFINES": "WX_NT_STORE=1"},
    "deep_plainst": {"WARPDB_EXTRA_DEFINES": "WX_DEEP_NT_STORE=0"},
    "deep_nolookback": {"WARPDB_EXTRA_DEFINES": "WX_DIAG_NO_LOOKBACK"},
    "deep_nostore": {"WARPDB_EXTRA_DEFINES": "WX_DIAG_NO_STORE"},
    "static_sched": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_COMPACT_TICKETS=0"},
    "nolb_unaligned": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_DIAG_NO_LOOKBACK=2"},
    "deep_dw12": {"WARPDB_COMPACT_SCHED": "deep", "WARPDB_COMPACT_DWAVES": "12"},
    "deep_dw15_g3": {"WARPDB_COMPACT_SCHED": "deep", "WARPDB_COMPACT_GROUPS": "3"},
    "deep_g2": {"WARPDB_COMPACT_GROUPS": "2"},
    "ticket": {"WARPDB_COMPACT_SCHED": "ticket"},
    "deep_retire_acqrel": {"WARPDB_EXTRA_DEFINES": "WX_RETIRE_ACQ_REL=1"},
    "deep_ticket_single": {"WARPDB_EXTRA_DEFINES": "WX_TICKET_PAIR=0"},
    "static": {"WARPDB_COMPACT_SCHED": "static"},
    "deep_g3": {"WARPDB_COMPACT_GROUPS": "3"},
    "deep_dw8": {"WARPDB_COMPACT_DWAVES": "8"},
    "deep_dw8_g2": {"WARPDB_COMPACT_DWAVES": "8", "WARPDB_COMPACT_GROUPS": "2"},
    "deep_dw6_2pc": {"WARPDB_COMPACT_DWAVES": "6", "WARPDB_COMPACT_BPC_FORCE": "2",
                     "WARPDB_EXTRA_DEFINES": "WX_COMPACT_MINBLOCKS=2"},
    "deep_dw5_g4_2pc": {"WARPDB_COMPACT_DWAVES": "5", "WARPDB_COMPACT_BPC_FORCE": "2",
                        "WARPDB_EXTRA_DEFINES": "WX_COMPACT_MINBLOCKS=2"},
    "dw12": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_COMPACT_DWAVES": "12"},
    "lb_sleep0": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_LB_SLEEP=0"},
    "lb_sleep1": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_LB_SLEEP=1"},
    "lb_sleep6": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_LB_SLEEP=6"},
    "lb_lanes2": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_LB_PER_LANE=2"},
    "prof": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_DIAG_PROFILE"},
    "prof_nostore": {"WARPDB_COMPACT_SCHED": "static", "WARPDB_EXTRA_DEFINES": "WX_DIAG_PROFILE,WX_DIAG_NO_STORE"},
}
if len(sys.argv) > 3:
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in sys.argv[3].split(",")}
KNOBS = ("WARPDB_COMPACT_SCHED", "WARPDB_COMPACT_GROUPS", "WARPDB_COMPACT_BPC", "WARPDB_EXTRA_DEFINES",
         "WARPDB_COMPACT_BPC_FORCE", "WARPDB_COMPACT_DWAVES")


def setenv(v):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(v)


def run(Lx):
    wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", Lx, wx.MODE_COMPACT,
                      out_v.data_ptr(), out_i.data_ptr(), 4, 0, d_count=cnt.data_ptr())


res = {k: [] for k in VARIANTS}
for name, v in VARIANTS.items():  # compile + warm
    setenv(v)
    t0 = time.time()
    run(L)
    run(L)
    wx.check(L)
    ok = "diag" if "DIAG" in str(v) else ("ok" if int(cnt.item()) == ref_count else f"BAD {int(cnt.item())} vs {ref_count}")
    print(f"{name:24s} warm {time.time() - t0:5.2f}s  count {ok}", flush=True)
wx.timing_read()
for r in range(rounds):
    for name, v in VARIANTS.items():
        setenv(v)
        run(Lt)
        ms, k = wx.timing_read()
        res[name].append(ms / k)
bytes_ = n * 8 + ref_count * 8
for name, ts in res.items():
    ts.sort()
    med = ts[len(ts) // 2]
    print(f"{name:24s} median {med:8.3f} ms  min {ts[0]:8.3f}  {bytes_ / med / 1e6:8.1f} GB/s  {n / med / 1e6:8.2f} Grows/s")

# references: read-only SUM over both columns, torch copy
setenv({})
wx.reduce_sum(table, "(price[idx] * quantity[idx])", None, L)
ts = []
for _ in range(rounds):
    wx.reduce_sum(table, "(price[idx] * quantity[idx])", None, Lt, want_host=False)
    ms, k = wx.timing_read()
    ts.append(ms / k)
ts.sort()
print(f"{'sum_read_8B':24s} median {ts[len(ts)//2]:8.3f} ms  {n * 8 / ts[len(ts)//2] / 1e6:8.1f} GB/s (read)")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
tmp = torch.empty_like(price)
tmp.copy_(price)
ts = []
for _ in range(rounds):
    e0.record()
    tmp.copy_(price)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
print(f"{'torch_copy_4B':24s} median {ts[len(ts)//2]:8.3f} ms  {n * 8 / ts[len(ts)//2] / 1e6:8.1f} GB/s (r+w)")
