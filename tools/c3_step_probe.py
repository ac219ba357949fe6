#!/usr/bin/env python3
"""Where the multi-rank C3-strong step's time goes (one rank, RCCL on a
one-rank communicator: run with WARPDB_EXCHANGE_ONE_RANK=1 MASTER_ADDR=127.0.0.1
MASTER_PORT=... WORLD_SIZE=1 RANK=0).  At the 8-GPU per-rank size (1.25e8
rows of price f32 + 1K int32 keys) it times, per step:

  eager      ShardedQuery.group_sum_device as bench.py runs it (partials,
             all-reduce, combine): wall time and the host's issue time
  local      the single-GPU call (wx_group_sum + finalize, no exchange)
  graph      the eager step captured once into a HIP graph and replayed
  graph-loc  the same for the local call

and checks that the replayed steps return the eager step's groups.
usage: python tools/c3_step_probe.py [rows] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from warpdb_amd import _warpexec as wx  # noqa: E402
from warpdb_amd import distributed as wd  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    key = torch.empty(n, dtype=torch.int32, device="cuda")
    L = wx.make_launch(stream=s.cuda_stream)
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
    sq = wd.ShardedQuery(wd.Shard({"price": price, "quantity": key}, 0, n))
    sqt = wd.ShardedQuery(wd.Shard({"price": price, "quantity": key}, 0, n), flags=wx.F_TIME)
    cap = 4096
    lok = torch.empty(cap, dtype=torch.int32, device="cuda")
    los = torch.empty(cap, dtype=torch.float64, device="cuda")
    loc = torch.empty(cap, dtype=torch.int64, device="cuda")
    lng = torch.empty(1, dtype=torch.int64, device="cuda")


def eager():
    return sq.group_sum_device("price[idx]", "quantity[idx]", None, 0, cap)


def eager_timed():  # bench.py's step: HIP events around wx_group_sum (WX_F_TIME)
    return sqt.group_sum_device("price[idx]", "quantity[idx]", None, 0, cap)


def local():
    wx.group_sum(sq.table, "price[idx]", "quantity[idx]", None, sq.launch, 0, cap, lok.data_ptr(), los.data_ptr(),
                 loc.data_ptr(), d_n_groups=lng.data_ptr(), want_count=False)


def run(fn, label):
    with torch.cuda.stream(s):
        for _ in range(20):
            fn()
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
    k_ms, nl = wx.timing_read()
    kern = f"  wx_group_sum {k_ms / nl * 1e3:7.1f} us" if nl else ""
    print(f"{label:12s} {(t2 - t0) / steps * 1e6:8.1f} us/step  host issue {(t1 - t0) / steps * 1e6:8.1f} us/step"
          + kern, flush=True)


def snapshot():
    ok, osm, oc, ng = eager()
    s.synchronize()
    g = int(ng.item())
    return g, ok[:g].clone(), oc[:g].clone(), osm[:g].clone()


with torch.cuda.stream(s):
    ref = snapshot()
print(f"rows {n}, {ref[0]} groups, world {dist.get_world_size()}, exchange {sq.exchange}, "
      f"own stream communicator {sq.stream_comm}",
      flush=True)
for r in range(2):
    run(eager, "eager")
    run(eager_timed, "eager-timed")
    run(local, "local")
for label, fn in (("graph", eager), ("graph-loc", local)):
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.stream(s):
            fn()
            s.synchronize()
        with torch.cuda.graph(g, stream=s):
            fn()
    except Exception as e:  # report and go on: the probe's question is whether capture works
        print(f"{label}: capture failed: {type(e).__name__}: {e}", flush=True)
        continue
    for r in range(2):
        run(g.replay, label)
    if fn is eager:
        with torch.cuda.stream(s):
            g.replay()
            s.synchronize()
        _, ok, osm, oc, ng = (None,) + sq._group_bufs(cap)[6:]
        gg = int(ng.item())
        same = gg == ref[0] and torch.equal(ok[:gg], ref[1]) and torch.equal(oc[:gg], ref[2]) and torch.allclose(
            osm[:gg], ref[3], rtol=1e-12, atol=0)
        print(f"graph replay result {'equals' if same else 'DIFFERS FROM'} the eager step's", flush=True)
torch.cuda.synchronize()
wd.release_stream_comms()
dist.destroy_process_group()
