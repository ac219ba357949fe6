#!/usr/bin/env python3
"""Benchmark of the WarpDB execution path on MI355X (BASELINE.json metric).

Default workload (BASELINE.json `metric`, SURVEY.md 8d C2 shape at the
metric's 1B rows): a synthetic 2-column float32 table (price U[0,40),
quantity integer-valued U{1..100}) of 1e9 rows per GPU, resident in HBM,
and the query `price * quantity WHERE price > 15` through the C ABI
(wx_project_filter, ordered compaction: value + int32 row index per passing
row).  One step = one query over the whole table.  With --gpus N (one process
per GPU, torchrun) each rank owns a contiguous 1e9-row shard (weak scaling);
the only exchange is an RCCL all-gather of the per-shard passing counts that
places every shard's rows in the global result (src/multi_gpu_utils.cpp:5-63
concatenates shards in device order).

Other workloads (--workload): sum (C4: price * 0.9 WHERE price > 20 with an
RCCL all-reduce of the SUM), group (C3: SUM(price) GROUP BY int32 quantity,
1K groups), topk (C5: ORDER BY price DESC LIMIT 5 with discount()).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "rows/sec + achieved HBM GB/s, 1B-row float32 project+filter, 1/2/4/8 GPU"
DISCOUNT_SRC = "__device__ float discount(float price, float rate) {\n    return price * rate;\n}\n"

WORKLOADS = {
    # name: (query, kernel name for rocprof, read bytes/row, column spec)
    "project": ("price * quantity WHERE price > 15", "wx_project_compact"),
    "sum": ("SELECT SUM(price * 0.9) FROM t WHERE price > 20", "wx_reduce_sum"),
    "group": ("SELECT SUM(price) FROM t GROUP BY quantity", "wx_group_sum"),
    "topk": ("SELECT discount(price, 0.9) FROM t ORDER BY price DESC LIMIT 5", "wx_topk_scan"),
    # WarpDB::query's own contract (src/warpdb.cpp:243-256): dense float[N],
    # 0.0f where WHERE fails, written in the same pass
    "dense": ("price * quantity WHERE price > 15", "wx_project_dense"),
    # ORDER BY without LIMIT (query_sql): the projection, then the radix sort
    # (jit_sort_float, src/jit.cpp:283-307); roofline over the sort's kernels
    "sort": ("SELECT price FROM t ORDER BY price", "wx_radix_hist + wx_radix_tile_k_f_a"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=float, default=1e9, help="rows per GPU")
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="project")
    p.add_argument("--cpu-sample", type=float, default=5e7, help="rows for the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def cpu_sort_baseline(sample: int):
    """ORDER BY on the host: the sample's values stable-sorted by numpy on one
    core (the reference's own sort is a one-thread GPU bubble sort,
    src/jit.cpp:283-307, with no CPU counterpart)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth  # noqa: E402

    v = synth.c2_table(sample)["price"]
    t0 = time.perf_counter()
    np.sort(v, kind="stable")
    dt = time.perf_counter() - t0
    return {"value": round(sample / dt, 1), "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": f"{sample} synthetic price values, numpy stable sort (radix for float32) on one core, {dt:.2f} s"}


def cpu_baseline(query: str, sample: int):
    """Reference CPU evaluator on the host: oracle/_ref (the reference's own
    eval_node, built from /root/reference) when present, else the C port."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if os.path.exists(harness):
        r = subprocess.run([harness, "bench", str(sample), query], capture_output=True, text=True, timeout=900)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode == 0 and line:
            d = json.loads(line[-1])
            return {"value": round(d["rows_per_s"], 1), "unit": "rows/s", "cores": 1, "kind": "reference",
                    "sample": f"{sample} synthetic rows (same generator), '{query}', reference eval_node "
                              f"(src/warpdb.cpp:111-155) single thread, {d['seconds']:.2f} s"}
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # noqa: E402  (checker only: the CPU baseline leg)
    import synth  # noqa: E402

    cols = synth.c2_table(sample)
    t = oracle_lib.HostTable(cols)
    t0 = time.perf_counter()
    oracle_lib.scan_baseline(t, query)
    dt = time.perf_counter() - t0
    del np
    return {"value": round(sample / dt, 1), "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": f"{sample} synthetic rows, '{query}', oracle/warpdb_oracle.c per-row interpreter "
                      f"single thread, {dt:.2f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from warpdb_amd import _warpexec as wx

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # RCCL over xGMI, one GPU per rank.  WARPDB_DIST_BACKEND=gloo lets several
    # ranks share one GPU (rehearsal of the multi-rank path on a 1-GPU box);
    # its exchanges go through host tensors.
    backend = os.environ.get("WARPDB_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def all_gather(out, inp):
        if backend == "gloo":
            parts = [torch.empty_like(inp, device="cpu") for _ in range(world)]
            dist.all_gather(parts, inp.cpu())
            out.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(out, inp)

    def all_reduce(t, op=dist.ReduceOp.SUM):
        if backend == "gloo":
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)

    def barrier():
        if world > 1:
            dist.barrier()

    n = int(args.rows)
    row_base = rank * n
    stream = torch.cuda.current_stream().cuda_stream
    L = wx.make_launch(device=local, stream=stream, custom_src=DISCOUNT_SRC)
    Lt = wx.make_launch(device=local, stream=stream, custom_src=DISCOUNT_SRC, flags=wx.F_TIME)

    price = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L, row_base=row_base)
    if args.workload == "group":
        qty = torch.empty(n, dtype=torch.int32, device="cuda")
        wx.fill_synthetic(qty.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L, row_base=row_base)
        qdt = wx.INT32
    else:
        qty = torch.empty(n, dtype=torch.float32, device="cuda")
        wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 2, 1, 1, 100, L, row_base=row_base)
        qdt = wx.FLOAT32
    table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()), wx.Column("quantity", qdt, qty.data_ptr())])
    query, kname = WORKLOADS[args.workload]
    if args.workload == "project" and os.environ.get("WARPDB_COMPACT_SCHED", "deep") == "deep":
        kname = "wx_project_compact_deep"
    counts = torch.zeros(1, dtype=torch.int64, device="cuda")
    gathered = torch.zeros(world, dtype=torch.int64, device="cuda")

    if args.workload == "project":
        out_v = torch.empty(n, dtype=torch.float32, device="cuda")
        out_i = torch.empty(n, dtype=torch.int32, device="cuda")

        def step(Lx):
            wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", Lx, wx.MODE_COMPACT,
                              out_v.data_ptr(), out_i.data_ptr(), 4, 0, d_count=counts.data_ptr())
            if world > 1:  # global placement of each shard's rows
                all_gather(gathered, counts)
    elif args.workload == "dense":
        out_v = torch.empty(n, dtype=torch.float32, device="cuda")

        def step(Lx):
            wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", Lx, wx.MODE_DENSE_FILL,
                              out_v.data_ptr(), 0, 4, 0)
    elif args.workload == "sort":
        out_v = torch.empty(n, dtype=torch.float32, device="cuda")

        def step(Lx):
            wx.project_filter(table, "price[idx]", None, L, wx.MODE_COMPACT, out_v.data_ptr(), 0, 4, 0,
                              d_count=counts.data_ptr())
            wx.sort_float(out_v.data_ptr(), n, True, Lx)  # synchronous, as jit_sort_float
    elif args.workload == "sum":
        res = torch.zeros(2, dtype=torch.float64, device="cuda")

        def step(Lx):
            wx.reduce_sum(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", Lx, d_out=res.data_ptr(),
                          want_host=False)
            if world > 1:
                all_reduce(res[:1])
    elif args.workload == "group":
        cap = 4096
        keys = torch.empty(cap, dtype=torch.int32, device="cuda")
        sums = torch.empty(cap, dtype=torch.float64, device="cuda")
        cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
        ng = torch.zeros(1, dtype=torch.int64, device="cuda")

        def step(Lx):
            wx.group_sum(table, "price[idx]", "quantity[idx]", None, Lx, 0, cap, keys.data_ptr(), sums.data_ptr(),
                         cnts.data_ptr(), d_n_groups=ng.data_ptr(), want_count=False)
            if world > 1:  # dense 1K-bin partials: keys are identical on every shard
                all_reduce(sums[:1024])
    else:
        tk = torch.empty(5, dtype=torch.float32, device="cuda")
        ti = torch.empty(5, dtype=torch.int64, device="cuda")
        tv = torch.empty(5, dtype=torch.float32, device="cuda")
        allk = torch.empty(world * 5, dtype=torch.float32, device="cuda")

        def step(Lx):
            wx.topk(table, "price[idx]", None, "discount(price[idx], 0.9f)", 5, True, Lx, tk.data_ptr(),
                    ti.data_ptr(), tv.data_ptr(), row_base=row_base, d_count=counts.data_ptr(), want_count=False)
            if world > 1:
                all_gather(allk, tk)

    for _ in range(args.warmup):
        step(L)
    wx.check(L)
    wx.timing_read()  # discard
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(Lt)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms, launches = wx.timing_read()
    wx.check(L)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        km = torch.tensor([kern_ms / max(1, launches)], dtype=torch.float64, device="cuda")
        all_reduce(km, op=dist.ReduceOp.MAX)
        kern_avg_ms = km.item()
    else:
        kern_avg_ms = kern_ms / max(1, launches)
    if args.workload == "sort":  # the sort's kernels as one unit: per step, not per launch
        kern_avg_ms *= launches / max(1, args.steps)

    # algorithmic bytes per launch of the dominant kernel
    passing = int(counts.item()) if args.workload in ("project",) else None
    if args.workload == "project":
        bytes_per_launch = n * 8 + passing * 8
    elif args.workload in ("sum", "topk"):
        bytes_per_launch = n * 4
    elif args.workload == "dense":
        bytes_per_launch = n * 12
    elif args.workload == "sort":  # histogram read + 4 passes of read + write
        bytes_per_launch = n * (4 + 4 * 8)
    else:
        bytes_per_launch = n * 8
    achieved = bytes_per_launch / (kern_avg_ms * 1e-3) / 1e9
    read_bytes = n * (4 if args.workload in ("sum", "topk") else 8)
    if args.workload == "sort":
        read_bytes = n * (4 + 4 * 4)

    total_rows = n * world * args.steps
    value = total_rows / elapsed
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            d = json.load(f)
        if d.get("rows"):
            traffic = round(d["hbm_bytes_per_launch"] * n / d["rows"])

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        q = "price * quantity WHERE price > 15" if args.workload in ("project", "dense") else {
            "sum": "price * 0.9 WHERE price > 20", "group": "price", "topk": "price", "sort": "price"}[args.workload]
        cpu = cpu_sort_baseline(int(args.cpu_sample)) if args.workload == "sort" else cpu_baseline(q, int(args.cpu_sample))

    if rank == 0:
        line = {
            "metric": METRIC if args.workload == "project" else f"rows/sec, 1B-row {args.workload}",
            "value": round(value, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded splitmix64 generator, generated in HBM)",
            "config": {"workload": f"{query} ({args.workload})", "rows_per_gpu": n, "total_rows": n * world,
                       "columns": "price f32, quantity " + ("i32" if qdt == wx.INT32 else "f32"),
                       "index": "int32 shard-local row index" if args.workload == "project" else None,
                       "parallelism": f"row-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": kname, "kernel_ms": round(kern_avg_ms, 4),
                         "bytes_per_launch": bytes_per_launch,
                         # BASELINE.md's "HBM-read roofline": input bytes only (8 B/row for
                         # project / group, 4 B/row for sum / top-K) over the same time
                         "read_only_frac": round(read_bytes / (kern_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "cpu_baseline": cpu,
        }
        if passing is not None:
            line["config"]["passing_rows_per_gpu"] = passing
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
