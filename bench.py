#!/usr/bin/env python3
"""Benchmark of the WarpDB execution path on MI355X (BASELINE.json metric).

Default workload (BASELINE.json `metric`, SURVEY.md 8(d) C2 shape at the
metric's 1B rows): a synthetic 2-column float32 table (price U[0,40),
quantity integer-valued U{1..100}) of 1e9 rows per GPU, resident in HBM,
and the query `price * quantity WHERE price > 15` through the C ABI
(ordered compaction: value + int32 shard-local row index per passing row).
One step = one query over the whole table.

Every step goes through the product's row-sharded path,
warpdb_amd.distributed.ShardedQuery, with the exchange each result needs
(one collective per query):
  project  all-gather of the per-shard passing counts (global placement)
  sum      all-reduce of {sum, count} as two doubles          (C4)
  group    ONE all-reduce of the key window + per-shard slots of out-of-window
           groups, merged on the device (wx_group_combine_slots)  (C3)
  topk     all-gather of one 520-byte candidate record per shard, merged on
           the device (wx_topk_merge)                             (C5)
  dense    none (WarpDB::query's dense contract, src/warpdb.cpp:243-256)
  sort     single GPU only (ORDER BY without LIMIT: projection + radix sort)

Scaling: --rows R is per GPU (weak, the default: 1e9); --total-rows T splits
T rows over the GPUs (strong; C4 is `--workload sum --total-rows 8e9`).
With --gpus N the driver runs one process per GPU under torchrun (RCCL): each
rank's exchanges run on its own RCCL communicator on the query stream
(include/warpcomm.h; `config.collectives` names it, WARPDB_STREAM_COMM=0
keeps torch.distributed's collectives).

--api runs the single-process C++ path instead (pywarpdb.ResidentShards:
one host thread and stream per device, ncclCommInitAll over devices
0..N-1 -- WarpDB::query_multi_gpu_sum / _group / _topk), for sum, group and
topk; its per-step time includes the collective and the host read-back.

Beside the headline (`secondary`, each line timed the same way and checked
after timing; `exchange_ms` = HIP events around the collective + device merge
on multi-rank runs, read from up to 50 steps after the timed ones;
`host_issue_ms` = the host's time to issue one step): SUM and GROUP BY on the
same shards, C2 at its own 1e8
rows per GPU, C5 (ORDER BY price DESC LIMIT 5 + discount()), and the
strong-scaled C3 (1e9 rows) and C4 (8e9 rows) lines over all GPUs.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Kernel arguments in device memory (a HIP runtime setting, read when HIP
# starts, so before torch is imported): the dependent kernels of a
# multi-rank GROUP BY step start sooner -- C3 strong at 1.25e8 rows per rank
# 0.1688 vs 0.1723-0.1731 ms per step, the 1e9-row lines unchanged
# (profiles/r03/s2/kernarg/).  An explicit setting in the environment wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "rows/sec + achieved HBM GB/s, 1B-row float32 project+filter, 1/2/4/8 GPU"
DISCOUNT_SRC = "__device__ float discount(float price, float rate) {\n    return price * rate;\n}\n"

# name: (query text, lowered expression, lowered condition, dominant kernel)
WORKLOADS = {
    "project": ("price * quantity WHERE price > 15", "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)",
                "wx_project_compact_deep"),
    "sum": ("SELECT SUM(price * 0.9) FROM t WHERE price > 20", "(price[idx] * 0.9f)", "(price[idx] > 20.0f)",
            "wx_reduce_sum"),
    "group": ("SELECT SUM(price) FROM t GROUP BY quantity", "price[idx]", "quantity[idx]", "wx_group_sum"),
    "topk": ("SELECT discount(price, 0.9) FROM t ORDER BY price DESC LIMIT 5", "price[idx]",
             "discount(price[idx], 0.9f)", "wx_topk_scan"),
    # WarpDB::query's own contract: dense float[N], 0.0f where WHERE fails
    "dense": ("price * quantity WHERE price > 15", "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)",
              "wx_project_dense"),
    # ORDER BY without LIMIT (query_sql): the projection, then the radix
    # sort (jit_sort_float, src/jit.cpp:283-307); roofline over the sort
    "sort": ("SELECT price FROM t ORDER BY price", "price[idx]", None, "wx_radix_hist + wx_radix_tile_k_fp_a"),
}
# bytes every row reads from HBM (the "HBM-read roofline" of BASELINE.md)
READ_BYTES = {"project": 8, "dense": 8, "group": 8, "sum": 4, "topk": 4, "sort": 4}
C4_TOTAL_ROWS = 8e9  # BASELINE.json configs[3]: 8B rows row-sharded over 1/2/4/8 GPUs
C3_TOTAL_ROWS = 1e9  # BASELINE.json configs[2]: 1B rows, GROUP BY 1K int32 keys (strong-scaled over N GPUs)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=float, default=1e9, help="rows per GPU (weak scaling)")
    p.add_argument("--total-rows", type=float, default=None, help="rows over all GPUs (strong scaling)")
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="project")
    p.add_argument("--api", action="store_true", help="single-process C++ multi-GPU path (sum, group)")
    p.add_argument("--cpu-sample", type=float, default=1e8,
                   help="rows for the CPU baseline sample (BASELINE.md's plan: 1e8)")
    p.add_argument("--cpu-threads", type=int, default=0, help="threads of the all-cores CPU run (0: all)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-check", action="store_true", help="skip the post-timing result check")
    p.add_argument("--no-secondary", action="store_true",
                   help="project only: skip the SUM / GROUP BY lines measured beside the headline")
    p.add_argument("--no-c4", action="store_true",
                   help="project only: skip the strong-scaled C4 SUM line (8e9 rows over all GPUs)")
    p.add_argument("--c4-rows", type=float, default=C4_TOTAL_ROWS,
                   help="rows over all GPUs of the C4 SUM line (BASELINE: 8e9)")
    p.add_argument("--no-c3", action="store_true",
                   help="project only: skip the strong-scaled C3 GROUP BY line (1e9 rows over all GPUs)")
    p.add_argument("--c3-rows", type=float, default=C3_TOTAL_ROWS,
                   help="rows over all GPUs of the strong-scaled C3 GROUP BY line (BASELINE: 1e9)")
    p.add_argument("--no-c2", action="store_true", help="project only: skip the C2 line (1e8 rows per GPU)")
    p.add_argument("--c2-rows", type=float, default=1e8, help="rows per GPU of the C2 line (BASELINE: 1e8)")
    p.add_argument("--no-c5", action="store_true",
                   help="project only: skip the C5 line (ORDER BY price DESC LIMIT 5 + discount())")
    p.add_argument("--keys", type=int, default=1024,
                   help="group: distinct int32 keys, uniform over [0, keys) (BASELINE C3: 1K)")
    return p.parse_args()


# ------------------------------------------------------------ CPU baseline
def host_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"cpu_model": model, "logical_cpus": os.cpu_count(), "usable_cpus": usable}


def cpu_threads_default() -> int:
    # the GPU box's share of the host (OMP_NUM_THREADS is set to it there)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return host_info()["usable_cpus"] or 1


def cores_reason(threads: int, info: dict) -> str:
    """Why the all-cores leg ran on `threads` threads."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) == threads and info.get("usable_cpus", 0) > threads:
        return (f"this one-GPU job's CPU share: the pool sets OMP_NUM_THREADS={env} per GPU; the host's "
                f"{info.get('usable_cpus')} logical CPUs are shared with the other GPUs' jobs, so more threads "
                f"would time other tenants' work, not the reference's")
    return f"every usable CPU of the host ({info.get('usable_cpus')})"


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
    return {"value": round(sample / dt, 1), "unit": "rows/s", "cores": 1, "kind": "port", "host": host_info(),
            "sample": f"{sample} synthetic price values, numpy stable sort (radix for float32) on one core, {dt:.2f} s"}


def cpu_baseline(query: str, sample: int, threads: int):
    """Reference CPU evaluator on the host: oracle/_ref (the reference's own
    eval_node, built from /root/reference) when present, else the C port.
    Single-threaded as the reference is; the all-cores run beside it splits
    the rows into contiguous ranges on std::threads."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if os.path.exists(harness):
        def run(t):
            r = subprocess.run([harness, "bench", str(sample), query, str(t)], capture_output=True, text=True,
                               timeout=900)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            return json.loads(line[-1]) if r.returncode == 0 and line else None

        one = run(1)
        if one:
            out = {"value": round(one["rows_per_s"], 1), "unit": "rows/s", "cores": 1, "kind": "reference",
                   "host": host_info(),
                   "sample": f"{sample} synthetic rows (same generator), '{query}', reference eval_node "
                             f"(src/warpdb.cpp:111-155) single thread, {one['seconds']:.2f} s"}
            if threads > 1:
                mt = run(threads)
                if mt:
                    info = host_info()
                    out["all_cores"] = {"value": round(mt["rows_per_s"], 1), "unit": "rows/s", "cores": threads,
                                        "seconds": round(mt["seconds"], 3),
                                        "why_cores": cores_reason(threads, info)}
            return out
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
    return {"value": round(sample / dt, 1), "unit": "rows/s", "cores": 1, "kind": "port", "host": host_info(),
            "sample": f"{sample} synthetic rows, '{query}', oracle/warpdb_oracle.c per-row interpreter "
                      f"single thread, {dt:.2f} s"}


def cpu_leg(args, workload):
    if args.no_cpu_baseline:
        return None
    q = {"project": "price * quantity WHERE price > 15", "dense": "price * quantity WHERE price > 15",
         "sum": "price * 0.9 WHERE price > 20", "group": "price", "topk": "price"}.get(workload)
    if workload == "sort":
        return cpu_sort_baseline(int(args.cpu_sample))
    return cpu_baseline(q, int(args.cpu_sample), args.cpu_threads or cpu_threads_default())


# ------------------------------------------------------------------ helpers
def columns_for(workload, keys=1024):
    """(name, dtype, seed, kind, lo, hi) of the columns a workload reads."""
    from warpdb_amd import _warpexec as wx

    price = ("price", wx.FLOAT32, 1, 0, 0.0, 40.0)
    if workload in ("sum", "topk", "sort"):
        return [price]
    if workload == "group":
        return [price, ("quantity", wx.INT32, 3, 1, 0, keys - 1)]  # C3: 1K int32 groups
    return [price, ("quantity", wx.FLOAT32, 2, 1, 1, 100)]


def line_common(args, world, n_total, elapsed, workload):
    return {
        "metric": METRIC if workload == "project" else f"rows/sec, {workload} ({WORKLOADS[workload][0]})",
        "value": round(n_total * args.steps / elapsed, 1),
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.total_rows else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded splitmix64 generator, generated in HBM)",
    }


def roofline(bytes_per_launch, kern_ms, read_bytes, kname, traffic, timing):
    traffic, traffic_source = traffic
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_source,
            "kernel": kname,
            "kernel_ms": round(kern_ms, 4), "bytes_per_launch": int(bytes_per_launch), "timing": timing,
            # BASELINE.md's "HBM-read roofline": input bytes only over the same time
            "read_only_frac": round(read_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


# PMC traffic profiles (profiles/pmc_<workload>.json, written by
# tools/pmc_record.py after tools/pmc_run.sh): per workload, the dominant
# kernels with their dispatches per query, and the kernel sources whose text
# the profile was collected against (wx_args.h + wx_common.hip + the family).
PMC_FAMILIES = {
    "project": ({"wx_project_compact_deep": 1}, ["wx_compact.hip"]),
    "dense": ({"wx_project_dense": 1}, ["wx_dense.hip"]),
    "sum": ({"wx_reduce_sum": 1}, ["wx_sum.hip"]),
    "group": ({"wx_group_sum": 1}, ["wx_group.hip"]),
    "topk": ({"wx_topk_scan": 1}, ["wx_topk.hip"]),
    "sort": ({"wx_radix_hist_": 1, "wx_radix_tile_": 4}, ["wx_radix.hip"]),
    "group_wide": ({"wx_group_part_": None}, ["wx_group_part.hip"]),  # every dispatch of the pipeline, once
}


def kernel_src_sha16(workload):
    import hashlib

    h = hashlib.sha256()
    kdir = os.path.join(ROOT, "warpdb_amd", "csrc", "kernels")
    for name in ["wx_args.h", "wx_common.hip"] + PMC_FAMILIES[workload][1]:
        with open(os.path.join(kdir, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(workload, n, keys=1024):
    """(HBM bytes per launch scaled to n rows, provenance).  The bytes are
    null when the profile is missing or was collected against other kernel
    sources than the ones in the tree (stale): re-run tools/pmc_run.sh."""
    if workload == "group" and keys > 2048:  # the many-key (partitioned) pipeline has its own passes
        workload = "group_wide"
    rel = f"profiles/pmc_{workload}.json"
    pmc = os.path.join(ROOT, rel)
    if not os.path.exists(pmc) or workload not in PMC_FAMILIES:
        return None, {"file": None}
    with open(pmc) as f:
        d = json.load(f)
    src = {"file": rel, "collected": d.get("collected"), "kernel_src_sha16": d.get("kernel_src_sha16"),
           "rows": d.get("rows")}
    cur = kernel_src_sha16(workload)
    src["current"] = d.get("kernel_src_sha16") == cur
    if not src["current"] or not d.get("rows"):
        src["stale_reason"] = f"kernel sources changed since collection (tree {cur})"
        return None, src
    return round(d["hbm_bytes_per_launch"] * n / d["rows"]), src


# ------------------------------------------------- result check
SECONDARY_WARM_S = 0.1  # secondary lines: warm-up steps worth >= 0.1 s beyond --warmup (clock ramp, timed())
CHECK_CHUNK = 1 << 28  # rows per torch pass of the check (bounds its temporaries)


def _mark(what):
    if os.environ.get("WARPDB_BENCH_VERBOSE"):
        print(f"[bench rank {os.environ.get('RANK', '0')}] {what} {time.strftime('%H:%M:%S')}", file=sys.stderr,
              flush=True)


def wd_group_doubles(world):
    from warpdb_amd import _warpexec as wx
    from warpdb_amd import distributed as wd

    return wx.group_slots_doubles(world, wd.group_slot_groups(world))


def group_capacity(keys):
    return max(4096, keys)


def self_check(workload, sq, cols, n, world, wd, torch, out_v=None, keys=1024):
    """One more query after the timed steps, its exchanged result checked
    against torch on each rank's shard (all-reduced): counts and row ids
    exact, float values bit for bit, double sums to 1e-12 relative.  Only
    elementwise ops, gathers and reductions -- no torch select / sort
    kernels, whose look-back scans crawl when several processes share a GPU.
    Raises (no JSON line) on a mismatch; returns a short description."""
    price = cols["price"]
    _, expr, aux, _ = WORKLOADS[workload]
    mark = _mark

    def red(x, op=torch.distributed.ReduceOp.SUM):
        t = torch.as_tensor(x, dtype=torch.float64, device="cuda").reshape(-1).clone()
        return wd.all_reduce_(t, op=op)  # the identity without a process group

    def chunks():
        for c0 in range(0, n, CHECK_CHUNK):
            yield c0, min(n, c0 + CHECK_CHUNK)

    if workload == "project":
        mark("check: compaction")
        vals, idx, off, total = sq.compact(expr, aux, idx_bytes=8)
        mark("check: compare")
        qty = cols["quantity"]
        want = sum(int((price[c0:c1] > 15.0).sum()) for c0, c1 in chunks())
        k = vals.numel()
        li = idx - sq.shard.row_base
        # a strictly ascending list of `want` passing shard rows IS the passing-row list
        ok = k == want and (k == 0 or (int(li[0]) >= 0 and int(li[-1]) < n))
        if ok and k:
            ok = bool((li[1:] > li[:-1]).all()) and bool((price[li] > 15.0).all())
        if not ok:
            raise SystemExit(f"check failed: compaction row ids ({k} rows, {want} passing)")
        if not torch.equal(vals.view(torch.int32), (price[li] * qty[li]).view(torch.int32)):
            raise SystemExit("check failed: compaction values differ")
        mark("check: all-reduce")
        if int(red(k)[0]) != total:
            raise SystemExit(f"check failed: global passing count {total}")
        return f"ok: {total} passing rows, ids and value bits equal torch on every shard"
    if workload == "dense":
        qty = cols["quantity"]
        for c0, c1 in chunks():
            p_, q_ = price[c0:c1], qty[c0:c1]
            want = torch.where(p_ > 15.0, p_ * q_, torch.zeros_like(p_))
            if not torch.equal(out_v[c0:c1].view(torch.int32), want.view(torch.int32)):
                raise SystemExit(f"check failed: dense output differs in rows [{c0}, {c1})")
        return "ok: dense output bits equal torch"
    if workload == "sort":
        for c0, c1 in chunks():
            a = out_v[c0:min(n, c1 + 1)]
            if not bool((a[1:] >= a[:-1]).all()):
                raise SystemExit(f"check failed: not sorted in [{c0}, {c1})")
        sums = red([price.double().sum().item(), out_v[:n].double().sum().item()])
        if abs(float(sums[0]) - float(sums[1])) > 1e-12 * abs(float(sums[0])):
            raise SystemExit("check failed: the sorted values are not a permutation of the input")
        return "ok: ascending, same sum as the input"
    if workload == "sum":
        got_s, got_c = sq.sum(expr, aux)
        acc = [0.0, 0]
        for c0, c1 in chunks():
            p_ = price[c0:c1]
            m = p_ > 20.0
            acc[0] += torch.where(m, p_ * 0.9, torch.zeros_like(p_)).double().sum().item()  # + 0.0 is exact
            acc[1] += int(m.sum().item())
        want = red(acc)
        if got_c != int(want[1]) or abs(got_s - float(want[0])) > 1e-12 * abs(float(want[0])):
            raise SystemExit(f"check failed: SUM {got_s} / {got_c} vs {float(want[0])} / {int(want[1])}")
        return f"ok: count {got_c} exact, sum {got_s:.6e} within 1e-12"
    if workload == "group":
        if keys > wd.GROUP_WINDOW_BINS:  # the timed many-key form: list records + wx_group_merge_lists
            gk, gs, gc = sq.group_sum_lists(expr, aux, None, group_capacity(keys))
        else:
            gk, gs, gc = sq.group_sum(expr, aux, None, 0, group_capacity(keys))
        key = cols["quantity"]
        ws = torch.zeros(keys, dtype=torch.float64, device="cuda")
        wc = torch.zeros(keys, dtype=torch.float64, device="cuda")
        for c0, c1 in chunks():
            # bincount (a privatised histogram) rather than index_add_, whose
            # per-row global atomics on 1K bins took ~15 s per 1e9-row check
            kk = key[c0:c1].long()
            ws += torch.bincount(kk, weights=price[c0:c1].double(), minlength=keys)[:keys]
            wc += torch.bincount(kk, minlength=keys)[:keys].double()
        ws, wc = red(ws), red(wc)
        # present keys in ascending order without a torch select kernel: the
        # result's keys must index bins holding rows, and their count must be
        # the number of such bins (keys ascending and inside [0, keys))
        m = gk.numel()
        kl = gk.long()
        ok = m == int((wc > 0).sum()) and (m == 0 or (int(kl[0]) >= 0 and int(kl[-1]) < keys))
        ok = ok and (m < 2 or bool((kl[1:] > kl[:-1]).all()))
        if not ok or not torch.equal(gc.double(), wc[kl]):
            raise SystemExit("check failed: GROUP BY keys / counts differ from torch")
        rel = (gs - ws[kl]).abs() / ws[kl].abs().clamp_min(1e-300)
        if m and float(rel.max()) > 1e-12:
            raise SystemExit("check failed: GROUP BY sums differ from torch beyond 1e-12")
        return f"ok: {m} groups, keys and counts exact, sums within 1e-12"
    if workload == "topk":
        tk, ti, tv = sq.topk(expr, None, aux, 5, True)
        # order statistics: the i-th best key t has <= i keys above it and >= i + 1 at or above it
        above = red([sum(int((price[c0:c1] > float(t)).sum()) for c0, c1 in chunks()) for t in tk.tolist()])
        at = red([sum(int((price[c0:c1] >= float(t)).sum()) for c0, c1 in chunks()) for t in tk.tolist()])
        if tk.numel() != 5 or any(int(above[i]) > i or int(at[i]) < i + 1 for i in range(5)):
            raise SystemExit(f"check failed: top-5 keys {tk.tolist()}")
        if not torch.equal(tv.view(torch.int32), (tk * 0.9).view(torch.int32)):
            raise SystemExit("check failed: discount(price, 0.9) values differ")
        return "ok: top-5 keys are the order statistics, discount() values bit-equal torch"
    return None


# ------------------------------------------------- one process per GPU
def main_ranks(args):
    import torch
    import torch.distributed as dist

    from warpdb_amd import _warpexec as wx
    from warpdb_amd import distributed as wd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # RCCL over xGMI, one GPU per rank.  WARPDB_DIST_BACKEND=gloo lets several
    # ranks share one GPU (rehearsal of the multi-rank path on a 1-GPU box);
    # its exchanges stage through host tensors.
    backend = os.environ.get("WARPDB_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    # WARPDB_EXCHANGE_ONE_RANK=1 (test hook): the exchanges run with one rank
    # too, so a one-GPU box runs the RCCL collectives of the multi-rank step
    coll = world > 1 or wd.exchange_one_rank()
    if coll:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    workload = args.workload
    if workload == "sort" and world > 1:
        raise SystemExit("--workload sort runs on one GPU (no distributed sort on the path)")

    n_total = int(args.total_rows) if args.total_rows else int(args.rows) * world
    b, e = wd.shard_range(n_total, world, rank)
    n = e - b
    stream = torch.cuda.current_stream().cuda_stream
    L = wx.make_launch(device=local, stream=stream, custom_src=DISCOUNT_SRC)
    cols = {}
    dmap = {wx.FLOAT32: torch.float32, wx.INT32: torch.int32}
    for name, dt, seed, kind, lo, hi in columns_for(workload, args.keys):
        t = torch.empty(max(1, n), dtype=dmap[dt], device="cuda")[:n]
        wx.fill_synthetic(t.data_ptr(), dt, n, seed, kind, lo, hi, L, row_base=b)
        cols[name] = t
    sq = wd.ShardedQuery(wd.Shard(cols, b, n), custom_src=DISCOUNT_SRC, flags=wx.F_TIME)
    query, expr, aux, kname = WORKLOADS[workload]
    if workload == "project" and os.environ.get("WARPDB_COMPACT_SCHED", "deep") == "ticket":
        kname = "wx_project_compact_ticket"
    counts = torch.zeros(1, dtype=torch.int64, device="cuda")

    if workload == "project":
        out_v = torch.empty(max(1, n), dtype=torch.float32, device="cuda")
        out_i = torch.empty(max(1, n), dtype=torch.int32, device="cuda")

        def step():
            sq.compact_device(expr, aux, out_v, out_i, 4, counts)
    elif workload == "dense":
        out_v = torch.empty(max(1, n), dtype=torch.float32, device="cuda")

        def step():
            wx.project_filter(sq.table, expr, aux, sq.launch, wx.MODE_DENSE_FILL, out_v.data_ptr(), 0, 4, 0)
    elif workload == "sort":
        out_v = torch.empty(max(1, n), dtype=torch.float32, device="cuda")

        # ORDER BY a bare float column with no WHERE: the sort reads the column
        # (the projection would be a copy), as WarpDB::query_sql does
        bare = re.fullmatch(r"(\w+)\[idx\]", expr)
        src = cols[bare.group(1)] if bare and bare.group(1) in cols and cols[bare.group(1)].dtype == torch.float32 \
            else None

        def step():
            if src is not None:
                wx.sort_float_from(src.data_ptr(), out_v.data_ptr(), n, True, sq.launch)  # synchronous
                return
            wx.project_filter(sq.table, expr, None, sq.launch_aux, wx.MODE_COMPACT, out_v.data_ptr(), 0, 4, 0,
                              d_count=counts.data_ptr())
            wx.sort_float(out_v.data_ptr(), n, True, sq.launch)  # synchronous, as jit_sort_float
    elif workload == "sum":
        res = torch.zeros(2, dtype=torch.float64, device="cuda")

        def step():
            sq.sum_device(expr, aux, res)
    elif workload == "group":
        def step():
            if coll and args.keys > wx.GROUP_WINDOW_BINS:
                # many keys: every shard's groups as one list record, ONE
                # all-gather, wx_group_merge_lists on the device
                sq.group_sum_lists_device(expr, aux, None, group_capacity(args.keys))
            else:
                sq.group_sum_device(expr, aux, None, 0, group_capacity(args.keys))
    else:
        def step():  # results stay in HBM like the other workloads' (no host round trip per query)
            sq.topk_merged_device(expr, None, aux, 5, True)

    verbose = os.environ.get("WARPDB_BENCH_VERBOSE")

    def mark(what):
        if verbose:
            print(f"[bench rank {rank}] {what} {time.strftime('%H:%M:%S')}", file=sys.stderr, flush=True)

    def timed(step_fn, warm_s=0.0, sq_ex=None):
        """W warm-up steps (secondary lines: and at least warm_s seconds of
        them), then exactly K steps between barrier + synchronize;
        (elapsed s, average timed-kernel ms, launches, exchange ms, host
        issue ms per step), max over ranks.  With sq_ex (a ShardedQuery), up
        to 50 more steps AFTER the timed region record events around each
        exchange (collective + device merge): its average is the fourth value
        (None on one rank).  Those events stay out of the timed steps: an
        event record with the default system-scope fence costs several us
        of stream time, ~10 % of a 1.25e8-row GROUP BY step."""
        for _ in range(args.warmup):
            step_fn()
        if warm_s > 0:
            # after any host-side pause (the previous line's check) the first
            # ~20 ms of launches run slower while the clocks ramp back up
            # (profiles/r03/thermal_group.txt: 1.18 vs 1.13 ms per GROUP BY)
            # the same number of extra steps on every rank (each step may hold a collective)
            torch.cuda.synchronize()
            w0 = time.perf_counter()
            step_fn()
            torch.cuda.synchronize()
            extra = min(2000, int(warm_s / max(1e-5, time.perf_counter() - w0)) + 1)
            if coll:
                t = torch.tensor([float(extra)], dtype=torch.float64, device="cuda")
                wd.all_reduce_(t, op=dist.ReduceOp.MAX)
                extra = int(t[0])
            for _ in range(extra):
                step_fn()
        wx.check(L)
        wx.timing_read()  # discard the warm-up launches
        mark("timed steps")
        if coll:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_fn()
        issued = time.perf_counter() - t0  # the host's time to issue the K steps
        torch.cuda.synchronize()
        if coll:
            dist.barrier()
        el = time.perf_counter() - t0
        k_ms, nl = wx.timing_read()
        wx.check(L)
        k_avg = k_ms / max(1, nl)
        ex_ms = None
        if sq_ex is not None and coll:  # exchange time: more steps after the timed region (same count on every rank)
            sq_ex.time_exchanges(min(50, args.steps))
            for _ in range(min(50, args.steps)):
                step_fn()
            ex_ms = sq_ex.exchange_ms()
            wx.timing_read()
            wx.check(L)
        if coll:
            t = torch.tensor([el, k_avg, -1.0 if ex_ms is None else ex_ms, issued], dtype=torch.float64,
                             device="cuda")
            wd.all_reduce_(t, op=dist.ReduceOp.MAX)
            el, k_avg, issued = float(t[0]), float(t[1]), float(t[3])
            ex_ms = None if float(t[2]) < 0 else round(float(t[2]), 4)
        return el, k_avg, nl, ex_ms, round(issued / max(1, args.steps) * 1e3, 4)

    mark("warm-up")
    elapsed, kern_avg_ms, launches, ex_main, issue_main = timed(step, sq_ex=sq)

    # algorithmic bytes per launch of the dominant kernel
    passing = int(counts.item()) if workload == "project" else None
    mark("check")
    check = None if args.no_check else self_check(workload, sq, cols, n, world, wd, torch,
                                                  out_v if workload in ("dense", "sort") else None, keys=args.keys)
    rb = READ_BYTES[workload]
    if workload == "project":
        bytes_per_launch = n * 8 + passing * 8  # 4 B value + 4 B int32 index per passing row
    elif workload == "dense":
        bytes_per_launch = n * 12
    elif workload == "group" and launches > args.steps:
        # many keys: the range-partitioned pipeline (probe, hist, scan, scatter,
        # LDS aggregation, emit) as one unit per step; algorithmic bytes are
        # still the 8 B/row the query reads (the roofline BASELINE prices)
        kern_avg_ms *= launches / max(1, args.steps)
        kname = "wx_group_part_* pipeline (sample + tiles + plan + agg + count + scan2 + emit)"
        bytes_per_launch = n * rb
    elif workload == "sort":  # histogram read + the tile passes that ran (read + write 4 B each)
        passes = max(0, round(launches / max(1, args.steps)) - 1)
        kern_avg_ms *= launches / max(1, args.steps)  # the sort's kernels as one unit: per step
        bytes_per_launch = n * (4 + 8 * passes)
        rb = 4 + 4 * passes
    else:
        bytes_per_launch = n * rb
    if rank == 0:
        line = line_common(args, world, n_total, elapsed, workload)
        line["config"] = {"workload": f"{query} ({workload})", "rows_per_gpu": n, "total_rows": n_total,
                          "columns": ", ".join(f"{c} {'i32' if t.dtype == torch.int32 else 'f32'}"
                                               for c, t in cols.items()),
                          "index": "int32 shard-local row index" if workload == "project" else None,
                          "exchange": {"project": "all-gather int64 counts", "sum": "all-reduce 2 x f64",
                                       "group": (f"one all-reduce of {wd_group_doubles(world)} x f64 (key window + "
                                                 f"{world} slots of out-of-window groups), wx_group_combine_slots"
                                                 if args.keys <= 2048 else
                                                 f"one all-gather of {world} group list records "
                                                 f"({group_capacity(args.keys)} groups each), wx_group_merge_lists"),
                                       "topk": "all-gather 520 B per shard, wx_topk_merge",
                                       "dense": "none", "sort": "none"}[workload] if coll else "none (1 GPU)",
                          "parallelism": f"row-sharded x{world}, one process per GPU"}
        if coll:
            line["config"]["collectives"] = ("RCCL on the query stream (the rank's own communicator, "
                                             "include/warpcomm.h)" if sq.stream_comm else
                                             f"torch.distributed ({dist.get_backend()})")
        if passing is not None:
            line["config"]["passing_rows_per_gpu"] = passing
        if workload == "sort":
            line["config"]["sort_input"] = ("the price column itself (ORDER BY a bare column, no WHERE: no projection "
                                            "copy, as WarpDB::query_sql)" if src is not None
                                            else "the compacted projection")
        line["check"] = check
        if ex_main is not None:
            line["exchange_ms"] = ex_main
        line["host_issue_ms"] = issue_main
        if workload == "group":
            line["config"]["distinct_keys"] = args.keys
        line["roofline"] = roofline(bytes_per_launch, kern_avg_ms, n * rb, kname, pmc_traffic(workload, n, args.keys),
                                    "HIP events around the dominant kernel on its stream (max over ranks)")
    # The other north-star aggregates on the same shards, timed the same way
    # (so the driver's 1/2/4/8-GPU runs also measure SUM -- C4's 8e9 rows at
    # 8 GPUs -- and GROUP BY scaling); reported beside the headline, not in it.
    secondary = {}

    def sec(key, wname, sqx, step_fn, cols_x, n_x, total_x, scaling, bytes_fn, extra=None):
        """One checked secondary line: timed like the headline, then its own
        self-check; `bytes_fn()` gives the dominant kernel's algorithmic
        bytes per launch on this rank (max over ranks is the kernel time)."""
        mark(f"secondary {key}")
        el_x, k_ms_x, _, ex_x, issue_x = timed(step_fn, SECONDARY_WARM_S, sq_ex=sqx)
        chk_x = None if args.no_check else self_check(wname, sqx, cols_x, n_x, world, wd, torch)
        d = {"query": WORKLOADS[wname][0]}
        d.update(extra or {})
        d.update({"value": round(total_x * args.steps / el_x, 1), "unit": "rows/s",
                  "ms_per_step": round(el_x / args.steps * 1e3, 4), "scaling": scaling,
                  "kernel": WORKLOADS[wname][3], "kernel_ms": round(k_ms_x, 4),
                  "frac": round(bytes_fn() / (k_ms_x * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "check": chk_x})
        if ex_x is not None:
            d["exchange_ms"] = ex_x
        d["host_issue_ms"] = issue_x
        secondary[key] = d

    if workload == "project" and not args.no_secondary:
        weak = "strong" if args.total_rows else "weak"
        qk = torch.empty(max(1, n), dtype=torch.int32, device="cuda")[:n]
        wx.fill_synthetic(qk.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L, row_base=b)
        for w2, cols2 in (("sum", {"price": cols["price"]}), ("group", {"price": cols["price"], "quantity": qk})):
            sq2 = wd.ShardedQuery(wd.Shard(cols2, b, n), custom_src=DISCOUNT_SRC, flags=wx.F_TIME)
            _, e2, a2, _ = WORKLOADS[w2]
            if w2 == "sum":
                res2 = torch.zeros(2, dtype=torch.float64, device="cuda")

                def step2():
                    sq2.sum_device(e2, a2, res2)
            else:
                def step2():
                    sq2.group_sum_device(e2, a2, None, 0, group_capacity(1024))
            sec(w2, w2, sq2, step2, cols2, n, n_total, weak, lambda: n * READ_BYTES[w2])
        del qk, sq2
        # C2 at its own size (BASELINE configs[1]: 100M rows): the first 1e8
        # rows of the resident columns (views, 1e8 per GPU), the same ordered
        # compaction + the count all-gather as the headline
        n2 = min(n, int(args.c2_rows))
        if n2 > 0 and not args.no_c2:
            cols2 = {"price": cols["price"][:n2], "quantity": cols["quantity"][:n2]}
            sq2 = wd.ShardedQuery(wd.Shard(cols2, b, n2), custom_src=DISCOUNT_SRC, flags=wx.F_TIME)
            cnt2 = torch.zeros(1, dtype=torch.int64, device="cuda")
            _, e2, a2, _ = WORKLOADS["project"]

            def step_c2():
                sq2.compact_device(e2, a2, out_v, out_i, 4, cnt2)
            sec("c2_1e8", "project", sq2, step_c2, cols2, n2, n2 * world, "weak",
                lambda: n2 * 8 + int(cnt2.item()) * 8,
                {"config": f"C2: {n2:.3g} rows per GPU (the first rows of the resident columns)",
                 "rows_per_gpu": n2})
            del sq2, cols2
        # C5 (BASELINE configs[4]): ORDER BY price DESC LIMIT 5 + discount()
        # over the 1e9-row price column on each rank; at N > 1 the record
        # all-gather + wx_topk_merge
        if not args.no_c5:
            sq5 = wd.ShardedQuery(wd.Shard({"price": cols["price"]}, b, n), custom_src=DISCOUNT_SRC, flags=wx.F_TIME)
            _, e5, a5, _ = WORKLOADS["topk"]

            def step_c5():
                sq5.topk_merged_device(e5, None, a5, 5, True)
            sec("c5_topk", "topk", sq5, step_c5, {"price": cols["price"]}, n, n_total, weak,
                lambda: n * READ_BYTES["topk"],
                {"config": f"C5: {n:.3g} rows per GPU, K = 5, discount() from the custom.cu hook"})
            del sq5
        # C3 as BASELINE states it, strong-scaled: 1e9 rows (price f32, 1K
        # int32 keys) over all ranks, 1e9 / N per GPU, each shard generated at
        # its global row numbers; GROUP BY + the one-collective exchange, so
        # the driver's 1/2/4/8-GPU runs measure GROUP BY speed-up on a fixed table.
        if not args.no_c3:
            c3_total = int(args.c3_rows)
            b3, e3 = wd.shard_range(c3_total, world, rank)
            n3 = e3 - b3
            p3 = torch.empty(max(1, n3), dtype=torch.float32, device="cuda")[:n3]
            k3 = torch.empty(max(1, n3), dtype=torch.int32, device="cuda")[:n3]
            wx.fill_synthetic(p3.data_ptr(), wx.FLOAT32, n3, 1, 0, 0.0, 40.0, L, row_base=b3)
            wx.fill_synthetic(k3.data_ptr(), wx.INT32, n3, 3, 1, 0, 1023, L, row_base=b3)
            cols3 = {"price": p3, "quantity": k3}
            sq3 = wd.ShardedQuery(wd.Shard(cols3, b3, n3), custom_src=DISCOUNT_SRC, flags=wx.F_TIME)
            _, e3x, a3x, _ = WORKLOADS["group"]

            def step3():
                sq3.group_sum_device(e3x, a3x, None, 0, group_capacity(1024))
            sec("c3_group_strong", "group", sq3, step3, cols3, n3, c3_total, "strong",
                lambda: n3 * READ_BYTES["group"],
                {"config": f"C3: {c3_total:.3g} rows over all GPUs (strong scaling)", "total_rows": c3_total,
                 "rows_per_gpu": n3})
            del p3, k3, sq3, cols3
        # C4 exactly as BASELINE states it: 8e9 rows over all ranks (strong
        # scaling, 8e9 / N per GPU; 32 GB resident at N = 1), SUM + all-reduce,
        # so the driver's 1/2/4/8-GPU runs measure C4's scaling curve.
        if not args.no_c4:
            c4_total = int(args.c4_rows)
            b4, e4 = wd.shard_range(c4_total, world, rank)
            n4 = e4 - b4
            p4 = torch.empty(max(1, n4), dtype=torch.float32, device="cuda")[:n4]
            wx.fill_synthetic(p4.data_ptr(), wx.FLOAT32, n4, 1, 0, 0.0, 40.0, L, row_base=b4)
            sq4 = wd.ShardedQuery(wd.Shard({"price": p4}, b4, n4), custom_src=DISCOUNT_SRC, flags=wx.F_TIME)
            _, e4x, a4x, _ = WORKLOADS["sum"]
            res4 = torch.zeros(2, dtype=torch.float64, device="cuda")

            def step4():
                sq4.sum_device(e4x, a4x, res4)
            sec("c4_sum_strong", "sum", sq4, step4, {"price": p4}, n4, c4_total, "strong",
                lambda: n4 * READ_BYTES["sum"],
                {"config": f"C4: {c4_total:.3g} rows over all GPUs (strong scaling)", "total_rows": c4_total,
                 "rows_per_gpu": n4})
            del p4, sq4
    if rank == 0:
        if secondary:
            line["secondary"] = secondary
        line["cpu_baseline"] = cpu_leg(args, workload) if world == 1 else None
        print(json.dumps(line), flush=True)
    if coll:
        torch.cuda.synchronize()
        wd.release_stream_comms()
        dist.destroy_process_group()


# ------------------------------------------- single process, C++ multi-GPU
def main_api(args):
    from warpdb_amd import _warpexec as wx
    from warpdb_amd import pywarpdb as pw

    workload = args.workload
    if workload not in ("sum", "group", "topk"):
        raise SystemExit("--api covers the C++ multi-GPU paths: --workload sum | group | topk")
    if workload == "topk":  # the C++ path reads the custom.cu hook from $WARPDB_CUSTOM_PATH (src/jit.cpp:65-73)
        import tempfile
        hook = os.path.join(tempfile.mkdtemp(prefix="warpdb_bench_"), "custom.cu")
        with open(hook, "w") as f:
            f.write(DISCOUNT_SRC)
        os.environ["WARPDB_CUSTOM_PATH"] = hook
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--api is one process driving every GPU; do not launch it under torchrun")
    devs = args.gpus
    n_total = int(args.total_rows) if args.total_rows else int(args.rows) * devs
    dmap = {wx.FLOAT32: pw.DataType.Float32, wx.INT32: pw.DataType.Int32}
    cols = [(nm, dmap[dt], seed, kind, lo, hi) for nm, dt, seed, kind, lo, hi in columns_for(workload)]
    shards = pw.ResidentShards.synthetic(n_total, cols, devs)
    query, expr, aux, kname = WORKLOADS[workload]

    if workload == "sum":
        def step():
            return shards.sum(expr, aux)
    elif workload == "group":
        def step():
            return shards.group_sum(expr, aux, "", 0)
    else:
        def step():
            return shards.topk(expr, "", aux, 5, True)

    for _ in range(args.warmup):
        step()
    # then warm-up worth >= 0.2 s more, as the torchrun lines do: the first
    # ~20 ms of launches after a host-side pause run below the clocks' rate
    # (profiles/r03/thermal_group.txt)
    w0 = time.perf_counter()
    step()
    for _ in range(min(2000, int(0.2 / max(1e-5, time.perf_counter() - w0)))):
        step()
    shards.take_timing()  # discard the warm-up's (nothing is timed yet)
    shards.set_timing(True, False)  # HIP events around each shard's main kernel (no system fence)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    elapsed = time.perf_counter() - t0
    shards.set_timing(False, False)
    kt = shards.take_timing()
    # the exchange (collective + merge, an event pair per device) from more
    # steps after the timed region, as the torchrun line reads exchange_ms
    shards.set_timing(False, True)
    for _ in range(min(50, args.steps)):
        step()
    shards.set_timing(False, False)
    ex_ms = shards.take_timing()["exchange_ms"]
    n_max = max(e - b for _, b, e in shards.ranges())
    line = line_common(args, shards.num_shards, n_total, elapsed, workload)
    line["config"] = {"workload": f"{query} ({workload})", "rows_per_gpu": n_max, "total_rows": n_total,
                      "api": "pywarpdb.ResidentShards (WarpDB::query_multi_gpu_sum / _group / _topk)",
                      "exchange": ({"sum": "ncclAllReduce 2 x f64",
                                    "group": f"ncclAllReduce {api_group_doubles(shards.num_shards)} x f64 (key window + "
                                             f"per-shard slots), wx_group_combine_slots",
                                    "topk": "ncclAllGather 520 B per shard, wx_topk_merge"}[workload] +
                                   " over ncclCommInitAll(devices 0..n-1)")
                                  if shards.num_shards > 1 or os.environ.get("WARPDB_EXCHANGE_ONE_RANK") == "1"
                                  else "none (1 GPU)",
                      "parallelism": f"row-sharded x{shards.num_shards}, one process, one thread + stream per GPU"}
    rb = READ_BYTES[workload]
    kern_ms = kt["kernel_ms"] if kt["launches"] else elapsed / args.steps * 1e3
    line["roofline"] = roofline(n_max * rb, kern_ms, n_max * rb, kname, pmc_traffic(workload, n_max),
                                "HIP events around each shard's main kernel on its device's stream "
                                "(ResidentShards.set_timing, WX_F_TIME), average over the timed steps, slowest device"
                                if kt["launches"] else "whole step (no kernel events were read)")
    line["kernel_launches"] = kt["launches"]
    line["exchange_ms"] = None if ex_ms is None else round(ex_ms, 4)
    line["check"] = api_check(workload, step(), n_total, shards)
    line["cpu_baseline"] = cpu_leg(args, workload) if shards.num_shards == 1 else None
    print(json.dumps(line), flush=True)


def api_group_doubles(shards):
    """ResidentShards::group_sum's exchange buffer (multi_gpu.cpp: 64 groups
    per slot, at most 4096 slot groups in all)."""
    from warpdb_amd import _warpexec as wx

    return wx.group_slots_doubles(shards, max(1, min(64, 4096 // shards)))


def api_check(workload, res, n_total, shards):
    """The C++ path's result against torch on the same rows, regenerated on
    the first GPU chunk by chunk (the shards' synthetic columns come from the
    same counter-based generator, wx_fill_synthetic, at their global row
    numbers): the torchrun line's checks -- counts exact, sums within 1e-12
    relative, top-5 keys the order statistics and discount() values
    bit-equal."""
    import numpy as np
    import torch

    from warpdb_amd import _warpexec as wx

    L = wx.make_launch(stream=torch.cuda.current_stream().cuda_stream)
    spec = {c[0]: c for c in columns_for(workload)}

    def chunks():
        for c0 in range(0, n_total, CHECK_CHUNK):
            c1 = min(n_total, c0 + CHECK_CHUNK)
            out = {}
            for nm, (_, dt, seed, kind, lo, hi) in spec.items():
                t = torch.empty(c1 - c0, dtype=torch.float32 if dt == wx.FLOAT32 else torch.int32, device="cuda")
                wx.fill_synthetic(t.data_ptr(), dt, c1 - c0, seed, kind, lo, hi, L, row_base=c0)
                out[nm] = t
            yield c0, c1, out

    if workload == "sum":
        got_s, got_c = res
        acc = [0.0, 0]
        for _, _, c in chunks():
            p_ = c["price"]
            m = p_ > 20.0
            acc[0] += torch.where(m, p_ * 0.9, torch.zeros_like(p_)).double().sum().item()
            acc[1] += int(m.sum().item())
        if got_c != acc[1] or abs(got_s - acc[0]) > 1e-12 * abs(acc[0]):
            raise SystemExit(f"check failed: SUM {got_s} / {got_c} vs {acc[0]} / {acc[1]}")
        return f"ok: count {got_c} exact, sum {got_s:.6e} within 1e-12 of torch"
    if workload == "group":
        gk, gs, gc = (np.asarray(x) for x in res)
        keys = int(spec["quantity"][5]) + 1
        ws = torch.zeros(keys, dtype=torch.float64, device="cuda")
        wc = torch.zeros(keys, dtype=torch.float64, device="cuda")
        for _, _, c in chunks():
            kk = c["quantity"].long()
            ws += torch.bincount(kk, weights=c["price"].double(), minlength=keys)[:keys]
            wc += torch.bincount(kk, minlength=keys)[:keys].double()
        ws, wc = ws.cpu().numpy(), wc.cpu().numpy()
        present = np.nonzero(wc > 0)[0]
        if not np.array_equal(gk.astype(np.int64), present) or not np.array_equal(gc.astype(np.float64), wc[present]):
            raise SystemExit("check failed: GROUP BY keys / counts differ from torch")
        rel = np.abs(gs - ws[present]) / np.maximum(np.abs(ws[present]), 1e-300)
        if len(rel) and float(rel.max()) > 1e-12:
            raise SystemExit("check failed: GROUP BY sums differ from torch beyond 1e-12")
        return f"ok: {len(gk)} groups, keys and counts exact, sums within 1e-12 of torch"
    tk, rows, tv = (np.asarray(x) for x in res)
    above = [0] * len(tk)
    at = [0] * len(tk)
    for _, _, c in chunks():
        p_ = c["price"]
        for i, t in enumerate(tk.tolist()):
            above[i] += int((p_ > float(t)).sum())
            at[i] += int((p_ >= float(t)).sum())
    if len(tk) != 5 or any(above[i] > i or at[i] < i + 1 for i in range(5)):
        raise SystemExit(f"check failed: top-5 keys {tk.tolist()}")
    want = (tk.astype(np.float32) * np.float32(0.9)).astype(np.float32)
    if not np.array_equal(tv.view(np.uint32), want.view(np.uint32)):
        raise SystemExit("check failed: discount(price, 0.9) values differ")
    return "ok: top-5 keys are the order statistics, discount() values bit-equal"


def main():
    args = parse()
    if args.api:
        main_api(args)
    else:
        main_ranks(args)


if __name__ == "__main__":
    main()
