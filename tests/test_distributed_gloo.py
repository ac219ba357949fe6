"""Multi-process (world_size 2, gloo, CPU) tests of the row-sharded path.

The per-shard compute is the oracle here (no GPU in this container); what is
under test is the sharding plan and every exchange of warpdb_amd.distributed
(count all-gather -> global placement, SUM all-reduce, GROUP BY merge, top-K
merge), whose combined result must equal the oracle over the whole table.
The same exchange code runs on RCCL in bench.py and ShardedQuery on GPUs.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def group_partials_emulated(keys, sums, counts, key_lo):
    """What wx_group_partials leaves for one shard (include/warpexec.h): the
    dense window [sums | counts as f64 | out-of-window group count] and the
    out-of-window groups.  The device kernel itself is covered by the GPU tests."""
    W = 2048
    win = np.zeros(2 * W + 1, np.float64)
    inside = (keys >= key_lo) & (keys < key_lo + W)
    win[keys[inside] - key_lo] = sums[inside]
    win[W + keys[inside] - key_lo] = counts[inside]
    win[2 * W] = float((~inside).sum())
    return win, keys[~inside].astype(np.int32), sums[~inside], counts[~inside]


def group_combine_emulated(win, key_lo, xk, xs, xc):
    """wx_group_combine's contract: ascending keys over window bins + extras."""
    W = 2048
    bins = np.nonzero(win[W:2 * W])[0]
    keys = np.concatenate([xk.astype(np.int64), bins + key_lo])
    sums = np.concatenate([xs, win[bins]])
    cnts = np.concatenate([xc, win[W + bins].astype(np.int64)])
    o = np.argsort(keys, kind="stable")
    return keys[o].astype(np.int32), sums[o], cnts[o]


def _worker(rank: int, world: int, port: int, n: int, errq):
    try:
        sys.path[:0] = [ROOT, HERE]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist

        import oracle_lib as ora
        import synth
        from warpdb_amd import distributed as wd

        dist.init_process_group("gloo", rank=rank, world_size=world)
        b, e = wd.shard_range(n, world, rank)
        full2, full3 = synth.c2_table(n), synth.c3_table(n)
        loc2 = ora.HostTable(synth.c2_table(e - b, row_base=b))
        loc3 = ora.HostTable(synth.c3_table(e - b, row_base=b))

        # compaction: local results + global placement
        v, i = ora.project_filter(loc2, "price * quantity", "price > 15")
        off, total, counts = wd.exchange_counts(len(i))
        rv, ri = ora.project_filter(ora.HostTable(full2), "price * quantity", "price > 15")
        assert total == len(ri)
        assert np.array_equal(ri[off: off + len(i)], i + b)
        assert np.array_equal(rv[off: off + len(v)].view(np.uint32), v.view(np.uint32))

        # SUM
        s, c = ora.reduce_sum(loc2, "price * 0.9", "price > 20")
        gs, gc = wd.allreduce_sum(s, c)
        rs, rc = ora.reduce_sum(ora.HostTable(full2), "price * 0.9", "price > 20")
        assert gc == rc and abs(gs - rs) <= 1e-9 * abs(rs)

        # GROUP BY: the general merge, and the product's exchange (dense
        # window all-reduce + merge of the out-of-window groups only).  With
        # key_lo = 512 half of the 1024 keys fall outside the window.
        k, sm, cn = ora.group_sum(loc3, "price", "quantity")
        gk, gsum, gcnt = wd.merge_groups(torch.from_numpy(k), torch.from_numpy(sm), torch.from_numpy(cn), len(k))
        rk, rsum, rcnt = ora.group_sum(ora.HostTable(full3), "price", "quantity")
        assert np.array_equal(gk.numpy(), rk) and np.array_equal(gcnt.numpy(), rcnt)
        assert np.array_equal(gsum.numpy(), rsum)  # exact: float values summed in double
        for key_lo in (0, 512, -5000):
            win, xk, xs, xc = group_partials_emulated(k, sm, cn, key_lo)
            wt = torch.from_numpy(win)
            wd.exchange_group_window(wt)
            n_extra_total = int(wt[2 * wd.GROUP_WINDOW_BINS].item())
            outside = int(((rk < key_lo) | (rk >= key_lo + wd.GROUP_WINDOW_BINS)).sum())
            assert (n_extra_total > 0) == (outside > 0) and n_extra_total >= outside  # shards' counts, summed
            mk = np.zeros(0, np.int32); ms = np.zeros(0); mc = np.zeros(0, np.int64)
            if n_extra_total:
                a, b_, c_ = wd.merge_groups(torch.from_numpy(xk), torch.from_numpy(xs), torch.from_numpy(xc), len(xk))
                mk, ms, mc = a.numpy(), b_.numpy(), c_.numpy()
            ck, cs, cc = group_combine_emulated(wt.numpy(), key_lo, mk, ms, mc)
            assert np.array_equal(ck, rk) and np.array_equal(cc, rcnt) and np.array_equal(cs, rsum), key_lo

        # SUM through the product's one-collective layout {sum, count as f64}
        out = torch.tensor([s, float(c)], dtype=torch.float64)
        wd.exchange_sum_device(out)
        assert int(out[1]) == rc and abs(float(out[0]) - rs) <= 1e-9 * abs(rs)

        # top-K with ties (quantised keys) in both directions
        for desc in (True, False):
            t = {"p": np.floor(synth.uniform_f32(e - b, 1, 0, 40, row_base=b)).astype(np.float32)}
            tk, ti, tv = ora.topk(ora.HostTable(t), "p", 5, desc)
            mk, mi, mv = wd.merge_topk(torch.from_numpy(tk), torch.from_numpy(ti + b), torch.from_numpy(tv),
                                       len(tk), 5, desc)
            full = {"p": np.floor(synth.uniform_f32(n, 1, 0, 40)).astype(np.float32)}
            rk2, ri2, _ = ora.topk(ora.HostTable(full), "p", 5, desc)
            assert np.array_equal(mk.numpy(), rk2) and np.array_equal(mi.numpy(), ri2)
            # the device-side merge (no host round trip): k slots per shard,
            # unused ones filled with junk and masked by the shard's count
            m = len(tk)
            pk = torch.full((5,), float("nan")); pi = torch.full((5,), -7, dtype=torch.int64)
            pv = torch.full((5,), 123.0)
            pk[:m] = torch.from_numpy(tk); pi[:m] = torch.from_numpy(ti + b); pv[:m] = torch.from_numpy(tv)
            dk, di, dv, dn = wd.merge_topk_device(pk, pi, pv, torch.tensor([m]), 5, desc)
            c = int(dn[0])
            assert c == len(rk2)
            assert np.array_equal(dk[:c].numpy().view(np.uint32), mk.numpy().view(np.uint32))
            assert np.array_equal(di[:c].numpy(), mi.numpy()) and np.array_equal(dv[:c].numpy(), mv.numpy())
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:  # report to the parent
        import traceback

        errq.put(f"rank {rank}: {ex!r}\n{traceback.format_exc()}")
        raise


@pytest.mark.parametrize("n", [1, 7, 100_003])
def test_two_rank_exchanges_match_oracle(n):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    msgs = []
    while not errq.empty():
        msgs.append(errq.get())
    assert all(p.exitcode == 0 for p in procs), "\n".join(msgs)


def test_shard_range_matches_plan():
    from warpdb_amd import distributed as wd
    from warpdb_amd import pywarpdb as pw

    for n, w in [(10, 4), (3, 8), (8_000_000_000, 8), (1_000_000_007, 2)]:
        plan = [(b, e) for _, b, e in pw.plan_shards(n, w)]
        ranges = [wd.shard_range(n, w, r) for r in range(w)]
        assert [r for r in ranges if r[0] < r[1]] == plan
