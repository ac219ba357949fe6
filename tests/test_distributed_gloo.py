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


def group_slots_emulated(win, xk, xs, xc, world, rank, slot_groups, n_extra=None):
    """What wx_group_partials_slots leaves for one shard: the window, then
    world slots of 1 + 3 * slot_groups doubles -- this shard's count and first
    slot_groups (key, sum, count) triples, zeros in every other slot."""
    sl = 1 + 3 * slot_groups
    slots = np.zeros(world * sl, np.float64)
    m = len(xk) if n_extra is None else n_extra
    slots[rank * sl] = m
    for j in range(min(len(xk), slot_groups)):
        slots[rank * sl + 1 + 3 * j: rank * sl + 4 + 3 * j] = (xk[j], xs[j], xc[j])
    return np.concatenate([win, slots])


def group_combine_slots_emulated(ex, world, slot_groups, key_lo):
    """wx_group_combine_slots' contract: -1 / -2 status, else the slots' groups
    summed per key in slot order and merged with the window (ascending keys)."""
    W = 2048
    sl = 1 + 3 * slot_groups
    slots = ex[2 * W + 1:].reshape(world, sl)
    cnt = slots[:, 0]
    if (cnt < 0).any():
        return -1
    if (cnt > slot_groups).any():
        return -2
    acc = {}
    for r in range(world):
        for j in range(int(cnt[r])):
            k, sm, c = slots[r, 1 + 3 * j: 4 + 3 * j]
            a = acc.setdefault(int(k), [0.0, 0])
            a[0] += sm
            a[1] += int(c)
    ks = sorted(acc)
    return group_combine_emulated(ex[:2 * W + 1], key_lo, np.array(ks, np.int32),
                                  np.array([acc[k][0] for k in ks]), np.array([acc[k][1] for k in ks], np.int64))


def group_list_record(keys, sums, counts, cap, count=None):
    """One shard's group list record (wx_group_merge_lists layout) as bytes:
    int64 count | int32 keys[cap] padded to 8 B | f64 sums[cap] | int64 counts[cap]."""
    from warpdb_amd import _warpexec as wx

    nbytes, so, co = wx.group_list_layout(cap)
    rec = np.zeros(nbytes, np.uint8)
    m = len(keys)
    rec[0:8] = np.array([m if count is None else count], np.int64).view(np.uint8)
    rec[8:8 + 4 * m] = np.asarray(keys, np.int32).view(np.uint8)
    rec[so:so + 8 * m] = np.asarray(sums, np.float64).view(np.uint8)
    rec[co:co + 8 * m] = np.asarray(counts, np.int64).view(np.uint8)
    return rec


def group_merge_lists_emulated(allr, n_lists, cap, window, key_lo):
    """wx_group_merge_lists' contract: -1 on a bad list count, else equal keys
    summed in list order, merged with the window's non-empty bins."""
    from warpdb_amd import _warpexec as wx

    nbytes, so, co = wx.group_list_layout(cap)
    recs = allr.reshape(n_lists, nbytes)
    acc = {}
    for rec in recs:
        m = int(rec[0:8].view(np.int64)[0])
        if m < 0 or m > cap:
            return -1
        ks, ss, cs = rec[8:8 + 4 * m].view(np.int32), rec[so:so + 8 * m].view(np.float64), rec[co:co + 8 * m].view(
            np.int64)
        for j in range(m):
            a = acc.setdefault(int(ks[j]), [None, 0])
            a[0] = ss[j] if a[0] is None else a[0] + ss[j]
            a[1] += int(cs[j])
    kk = sorted(acc)
    xk, xs, xc = (np.array(kk, np.int32), np.array([acc[k][0] for k in kk], np.float64),
                  np.array([acc[k][1] for k in kk], np.int64))
    if window is None:
        return xk, xs, xc
    return group_combine_emulated(window, key_lo, xk, xs, xc)


def topk_record(keys, vals, rows):
    """One wx_topk_record (include/warpexec.h) as bytes: unused slots junk."""
    rec = np.zeros(520, np.uint8)
    kk = np.full(32, np.nan, np.float32); vv = np.full(32, 123.0, np.float32); rr = np.full(32, -7, np.int64)
    m = len(keys)
    kk[:m], vv[:m], rr[:m] = keys, vals, rows
    rec[0:128] = kk.view(np.uint8); rec[128:256] = vv.view(np.uint8); rec[256:512] = rr.view(np.uint8)
    rec[512:520] = np.array([m], np.int64).view(np.uint8)
    return rec


def topk_merge_emulated(allr, k, desc):
    """wx_topk_merge's contract over gathered records: better key first (NaN
    last, -0.0 == +0.0), then the smaller row."""
    recs = allr.reshape(-1, 520)
    cand = []
    for rec in recs:
        m = int(rec[512:520].view(np.int64)[0])
        ks, vs, rs = rec[0:128].view(np.float32), rec[128:256].view(np.float32), rec[256:512].view(np.int64)
        cand += [(ks[j], vs[j], rs[j]) for j in range(m)]

    def order(c):
        key = float(c[0])
        return (1 if np.isnan(key) else 0, 0.0 if np.isnan(key) else (-key if desc else key) + 0.0, int(c[2]))

    cand.sort(key=order)
    cand = cand[:k]
    return (np.array([c[0] for c in cand], np.float32), np.array([c[2] for c in cand], np.int64),
            np.array([c[1] for c in cand], np.float32))


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
        # host-staged exchanges build no RCCL communicator of their own (a
        # collective decision: every rank returns the same without a call)
        assert wd.enable_stream_comm() is False and wd.stream_comm() is None
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
        # every shard's whole group list, ONE all-gather of the fixed-size
        # records, the wx_group_merge_lists contract (no window)
        CAP = 1100
        allr = wd.all_gather(torch.from_numpy(group_list_record(k, sm, cn, CAP)))
        gk, gsum, gcnt = group_merge_lists_emulated(allr.numpy(), world, CAP, None, 0)
        rk, rsum, rcnt = ora.group_sum(ora.HostTable(full3), "price", "quantity")
        assert np.array_equal(gk, rk) and np.array_equal(gcnt, rcnt)
        assert np.allclose(gsum, rsum, rtol=1e-12, atol=0)
        for key_lo in (0, 512, -5000):
            win, xk, xs, xc = group_partials_emulated(k, sm, cn, key_lo)
            wt = torch.from_numpy(win)
            wd.exchange_group_window(wt)
            n_extra_total = int(wt[2 * wd.GROUP_WINDOW_BINS].item())
            outside = int(((rk < key_lo) | (rk >= key_lo + wd.GROUP_WINDOW_BINS)).sum())
            assert (n_extra_total > 0) == (outside > 0) and n_extra_total >= outside  # shards' counts, summed
            mk = np.zeros(0, np.int32); ms = np.zeros(0); mc = np.zeros(0, np.int64)
            if n_extra_total:
                allr = wd.all_gather(torch.from_numpy(group_list_record(xk, xs, xc, CAP)))
                mk, ms, mc = group_merge_lists_emulated(allr.numpy(), world, CAP, None, 0)
            ck, cs, cc = group_combine_emulated(wt.numpy(), key_lo, mk, ms, mc)
            assert np.array_equal(ck, rk) and np.array_equal(cc, rcnt), key_lo
            assert np.allclose(cs, rsum, rtol=1e-12, atol=0), key_lo

        # SUM through the product's one-collective layout {sum, count as f64}
        out = torch.tensor([s, float(c)], dtype=torch.float64)
        wd.exchange_sum_device(out)
        assert int(out[1]) == rc and abs(float(out[0]) - rs) <= 1e-9 * abs(rs)

        # GROUP BY in ONE collective (wx_group_partials_slots layout): the
        # window all-reduce also gathers every shard's slot of out-of-window
        # groups; slot sizes 64 (all fit) and 1 (overflow -> the -2 merge path)
        for key_lo in (0, 512, -5000):
            win, xk, xs, xc = group_partials_emulated(k, sm, cn, key_lo)
            for S in (64, 1):
                ex = torch.from_numpy(group_slots_emulated(win, xk, xs, xc, world, rank, S))
                wd.all_reduce_(ex)
                counts = wd.group_slot_counts(ex, world, S)
                assert wd.group_exchange_error(counts, 1 << 16) is None
                res = group_combine_slots_emulated(ex.numpy(), world, S, key_lo)
                if res == -2:  # the fallback: every shard's whole list record, one all-gather, the list merge
                    assert max(counts) > S
                    allr = wd.all_gather(torch.from_numpy(group_list_record(xk, xs, xc, CAP)))
                    res = group_merge_lists_emulated(allr.numpy(), world, CAP, ex.numpy()[:2 * 2048 + 1], key_lo)
                else:
                    assert max(counts) <= S
                ck, cs, cc = res
                assert np.array_equal(ck, rk) and np.array_equal(cc, rcnt), (key_lo, S)
                assert np.allclose(cs, rsum, rtol=1e-12, atol=0), (key_lo, S)
        # an overflow on ONE shard only is seen by every rank in the combined
        # buffer, so both raise the same error (no rank waits alone in a collective)
        win, xk, xs, xc = group_partials_emulated(k, sm, cn, 512)
        bad = {0: None, 1: -1}.get(rank)
        ex = torch.from_numpy(group_slots_emulated(win, xk, xs, xc, world, rank, 64, n_extra=bad))
        wd.all_reduce_(ex)
        errs = wd.group_exchange_error(wd.group_slot_counts(ex, world, 64), 1 << 16)
        assert errs is not None and "shard 1" in errs, errs
        # a list overflow on ONE shard: every rank's merge of the gathered records returns -1
        allr = wd.all_gather(torch.from_numpy(group_list_record(xk, xs, xc, CAP, count=bad)))
        assert (group_merge_lists_emulated(allr.numpy(), world, CAP, None, 0) == -1) == (world > 1)
        cap_small = wd.group_exchange_error(wd.group_slot_counts(
            torch.from_numpy(group_slots_emulated(win, xk, xs, xc, 1, 0, 64)), 1, 64), 3)
        assert (cap_small is not None) == (len(xk) > 3)

        # top-K with ties (quantised keys) in both directions: each shard's
        # wx_topk_record, ONE all-gather of the records, the wx_topk_merge contract
        for desc in (True, False):
            t = {"p": np.floor(synth.uniform_f32(e - b, 1, 0, 40, row_base=b)).astype(np.float32)}
            tk, ti, tv = ora.topk(ora.HostTable(t), "p", 5, desc)
            rec = torch.from_numpy(topk_record(tk, tv, ti + b))
            allr = wd.exchange_topk_records(rec)
            assert allr.numel() == 520 * world
            mk, mi, mv = topk_merge_emulated(allr.numpy(), 5, desc)
            full = {"p": np.floor(synth.uniform_f32(n, 1, 0, 40)).astype(np.float32)}
            rk2, ri2, _ = ora.topk(ora.HostTable(full), "p", 5, desc)
            assert np.array_equal(mk.view(np.uint32), rk2.view(np.uint32)) and np.array_equal(mi, ri2)
            assert np.array_equal(mv.view(np.uint32), rk2.view(np.uint32))  # SELECT = the key here
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


def _registry_worker(port: int, errq):
    try:
        sys.path[:0] = [ROOT, HERE]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from warpdb_amd import distributed as wd

        dist.init_process_group("gloo", rank=0, world_size=1)
        assert wd.enable_stream_comm() is False and wd.stream_comm() is None
        first = wd._COMMS["WORLD"][0]
        dist.destroy_process_group()
        # a new default group: the same registry key ("WORLD"), another object
        dist.init_process_group("gloo", rank=0, world_size=1)
        assert wd.stream_comm() is None and "WORLD" not in wd._COMMS  # the stale entry is dropped
        assert wd.enable_stream_comm() is False and wd._COMMS["WORLD"][0] is not first
        # an entry left by an earlier group never hands out its communicator
        wd._COMMS["WORLD"] = (first, 1, 0, object())
        assert wd.stream_comm() is None
        wd._COMMS["WORLD"] = (dist.distributed_c10d._get_default_group(), 2, 0, object())  # other size
        assert wd.stream_comm() is None
        wd.release_stream_comms()
        dist.destroy_process_group()
    except BaseException as ex:  # noqa: BLE001
        import traceback

        errq.put(f"{ex!r}\n{traceback.format_exc()}")
        raise


def test_stream_comm_registry_follows_the_process_group():
    """a communicator cached for one process group is never reused
    by a later group of the same name (torch reuses names; the default group
    is always "WORLD") -- the entry is re-checked against the group object,
    its size and rank on every lookup."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    p = ctx.Process(target=_registry_worker, args=(_free_port(), errq))
    p.start()
    p.join(timeout=120)
    msgs = []
    while not errq.empty():
        msgs.append(errq.get())
    assert p.exitcode == 0, "\n".join(msgs)


def test_shard_range_matches_plan():
    from warpdb_amd import distributed as wd
    from warpdb_amd import pywarpdb as pw

    for n, w in [(10, 4), (3, 8), (8_000_000_000, 8), (1_000_000_007, 2)]:
        plan = [(b, e) for _, b, e in pw.plan_shards(n, w)]
        ranges = [wd.shard_range(n, w, r) for r in range(w)]
        assert [r for r in ranges if r[0] < r[1]] == plan


def test_enable_stream_comm_without_process_group():
    """with no process group initialised, the public
    enable_stream_comm returns False (nothing to exchange over) instead of
    raising from torch's default-group lookup."""
    import torch.distributed as dist

    from warpdb_amd import distributed as wd

    if dist.is_initialized():
        pytest.skip("a process group is initialised in this process")
    assert wd.enable_stream_comm() is False
    assert wd.stream_comm() is None
