"""GPU tests of the round-3 exchange kernels of the row-sharded path.

* wx_group_partials_slots + an element-wise sum of the shards' buffers (what
  the ONE all-reduce computes) + wx_group_combine_slots, against the oracle
  over the whole table: 1..64 shards (views of one table on cuda:0), keys
  inside and outside the dense window, slots large enough and too small (the
  -2 status, then the variable-size merge and wx_group_combine), and a
  shard's general-key table overflow (-1).
* wx_topk_merge over real per-shard wx_topk records, against the oracle:
  heavy ties, NaN, +/-0.0, fewer rows than K, both directions, K = 1..32.
* The multi-rank bench under torchrun with RCCL (the default backend) when
  more than one GPU is visible -- skipped on a one-GPU box.
* The same multi-rank step, ResidentShards and WarpDB::query_multi_gpu_*
  with a ONE-rank communicator (WARPDB_EXCHANGE_ONE_RANK=1): on a one-GPU
  box this executes the RCCL all-reduce / all-gather calls and the buffers
  they hand to the exchange kernels.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as ora
import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from warpdb_amd import _warpexec as wx  # noqa: E402
from test_gpu_parity import dev_table, launch, bits  # noqa: E402
from test_gpu_multi import _shard_views  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = wx.GROUP_WINDOW_BINS


def _slots_partials(table, world, rank, S, key_lo, cond=None, cap=1 << 14):
    nd = wx.group_slots_doubles(world, S)
    ex = torch.full((nd,), float("nan"), dtype=torch.float64, device="cuda")
    xk = torch.empty(cap, dtype=torch.int32, device="cuda")
    xs = torch.empty(cap, dtype=torch.float64, device="cuda")
    xc = torch.empty(cap, dtype=torch.int64, device="cuda")
    nx = wx.group_partials_slots(table, "price[idx]", "quantity[idx]", cond, launch(), key_lo, ex.data_ptr(), world,
                                 rank, S, cap, xk.data_ptr(), xs.data_ptr(), xc.data_ptr(), want_count=True)
    return ex, xk, xs, xc, nx


def _combine_slots(ex, world, S, key_lo, cap=1 << 14):
    ok = torch.empty(cap, dtype=torch.int32, device="cuda")
    os_ = torch.empty(cap, dtype=torch.float64, device="cuda")
    oc = torch.empty(cap, dtype=torch.int64, device="cuda")
    ng = torch.empty(1, dtype=torch.int64, device="cuda")
    wx.group_combine_slots(ex.data_ptr(), world, S, key_lo, launch(), cap, ok.data_ptr(), os_.data_ptr(),
                           oc.data_ptr(), d_n_groups=ng.data_ptr())
    torch.cuda.synchronize()
    return ok, os_, oc, int(ng.item())


@pytest.mark.parametrize("shards,S", [(1, 64), (2, 64), (3, 64), (8, 64), (8, 1), (8, 512), (64, 64), (2, 4096 // 2)])
@pytest.mark.parametrize("key_lo", [0, 512, -100_000, 900])
def test_group_slots_match_oracle(shards, S, key_lo):
    n = 300_007
    cols = synth.c3_table(n)
    total = None
    lists = []
    sl = 1 + 3 * S
    for r, (_, t) in enumerate(_shard_views(cols, shards)):
        if t is None:  # an empty shard still contributes its (zero) buffer
            t = wx.Table(0, [wx.Column("price", wx.FLOAT32, 0), wx.Column("quantity", wx.INT32, 0)])
        ex, xk, xs, xc, nx = _slots_partials(t, shards, r, S, key_lo, cond="(price[idx] < 35.0f)")
        assert not torch.isnan(ex).any()
        h = ex.cpu().numpy()
        slots = h[wx.GROUP_EXCHANGE_DOUBLES:].reshape(shards, sl)
        assert slots[r, 0] == nx and int(h[2 * W]) == nx
        assert not np.any(np.delete(slots, r, axis=0))  # the other shards' slots are zero
        m = min(nx, S)  # the slot holds the first S groups, ascending
        trip = slots[r, 1:1 + 3 * m].reshape(m, 3)
        assert np.array_equal(trip[:, 0], xk[:m].cpu().numpy()) and np.array_equal(trip[:, 1], xs[:m].cpu().numpy())
        assert np.array_equal(trip[:, 2], xc[:m].cpu().numpy())
        total = ex.clone() if total is None else total + ex  # the all-reduce
        lists.append((xk[:nx], xs[:nx], xc[:nx]))
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", "price < 35")
    ok, os_, oc, g = _combine_slots(total, shards, S, key_lo)
    if g == wx.GROUP_NEEDS_MERGE:  # some shard's groups outgrew its slot: the list-record merge
        assert max(x[0].numel() for x in lists) > S
        cap = 1 << 14
        recs = _list_records([(a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy()) for a, b, c in lists], cap)
        g = wx.group_merge_lists(recs.data_ptr(), shards, cap, total.data_ptr(), key_lo, launch(), cap,
                                 ok.data_ptr(), os_.data_ptr(), oc.data_ptr(), want_count=True)
    else:
        assert max(x[0].numel() for x in lists) <= S
    assert np.array_equal(ok[:g].cpu().numpy(), rk) and np.array_equal(oc[:g].cpu().numpy(), rc)
    np.testing.assert_allclose(os_[:g].cpu().numpy(), rs, rtol=1e-12, atol=0)
    if shards == 1:
        assert np.array_equal(os_[:g].cpu().numpy(), rs)


def test_group_slots_deterministic_and_exact_sum_order():
    """Equal keys from several slots add in slot order: two combines of the
    same buffer are bit-identical, and a key present in every slot sums to
    the slot-order double sum."""
    world, S = 4, 8
    nd = wx.group_slots_doubles(world, S)
    ex = torch.zeros(nd, dtype=torch.float64)
    sl = 1 + 3 * S
    vals = [1e16, 1.0, -1e16, 1.0]  # order-sensitive in double
    for r in range(world):
        base = wx.GROUP_EXCHANGE_DOUBLES + r * sl
        ex[base] = 2
        ex[base + 1: base + 4] = torch.tensor([-7.0, vals[r], 1.0], dtype=torch.float64)
        ex[base + 4: base + 7] = torch.tensor([5000.0 + r, 2.0, 3.0], dtype=torch.float64)
    exd = ex.cuda()
    a = _combine_slots(exd, world, S, 0)
    b = _combine_slots(exd, world, S, 0)
    assert a[3] == b[3] == 5
    assert torch.equal(a[1][:5], b[1][:5])
    want = ((1e16 + 1.0) + -1e16) + 1.0
    assert a[0][:5].cpu().tolist() == [-7, 5000, 5001, 5002, 5003]
    assert a[1][0].item() == want and a[2][0].item() == 4
    assert a[1][1:5].cpu().tolist() == [2.0] * 4 and a[2][1:5].cpu().tolist() == [3] * 4


def test_group_slots_table_overflow_is_minus_one():
    """More than 4096 distinct out-of-window keys with capacity <= 4096: the
    shard's table cannot be sorted for the finalize (-1 in its slot), and
    the combine reports -1 whatever the other slots hold."""
    n = 20_000
    cols = {"price": np.ones(n, np.float32), "quantity": (np.arange(n) % 9000).astype(np.int32)}
    table, _ = dev_table(cols)
    cap = 4096
    ex = torch.full((wx.group_slots_doubles(2, 64),), float("nan"), dtype=torch.float64, device="cuda")
    xk = torch.empty(cap, dtype=torch.int32, device="cuda")
    xs = torch.empty(cap, dtype=torch.float64, device="cuda")
    xc = torch.empty(cap, dtype=torch.int64, device="cuda")
    wx.group_partials_slots(table, "price[idx]", "quantity[idx]", None, launch(0), 0, ex.data_ptr(), 2, 1, 64, cap,
                            xk.data_ptr(), xs.data_ptr(), xc.data_ptr())  # asynchronous: no error raised here
    with pytest.raises(wx.WarpExecError) as e:  # the shard's own flag, reported (and cleared) by the check
        wx.check(launch())
    assert e.value.status == wx.WX_ERR_UNSUPPORTED
    h = ex.cpu().numpy()
    assert h[wx.GROUP_EXCHANGE_DOUBLES + (1 + 3 * 64)] == -1.0
    assert _combine_slots(ex, 2, 64, 0)[3] == -1


def test_group_slots_bad_arguments():
    ex = torch.zeros(wx.group_slots_doubles(2, 64), dtype=torch.float64, device="cuda")
    for world, S in ((0, 64), (2, 0), (2, 4096), (2000, 1)):
        with pytest.raises(wx.WarpExecError) as e:
            wx.group_combine_slots(ex.data_ptr(), world, S, 0, launch(), 0, 0, 0, 0)
        assert e.value.status == wx.WX_ERR_INVALID


def _list_records(groups, cap, counts=None):
    """Gathered group list records (wx_group_merge_lists layout) on the
    device from per-list (keys, sums, counts) arrays; counts[r] overrides a
    record's count word."""
    nbytes, so, co = wx.group_list_layout(cap)
    buf = np.zeros(max(1, len(groups)) * nbytes, np.uint8)
    for r, (k, sm, c) in enumerate(groups):
        rec = buf[r * nbytes:(r + 1) * nbytes]
        m = len(k)
        cw = m if counts is None or counts[r] is None else counts[r]
        rec[0:8] = np.array([cw], np.int64).view(np.uint8)
        rec[8:8 + 4 * m] = np.asarray(k, np.int32).view(np.uint8)
        rec[so:so + 8 * m] = np.asarray(sm, np.float64).view(np.uint8)
        rec[co:co + 8 * m] = np.asarray(c, np.int64).view(np.uint8)
    return torch.from_numpy(buf).cuda()


def _merge_lists_ref(groups, window=None, key_lo=0):
    """wx_group_merge_lists' contract: equal keys summed in list order (the
    first list's sum, then the others added), merged with the non-empty bins
    of the window (ascending keys)."""
    acc = {}
    for k, sm, c in groups:
        for j in range(len(k)):
            a = acc.get(int(k[j]))
            acc[int(k[j])] = [float(sm[j]), int(c[j])] if a is None else [a[0] + float(sm[j]), a[1] + int(c[j])]
    if window is not None:
        for b in range(W):
            if window[W + b] != 0.0:
                assert key_lo + b not in acc
                acc[key_lo + b] = [float(window[b]), int(window[W + b])]
    ks = sorted(acc)
    return (np.array(ks, np.int64), np.array([acc[x][0] for x in ks], np.float64),
            np.array([acc[x][1] for x in ks], np.int64))


def _merge_lists(recs, n_lists, cap, window=None, key_lo=0, capacity=1 << 16):
    ok = torch.full((max(1, capacity),), -7, dtype=torch.int32, device="cuda")
    os_ = torch.empty(max(1, capacity), dtype=torch.float64, device="cuda")
    oc = torch.empty(max(1, capacity), dtype=torch.int64, device="cuda")
    ng = torch.empty(1, dtype=torch.int64, device="cuda")
    wx.group_merge_lists(recs.data_ptr(), n_lists, cap, window.data_ptr() if window is not None else 0, key_lo,
                         launch(), capacity, ok.data_ptr(), os_.data_ptr(), oc.data_ptr(), d_n_groups=ng.data_ptr())
    torch.cuda.synchronize()
    return ok, os_, oc, int(ng.item())


def _random_lists(rng, n_lists, cap, lo, hi, window_lo=None):
    """n_lists sorted unique key lists of random length <= cap over [lo, hi),
    none inside [window_lo, window_lo + W); random sums (signs, magnitudes)."""
    out = []
    for _ in range(n_lists):
        m = int(rng.integers(0, cap + 1))
        pool = np.arange(lo, hi, dtype=np.int64)
        if window_lo is not None:
            pool = pool[(pool < window_lo) | (pool >= window_lo + W)]
        m = min(m, pool.size)
        k = np.sort(rng.choice(pool, m, replace=False))
        sm = rng.standard_normal(m) * 10.0 ** rng.integers(-3, 12, m)
        c = rng.integers(1, 1 << 40, m)
        out.append((k, sm, c))
    return out


@pytest.mark.parametrize("n_lists,cap", [(1, 1), (1, 1000), (2, 7), (3, 1000), (8, 5000), (64, 300), (17, 1)])
@pytest.mark.parametrize("with_window", [False, True])
def test_group_merge_lists_matches_reference(n_lists, cap, with_window):
    """Random overlapping sorted lists (some empty), with and without a
    window: keys, counts and sum BITS equal the list-order reference."""
    rng = np.random.default_rng(n_lists * 1000 + cap + with_window)
    key_lo = int(rng.integers(-3000, 3000)) if with_window else 0
    groups = _random_lists(rng, n_lists, cap, -6000, 6000, key_lo if with_window else None)
    window = None
    if with_window:
        w = np.zeros(2 * W + 1)
        used = rng.random(W) < 0.3
        w[:W][used] = rng.standard_normal(int(used.sum())) * 1e6
        w[W:2 * W][used] = rng.integers(1, 1000, int(used.sum()))
        window = torch.from_numpy(w).cuda()
    recs = _list_records(groups, cap)
    ok, os_, oc, g = _merge_lists(recs, n_lists, cap, window, key_lo)
    rk, rs, rc = _merge_lists_ref(groups, window.cpu().numpy() if window is not None else None, key_lo)
    assert g == len(rk)
    assert np.array_equal(ok[:g].cpu().numpy(), rk) and np.array_equal(oc[:g].cpu().numpy(), rc)
    assert np.array_equal(os_[:g].cpu().numpy().view(np.uint64), rs.view(np.uint64))  # bit for bit, list order
    again = _merge_lists(recs, n_lists, cap, window, key_lo)  # deterministic
    assert again[3] == g and torch.equal(again[1][:g], os_[:g])


def test_group_merge_lists_bad_counts_and_capacity():
    rng = np.random.default_rng(3)
    groups = _random_lists(rng, 4, 100, 0, 1000)
    for bad in (-1, 101, 1 << 40):  # a shard whose table / list overflowed: -1 for everyone
        recs = _list_records(groups, 100, counts=[None, bad, None, None])
        assert _merge_lists(recs, 4, 100)[3] == -1
        with pytest.raises(wx.WarpExecError) as e:
            wx.group_merge_lists(recs.data_ptr(), 4, 100, 0, 0, launch(), 0, 0, 0, 0, want_count=True)
        assert e.value.status == wx.WX_ERR_CAPACITY
    # fewer output slots than groups: the first `capacity` written, the full count reported
    recs = _list_records(groups, 100)
    rk, rs, rc = _merge_lists_ref(groups)
    ok, os_, oc, g = _merge_lists(recs, 4, 100, capacity=5)
    assert g == len(rk) and np.array_equal(ok[:5].cpu().numpy(), rk[:5])
    with pytest.raises(wx.WarpExecError) as e:
        wx.group_merge_lists(recs.data_ptr(), 4, 100, 0, 0, launch(), 5, ok.data_ptr(), os_.data_ptr(),
                             oc.data_ptr(), want_count=True)
    assert e.value.status == wx.WX_ERR_CAPACITY
    # all lists empty, window only
    w = np.zeros(2 * W + 1)
    w[[0, 5, W - 1]] = [1.5, -2.0, 3.0]
    w[[W, W + 5, 2 * W - 1]] = [1, 2, 3]
    recs = _list_records([(np.zeros(0), np.zeros(0), np.zeros(0))] * 3, 10)
    ok, os_, oc, g = _merge_lists(recs, 3, 10, torch.from_numpy(w).cuda(), -100)
    assert g == 3 and ok[:3].cpu().tolist() == [-100, -95, -100 + W - 1] and os_[:3].cpu().tolist() == [1.5, -2.0, 3.0]
    for n_lists, cap in ((0, 10), (1025, 1), (2, 0)):
        with pytest.raises(wx.WarpExecError) as e:
            wx.group_merge_lists(recs.data_ptr(), n_lists, cap, 0, 0, launch(), 0, 0, 0, 0)
        assert e.value.status == wx.WX_ERR_INVALID


@pytest.mark.parametrize("shards", [1, 2, 5, 8])
def test_group_merge_lists_many_keys_against_oracle(shards, monkeypatch):
    """The many-key row-sharded GROUP BY as ShardedQuery.group_sum_lists runs
    it: every shard's whole wx_group_sum (the range-partitioned kernels above
    2^20 rows) written into its list record, the records gathered, merged on
    the device -- against the oracle over the whole table (2^21 + 7 rows,
    200 000 distinct keys)."""
    monkeypatch.setenv("WARPDB_GP_MIN_ROWS", "1")
    n = (1 << 21) + 7
    cols = {"price": synth.uniform_f32(n, 1, 0.0, 40.0),
            "quantity": synth.uniform_int(n, 3, -100_000, 99_999).astype(np.int32)}
    cap = 1 << 18
    nbytes, so, co = wx.group_list_layout(cap)
    recs = torch.zeros(shards * nbytes, dtype=torch.uint8, device="cuda")
    for r, (_, t) in enumerate(_shard_views(cols, shards)):
        rec = recs[r * nbytes:(r + 1) * nbytes]
        if t is None:
            continue  # an empty shard: count 0
        wx.group_sum(t, "price[idx]", "quantity[idx]", "(price[idx] < 30.0f)", launch(), 0, cap,
                     rec[8:8 + 4 * cap].view(torch.int32).data_ptr(), rec[so:so + 8 * cap].view(torch.float64).data_ptr(),
                     rec[co:co + 8 * cap].view(torch.int64).data_ptr(), d_n_groups=rec[0:8].view(torch.int64).data_ptr())
    ok, os_, oc, g = _merge_lists(recs, shards, cap, capacity=cap)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", "price < 30")
    assert g == len(rk)
    assert np.array_equal(ok[:g].cpu().numpy(), rk) and np.array_equal(oc[:g].cpu().numpy(), rc)
    np.testing.assert_allclose(os_[:g].cpu().numpy(), rs, rtol=1e-12, atol=0)


def _records(host, shards, k, desc, cond=None, select=None):
    """Each shard's real wx_topk output written into its wx_topk_record."""
    n = len(next(iter(host.values())))
    views = _shard_views(host, shards)
    recs = torch.zeros(shards * wx.TOPK_RECORD_BYTES, dtype=torch.uint8, device="cuda")
    for r, (b, t) in enumerate(views):
        rec = recs[r * wx.TOPK_RECORD_BYTES:(r + 1) * wx.TOPK_RECORD_BYTES]
        rec[:128].view(torch.float32).fill_(float("nan"))  # junk beyond the count
        rec[256:512].view(torch.int64).fill_(-5)
        if t is None:
            continue
        wx.topk(t, "price[idx]", cond, select, k, desc, launch(), rec[:128].data_ptr(), rec[256:512].data_ptr(),
                rec[128:256].data_ptr(), row_base=b, d_count=rec[512:520].data_ptr(), want_count=False)
    torch.cuda.synchronize()
    assert n >= 0
    return recs


@pytest.mark.parametrize("rows", [3, 1000, 300_007])
@pytest.mark.parametrize("shards", [1, 2, 3, 8, 128])
@pytest.mark.parametrize("k,desc", [(5, True), (5, False), (32, True), (1, False)])
def test_topk_merge_matches_oracle(rows, shards, k, desc):
    if shards * k > wx.TOPK_MERGE_MAX:
        pytest.skip("n_records * k above the merge bound")
    i = np.arange(rows)
    price = ((i // 7) % 13).astype(np.float32) - 6.0  # heavy ties
    price[i % 97 == 5] = np.nan
    price[i % 89 == 3] = -0.0
    qty = (i % 5).astype(np.float32)
    host = {"price": price, "quantity": qty}
    recs = _records(host, shards, k, desc, cond="(quantity[idx] > 0.0f)", select="(price[idx] * quantity[idx])")
    out_k = torch.empty(k, dtype=torch.float32, device="cuda")
    out_i = torch.empty(k, dtype=torch.int64, device="cuda")
    out_v = torch.empty(k, dtype=torch.float32, device="cuda")
    cnt = wx.topk_merge(recs.data_ptr(), shards, k, desc, launch(), out_k.data_ptr(), out_i.data_ptr(),
                        out_v.data_ptr(), want_count=True)
    ok_, oi, ov = ora.topk(ora.HostTable(host), "price", k, desc, cond="quantity > 0", select_expr="price * quantity")
    assert cnt == len(oi)
    assert np.array_equal(out_i[:cnt].cpu().numpy(), oi)
    assert np.array_equal(bits(out_k[:cnt].cpu().numpy()), bits(ok_))
    assert np.array_equal(bits(out_v[:cnt].cpu().numpy()), bits(ov))


def test_topk_merge_bounds():
    recs = torch.zeros(wx.TOPK_RECORD_BYTES * 200, dtype=torch.uint8, device="cuda")
    with pytest.raises(wx.WarpExecError) as e:
        wx.topk_merge(recs.data_ptr(), 200, 32, True, launch())
    assert e.value.status == wx.WX_ERR_UNSUPPORTED
    with pytest.raises(wx.WarpExecError):
        wx.topk_merge(recs.data_ptr(), 2, 33, True, launch())
    assert wx.topk_merge(recs.data_ptr(), 0, 5, True, launch(), want_count=True) == 0


# ------------------------------------------- RCCL: one process per GPU (>= 2 GPUs)
def _ngpus():
    return torch.cuda.device_count()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="one GPU visible: the RCCL runs need a multi-GPU box")
@pytest.mark.parametrize("workload,extra", [
    ("project", ["--rows", "2e7", "--c4-rows", "40000001"]),
    ("sum", ["--total-rows", "40000001"]),
    ("group", ["--rows", "1e7"]),
    ("group", ["--total-rows", "2e7"]),
    ("group", ["--rows", "4e6", "--keys", "100000"]),  # many keys: list records, one all-gather, the list merge
    ("topk", ["--rows", "1e7"]),
])
def test_bench_rccl_ranks(workload, extra):
    """bench.py under torchrun with the default (RCCL) backend, one rank per
    visible GPU (at most 8): the product's exchanges over xGMI, each line's
    own result check."""
    _bench_ranks(min(8, _ngpus()), workload, extra)


def _bench_ranks(n, workload, extra, env_extra=None):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k != "WARPDB_DIST_BACKEND"}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", str(n), "--workload", workload, "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", *extra],
                       capture_output=True, text=True, cwd=ROOT, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][-1]
    assert d["n_gpus"] == n and d["value"] > 0 and str(d["check"]).startswith("ok"), d
    for v in (d.get("secondary") or {}).values():
        assert str(v["check"]).startswith("ok"), v
    return d


@pytest.mark.parametrize("workload,extra", [
    ("project", ["--rows", "1e7", "--c4-rows", "20000001", "--c3-rows", "10000001"]),
    ("sum", ["--total-rows", "20000001"]),
    ("group", ["--rows", "1e7"]),
    ("group", ["--rows", "3e6", "--keys", "3000"]),  # keys beyond the window: the list records and merge
    ("group", ["--rows", "4e6", "--keys", "100000"]),  # the range-partitioned shard GROUP BY into the records
    ("topk", ["--rows", "1e7"]),
])
def test_bench_rccl_one_rank(workload, extra):
    """The multi-rank step of bench.py on a one-rank RCCL communicator
    (WARPDB_EXCHANGE_ONE_RANK=1, default backend): the rank's own RCCL
    communicator on the query stream (include/warpcomm.h) with the exchange
    buffers the 8-GPU run hands over (counts, {sum, count}, window + slots,
    top-K records), the exchange kernels behind them, every line self-checked."""
    d = _bench_ranks(1, workload, extra, {"WARPDB_EXCHANGE_ONE_RANK": "1"})
    assert d["config"]["exchange"] != "none (1 GPU)", d["config"]
    assert "own communicator" in d["config"]["collectives"], d["config"]


@pytest.mark.parametrize("workload,extra", [
    ("project", ["--rows", "1e7", "--no-c4", "--c3-rows", "10000001"]),
    ("group", ["--rows", "3e6", "--keys", "3000"]),
    ("topk", ["--rows", "1e7"]),
])
def test_bench_rccl_one_rank_torch_collectives(workload, extra):
    """The same with WARPDB_STREAM_COMM=0: torch.distributed's all_reduce /
    all_gather_into_tensor (RCCL on the process group's stream), the path
    every rank falls back to when a communicator of its own cannot be built."""
    d = _bench_ranks(1, workload, extra, {"WARPDB_EXCHANGE_ONE_RANK": "1", "WARPDB_STREAM_COMM": "0"})
    assert d["config"]["collectives"].startswith("torch.distributed"), d["config"]


@pytest.mark.parametrize("workload", ["sum", "group", "topk"])
def test_bench_api_rccl_one_device(workload):
    """ResidentShards (the C++ multi-GPU path) with a one-device
    ncclCommInitAll communicator: ncclAllReduce / ncclAllGather run."""
    env = dict(os.environ, WARPDB_EXCHANGE_ONE_RANK="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--api", "--gpus", "1", "--workload", workload,
                        "--rows", "1e7", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"],
                       capture_output=True, text=True, cwd=ROOT, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][-1]
    assert str(d["check"]).startswith("ok") and "nccl" in d["config"]["exchange"], d


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="one GPU visible: the RCCL runs need a multi-GPU box")
def test_warpdb_multi_gpu_all_devices_against_oracle(tmp_path):
    """WarpDB::query_multi_gpu{,_sum,_group,_topk} over every visible GPU
    (ncclCommInitAll, one thread + stream per device) against the oracle."""
    _warpdb_multi_against_oracle(tmp_path)


def test_warpdb_multi_gpu_one_device_rccl_against_oracle(tmp_path, monkeypatch):
    """The same on one device with its exchanges on a one-device RCCL
    communicator (WARPDB_EXCHANGE_ONE_RANK=1)."""
    monkeypatch.setenv("WARPDB_EXCHANGE_ONE_RANK", "1")
    _warpdb_multi_against_oracle(tmp_path)


def _warpdb_multi_against_oracle(tmp_path):
    from warpdb_amd import pywarpdb as pw

    m = 200_003
    small = synth.c2_table(m)
    small["quantity"] = small["quantity"].astype(np.float32)
    path = tmp_path / "t.csv"
    with open(path, "w") as f:
        f.write("price,quantity\n")
        for p_, q_ in zip(small["price"].tolist(), small["quantity"].tolist()):
            f.write(f"{p_!r},{q_!r}\n")
    db = pw.WarpDB(str(path))
    hs = ora.HostTable(small)
    r = np.asarray(db.query_multi_gpu("price * quantity WHERE price > 15"), np.float32)
    assert np.array_equal(bits(r), bits(ora.dense(hs, "price * quantity", "price > 15", np.zeros(m, np.float32))))
    s2, c2 = db.query_multi_gpu_sum("price * 0.9 WHERE price > 20")
    es2, ec2 = ora.reduce_sum(hs, "price * 0.9", "price > 20")
    assert c2 == ec2 and abs(s2 - es2) <= 1e-12 * abs(es2)
    # key window at 5000: all 100 keys fall outside it, more than a slot holds
    # (-2), so the shards' group list records are all-gathered (RCCL with the
    # one-rank hook) and merged by wx_group_merge_lists
    for sql, lo in (("SELECT SUM(price) FROM t GROUP BY quantity", 0),
                    ("SELECT SUM(price) FROM t GROUP BY quantity", 5000)):
        k, s, c = db.query_multi_gpu_group(sql, lo)
        rk, rs, rc = ora.group_sum(hs, "price", "quantity")
        assert np.array_equal(k, rk) and np.array_equal(c, rc)
        np.testing.assert_allclose(s, rs, rtol=1e-12, atol=0)
    k2, rows2, v2 = db.query_multi_gpu_topk("SELECT price FROM t ORDER BY price DESC LIMIT 7")
    ok2, oi2, ov2 = ora.topk(hs, "price", 7, True, select_expr="price")
    assert np.array_equal(rows2, oi2) and np.array_equal(bits(v2), bits(ov2))
    # OFFSET + LIMIT beyond the 32-candidate records: the shards' sorted heads
    # (wx_order_head), one all-gather of head records, wx_head_merge
    k3, rows3, v3 = db.query_multi_gpu_topk(
        "SELECT price * quantity FROM t WHERE quantity < 60 ORDER BY price ASC LIMIT 300 OFFSET 40")
    ok3, oi3, ov3 = ora.topk(hs, "price", 340, False, cond="quantity < 60", select_expr="price * quantity")
    assert np.array_equal(rows3, oi3[40:]) and np.array_equal(bits(k3), bits(ok3[40:]))
    assert np.array_equal(bits(v3), bits(ov3[40:]))


def test_stream_comm_fallback_is_collective(monkeypatch):
    """A rank whose own communicator cannot be built (here: the id call
    raises) makes every rank keep torch.distributed's collectives, with a
    warning; the exchanges then still run and agree with the local result.
    One-rank RCCL process group in this process (WARPDB_EXCHANGE_ONE_RANK)."""
    import torch.distributed as dist

    from warpdb_amd import _warpcomm as wc
    from warpdb_amd import distributed as wd

    for k, v in {"MASTER_ADDR": "127.0.0.1", "WORLD_SIZE": "1", "RANK": "0", "WARPDB_EXCHANGE_ONE_RANK": "1"}.items():
        monkeypatch.setenv(k, v)
    torch.cuda.set_device(0)
    # the store binds its own free port (a probed port can be taken by another
    # process before the store listens: EADDRINUSE once on a shared box)
    store = dist.TCPStore("127.0.0.1", 0, 1, is_master=True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        def broken():
            raise RuntimeError("no id for this test")

        monkeypatch.setattr(wc, "unique_id", broken)
        wd.release_stream_comms()
        with pytest.warns(RuntimeWarning, match="exchanges use torch.distributed"):
            assert wd.enable_stream_comm() is False
        assert wd.stream_comm() is None
        n = 300_001
        cols = synth.c2_table(n)
        price = torch.from_numpy(cols["price"]).cuda()
        sq = wd.ShardedQuery(wd.Shard({"price": price}, 0, n))
        assert sq.exchange and not sq.stream_comm
        s_, c_ = sq.sum("(price[idx] * 0.9f)", "(price[idx] > 20.0f)")
        rs, rc = ora.reduce_sum(ora.HostTable({"price": cols["price"]}), "price * 0.9", "price > 20")
        assert c_ == rc
        assert s_ == pytest.approx(rs, rel=1e-12)
    finally:
        torch.cuda.synchronize()
        wd.release_stream_comms()
        dist.destroy_process_group()
