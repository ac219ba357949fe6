"""GPU tests of GROUP BY with many distinct keys (round 3).

wx_group_sum with a capacity above 4096 finds the passing rows' key range
first (the previous call's range, a sample, or an exact pass): a range that
fits the 2048-key LDS window moves the window onto it; a range up to 2^24
keys takes the range-partitioned kernels (tiles sorted in place by partition
+ run directory -> plan -> LDS aggregation per work item -> count -> emit,
wx_group_part.hip; rows outside a guessed range send the query
round again over the exact range); wider ranges keep the window + global
hash.  Every form against the oracle's
std::map-order double sums (tests/sql_features_test.cpp:14-19 intent): keys
and counts exact, sums to 1e-12 relative (double sums of float values in a
different order; exact whenever the bit-span bound of DESIGN.md 5.2 holds).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib as ora

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from warpdb_amd import _warpexec as wx  # noqa: E402
from test_gpu_parity import dev_table, launch  # noqa: E402

N = 1_500_007  # above the partitioned path's 2^20-row floor, ragged


def _table(keys, seed=7):
    rng = np.random.default_rng(seed)
    price = rng.uniform(0.0, 40.0, len(keys)).astype(np.float32)
    return {"price": price, "quantity": keys.astype(np.int32)}


def _gpu_group(cols, key_expr="quantity[idx]", cond=None, cap=1 << 21, key_lo=0, val="price[idx]"):
    table, _ = dev_table(cols)
    k = torch.empty(cap, dtype=torch.int32, device="cuda")
    s = torch.empty(cap, dtype=torch.float64, device="cuda")
    c = torch.empty(cap, dtype=torch.int64, device="cuda")
    g = wx.group_sum(table, val, key_expr, cond, launch(), key_lo, cap, k.data_ptr(), s.data_ptr(), c.data_ptr())
    return k[:g].cpu().numpy(), s[:g].cpu().numpy(), c[:g].cpu().numpy()


def _check(cols, key_expr="quantity", cond=None, **kw):
    lowered_key = kw.pop("lowered_key", "quantity[idx]")
    lowered_cond = kw.pop("lowered_cond", None)
    gk, gs, gc = _gpu_group(cols, lowered_key, lowered_cond, **kw)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", key_expr, cond, capacity=1 << 22)
    assert np.array_equal(gk, rk) and np.array_equal(gc, rc)
    np.testing.assert_allclose(gs, rs, rtol=1e-12, atol=0)
    return len(gk)


@pytest.mark.parametrize("lo,span", [(0, 1_000_000), (-500_000, 100_000), (7, 4_097), (-(2 ** 31), 300_000),
                                     (2 ** 31 - 200_000, 200_000), (0, 2 ** 24), (0, 2 ** 26)])
def test_partitioned_uniform_keys(lo, span):
    i = np.arange(N, dtype=np.int64)
    keys = lo + ((i * 2654435761) % span)
    if span >= 2 ** 24:  # its two ends present, sparse inside: 2^24 is the widest partitioned range (2048
        # partitions), 2^26 takes the window + global hash
        keys = lo + ((i * 2654435761) % 5000) * (span // 5000)
        keys[0], keys[1] = lo, lo + span - 1
    n = _check(_table(keys))
    assert n == len(np.unique(keys))


def test_partitioned_with_where_and_key_expression():
    i = np.arange(N, dtype=np.int64)
    cols = _table((i * 7919) % 400_000)
    _check(cols, key_expr="quantity * 3 - 5", cond="price < 30", lowered_key="((quantity[idx] * 3) - 5)",
           lowered_cond="(price[idx] < 30.0f)")


def test_relocated_window_and_wide_fallback():
    i = np.arange(N, dtype=np.int64)
    # 1500 keys far outside the caller's window: the window moves onto them
    _check(_table(100_000 + i % 1500))
    # a range wider than 2^26: window + global hash (5000 sparse keys)
    keys = (i % 5000) * 100_000 - 250_000_000
    _check(_table(keys), cap=8192)


def test_partitioned_empty_where_and_capacity():
    i = np.arange(N, dtype=np.int64)
    cols = _table(i % 200_000)
    gk, _, _ = _gpu_group(cols, cond="(price[idx] > 100.0f)")
    assert len(gk) == 0
    table, _ = dev_table(cols)
    cap = 5000
    k = torch.empty(cap, dtype=torch.int32, device="cuda")
    s = torch.empty(cap, dtype=torch.float64, device="cuda")
    c = torch.empty(cap, dtype=torch.int64, device="cuda")
    with pytest.raises(wx.WarpExecError) as e:
        wx.group_sum(table, "price[idx]", "quantity[idx]", None, launch(), 0, cap, k.data_ptr(), s.data_ptr(),
                     c.data_ptr())
    assert e.value.status == wx.WX_ERR_CAPACITY
    # the dense accumulators were left clean: the next query is exact
    _check(cols)


def test_partitioned_matches_window_hash_path(monkeypatch):
    i = np.arange(N, dtype=np.int64)
    cols = _table((i * 31) % 60_000)
    a = _gpu_group(cols)
    monkeypatch.setenv("WARPDB_GROUP_PARTITION", "0")
    b = _gpu_group(cols)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2])
    np.testing.assert_allclose(a[1], b[1], rtol=1e-12, atol=0)


def test_partitioned_float_and_int64_columns():
    i = np.arange(N, dtype=np.int64)
    rng = np.random.default_rng(3)
    cols = {"price": rng.uniform(-5, 5, N).astype(np.float64), "quantity": ((i * 13) % 250_000).astype(np.int64)}
    gk, gs, gc = _gpu_group(cols)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", None, capacity=1 << 22)
    assert np.array_equal(gk, rk) and np.array_equal(gc, rc)
    np.testing.assert_allclose(gs, rs, rtol=1e-9, atol=1e-9)  # float(double) values summed in double


@pytest.mark.parametrize("guess", ["1", "0"])
def test_partitioned_sample_misses_outliers(guess, monkeypatch):
    """The first pass runs over a range guessed from a 65 536-row sample:
    rare keys far outside it (never sampled) must send the query through
    the exact-range pass, and a selective WHERE leaves the sample few rows."""
    monkeypatch.setenv("WARPDB_GP_GUESS", guess)
    i = np.arange(N, dtype=np.int64)
    keys = (i * 48271) % 100_000
    keys[[17, 900_001, N - 2]] = [3_000_000, -2_000_000, 5_000_000]  # between sampled rows
    cols = _table(keys)
    _check(cols)
    _check(cols, cond="price > 39.9", lowered_cond="(price[idx] > 39.9f)")


def test_partitioned_selective_where_exact_probe():
    """a WHERE so selective that the 65 536-row sample sees
    no passing row sends the query through the exact min / max pass, which
    must visit every row -- here the passing rows, and the extreme keys, sit
    only at quad offsets 256..511 (mod 1024) that a 256-thread launch of a
    512-thread loop once skipped.  About 1700 partitions (span ~1.4e7)."""
    n = N
    i = np.arange(n, dtype=np.int64)
    keys = (i * 7919) % 300_000
    flag = np.zeros(n, np.float32)
    sel = ((i // 4) % 1024 >= 256) & ((i // 4) % 1024 < 512)
    s = np.arange(65536, dtype=np.int64)
    sampled = s * (n // 65536) + (s * (n % 65536)) // 65536  # wx_group_part_sample's rows
    sel[sampled] = False
    flag[sel] = 1.0
    rows = np.flatnonzero(sel)
    keys[rows[5]], keys[rows[len(rows) // 2]] = -5_000_000, 9_000_000
    cols = _table(keys)
    cols["flag"] = flag
    m = _check(cols, cond="flag > 0", lowered_cond="(flag[idx] > 0.0f)")
    assert m == len(np.unique(keys[sel]))


def test_partitioned_memo_survives_rewritten_table():
    """The key range is remembered per (expressions, columns, rows) and only
    ever used as a guess: the same query again, then over the same buffers
    rewritten in place with keys outside the remembered range (the pass
    counts them and goes round again over the exact range), then with few
    keys (the window path)."""
    i = np.arange(N, dtype=np.int64)
    cols = _table((i * 31) % 500_000)
    table, tensors = dev_table(cols)
    cap = 1 << 20

    def run():
        k = torch.empty(cap, dtype=torch.int32, device="cuda")
        s = torch.empty(cap, dtype=torch.float64, device="cuda")
        c = torch.empty(cap, dtype=torch.int64, device="cuda")
        g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, launch(), 0, cap, k.data_ptr(), s.data_ptr(),
                         c.data_ptr())
        return k[:g].cpu().numpy(), s[:g].cpu().numpy(), c[:g].cpu().numpy()

    def want():
        return ora.group_sum(ora.HostTable(cols), "price", "quantity", None, capacity=1 << 22)

    for keys in ((i * 31) % 500_000, (i * 31) % 500_000, 3_000_000 + (i * 17) % 900_000, 40 + i % 700,
                 (i * 13) % 250_000):
        cols["quantity"] = keys.astype(np.int32)
        tensors["quantity"].copy_(torch.from_numpy(cols["quantity"]))
        gk, gs, gc = run()
        rk, rs, rc = want()
        assert np.array_equal(gk, rk) and np.array_equal(gc, rc)
        np.testing.assert_allclose(gs, rs, rtol=1e-12, atol=0)


def test_partitioned_skewed_keys():
    """Half the rows on one key, the rest spread over 600 000 keys: one
    partition far heavier than the others (its work items stay whole
    workgroup ranges)."""
    i = np.arange(N, dtype=np.int64)
    keys = np.where(i % 2 == 0, 123_456, (i * 2654435761) % 600_000)
    _check(_table(keys))
