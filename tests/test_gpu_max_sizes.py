"""GPU tests at the ABI's size limits: tables past 2^31 rows, sorts of 2^32 - 1 keys.

The reference counts rows in `int` (`include/csv_loader.hpp:20`, the kernel's
`int N`, `src/jit.cpp:55-61`), so C4's 8e9 rows overflow it; here row counts
are int64 end to end.  These sizes are far beyond what the oracle finishes in
seconds, so the checks are the size-independent properties of each operation,
computed by torch on the device: the compaction is the ascending list of rows
whose condition holds and their projected values; SUM and GROUP BY agree with
a float64 torch reduction (different summation order, hence the relative
tolerance) and their counts are exact; top-K holds the K largest values with
the smallest-index tie-break; a sort is ordered and a permutation of its input.
"""
from __future__ import annotations

import pytest

import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from warpdb_amd import _warpexec as wx  # noqa: E402

N_BIG = (1 << 31) + 4099  # past INT32_MAX, and not a multiple of any tile
CHUNK = 1 << 28


def launch():
    return wx.make_launch(device=0, stream=torch.cuda.current_stream().cuda_stream, flags=wx.F_SYNC)


@pytest.fixture(scope="module")
def big_c2():
    n = N_BIG
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    qty = torch.empty(n, dtype=torch.float32, device="cuda")
    L = launch()
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, synth.SEED_PRICE, 0, 0.0, 40.0, L)
    wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, synth.SEED_QTY, 1, 1, 100, L)
    table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()),
                         wx.Column("quantity", wx.FLOAT32, qty.data_ptr())])
    yield table, price, qty
    del price, qty
    torch.cuda.empty_cache()


def test_compaction_past_int32_rows(big_c2):
    table, price, qty = big_c2
    n = table.n_rows
    vals = torch.empty(n, dtype=torch.float32, device="cuda")
    idx = torch.empty(n, dtype=torch.int64, device="cuda")
    row_base = 5 << 32  # a shard of a larger table: indices are row_base + row
    cnt = wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", launch(),
                            wx.MODE_COMPACT, vals.data_ptr(), idx.data_ptr(), 8, row_base, want_count=True)
    with pytest.raises(wx.WarpExecError):  # int32 indices cannot hold rows past INT32_MAX
        wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", launch(),
                          wx.MODE_COMPACT, vals.data_ptr(), idx.data_ptr(), 4, 0, want_count=True)
    out = 0
    for lo in range(0, n, CHUNK):
        hi = min(n, lo + CHUNK)
        mask = price[lo:hi] > 15.0
        m = int(mask.sum().item())
        ref_idx = torch.nonzero(mask).flatten() + (row_base + lo)
        assert torch.equal(idx[out:out + m], ref_idx), lo
        assert torch.equal(vals[out:out + m], (price[lo:hi] * qty[lo:hi])[mask]), lo
        out += m
    assert cnt == out
    assert int(idx[cnt - 1].item()) - row_base > (1 << 31)
    del vals, idx


def test_sum_past_int32_rows(big_c2):
    table, price, _ = big_c2
    s, c = wx.reduce_sum(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", launch())
    rs, rc = 0.0, 0
    for lo in range(0, table.n_rows, CHUNK):
        p = price[lo:lo + CHUNK]
        mask = p > 20.0
        rc += int(mask.sum().item())
        rs += float((p * 0.9)[mask].double().sum().item())
    assert c == rc
    assert s == pytest.approx(rs, rel=1e-12)


def _rows_where(t, pred):
    return torch.cat([torch.nonzero(pred(t[lo:lo + CHUNK])).flatten() + lo for lo in range(0, t.numel(), CHUNK)])


def test_topk_past_int32_rows(big_c2):
    table, price, _ = big_c2
    k = 32
    keys = torch.empty(k, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    vals = torch.empty(k, device="cuda")
    m = wx.topk(table, "price[idx]", None, "price[idx]", k, True, launch(), keys.data_ptr(), idx.data_ptr(),
                vals.data_ptr())
    assert m == k
    cand = torch.cat([price[lo:lo + CHUNK].topk(k).values for lo in range(0, table.n_rows, CHUNK)])
    assert torch.equal(keys, cand.topk(k).values)
    assert torch.equal(price[idx], keys) and torch.equal(vals, keys)
    # smallest-index tie-break at the K-th value: every row above it, then the first rows equal to it
    # (torch.nonzero is taken chunk by chunk: it fails on tensors past 2^31 elements)
    t = keys[-1]
    rows_above = _rows_where(price, lambda c: c > t)
    above = rows_above.numel()
    ties = _rows_where(price, lambda c: c == t)[:k - above]
    assert torch.equal(idx[:above].sort().values, rows_above)
    assert torch.equal(idx[above:], ties)


def test_group_sum_past_int32_rows():
    n = N_BIG
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    key = torch.empty(n, dtype=torch.int32, device="cuda")
    L = launch()
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, 1023, L)
    table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()),
                         wx.Column("quantity", wx.INT32, key.data_ptr())])
    cap = 2048
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, L, 0, cap, keys.data_ptr(), sums.data_ptr(),
                     cnts.data_ptr())
    rsum = torch.zeros(1024, dtype=torch.float64, device="cuda")
    rcnt = torch.zeros(1024, dtype=torch.int64, device="cuda")
    for lo in range(0, n, CHUNK):
        kk = key[lo:lo + CHUNK].long()
        rsum.index_add_(0, kk, price[lo:lo + CHUNK].double())
        rcnt += torch.bincount(kk, minlength=1024)
    present = torch.nonzero(rcnt).flatten()
    assert g == present.numel()
    assert torch.equal(keys[:g].long(), present)
    assert torch.equal(cnts[:g], rcnt[present])
    assert torch.allclose(sums[:g], rsum[present], rtol=1e-12, atol=0)
    del price, key
    torch.cuda.empty_cache()


def test_group_sum_many_keys_past_int32_rows():
    """The range-partitioned GROUP BY (10^6 keys, capacity 2^20) past 2^31
    rows: tile indices, run directory, per-partition totals and the items'
    tile ranges in 64-bit, against torch's bincount over the same table."""
    n = N_BIG
    nk = 1_000_000
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    key = torch.empty(n, dtype=torch.int32, device="cuda")
    L = launch()
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 1, 0, 0.0, 40.0, L)
    wx.fill_synthetic(key.data_ptr(), wx.INT32, n, 3, 1, 0, nk - 1, L)
    table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()),
                         wx.Column("quantity", wx.INT32, key.data_ptr())])
    cap = 1 << 20
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, L, 0, cap, keys.data_ptr(), sums.data_ptr(),
                     cnts.data_ptr())
    rsum = torch.zeros(nk, dtype=torch.float64, device="cuda")
    rcnt = torch.zeros(nk, dtype=torch.int64, device="cuda")
    for lo in range(0, n, CHUNK):
        kk = key[lo:lo + CHUNK].long()
        rsum += torch.bincount(kk, weights=price[lo:lo + CHUNK].double(), minlength=nk)
        rcnt += torch.bincount(kk, minlength=nk)
    present = torch.nonzero(rcnt).flatten()
    assert g == present.numel()
    assert torch.equal(keys[:g].long(), present)
    assert torch.equal(cnts[:g], rcnt[present])
    assert torch.allclose(sums[:g], rsum[present], rtol=1e-12, atol=0)
    del price, key
    torch.cuda.empty_cache()


def _multiset(t):
    """(sum, sum of squares) of the 32-bit patterns, as int64 (wrapping), chunk by chunk."""
    s = q = 0
    for lo in range(0, t.numel(), CHUNK):
        b = t[lo:lo + CHUNK].view(torch.int32).to(torch.int64)
        s += int(b.sum().item())
        q += int((b * b).sum().item())
    return s & 0xFFFFFFFFFFFFFFFF, q & 0xFFFFFFFFFFFFFFFF


def _ordered(t):
    n = t.numel()
    for lo in range(0, n - 1, CHUNK):
        hi = min(n - 1, lo + CHUNK)
        if not bool((t[lo + 1:hi + 1] >= t[lo:hi]).all().item()):
            return False
    return True


def test_sort_float_max_count():
    # the ABI's largest sort: 2^32 - 1 keys, every 32-bit destination in use
    n = (1 << 32) - 1
    t = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(t.data_ptr(), wx.FLOAT32, n, 23, 0, -1000.0, 1000.0, launch())
    before = _multiset(t)
    wx.sort_float(t.data_ptr(), n, True, launch())
    assert _ordered(t)
    assert _multiset(t) == before
    with pytest.raises(wx.WarpExecError):
        wx.sort_float(t.data_ptr(), n + 1, True, launch())
    del t
    torch.cuda.empty_cache()


def test_sort_pairs_past_int32():
    # key + payload past INT32_MAX: the payload must follow its key (payload = row number as float bits)
    n = (1 << 31) + 77
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    wx.fill_synthetic(keys.data_ptr(), wx.INT32, n, 29, 1, 0, 65535, launch())
    vals = torch.arange(n, dtype=torch.int64, device="cuda").to(torch.int32).view(torch.float32)
    orig = keys.clone()
    wx.sort_pairs(keys.data_ptr(), vals.data_ptr(), n, True, launch())
    rows = vals.view(torch.int32).to(torch.int64)  # row numbers < 2^32 fit in the low 32 bits
    rows = torch.where(rows < 0, rows + (1 << 32), rows)
    for lo in range(0, n, CHUNK):
        hi = min(n, lo + CHUNK)
        assert torch.equal(orig[rows[lo:hi]], keys[lo:hi]), lo
        # stable: equal keys keep ascending row order
        if hi - lo > 1:
            same = keys[lo + 1:hi] == keys[lo:hi - 1]
            assert bool((rows[lo + 1:hi][same] > rows[lo:hi - 1][same]).all().item()), lo
    assert _ordered(keys)
