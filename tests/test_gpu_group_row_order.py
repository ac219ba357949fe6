"""GROUP BY with WX_F_ROW_ORDER: each group's sum folded in ascending row
order, one double add per row -- the reference's std::map fold
(src/warpdb.cpp:373-385: `g.sum += val` over the rows in order) to the bit.

The ordinary GROUP BY adds a group's values in whatever order the workgroups
and the LDS atomics take them, so its double sums can differ from the
reference's in the last bits when the values span many binades (its tests
compare at 1e-12).  Here the tables are built so that order matters --
values of 1e7, 1 and 1e-3 scales mixed within every group -- and the
row-order sums must equal the oracle's (oracle/warpdb_oracle.c, the same
sequential double fold) bit for bit, on every path the groups can take
(LDS window, window + general-key hash, range-partitioned), with a WHERE,
negative and skewed keys, MIN / MAX beside the sums, and run to run.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib as ora

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from warpdb_amd import _warpexec as wx  # noqa: E402
from test_gpu_parity import dev_table  # noqa: E402


def launch(flags=wx.F_ROW_ORDER):
    return wx.make_launch(device=0, stream=torch.cuda.current_stream().cuda_stream, flags=flags)


def spread_values(rng, n):
    """Values over many binades: 1e7-, 1- and 1e-3-scale rows interleaved."""
    scale = rng.choice(np.array([1e7, 1.0, 1e-3], np.float32), n)
    return (rng.uniform(0.0, 1.0, n).astype(np.float32) * scale).astype(np.float32)


def run(cols, cond_c, cap, agg=False, flags=wx.F_ROW_ORDER):
    t, _ = dev_table(cols)
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    if agg:
        mins = torch.empty(cap, dtype=torch.float32, device="cuda")
        maxs = torch.empty(cap, dtype=torch.float32, device="cuda")
        g = wx.group_agg(t, "price[idx]", "quantity[idx]", cond_c, launch(flags), 0, cap, keys.data_ptr(),
                         sums.data_ptr(), cnts.data_ptr(), mins.data_ptr(), maxs.data_ptr())
        return (g, keys[:g].cpu().numpy(), sums[:g].cpu().numpy(), cnts[:g].cpu().numpy(),
                mins[:g].cpu().numpy(), maxs[:g].cpu().numpy())
    g = wx.group_sum(t, "price[idx]", "quantity[idx]", cond_c, launch(flags), 0, cap, keys.data_ptr(),
                     sums.data_ptr(), cnts.data_ptr())
    return g, keys[:g].cpu().numpy(), sums[:g].cpu().numpy(), cnts[:g].cpu().numpy()


def bits(a):
    return np.asarray(a, np.float64).view(np.uint64)


@pytest.mark.parametrize("n,keys,cond,min_rows", [
    (300_001, (0, 1024), None, None),                  # the LDS window
    (300_001, (0, 100_000), None, None),               # window + general-key hash
    (300_001, (-500, 501), "(price[idx] > 0.5f)", None),  # negative keys, a WHERE
    ((1 << 21) + 7, (0, 100_000), None, "0"),          # range-partitioned first step
])
def test_row_order_sums_equal_sequential_fold(n, keys, cond, min_rows, monkeypatch):
    if min_rows is not None:
        monkeypatch.setenv("WARPDB_GP_MIN_ROWS", min_rows)
    rng = np.random.default_rng(n + keys[1])
    cols = {"price": spread_values(rng, n), "quantity": rng.integers(keys[0], keys[1], n).astype(np.int32)}
    cap = 1 << 17
    g, k, s, c = run(cols, cond, cap)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity",
                               {None: None, "(price[idx] > 0.5f)": "price > 0.5"}[cond], capacity=cap)
    assert g == len(rk)
    assert np.array_equal(k, rk) and np.array_equal(c, rc)
    assert np.array_equal(bits(s), bits(rs))


def test_row_order_skewed_and_reproducible():
    # 90 % of the rows on one key (a long dependent chain), the rest spread
    n = 2_000_003
    rng = np.random.default_rng(5)
    q = np.where(rng.random(n) < 0.9, 7, rng.integers(0, 3000, n)).astype(np.int32)
    cols = {"price": spread_values(rng, n), "quantity": q}
    g, k, s, c = run(cols, None, 4096)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", capacity=4096)
    assert g == len(rk) and np.array_equal(k, rk) and np.array_equal(c, rc)
    assert np.array_equal(bits(s), bits(rs))
    g2, k2, s2, c2 = run(cols, None, 4096)
    assert g2 == g and np.array_equal(bits(s2), bits(s))


def test_row_order_with_min_max():
    n = 200_003
    rng = np.random.default_rng(11)
    cols = {"price": spread_values(rng, n), "quantity": rng.integers(0, 5000, n).astype(np.int32)}
    g, k, s, c, mn, mx = run(cols, None, 8192, agg=True)
    rk, rs, rc, rmn, rmx = ora.group_agg(ora.HostTable(cols), "price", "quantity", capacity=8192)
    assert g == len(rk) and np.array_equal(k, rk) and np.array_equal(c, rc)
    assert np.array_equal(bits(s), bits(rs))
    assert np.array_equal(mn.view(np.uint32), rmn.view(np.uint32))
    assert np.array_equal(mx.view(np.uint32), rmx.view(np.uint32))


def test_row_order_edge_cases():
    rng = np.random.default_rng(3)
    one = {"price": np.array([2.5], np.float32), "quantity": np.array([-4], np.int32)}
    g, k, s, c = run(one, None, 16)
    assert g == 1 and k[0] == -4 and s[0] == 2.5 and c[0] == 1
    n = 10_000
    cols = {"price": spread_values(rng, n), "quantity": rng.integers(0, 10, n).astype(np.int32)}
    g, *_ = run(cols, "(price[idx] < -1.0f)", 16)  # nothing passes
    assert g == 0
    with pytest.raises(wx.WarpExecError):  # more groups than capacity: the same error as without the flag
        run(cols, None, 4)


def test_plain_sums_order_free_within_tolerance():
    # the ordinary path on the same data: counts exact, sums within 1e-12 of
    # the sequential fold (they may differ in the last bits -- the reason
    # for the flag)
    n = 300_001
    rng = np.random.default_rng(17)
    cols = {"price": spread_values(rng, n), "quantity": rng.integers(0, 1024, n).astype(np.int32)}
    g, k, s, c = run(cols, None, 4096, flags=0)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", capacity=4096)
    assert np.array_equal(k, rk) and np.array_equal(c, rc)
    assert np.allclose(s, rs, rtol=1e-12, atol=0)


def test_row_order_general_path_keys_with_nan_bit_patterns():
    """the general row-order path carries each int key's bits
    through the float-valued compaction (__int_as_float).  Keys whose bits
    are signalling / quiet NaN patterns, infinities and -0.0 must come back
    unchanged (the compaction only moves bits).  Keys this far apart (span >
    2048) take the general path, not the key-span counting scatter."""
    n = 200_003
    rng = np.random.default_rng(29)
    special = np.array([-8388607, -4194305, -4194304, -8388608, 2139095041, 2143289343, 2143289344, 2139095040,
                        -2147483648, 0, 1, 7], np.int64).astype(np.int32)  # sNaN, qNaN, -inf, +inf, -0.0, ... bits
    q = special[rng.integers(0, len(special), n)]
    cols = {"price": spread_values(rng, n), "quantity": q}
    g, k, s, c = run(cols, None, 4096)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", capacity=4096)
    assert g == len(rk) == len(special)
    assert np.array_equal(k, rk) and np.array_equal(c, rc)
    assert np.array_equal(bits(s), bits(rs))


def _adversarial_groups(rng, n):
    """Per-group value streams that push the exact block-parallel fold
    (wx::fold_exact) onto every branch: round-half-even ties against a large
    running sum, sums that cancel through zero and hover at a power of two,
    binade crossings both ways, negative sums, NaN / Inf, denormal floats,
    overflow, and plain prices (the fast path)."""
    g = rng.integers(0, 10, n).astype(np.int32)
    v = np.empty(n, np.float32)
    for key in range(10):
        m = int((g == key).sum())
        if key == 0:    # ties: 2^30 first, then odd / even multiples of 2^-23 (half of u = 2^-22)
            x = rng.integers(-8, 9, m).astype(np.float32) * np.float32(2.0 ** -23)
            x[0] = 2.0 ** 30
        elif key == 1:  # cancellation through zero
            x = np.where(rng.random(m) < 0.5, 1e7, -1e7).astype(np.float32) + rng.uniform(-1, 1, m).astype(np.float32)
        elif key == 2:  # prices
            x = rng.uniform(0.0, 40.0, m).astype(np.float32)
        elif key == 3:  # a NaN midway
            x = rng.uniform(0.0, 40.0, m).astype(np.float32)
            x[m // 2] = np.float32("nan")
        elif key == 4:  # +inf, then -inf: NaN
            x = rng.uniform(0.0, 1.0, m).astype(np.float32)
            x[m // 3] = np.float32("inf")
            x[2 * m // 3] = np.float32("-inf")
        elif key == 5:  # denormals and tiny values under a large sum
            x = (rng.integers(1, 1 << 20, m).astype(np.float32) * np.float32(2.0 ** -149)).astype(np.float32)
            x[::97] = np.float32(3.0e6)
        elif key == 6:  # hovering at 2^20: +-x steps across the power of two
            x = (rng.choice(np.array([1.0, -1.0], np.float32), m) * rng.uniform(0.0, 3.0, m)).astype(np.float32)
            x[0] = 2.0 ** 20
        elif key == 7:  # negative sums crossing binades
            x = -rng.uniform(0.0, 1000.0, m).astype(np.float32)
        elif key == 8:  # float-max values: a double sum far above the float range
            x = np.full(m, 3.0e38, np.float32)
        else:           # mixed scales (the spread_values mix), negative too
            x = spread_values(rng, m) * rng.choice(np.array([1.0, -1.0], np.float32), m)
        v[g == key] = x
    return v, g


@pytest.mark.parametrize("path", ["span", "general"])
def test_row_order_exact_fold_adversarial(path):
    n = 400_003
    rng = np.random.default_rng(41)
    v, g = _adversarial_groups(rng, n)
    keys = g if path == "span" else g * 1000  # a key span > 2048 takes the general path
    cols = {"price": v, "quantity": keys.astype(np.int32)}
    got_g, k, s, c = run(cols, None, 64)
    assert got_g == 10 and np.array_equal(k, np.unique(keys))
    for i, key in enumerate(np.unique(keys)):
        want = np.add.accumulate(v[keys == key].astype(np.float64))[-1]  # the sequential fold, row order
        assert c[i] == int((keys == key).sum())
        if np.isnan(want):
            assert np.isnan(s[i]), (key, s[i])
        else:
            assert bits(s[i]) == bits(want), (key, s[i], want)


@pytest.mark.parametrize("outlier", [None, 1000, 5000, -3000])
def test_row_order_direct_span_guess(outlier, monkeypatch):
    """The span path without the ordinary call: the 2048-key span is guessed
    from a strided sample (or the memo), so a key the sample misses either
    still falls inside the centred span (1000) or makes the count kernel flag
    the miss and the call fall back to the ordinary call first (5000, -3000:
    then the general path, the keys spanning > 2048).  Equal, bit for bit, to
    the oracle and to the ordinary-call-first span path."""
    n = 500_003
    rng = np.random.default_rng(47)
    q = rng.integers(0, 100, n).astype(np.int32)
    if outlier is not None:
        q[n // 2 + 1] = outlier  # one row: a 65 536-row strided sample misses it
    cols = {"price": spread_values(rng, n), "quantity": q}
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", capacity=4096)
    for mode in ("span", "ordinary"):
        monkeypatch.setenv("WARPDB_GROUP_ROWS", mode)
        for _ in range(2):  # the second call takes the memo's range
            g, k, s, c = run(cols, None, 4096)
            assert g == len(rk) and np.array_equal(k, rk) and np.array_equal(c, rc), mode
            assert np.array_equal(bits(s), bits(rs)), mode


@pytest.mark.parametrize("path", ["span", "general"])
@pytest.mark.parametrize("values", ["prices", "spread", "ties"])
def test_row_order_big_group_chunked(path, values):
    """A group of more than WX_XF_BIG (4 Mi) rows is folded in 64 Ki-value
    chunks (wx_xf_big_*: approximate chunk sums, exact chunk sums under a
    guessed binade, applied in order after checking it, fold_exact for the
    rest) instead of one wave streaming it alone; the sums stay bit-equal
    to the sequential fold, with prices (chunks mostly applied whole), with
    mixed 1e7 / 1 / 1e-3 scales (chunks mostly refolded), and with half the
    values ties against a 2^33 running sum (the tie scan of every block and
    chunk)."""
    n = 10_000_003
    rng = np.random.default_rng(53)
    q = np.where(rng.random(n) < 0.85, 7, rng.integers(0, 1000, n)).astype(np.int32)
    if path == "general":
        q = q * 1000  # a key span > 2048
    if values == "prices":
        v = rng.uniform(0.0, 40.0, n).astype(np.float32)
    elif values == "spread":
        v = spread_values(rng, n)
    else:  # half of the values ties against the running sum: multiples of 2^-20 under a 1.5 * 2^33 sum (u = 2^-19)
        v = (rng.integers(-8, 9, n).astype(np.float32) * np.float32(2.0 ** -20)).astype(np.float32)
        v[np.flatnonzero(q == (7000 if path == "general" else 7))[0]] = np.float32(1.5 * 2.0 ** 33)  # mid-binade
    cols = {"price": v, "quantity": q}
    g, k, s, c = run(cols, None, 4096)
    uk = np.unique(q)
    assert g == len(uk) and np.array_equal(k, uk)
    big = int(np.argmax(c))
    assert c[big] > 4 * (1 << 20)
    for i in (big, 0, g - 1):
        want = np.add.accumulate(v[q == k[i]].astype(np.float64))[-1]
        assert c[i] == int((q == k[i]).sum())
        assert bits(s[i]) == bits(want), (i, s[i], want)


@pytest.mark.parametrize("lo,width", [(0, 2048), (0, 2049), (2**31 - 2048, 2048), (-2**31, 2048), (-2**31, 2049),
                                      (-1024, 2048)])
@pytest.mark.parametrize("mode", ["span", "ordinary"])
def test_row_order_key_span_boundaries(lo, width, mode, monkeypatch):
    """Keys spanning exactly the 2048 bins of the key-span scatter (at 0, at
    the int32 extremes, straddling 0) take it; one key more takes the
    general path.  The lowest and highest key each appear once, in the
    middle of the table (a strided sample misses them: the direct path's
    miss flag and fallback at the int32 extremes), and a WHERE drops rows.
    Equal to the oracle's sequential fold bit for bit."""
    monkeypatch.setenv("WARPDB_GROUP_ROWS", mode)
    n = 300_007
    rng = np.random.default_rng(lo % 1000 + width)
    q = rng.integers(lo + 1, lo + width - 1, n, dtype=np.int64)
    q[n // 2 + 3] = lo
    q[n // 2 + 5] = lo + width - 1
    cols = {"price": spread_values(rng, n), "quantity": q.astype(np.int32)}
    cols["price"][n // 2 + 3] = 3.0  # the extreme keys' rows pass the WHERE
    cols["price"][n // 2 + 5] = 4.0
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", "price > 0.25", capacity=4096)
    assert rk[0] == lo and rk[-1] == lo + width - 1
    for _ in range(2):  # the second call takes the memo's range
        g, k, s, c = run(cols, "(price[idx] > 0.25f)", 4096)
        assert g == len(rk) and np.array_equal(k, rk) and np.array_equal(c, rc)
        assert np.array_equal(bits(s), bits(rs))


@pytest.mark.parametrize("kind", ["int_expr", "float_col", "int_col", "int_col_where", "val_expr", "int_val"])
def test_row_order_general_key_sources(kind, monkeypatch):
    """The general path's keys and values: a bare int32 key column with no
    WHERE is sorted straight from the column (no key projection), a bare
    float32 value column with no WHERE rides as the sort's payload straight
    from the column (no value projection); a key expression, a float key
    column (cast to int), a value expression, an int value column (converted
    to float) or a WHERE go through the compactions.  Groups of every size class: one lane each (<= 4096 rows),
    one wave each, and (with WARPDB_FOLD_SMALL=0) one wave for all.  Equal
    to the oracle's sequential fold bit for bit."""
    n = 700_001
    rng = np.random.default_rng(61)
    q = rng.integers(0, 50_000, n).astype(np.int32)
    q[rng.random(n) < 0.3] = 12_345  # one group of ~210 000 rows (a wave), the rest ~10 rows (lanes)
    cols = {"price": spread_values(rng, n), "quantity": q}
    key_gpu, key_ora, cond_gpu, cond_ora = "quantity[idx]", "quantity", None, None
    val_gpu, val_ora = "price[idx]", "price"
    if kind == "val_expr":
        val_gpu, val_ora = "(price[idx] * 3.0f)", "price * 3"
    elif kind == "int_val":
        cols["units"] = rng.integers(-1000, 1000, n).astype(np.int32)
        val_gpu, val_ora = "units[idx]", "units"
    if kind == "int_expr":
        key_gpu, key_ora = "(quantity[idx] * 3)", "quantity * 3"
    elif kind == "float_col":
        cols["quantity"] = q.astype(np.float32)
    elif kind == "int_col_where":
        cond_gpu, cond_ora = "(price[idx] > 0.25f)", "price > 0.25"
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), val_ora, key_ora, cond_ora, capacity=1 << 17)
    t, _ = dev_table(cols)
    cap = 1 << 17
    for small in ("", "0"):
        monkeypatch.setenv("WARPDB_FOLD_SMALL", small)
        keys = torch.empty(cap, dtype=torch.int32, device="cuda")
        sums = torch.empty(cap, dtype=torch.float64, device="cuda")
        cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
        g = wx.group_sum(t, val_gpu, key_gpu, cond_gpu, launch(), 0, cap, keys.data_ptr(), sums.data_ptr(),
                         cnts.data_ptr())
        assert g == len(rk)
        assert np.array_equal(keys[:g].cpu().numpy(), rk) and np.array_equal(cnts[:g].cpu().numpy(), rc)
        assert np.array_equal(bits(sums[:g].cpu().numpy()), bits(rs)), small


@pytest.mark.parametrize("mode", ["span", "general", "ordinary"])
def test_row_order_wide_keys_capacity_and_empty(mode, monkeypatch):
    """Keys spanning more than 2048 take the general path; without MIN / MAX
    and no ordinary call (span / general modes) its groups come from the
    sorted keys' runs.  More groups than the capacity is the ordinary call's
    capacity error, and a WHERE nothing passes gives no groups, on every
    route."""
    monkeypatch.setenv("WARPDB_GROUP_ROWS", mode)
    n = 200_003
    rng = np.random.default_rng(67)
    cols = {"price": spread_values(rng, n), "quantity": (rng.integers(0, 5000, n) * 7).astype(np.int32)}
    with pytest.raises(wx.WarpExecError):
        run(cols, None, 100)
    g, *_ = run(cols, "(price[idx] < -1.0f)", 100)
    assert g == 0
    g, k, s, c = run(cols, None, 8192)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", capacity=8192)
    assert g == len(rk) and np.array_equal(k, rk) and np.array_equal(c, rc)
    assert np.array_equal(bits(s), bits(rs))


def test_shutdown_releases_every_workspace_buffer():
    """wx_shutdown frees every buffer the workspaces allocated (it once freed
    a fixed list that missed the partitioned GROUP BY's staging, the group
    lists and the row-order fold's buffers), and the library works again
    afterwards.  The row-order general path (keys spanning > 2048) holds
    ≈ 16 B per row (sorted keys and values, the sort's scratch), the
    partitioned GROUP BY (10^5 keys, capacity > 4096) 6 B per row of
    staging: at least 20 B per row must come back."""
    lib = wx.load()
    n = 16_000_003
    rng = np.random.default_rng(71)
    cols = {"price": rng.uniform(0, 40, n).astype(np.float32),
            "quantity": rng.integers(0, 100_000, n).astype(np.int32)}
    t, _ = dev_table(cols)
    cap = 1 << 17
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")

    def query(flags):
        return wx.group_sum(t, "price[idx]", "quantity[idx]", None, launch(flags), 0, cap, keys.data_ptr(),
                            sums.data_ptr(), cnts.data_ptr())

    g_plain = query(0)
    g_rows = query(wx.F_ROW_ORDER)
    assert g_plain == g_rows == len(np.unique(cols["quantity"]))
    torch.cuda.synchronize()
    free_before = torch.cuda.mem_get_info()[0]
    lib.wx_shutdown()
    torch.cuda.synchronize()
    free_after = torch.cuda.mem_get_info()[0]
    assert free_after - free_before >= 20 * n, (free_before, free_after)
    s_before = sums[:g_rows].clone()
    assert query(wx.F_ROW_ORDER) == g_rows  # the workspaces and modules come back
    assert torch.equal(sums[:g_rows].view(torch.int64), s_before.view(torch.int64))


@pytest.mark.parametrize("rows", [1, 2, 63, 64, 65])
def test_row_order_general_tiny_tables(rows, monkeypatch):
    """The general path's run-length encoding and folds at tables of one row,
    two rows and around one 64-row chunk (bare key and value columns: no
    projections; the sort skipped for a single row)."""
    monkeypatch.setenv("WARPDB_GROUP_ROWS", "general")
    rng = np.random.default_rng(rows)
    cols = {"price": spread_values(rng, rows), "quantity": rng.integers(-3, 3, rows).astype(np.int32) * 5000}
    g, k, s, c = run(cols, None, 64)
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", capacity=64)
    assert g == len(rk) and np.array_equal(k, rk) and np.array_equal(c, rc)
    assert np.array_equal(bits(s), bits(rs))
