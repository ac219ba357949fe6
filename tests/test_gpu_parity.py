"""GPU parity tests: the HIP path through the C ABI against the CPU oracle.

Every test here calls libwarpexec.so (include/warpexec.h) with device
buffers and compares against oracle/liboracle.so on the same seeded inputs.
Bar: bit-exact for compaction indices, projections and double sums (the
build uses -ffp-contract=off); order of GROUP BY / top-K results exact.
Sizes are chosen so the oracle finishes in seconds; the 2^28-row case checks
size-independent properties instead.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle_lib as ora
import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from warpdb_amd import _warpexec as wx  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
DISCOUNT_SRC = "__device__ float discount(float price, float rate) {\n    return price * rate;\n}\n"
_TD = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
       np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}


def dev_table(cols, offset=0):
    """Upload numpy columns; `offset` elements of padding make pointers unaligned."""
    tensors = {}
    for k, v in cols.items():
        t = torch.empty(len(v) + offset, dtype=_TD[v.dtype], device="cuda")
        if len(v):
            t[offset:].copy_(torch.from_numpy(v))
        tensors[k] = t[offset:]
    n = len(next(iter(cols.values())))
    dt = {torch.int32: wx.INT32, torch.int64: wx.INT64, torch.float32: wx.FLOAT32, torch.float64: wx.FLOAT64}
    table = wx.Table(n, [wx.Column(k, dt[t.dtype], t.data_ptr() if n else 0) for k, t in tensors.items()],
                     owners=list(tensors.values()))
    return table, tensors


def launch(flags=wx.F_SYNC, custom=DISCOUNT_SRC):
    return wx.make_launch(device=0, stream=torch.cuda.current_stream().cuda_stream, custom_src=custom,
                          flags=flags)


def gpu_compact(table, expr, cond, idx_bytes=8, row_base=0):
    n = table.n_rows
    vals = torch.full((max(1, n),), float("nan"), dtype=torch.float32, device="cuda")
    idx = torch.full((max(1, n),), -1, dtype=torch.int64 if idx_bytes == 8 else torch.int32, device="cuda")
    cnt = wx.project_filter(table, expr, cond, launch(), wx.MODE_COMPACT, vals.data_ptr(), idx.data_ptr(),
                            idx_bytes, row_base, want_count=True)
    return vals[:cnt].cpu().numpy(), idx[:cnt].cpu().numpy()


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def read_csv(path):
    import csv

    with open(path) as f:
        r = list(csv.reader(f))
    names = r[0]
    return {n: np.array([float(row[i]) for row in r[1:]], np.float32) for i, n in enumerate(names)}


# ------------------------------------------------------------------ goldens
def load_golden():
    import json

    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", range(len(load_golden()["project"])))
def test_golden_project(case):
    g = load_golden()["project"][case]
    cols = read_csv(os.path.join(GOLDEN, g["csv"]))
    table, _ = dev_table(cols)
    expr, cond = ora.split_where(g["query"])
    e = ora.lower(expr)
    c = ora.lower(cond) if cond.strip() else None
    vals, idx = gpu_compact(table, e, c)
    assert idx.tolist() == g["idx"]
    assert [float.hex(float(v)) for v in vals] == [float.hex(float.fromhex(x)) for x in g["vals"]]


def test_dense_mode_leaves_unselected_rows():
    cols = read_csv(os.path.join(GOLDEN, "test.csv"))
    table, _ = dev_table(cols)
    out = torch.full((4,), -7.0, device="cuda")
    wx.project_filter(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", launch(), wx.MODE_DENSE,
                      out.data_ptr())
    assert out.cpu().tolist() == [-7.0, -7.0, -7.0, 27.0]
    wx.project_filter(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", launch(), wx.MODE_DENSE_FILL,
                      out.data_ptr())
    assert out.cpu().tolist() == [0.0, 0.0, 0.0, 27.0]
    wx.project_filter(table, "(price[idx] * 0.9f)", None, launch(), wx.MODE_DENSE, out.data_ptr())
    ref = ora.dense(ora.HostTable(cols), "price * 0.9", None, np.zeros(4, np.float32))
    assert (bits(out.cpu().numpy()) == bits(ref)).all()


@pytest.mark.parametrize("n", [1, 4095, 4097, 4 * 256 * 4 * 7 + 5, 1_000_003])
@pytest.mark.parametrize("offset", [0, 1])
def test_dense_vs_oracle(n, offset):
    # src/jit.cpp:55-61: out[idx] = expr where cond; unselected rows untouched
    # (MODE_DENSE) or 0.0f (MODE_DENSE_FILL, WarpDB::query's zeroed result)
    cols = synth.c2_table(n)
    table, _ = dev_table(cols, offset)
    ht = ora.HostTable(cols)
    sentinel = np.full(n, -7.0, np.float32)
    for mode, fill in ((wx.MODE_DENSE, sentinel), (wx.MODE_DENSE_FILL, np.zeros(n, np.float32))):
        buf = torch.full((n + offset,), -7.0, dtype=torch.float32, device="cuda")
        out = buf[offset:]
        wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", launch(), mode,
                          out.data_ptr())
        ref = ora.dense(ht, "price * quantity", "price > 15", fill)
        assert (bits(out.cpu().numpy()) == bits(ref)).all()
        if offset:
            assert buf[0].item() == -7.0


@pytest.mark.parametrize("mode", ["masked", "fill"])
def test_dense_many_spans_per_workgroup(mode):
    # 2^23 + 5 rows: every workgroup walks several whole spans through the
    # software-pipelined loop (masked mode: old output quads read and blended)
    # and then the ragged tail; unselected rows keep a per-row sentinel
    n = (1 << 23) + 5
    cols = synth.c2_table(n)
    table, t = dev_table(cols)
    price, qty = t["price"], t["quantity"]
    sentinel = torch.arange(n, dtype=torch.float32, device="cuda") * -1.0 - 0.5
    out = sentinel.clone()
    m = wx.MODE_DENSE if mode == "masked" else wx.MODE_DENSE_FILL
    wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", launch(), m, out.data_ptr())
    keep = sentinel if mode == "masked" else torch.zeros_like(sentinel)
    want = torch.where(price > 15.0, price * qty, keep)
    assert torch.equal(out.view(torch.int32), want.view(torch.int32))


def test_jit_arch_identity_raw_expression():
    # tests/jit_arch_test.cpp:6-38: the un-lowered expression "price" -> 2.0
    table, _ = dev_table({"price": np.array([2.0], np.float32), "quantity": np.array([0], np.int32)})
    out = torch.zeros(1, device="cuda")
    wx.project_filter(table, "price", "", launch(), wx.MODE_DENSE, out.data_ptr())
    assert out.item() == 2.0
    wx.project_filter(table, "price + 1", "", launch(), wx.MODE_DENSE, out.data_ptr())
    assert out.item() == 3.0


def test_compile_error_then_recovery():
    # tests/jit_error_test.cpp:19-33
    table, _ = dev_table({"price": np.array([1.5], np.float32), "quantity": np.array([2], np.int32)})
    out = torch.zeros(1, device="cuda")
    with pytest.raises(wx.WarpExecError) as ei:
        wx.project_filter(table, "invalid@", "", launch(), wx.MODE_DENSE, out.data_ptr())
    assert ei.value.status == wx.WX_ERR_COMPILE
    assert "Kernel compilation failed" in str(ei.value)
    wx.project_filter(table, "price + 1", "", launch(), wx.MODE_DENSE, out.data_ptr())
    assert out.item() == 2.5


# ------------------------------------------------------- synthetic parity
@pytest.mark.parametrize("sched", ["deep", "ticket"])
@pytest.mark.parametrize("n", [0, 1, 5, 4095, 4096, 4097, 12289, 65536 + 3, 1_000_003])
def test_compact_c2_shape_vs_oracle(n, sched, monkeypatch):
    # both compaction schedules (the default pipeline and the one-tile-per-workgroup fallback)
    monkeypatch.setenv("WARPDB_COMPACT_SCHED", sched)
    cols = synth.c2_table(n)
    table, _ = dev_table(cols)
    vals, idx = gpu_compact(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)")
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * quantity", "price > 15")
    assert np.array_equal(idx, ri)
    assert np.array_equal(bits(vals), bits(rv))


@pytest.mark.parametrize("n", [3_158_017, 12_582_912])
def test_compact_many_tiles_row_base_vs_oracle(n):
    # more tiles than workgroups (several pipeline iterations each), a ragged
    # or whole last tile, and a row base in the stored indices
    cols = synth.c2_table(n, row_base=77)
    table, _ = dev_table(cols)
    vals, idx = gpu_compact(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", row_base=77)
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * quantity", "price > 15")
    assert np.array_equal(idx, ri + 77)
    assert np.array_equal(bits(vals), bits(rv))


@pytest.mark.parametrize("cond", ["price > 100", "price >= 0", "price > 10 AND quantity < 50",
                                  "price < 1 OR price > 39", "quantity = 7"])
def test_compact_selectivity_extremes(cond):
    n = 300_001
    cols = synth.c2_table(n)
    table, _ = dev_table(cols)
    vals, idx = gpu_compact(table, ora.lower("price * 0.9 + quantity"), ora.lower(cond))
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * 0.9 + quantity", cond)
    assert np.array_equal(idx, ri)
    assert np.array_equal(bits(vals), bits(rv))


@pytest.mark.parametrize("n,offset", [(0, 0), (5, 0), (300_001, 0), (300_001, 1)])
def test_compact_without_where(n, offset):
    # no WHERE and no indices: every row in order (run as the dense projection);
    # with indices: the compaction kernel, indices 0..n-1
    cols = synth.c2_table(n)
    table, _ = dev_table(cols, offset=offset)
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * quantity + 1", None)
    out = torch.full((max(1, n) + 1,), float("nan"), device="cuda")
    vals = out[offset:offset + max(1, n)]
    cnt = wx.project_filter(table, ora.lower("price * quantity + 1"), None, launch(), wx.MODE_COMPACT,
                            vals.data_ptr(), 0, 8, 0, want_count=True)
    assert cnt == n == len(rv)
    assert np.array_equal(bits(vals[:n].cpu().numpy()), bits(rv))
    dc = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    wx.project_filter(table, ora.lower("price * quantity + 1"), None, launch(), wx.MODE_COMPACT, 0, 0, 8, 0,
                      d_count=dc.data_ptr())
    assert int(dc.item()) == n
    v2, i2 = gpu_compact(table, ora.lower("price * quantity + 1"), None)
    assert np.array_equal(i2, ri) and np.array_equal(bits(v2), bits(rv))


def test_compact_int32_index_and_row_base():
    n = 123_457
    cols = synth.c2_table(n, row_base=1000)
    table, _ = dev_table(cols)
    vals, idx = gpu_compact(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", idx_bytes=4, row_base=1000)
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * 0.9", "price > 20")
    assert np.array_equal(idx.astype(np.int64), ri + 1000)
    assert np.array_equal(bits(vals), bits(rv))


def test_compact_unaligned_columns():
    n = 100_003
    cols = synth.c2_table(n)
    table, _ = dev_table(cols, offset=1)
    vals, idx = gpu_compact(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)")
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * quantity", "price > 15")
    assert np.array_equal(idx, ri)
    assert np.array_equal(bits(vals), bits(rv))


def test_mixed_types_follow_jit_semantics():
    n = 50_000
    rng = np.random.default_rng(7)
    cols = {
        "a": rng.integers(-1000, 1000, n).astype(np.int32),
        "b": rng.integers(1, 50, n).astype(np.int32),
        "c": rng.uniform(-5, 5, n).astype(np.float64),
        "d": rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64),
    }
    table, _ = dev_table(cols)
    for e_sql, e_c, c_sql, c_c in [
        ("a / b", "(a[idx] / b[idx])", "a > 0", "(a[idx] > 0.0f)"),
        ("c * a + 1", "((c[idx] * a[idx]) + 1.0f)", "c < 2.5", "(c[idx] < 2.5f)"),
        ("d / 3", "(d[idx] / 3.0f)", "d != b", "(d[idx] != b[idx])"),
    ]:
        vals, idx = gpu_compact(table, e_c, c_c)
        rv, ri = ora.project_filter(ora.HostTable(cols), e_sql, c_sql, sem=ora.SEM_JIT)
        assert np.array_equal(idx, ri), e_sql
        assert np.array_equal(bits(vals), bits(rv)), e_sql


def test_large_compaction_properties():
    """2^28 rows: ordering, count and values checked against torch on device."""
    n = 1 << 28
    price = torch.empty(n, dtype=torch.float32, device="cuda")
    qty = torch.empty(n, dtype=torch.float32, device="cuda")
    L = launch()
    wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, synth.SEED_PRICE, 0, 0.0, 40.0, L)
    wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, synth.SEED_QTY, 1, 1, 100, L)
    head = synth.c2_table(4096)
    assert np.array_equal(price[:4096].cpu().numpy(), head["price"])
    assert np.array_equal(qty[:4096].cpu().numpy(), head["quantity"])
    table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()),
                         wx.Column("quantity", wx.FLOAT32, qty.data_ptr())])
    vals = torch.empty(n, dtype=torch.float32, device="cuda")
    idx = torch.empty(n, dtype=torch.int32, device="cuda")
    cnt = wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", L, wx.MODE_COMPACT,
                            vals.data_ptr(), idx.data_ptr(), 4, 0, want_count=True)
    mask = price > 15.0
    assert cnt == int(mask.sum().item())
    ref_idx = torch.nonzero(mask).flatten().to(torch.int32)
    assert torch.equal(idx[:cnt], ref_idx)
    assert torch.equal(vals[:cnt], (price * qty)[mask])


# ------------------------------------------------------------------ SUM
@pytest.mark.parametrize("n", [0, 3, 4096 * 7 + 1, 2_000_003])
def test_sum_vs_oracle(n):
    cols = synth.c2_table(n)
    table, _ = dev_table(cols)
    s, c = wx.reduce_sum(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", launch())
    rs, rc = ora.reduce_sum(ora.HostTable(cols), "price * 0.9", "price > 20")
    assert c == rc
    assert s == rs  # float values summed in double: exact at these sizes


# -------------------------------------------------------------- GROUP BY
@pytest.mark.parametrize("n", [1, 1000, 2_000_003])
def test_group_sum_c3_shape(n):
    cols = synth.c3_table(n)
    table, _ = dev_table(cols)
    cap = 4096
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, launch(), 0, cap, keys.data_ptr(),
                     sums.data_ptr(), cnts.data_ptr())
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity")
    assert g == len(rk)
    assert np.array_equal(keys[:g].cpu().numpy(), rk)
    assert np.array_equal(sums[:g].cpu().numpy(), rs)
    assert np.array_equal(cnts[:g].cpu().numpy(), rc)


def test_group_sum_keys_outside_window_and_filter():
    n = 400_000
    rng = np.random.default_rng(11)
    cols = {"price": synth.uniform_f32(n, 1, 0.0, 40.0),
            "k": rng.choice(np.array([-5, -1, 0, 7, 2047, 2048, 5000, 1 << 30, -(1 << 31)], np.int32), n)}
    table, _ = dev_table(cols)
    cap = 64
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    for _ in range(2):  # second call checks the tables were left clean
        g = wx.group_sum(table, "(price[idx] * 2.0f)", "k[idx]", "(price[idx] < 30.0f)", launch(), 0, cap,
                         keys.data_ptr(), sums.data_ptr(), cnts.data_ptr())
        rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price * 2", "k", "price < 30")
        assert g == len(rk)
        assert np.array_equal(keys[:g].cpu().numpy(), rk)
        assert np.array_equal(sums[:g].cpu().numpy(), rs)
        assert np.array_equal(cnts[:g].cpu().numpy(), rc)


def test_group_sum_reference_golden():
    # tests/sql_features_test.cpp:11-22 on data/test.csv: keys 2,3,4,5
    cols = read_csv(os.path.join(GOLDEN, "test.csv"))
    table, _ = dev_table(cols)
    keys = torch.empty(8, dtype=torch.int32, device="cuda")
    sums = torch.empty(8, dtype=torch.float64, device="cuda")
    cnts = torch.empty(8, dtype=torch.int64, device="cuda")
    g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, launch(), 0, 8, keys.data_ptr(),
                     sums.data_ptr(), cnts.data_ptr())
    assert g == 4
    assert keys[:4].cpu().tolist() == [2, 3, 4, 5]
    assert sums[:4].cpu().tolist() == [15.25, 10.5, 20.0, 30.0]


def _nan_minus_zero(n, seed):
    """float32 values with NaNs, -0.0 and ties (MIN / MAX edge cases)."""
    u = synth.uniform_f32(n, seed + 100, 0.0, 1.0)
    v = np.round(synth.uniform_f32(n, seed, -50.0, 50.0), 1).astype(np.float32)
    v[u < 0.02] = np.nan
    v[(u >= 0.02) & (u < 0.05)] = np.float32(-0.0)
    return v


@pytest.mark.parametrize("cond,ocond", [(None, None), ("(price[idx] > 20.0f)", "price > 20"),
                                        ("(price[idx] > 1000.0f)", "price > 1000")])
def test_reduce_stats_vs_oracle(cond, ocond):
    # ungrouped SUM / COUNT / MIN / MAX (query_sql aggregates, optimizer stats)
    n = 1_000_003
    cols = {"price": synth.uniform_f32(n, 1, 0.0, 40.0), "v": _nan_minus_zero(n, 5)}
    table, _ = dev_table(cols)
    for expr, oexpr in (("(price[idx] * 0.9f)", "price * 0.9"), ("v[idx]", "v")):
        s, c, mn, mx = wx.reduce_stats(table, expr, cond, launch())
        rs, rc, rmn, rmx = ora.stats(ora.HostTable(cols), oexpr, ocond)
        assert c == rc
        assert (s == rs) or (np.isnan(s) and np.isnan(rs))
        assert np.array_equal(bits(np.float32(mn)), bits(rmn)) or (np.isnan(mn) and np.isnan(rmn))
        assert np.array_equal(bits(np.float32(mx)), bits(rmx)) or (np.isnan(mx) and np.isnan(rmx))
    # the plain SUM entry point is unchanged by the MIN / MAX build
    s2, c2 = wx.reduce_sum(table, "(price[idx] * 0.9f)", cond, launch())
    assert (s2, c2) == ora.reduce_sum(ora.HostTable(cols), "price * 0.9", ocond)


def test_group_agg_minmax_vs_oracle():
    n = 600_001
    rng = np.random.default_rng(3)
    keys_pool = np.concatenate([np.arange(0, 1024, dtype=np.int32),
                                np.array([-7, 2048, 99_999, -(1 << 31)], np.int32)])
    cols = {"v": _nan_minus_zero(n, 7), "k": rng.choice(keys_pool, n).astype(np.int32),
            "price": synth.uniform_f32(n, 1, 0.0, 40.0)}
    table, _ = dev_table(cols)
    cap = 2048
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    mins = torch.empty(cap, dtype=torch.float32, device="cuda")
    maxs = torch.empty(cap, dtype=torch.float32, device="cuda")
    for cond, ocond in ((None, None), ("(price[idx] < 10.0f)", "price < 10"), (None, None)):
        g = wx.group_agg(table, "v[idx]", "k[idx]", cond, launch(), 0, cap, keys.data_ptr(), sums.data_ptr(),
                         cnts.data_ptr(), mins.data_ptr(), maxs.data_ptr())
        rk, rs, rc, rmn, rmx = ora.group_agg(ora.HostTable(cols), "v", "k", ocond)
        assert g == len(rk)
        assert np.array_equal(keys[:g].cpu().numpy(), rk)
        assert np.array_equal(cnts[:g].cpu().numpy(), rc)
        assert np.array_equal(sums[:g].cpu().numpy(), rs, equal_nan=True)
        assert np.array_equal(mins[:g].cpu().numpy(), rmn, equal_nan=True)
        assert np.array_equal(maxs[:g].cpu().numpy(), rmx, equal_nan=True)
        assert not np.signbit(mins[:g].cpu().numpy()[mins[:g].cpu().numpy() == 0]).any()
    # a plain GROUP BY SUM after MIN / MAX calls sees clean tables
    g = wx.group_sum(table, "price[idx]", "k[idx]", None, launch(), 0, cap, keys.data_ptr(), sums.data_ptr(),
                     cnts.data_ptr())
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "k")
    assert g == len(rk) and np.array_equal(sums[:g].cpu().numpy(), rs)


@pytest.mark.parametrize("minmax", [False, True])
def test_group_many_general_keys(minmax):
    # > 4096 distinct keys outside the LDS window: device-sorted finalize
    n = 1_000_003
    rng = np.random.default_rng(17)
    keys = (rng.integers(0, 150_000, n) * 7 - 500_000).astype(np.int32)
    in_window = rng.uniform(size=n) < 0.2
    keys[in_window] = rng.integers(0, 2048, int(in_window.sum())).astype(np.int32)
    cols = {"price": synth.uniform_f32(n, 1, 0.0, 40.0), "k": keys}
    table, _ = dev_table(cols)
    cap = 200_000
    dk = torch.empty(cap, dtype=torch.int32, device="cuda")
    ds = torch.empty(cap, dtype=torch.float64, device="cuda")
    dc = torch.empty(cap, dtype=torch.int64, device="cuda")
    dmn = torch.empty(cap, dtype=torch.float32, device="cuda")
    dmx = torch.empty(cap, dtype=torch.float32, device="cuda")
    for _ in range(2):  # the second call checks the tables were left clean
        if minmax:
            g = wx.group_agg(table, "price[idx]", "k[idx]", None, launch(), 0, cap, dk.data_ptr(), ds.data_ptr(),
                             dc.data_ptr(), dmn.data_ptr(), dmx.data_ptr())
            rk, rs, rc, rmn, rmx = ora.group_agg(ora.HostTable(cols), "price", "k")
            assert np.array_equal(dmn[:g].cpu().numpy(), rmn) and np.array_equal(dmx[:g].cpu().numpy(), rmx)
        else:
            g = wx.group_sum(table, "price[idx]", "k[idx]", None, launch(), 0, cap, dk.data_ptr(), ds.data_ptr(),
                             dc.data_ptr())
            rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "k")
        assert g == len(rk) and g > 100_000
        assert np.array_equal(dk[:g].cpu().numpy(), rk)
        assert np.array_equal(ds[:g].cpu().numpy(), rs)
        assert np.array_equal(dc[:g].cpu().numpy(), rc)


def test_group_capacity_error():
    cols = synth.c3_table(10_000)
    table, _ = dev_table(cols)
    keys = torch.empty(10, dtype=torch.int32, device="cuda")
    sums = torch.empty(10, dtype=torch.float64, device="cuda")
    cnts = torch.empty(10, dtype=torch.int64, device="cuda")
    with pytest.raises(wx.WarpExecError) as ei:
        wx.group_sum(table, "price[idx]", "quantity[idx]", None, launch(), 0, 10, keys.data_ptr(),
                     sums.data_ptr(), cnts.data_ptr())
    assert ei.value.status == wx.WX_ERR_CAPACITY
    # engine still healthy afterwards
    big = torch.empty(2048, dtype=torch.int32, device="cuda")
    bs = torch.empty(2048, dtype=torch.float64, device="cuda")
    bc = torch.empty(2048, dtype=torch.int64, device="cuda")
    g = wx.group_sum(table, "price[idx]", "quantity[idx]", None, launch(), 0, 2048, big.data_ptr(),
                     bs.data_ptr(), bc.data_ptr())
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity")
    assert g == len(rk) and np.array_equal(bs[:g].cpu().numpy(), rs)


# ---------------------------------------------------------------- top-K
@pytest.mark.parametrize("k,desc", [(5, True), (1, True), (5, False), (32, True)])
def test_topk_vs_oracle(k, desc):
    n = 1_000_003
    cols = synth.c2_table(n)
    table, _ = dev_table(cols)
    keys = torch.empty(k, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    vals = torch.empty(k, device="cuda")
    m = wx.topk(table, "price[idx]", None, "discount(price[idx], 0.9f)", k, desc, launch(), keys.data_ptr(),
                idx.data_ptr(), vals.data_ptr())
    rk, ri, rv = ora.topk(ora.HostTable(cols), "price", k, desc, select_expr="discount(price, 0.9)")
    assert m == len(rk)
    assert np.array_equal(bits(keys[:m].cpu().numpy()), bits(rk))
    assert np.array_equal(idx[:m].cpu().numpy(), ri)
    assert np.array_equal(bits(vals[:m].cpu().numpy()), bits(rv))


def test_topk_ties_and_filter():
    n = 200_000
    cols = {"price": np.floor(synth.uniform_f32(n, 1, 0.0, 40.0)).astype(np.float32),
            "quantity": synth.uniform_int(n, 2, 1, 100).astype(np.float32)}
    table, _ = dev_table(cols)
    k = 7
    keys = torch.empty(k, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    m = wx.topk(table, "(price[idx] + quantity[idx])", "(quantity[idx] < 50.0f)", None, k, True, launch(),
                keys.data_ptr(), idx.data_ptr())
    rk, ri, _ = ora.topk(ora.HostTable(cols), "price + quantity", k, True, cond="quantity < 50")
    assert m == k
    assert np.array_equal(idx[:m].cpu().numpy(), ri)
    assert np.array_equal(keys[:m].cpu().numpy(), rk)


@pytest.mark.parametrize("desc", [True, False])
@pytest.mark.parametrize("k", [1, 5, 32])
def test_topk_heavy_ties_nan_signed_zero(k, desc):
    # few distinct keys (every key tied thousands of times), NaNs and -0.0/+0.0,
    # ragged row count: the wave threshold must keep the smallest row indices
    n = 4_000_037
    u = synth.uniform_f32(n, 9, 0.0, 1.0)
    p = np.floor(synth.uniform_f32(n, 1, -3.0, 3.0)).astype(np.float32)
    p[u < 0.01] = np.nan
    p[(u >= 0.01) & (u < 0.3)] = np.float32(-0.0)
    cols = {"price": p, "quantity": synth.uniform_int(n, 2, 1, 100).astype(np.float32)}
    table, _ = dev_table(cols)
    keys = torch.empty(k, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    for cond, ocond in ((None, None), ("(quantity[idx] > 50.0f)", "quantity > 50")):
        m = wx.topk(table, "price[idx]", cond, None, k, desc, launch(), keys.data_ptr(), idx.data_ptr())
        rk, ri, _ = ora.topk(ora.HostTable(cols), "price", k, desc, cond=ocond)
        assert m == len(rk)
        assert np.array_equal(idx[:m].cpu().numpy(), ri)
        assert np.array_equal(bits(keys[:m].cpu().numpy()), bits(rk))


@pytest.mark.parametrize("layout", ["one_lane", "sorted", "reverse"])
@pytest.mark.parametrize("k", [9, 16, 32])
def test_topk_large_k_spill_paths(k, layout):
    # K > 8 keeps 8 rows per lane and spills the rest to the wave's list:
    # the winners packed into one lane's rows (quad q = 5 + 256 u of the first
    # 2 048-quad span: 32 of them, 16 more in quad 6 + 256 u), every row a new
    # best (sorted input, descending order) or a new worst (reversed)
    n = 1_000_003
    p = synth.uniform_f32(n, 21, 0.0, 40.0)
    if layout == "one_lane":
        rows = [4 * (5 + 256 * u) + e for u in range(8) for e in range(4)]
        rows += [4 * (6 + 256 * u) + e for u in range(4) for e in range(4)]
        p[np.array(rows)] = np.float32(100.0) + np.arange(len(rows), dtype=np.float32)[::-1]
    elif layout == "sorted":
        p = np.sort(p)
    else:
        p = np.sort(p)[::-1].copy()
    cols = {"price": p.astype(np.float32), "quantity": synth.uniform_int(n, 2, 1, 100).astype(np.float32)}
    table, _ = dev_table(cols)
    keys = torch.empty(k, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    for desc in (True, False):
        for cond, ocond in ((None, None), ("(quantity[idx] > 50.0f)", "quantity > 50")):
            m = wx.topk(table, "price[idx]", cond, None, k, desc, launch(), keys.data_ptr(), idx.data_ptr())
            rk, ri, _ = ora.topk(ora.HostTable(cols), "price", k, desc, cond=ocond)
            assert m == len(rk)
            assert np.array_equal(idx[:m].cpu().numpy(), ri)
            assert np.array_equal(bits(keys[:m].cpu().numpy()), bits(rk))


@pytest.mark.parametrize("data", ["ties", "nan", "sorted"])
@pytest.mark.parametrize("k", [1, 5, 32])
def test_topk_seed_pass(k, data, monkeypatch):
    # WX_TOPK_SEED=2 forces the seed pass (wx_topk_seed + a seed finalize into
    # bound slot 0) on a table below its default 2^24 rows.  Heavy ties: the
    # seed equals the winners' key, and the winners are the smallest row
    # indices among thousands of equal keys, most of them outside the sample.
    monkeypatch.setenv("WARPDB_EXTRA_DEFINES", "WX_TOPK_SEED=2")
    n = 300_003
    p = synth.uniform_f32(n, 33, 0.0, 40.0)
    if data == "ties":
        p = (np.round(p * 2.0) / 2.0).astype(np.float32)
    elif data == "nan":
        p[::7] = np.float32("nan")
        p[1::11] = np.float32(-0.0)
    else:
        p = np.sort(p)
    cols = {"price": p.astype(np.float32), "quantity": synth.uniform_int(n, 3, 1, 100).astype(np.float32)}
    table, _ = dev_table(cols)
    keys = torch.empty(k, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    for desc in (True, False):
        for cond, ocond in ((None, None), ("(quantity[idx] > 50.0f)", "quantity > 50")):
            m = wx.topk(table, "price[idx]", cond, None, k, desc, launch(), keys.data_ptr(), idx.data_ptr())
            rk, ri, _ = ora.topk(ora.HostTable(cols), "price", k, desc, cond=ocond)
            assert m == len(rk)
            assert np.array_equal(idx[:m].cpu().numpy(), ri)
            assert np.array_equal(bits(keys[:m].cpu().numpy()), bits(rk))


def test_topk_seed_pass_default_size():
    # the default seed rule (K >= 5 over tables of 2^24 rows and more; K = 4
    # runs without it), ties at the winners
    n = (1 << 24) + 5
    p = (np.round(synth.uniform_f32(n, 34, 0.0, 40.0) * 4.0) / 4.0).astype(np.float32)
    cols = {"price": p}
    table, _ = dev_table(cols)
    keys = torch.empty(32, device="cuda")
    idx = torch.empty(32, dtype=torch.int64, device="cuda")
    for k, desc in ((4, True), (5, True), (5, False), (9, True), (32, False)):
        m = wx.topk(table, "price[idx]", None, None, k, desc, launch(), keys.data_ptr(), idx.data_ptr())
        rk, ri, _ = ora.topk(ora.HostTable(cols), "price", k, desc)
        assert m == len(rk) == k
        assert np.array_equal(idx[:m].cpu().numpy(), ri)
        assert np.array_equal(bits(keys[:m].cpu().numpy()), bits(rk))


def test_topk_fewer_rows_than_k():
    cols = read_csv(os.path.join(GOLDEN, "test.csv"))
    table, _ = dev_table(cols)
    keys = torch.empty(5, device="cuda")
    m = wx.topk(table, "price[idx]", None, None, 5, True, launch(), keys.data_ptr())
    assert m == 4
    assert keys[:4].cpu().tolist() == [30.0, 20.0, 15.25, 10.5]  # SURVEY.md 8c, C5 golden


# ----------------------------------------------------------------- sorts
@pytest.mark.parametrize("n", [1, 17, 2048, 5000, 70_000])
def test_sort_float_and_pairs(n):
    rng = np.random.default_rng(n)
    v = np.round(rng.uniform(-100, 100, n), 1).astype(np.float32)
    for asc in (True, False):
        t = torch.from_numpy(v.copy()).cuda()
        wx.sort_float(t.data_ptr(), n, asc, launch())
        ref = np.sort(v) if asc else -np.sort(-v)
        assert np.array_equal(t.cpu().numpy(), ref)
    keys = rng.integers(-50, 50, n).astype(np.int32)
    for asc in (True, False):
        tk = torch.from_numpy(keys.copy()).cuda()
        tv = torch.from_numpy(v.copy()).cuda()
        wx.sort_pairs(tk.data_ptr(), tv.data_ptr(), n, asc, launch())
        order = np.argsort(keys if asc else -keys.astype(np.int64), kind="stable")
        assert np.array_equal(tk.cpu().numpy(), keys[order])
        assert np.array_equal(tv.cpu().numpy(), v[order])


def _sort_input(n, seed):
    # heavy ties, NaN, -0.0 / +0.0, infinities: the order key must keep equal
    # keys in input order (stable) and NaN last in both directions
    u = synth.uniform_f32(n, seed, 0.0, 1.0)
    v = np.floor(synth.uniform_f32(n, seed + 1, -1000.0, 1000.0)).astype(np.float32) / np.float32(8.0)
    v[u < 0.01] = np.nan
    v[(u >= 0.01) & (u < 0.05)] = np.float32(-0.0)
    v[(u >= 0.05) & (u < 0.09)] = np.float32(0.0)
    v[(u >= 0.09) & (u < 0.095)] = np.float32(np.inf)
    v[(u >= 0.095) & (u < 0.1)] = np.float32(-np.inf)
    return v


# the bitonic path is a cross-check at small sizes only
# radix tile edges: key tiles hold 512 x 32 = 16 384 keys, key + payload tiles 512 x 20 = 10 240
@pytest.mark.parametrize("sort,n", [("radix", n) for n in (8191, 10240, 10241, 16383, 16384, 16385, 24577,
                                                           3 * 16384 + 1, 3_000_017)]
                         + [("bitonic", 8191)])
def test_sort_float_stable_nan_signed_zero(n, sort, monkeypatch):
    monkeypatch.setenv("WARPDB_SORT", sort)
    v = _sort_input(n, 11)
    for asc in (True, False):
        t = torch.from_numpy(v.copy()).cuda()
        wx.sort_float(t.data_ptr(), n, asc, launch())
        ref = v[np.argsort(v if asc else -v, kind="stable")]
        assert np.array_equal(bits(t.cpu().numpy()), bits(ref))


@pytest.mark.parametrize("n", [16385, 1_000_003])
@pytest.mark.parametrize("special", [None, "neg_zero_last", "nan_first", "neg_zero_tail"])
def test_sort_float_plain_flip_equals_general_map(n, special, monkeypatch):
    """The radix tiles' plain order flip (taken when the histogram pass saw no
    NaN and no -0.0) sorts exactly as the general order map: +0.0, infinities
    and heavy ties included; one NaN or -0.0 anywhere -- also in the last,
    scalar-loaded elements -- makes the pass take the general map."""
    v = _sort_input(n, 31)
    v[np.isnan(v)] = np.float32(np.inf)
    v[(v == 0) & np.signbit(v)] = np.float32(0.0)
    if special == "neg_zero_last":
        v[-1] = np.float32(-0.0)
    elif special == "nan_first":
        v[0] = np.float32(np.nan)
    elif special == "neg_zero_tail":
        v[n - (n % 4 or 1)] = np.float32(-0.0)
    for asc in (True, False):
        ref = v[np.argsort(v if asc else -v, kind="stable")]
        for plain in ("1", "0"):
            monkeypatch.setenv("WARPDB_RS_PLAIN", plain)
            t = torch.from_numpy(v.copy()).cuda()
            wx.sort_float(t.data_ptr(), n, asc, launch())
            assert np.array_equal(bits(t.cpu().numpy()), bits(ref)), (plain, asc)


@pytest.mark.parametrize("n", [10241, 1_000_003])
def test_sort_ranking_modes_agree(n, monkeypatch):
    """The tiles' in-wave ranking by one LDS add per key (WARPDB_RS_LEAD=0),
    with lane 0's digit group ranked by one ballot (1, the default) and chosen
    per pass from the histogram (auto), and the peer-mask ranking (the
    non-gfx950 build) all give the oracle's stable order:
    float keys with heavy ties, and int key + row payload pairs whose keys
    skew one digit (a few small values) next to a full-range digit."""
    monkeypatch.setenv("WARPDB_SORT", "radix")
    v = _sort_input(n, 41)
    rng = np.random.default_rng(n)
    keys = np.where(rng.random(n) < 0.7, rng.integers(0, 3, n), rng.integers(-2**31, 2**31 - 1, n)).astype(np.int32)
    rows = np.arange(n, dtype=np.int32)
    for asc in (True, False):
        ref = v[np.argsort(v if asc else -v, kind="stable")]
        order = np.argsort(keys if asc else -keys.astype(np.int64), kind="stable")
        # "peer": the peer-mask ranking (WX_RS_RANK_ATOMIC=0), what any target
        # other than gfx950 builds (the atomic form's stability rests on the
        # LDS returning same-address adds in lane order, observed on gfx950)
        for lead in ("0", "1", "auto", "peer"):
            monkeypatch.setenv("WARPDB_RS_RANK_ATOMIC", "0" if lead == "peer" else "")
            monkeypatch.setenv("WARPDB_RS_LEAD", "1" if lead == "peer" else lead)
            t = torch.from_numpy(v.copy()).cuda()
            wx.sort_float(t.data_ptr(), n, asc, launch())
            assert np.array_equal(bits(t.cpu().numpy()), bits(ref)), (lead, asc)
            tk = torch.from_numpy(keys.copy()).cuda()
            tv = torch.from_numpy(rows.copy()).cuda()
            wx.sort_pairs(tk.data_ptr(), tv.data_ptr(), n, asc, launch())
            assert np.array_equal(tk.cpu().numpy(), keys[order]), (lead, asc)
            assert np.array_equal(tv.cpu().numpy(), rows[order]), (lead, asc)


@pytest.mark.parametrize("sort,n,data", [("radix", n, "mixed") for n in (1, 2, 8191, 16385, 3 * 16384 + 1, 1_000_003)]
                         + [("radix", 70_001, "constant"), ("radix", 70_001, "small_ints"),
                            ("bitonic", 8191, "mixed")])
def test_sort_float_from_column(sort, n, data, monkeypatch):
    # ORDER BY a bare column: the sort reads the column and writes a separate
    # buffer; the result equals the in-place sort's bit for bit, the column is
    # untouched, whatever number of passes runs (constant keys skip all four,
    # small integers three) and whichever buffer the last pass lands in
    monkeypatch.setenv("WARPDB_SORT", sort)
    if data == "mixed":
        v = _sort_input(n, 23)
    elif data == "constant":
        v = np.full(n, 7.5, dtype=np.float32)
    else:
        v = synth.uniform_int(n, 9, 0, 99).astype(np.float32)
    for asc in (True, False):
        src = torch.from_numpy(v.copy()).cuda()
        dst = torch.full((n,), 12345.0, device="cuda")
        wx.sort_float_from(src.data_ptr(), dst.data_ptr(), n, asc, launch())
        ref = v[np.argsort(v if asc else -v, kind="stable")]
        assert np.array_equal(bits(dst.cpu().numpy()), bits(ref))
        assert np.array_equal(bits(src.cpu().numpy()), bits(v)), "the source column was written"
        same = torch.from_numpy(v.copy()).cuda()  # src == dst: in place
        wx.sort_float_from(same.data_ptr(), same.data_ptr(), n, asc, launch())
        assert np.array_equal(bits(same.cpu().numpy()), bits(ref))


@pytest.mark.parametrize("n", [10240, 10241, 12288, 12289, 2 * 10240 + 1, 100_003, 2_500_001])
@pytest.mark.parametrize("span", ["narrow", "full"])
def test_sort_pairs_radix_stable(n, span):
    # narrow keys leave three digits constant (those passes are skipped);
    # full-range keys include INT_MIN / INT_MAX.  Payload = input position,
    # so the payload order proves stability.
    if span == "narrow":
        keys = synth.uniform_int(n, 5, 0, 99).astype(np.int32)
    else:
        keys = (synth.uniform_int(n, 6, 0, (1 << 32) - 1).astype(np.int64) - (1 << 31)).astype(np.int32)
        keys[:3] = [np.iinfo(np.int32).min, np.iinfo(np.int32).max, 0]
        keys[n // 2:n // 2 + 1000] = 7  # a long run of ties
    pos = np.arange(n, dtype=np.float32)
    for asc in (True, False):
        tk = torch.from_numpy(keys.copy()).cuda()
        tv = torch.from_numpy(pos.copy()).cuda()
        wx.sort_pairs(tk.data_ptr(), tv.data_ptr(), n, asc, launch())
        order = np.argsort(keys if asc else -keys.astype(np.int64), kind="stable")
        assert np.array_equal(tk.cpu().numpy(), keys[order])
        assert np.array_equal(tv.cpu().numpy(), pos[order])


@pytest.mark.parametrize("data", ["uniform", "ties_nan"])
@pytest.mark.parametrize("limit", [0, 1, 1000, 777_777, 5_000_000])
def test_sort_limit_head_matches_full_sort(data, limit):
    # ORDER BY .. LIMIT: the first `limit` positions equal the stable full
    # sort's (uniform data takes the top-digit head path for small limits)
    n = 3_000_017
    v = synth.uniform_f32(n, 41, 0.0, 40.0) if data == "uniform" else _sort_input(n, 43)
    pos = np.arange(n, dtype=np.float32)
    k = min(limit, n)
    for asc in (True, False):
        order = np.argsort(v if asc else -v, kind="stable")[:k]
        t = torch.from_numpy(v.copy()).cuda()
        wx.sort_float_limit(t.data_ptr(), n, limit, asc, launch())
        assert np.array_equal(bits(t[:k].cpu().numpy()), bits(v[order]))
        tk = torch.from_numpy(v.copy()).cuda()
        tv = torch.from_numpy(pos.copy()).cuda()
        wx.sort_by_key_limit(tk.data_ptr(), tv.data_ptr(), n, limit, asc, launch())
        assert np.array_equal(tv[:k].cpu().numpy(), pos[order])


@pytest.mark.parametrize("n", [3, 10241, 400_007])
def test_sort_float_unaligned_view(n):
    # a sort of a tensor view 4 bytes into its allocation (scalar histogram
    # loads); the element before the view must stay untouched
    v = _sort_input(n, 31)
    buf = torch.full((n + 1,), -123.0, dtype=torch.float32, device="cuda")
    buf[1:].copy_(torch.from_numpy(v))
    wx.sort_float(buf[1:].data_ptr(), n, False, launch())
    assert np.array_equal(bits(buf[1:].cpu().numpy()), bits(v[np.argsort(-v, kind="stable")]))
    assert buf[0].item() == -123.0


@pytest.mark.parametrize("n", [5, 16385, 400_007])
@pytest.mark.parametrize("src_off,dst_off", [(1, 0), (0, 3), (2, 1)])
def test_sort_float_from_unaligned(n, src_off, dst_off):
    # ORDER BY a bare column whose source and destination start 4-12 bytes
    # past a 16-byte boundary (independently): the column-reading histogram
    # and first pass take their scalar paths; neighbours stay untouched
    v = _sort_input(n, 37)
    sbuf = torch.full((n + 4,), -321.0, dtype=torch.float32, device="cuda")
    sbuf[src_off:src_off + n].copy_(torch.from_numpy(v))
    dbuf = torch.full((n + 4,), -654.0, dtype=torch.float32, device="cuda")
    for asc in (True, False):
        wx.sort_float_from(sbuf[src_off:].data_ptr(), dbuf[dst_off:].data_ptr(), n, asc, launch())
        ref = v[np.argsort(v if asc else -v, kind="stable")]
        assert np.array_equal(bits(dbuf[dst_off:dst_off + n].cpu().numpy()), bits(ref))
        assert np.array_equal(bits(sbuf[src_off:src_off + n].cpu().numpy()), bits(v)), "the column was written"
        d = dbuf.cpu().numpy()
        assert np.all(d[:dst_off] == -654.0) and np.all(d[dst_off + n:] == -654.0)
        s = sbuf.cpu().numpy()
        assert np.all(s[:src_off] == -321.0) and np.all(s[src_off + n:] == -321.0)


@pytest.mark.parametrize("sort,n", [("radix", n) for n in (1, 12289, 1_000_003)]
                         + [("bitonic", n) for n in (1, 12289)])
def test_sort_by_key_stable(n, sort, monkeypatch):
    # the keyed sort behind query_sql ORDER BY <other expression>: float keys
    # with NaN / +-0 / ties, payload = input position (proves stability);
    # the bitonic path is a cross-check at small sizes only
    monkeypatch.setenv("WARPDB_SORT", sort)
    k = _sort_input(n, 23)
    pos = np.arange(n, dtype=np.float32)
    for asc in (True, False):
        tk = torch.from_numpy(k.copy()).cuda()
        tv = torch.from_numpy(pos.copy()).cuda()
        wx.sort_by_key(tk.data_ptr(), tv.data_ptr(), n, asc, launch())
        order = np.argsort(k if asc else -k, kind="stable")
        assert np.array_equal(bits(tk.cpu().numpy()), bits(k[order]))
        assert np.array_equal(tv.cpu().numpy(), pos[order])


def test_sort_radix_large_properties():
    # 2^27 + 5 keys (16 385 tiles per pass): sortedness, and the multiset is
    # unchanged (sum of bit patterns and of squares of bit patterns as int64)
    n = (1 << 27) + 5
    t = torch.empty(n, dtype=torch.float32, device="cuda")
    wx.fill_synthetic(t.data_ptr(), wx.FLOAT32, n, 21, 0, -50.0, 50.0, launch())
    b0 = t.view(torch.int32).to(torch.int64)
    s0, q0 = b0.sum().item(), (b0 * b0).sum().item()
    wx.sort_float(t.data_ptr(), n, True, launch())
    assert bool((t[1:] >= t[:-1]).all().item())
    b1 = t.view(torch.int32).to(torch.int64)
    assert (b1.sum().item(), (b1 * b1).sum().item()) == (s0, q0)


# ------------------------------------------------------- concurrent streams
def test_concurrent_streams_from_threads():
    """Four host threads, one HIP stream each, interleave compaction, SUM, top-K
    and radix sorts on their own tables; every result equals the serial one.
    The runtime keeps one workspace per (device, stream) and locks only its
    shared maps (warpexec.cpp `workspace`), so this must not race."""
    import threading

    n_threads, iters = 4, 6
    sizes = [1_000_003, 2_500_001, 777_777, 1_300_000]
    jobs = []
    for t in range(n_threads):
        n = sizes[t]
        price = torch.empty(n, dtype=torch.float32, device="cuda")
        qty = torch.empty(n, dtype=torch.float32, device="cuda")
        L = launch()
        wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 100 + t, 0, 0.0, 40.0, L)
        wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 200 + t, 1, 1, 100, L)
        table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()),
                             wx.Column("quantity", wx.FLOAT32, qty.data_ptr())])
        mask = price > 15.0
        want = {"idx": torch.nonzero(mask).flatten(), "vals": (price * qty)[mask],
                "sorted": torch.sort(price).values}
        s, c = wx.reduce_sum(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", L)
        want["sum"] = (s, c)
        k = torch.empty(5, device="cuda")
        i = torch.empty(5, dtype=torch.int64, device="cuda")
        v = torch.empty(5, device="cuda")
        wx.topk(table, "price[idx]", None, "discount(price[idx], 0.9f)", 5, True, L, k.data_ptr(), i.data_ptr(),
                v.data_ptr())
        want["topk"] = (k.clone(), i.clone(), v.clone())
        bufs = {"vals": torch.empty(n, device="cuda"), "idx": torch.empty(n, dtype=torch.int64, device="cuda"),
                "sort": torch.empty(n, device="cuda"), "k": torch.empty(5, device="cuda"),
                "i": torch.empty(5, dtype=torch.int64, device="cuda"), "v": torch.empty(5, device="cuda")}
        jobs.append((table, price, qty, want, bufs, torch.cuda.Stream()))
    torch.cuda.synchronize()
    errors = []

    def work(j):
        table, price, _, want, b, stream = jobs[j]
        op, it = "setup", -1
        try:
            with torch.cuda.stream(stream):
                L = wx.make_launch(device=0, stream=stream.cuda_stream, custom_src=DISCOUNT_SRC, flags=wx.F_SYNC)
                for it in range(iters):
                    op = "compact"
                    cnt = wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", L,
                                            wx.MODE_COMPACT, b["vals"].data_ptr(), b["idx"].data_ptr(), 8, 0,
                                            want_count=True)
                    assert cnt == want["idx"].numel()
                    assert torch.equal(b["idx"][:cnt], want["idx"]) and torch.equal(b["vals"][:cnt], want["vals"])
                    op = "sum"
                    assert wx.reduce_sum(table, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", L) == want["sum"]
                    op = "topk"
                    wx.topk(table, "price[idx]", None, "discount(price[idx], 0.9f)", 5, True, L, b["k"].data_ptr(),
                            b["i"].data_ptr(), b["v"].data_ptr())
                    assert all(torch.equal(x, y) for x, y in zip((b["k"], b["i"], b["v"]), want["topk"]))
                    op = "sort"
                    b["sort"].copy_(price)
                    wx.sort_float(b["sort"].data_ptr(), table.n_rows, True, L)
                    assert torch.equal(b["sort"], want["sorted"]), it
                stream.synchronize()
        except Exception as e:  # noqa: BLE001 - reported by the main thread
            errors.append((j, op, it, repr(e)))

    th = [threading.Thread(target=work, args=(j,)) for j in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_workspace_growth_on_fresh_stream_under_load():
    """A fresh stream's workspace is created and grown (look-back status
    words, tickets, radix status) while three other streams keep the GPU busy
    and the null stream is held by a spin kernel.  The zero-fills of fresh
    workspace buffers must be ordered before the first kernel that reads them
    (warpexec.cpp `ensure`: hipMemsetAsync on the workspace stream; the
    round-5 abort came from null-stream fills)."""
    import threading

    stop = threading.Event()
    errors = []

    def busy(j):
        n = 4_000_000 + 17 * j
        price = torch.empty(n, dtype=torch.float32, device="cuda")
        qty = torch.empty(n, dtype=torch.float32, device="cuda")
        L0 = launch()
        wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 300 + j, 0, 0.0, 40.0, L0)
        wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 400 + j, 1, 1, 100, L0)
        torch.cuda.synchronize()
        table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()),
                             wx.Column("quantity", wx.FLOAT32, qty.data_ptr())])
        want = int((price > 10.0).sum())
        vals = torch.empty(n, device="cuda")
        idx = torch.empty(n, dtype=torch.int64, device="cuda")
        stream = torch.cuda.Stream()
        try:
            with torch.cuda.stream(stream):
                L = wx.make_launch(device=0, stream=stream.cuda_stream, flags=wx.F_SYNC)
                while not stop.is_set():
                    cnt = wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 10.0f)", L,
                                            wx.MODE_COMPACT, vals.data_ptr(), idx.data_ptr(), 8, 0, want_count=True)
                    assert cnt == want
                stream.synchronize()
        except Exception as e:  # noqa: BLE001 - reported by the main thread
            errors.append(("busy", j, repr(e)))

    th = [threading.Thread(target=busy, args=(j,)) for j in range(3)]
    for t in th:
        t.start()
    try:
        for rep, n in enumerate([100_003, 1_000_003, 4_000_037, 9_000_011]):
            price = torch.empty(n, dtype=torch.float32, device="cuda")
            qty = torch.empty(n, dtype=torch.float32, device="cuda")
            L0 = launch()
            wx.fill_synthetic(price.data_ptr(), wx.FLOAT32, n, 500 + rep, 0, 0.0, 40.0, L0)
            wx.fill_synthetic(qty.data_ptr(), wx.FLOAT32, n, 600 + rep, 1, 1, 100, L0)
            torch.cuda.synchronize()
            table = wx.Table(n, [wx.Column("price", wx.FLOAT32, price.data_ptr()),
                                 wx.Column("quantity", wx.FLOAT32, qty.data_ptr())])
            mask = price > 15.0
            want_idx = torch.nonzero(mask).flatten()
            want_vals = (price * qty)[mask]
            want_sorted = torch.sort(price).values
            # a fresh stream per size: a new workspace, grown on its first use
            stream = torch.cuda.Stream()
            vals = torch.empty(n, device="cuda")
            idx = torch.empty(n, dtype=torch.int64, device="cuda")
            keys = price.clone()
            torch.cuda.synchronize()
            torch.cuda._sleep(50_000_000)  # hold the null stream (~20-50 ms)
            with torch.cuda.stream(stream):
                L = wx.make_launch(device=0, stream=stream.cuda_stream, flags=wx.F_SYNC)
                cnt = wx.project_filter(table, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", L,
                                        wx.MODE_COMPACT, vals.data_ptr(), idx.data_ptr(), 8, 0, want_count=True)
                wx.sort_float(keys.data_ptr(), n, True, L)
                stream.synchronize()
            torch.cuda.synchronize()
            assert cnt == want_idx.numel(), (n, cnt)
            assert torch.equal(idx[:cnt], want_idx) and torch.equal(vals[:cnt], want_vals), n
            assert torch.equal(keys, want_sorted), n
    finally:
        stop.set()
        for t in th:
            t.join()
    assert not errors, errors


@pytest.mark.parametrize("skew", [0.0, 0.5, 0.95, 1.0])
def test_group_sum_skewed_keys_wave_combined(skew):
    """GROUP BY with most rows on one key: a wave whose lanes share a window
    bin adds their summed values once (WX_GROUP_LEAD) instead of one LDS
    atomic per row.  Keys, counts exact; sums within 1e-12 of the oracle."""
    n = 1_000_003
    rng = np.random.default_rng(61)
    q = np.where(rng.random(n) < skew, 7, rng.integers(0, 1000, n)).astype(np.int32)
    cols = {"price": synth.uniform_f32(n, 62, 0.0, 40.0), "quantity": q}
    table, _ = dev_table(cols)
    cap = 4096
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    for cond, ocond in ((None, None), ("(price[idx] > 10.0f)", "price > 10")):
        g = wx.group_sum(table, "price[idx]", "quantity[idx]", cond, launch(), 0, cap, keys.data_ptr(),
                         sums.data_ptr(), cnts.data_ptr())
        rk, rs, rc = ora.group_sum(ora.HostTable(cols), "price", "quantity", ocond, capacity=cap)
        assert g == len(rk)
        assert np.array_equal(keys[:g].cpu().numpy(), rk) and np.array_equal(cnts[:g].cpu().numpy(), rc)
        assert np.allclose(sums[:g].cpu().numpy(), rs, rtol=1e-12, atol=0)
