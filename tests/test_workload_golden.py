"""Parity at workload scale, pinned to the reference's own output.

tests/golden/workload_*.npz hold what the reference's CPU path computed
(oracle/_ref/ref_harness, i.e. the reference's load_csv_to_host / eval_node
compiled from /root/reference) on 100 000-row synthetic tables of the
BASELINE.json shapes; tests/golden/make_workload_golden.py made them.

CPU tests: the table regenerated here hashes to the CSV the reference read,
and the oracle (oracle/warpdb_oracle.c) equals the reference's result.
GPU tests: the HIP path through the C ABI equals the reference's result
directly -- compaction indices and float bits, GROUP BY keys / counts / double
sums, top-K rows and keys.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import pytest

import oracle_lib as ora
import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, GOLDEN)
import make_workload_golden as mk  # noqa: E402  (generator + CSV formatting of the fixtures)

with open(os.path.join(GOLDEN, "workload_golden.json")) as _f:
    META = json.load(_f)
N = META["rows"]


def table(name):
    if name in ("c2", "c4"):
        return synth.c2_table(N), ()
    if name == "c3":
        return synth.c3_table(N), ("quantity",)
    if name == "c3w":
        return mk.c3w_table(N), ("quantity",)
    if name == "c3o":
        return mk.c3o_table(N), ("quantity",)
    return mk.c5_table(N), ()


def fixture(name):
    return np.load(os.path.join(GOLDEN, f"workload_{name}.npz"))


def compaction_fixture(name):
    f = fixture(name)
    idx = np.nonzero(np.unpackbits(f["mask"])[:N])[0].astype(np.int64)
    return idx, f["bits"]


@pytest.mark.parametrize("name", ["c2", "c3", "c3w", "c3o", "c4", "c5"])
def test_regenerated_table_is_the_reference_input(name):
    cols, ints = table(name)
    text = mk.csv_text(cols, ints)
    assert hashlib.sha256(text.encode()).hexdigest() == META["cases"][name]["csv_sha256"]


@pytest.mark.parametrize("name", ["c2", "c4"])
def test_oracle_equals_reference_compaction(name):
    cols, _ = table(name)
    e, c = ora.split_where(META["cases"][name]["query"])
    vals, idx = ora.project_filter(ora.HostTable(cols), e, c, sem=ora.SEM_CPU)
    ridx, rbits = compaction_fixture(name)
    assert len(ridx) == META["cases"][name]["passing"]
    assert np.array_equal(idx, ridx)
    assert np.array_equal(vals.view(np.uint32), rbits)


@pytest.mark.parametrize("name", ["c3", "c3w", "c3o"])
def test_oracle_equals_reference_group_by(name):
    cols, _ = table(name)
    k, s, c = ora.group_sum(ora.HostTable(cols), "price", "quantity", sem=ora.SEM_CPU)
    f = fixture(name)
    assert len(k) == META["cases"][name]["groups"]
    assert np.array_equal(k, f["keys"]) and np.array_equal(c, f["counts"])
    assert np.array_equal(s, f["sums"])  # c3 / c3w: exact in any order; c3o: the same row-order fold


def _fold(vals, order):
    s = 0.0
    for v in vals[order]:
        s += float(v)  # one double add per value, in the given order
    return s


def test_c3o_sums_depend_on_the_fold_order():
    """workload_c3o.npz tells fold orders apart: its bits are the reference's
    row-order std::map fold (src/warpdb.cpp:373-385), and the same values
    added in another order -- reversed, or sorted by magnitude, as an atomic
    path's scheduling may take them -- give other bits in most groups.  So
    the ordinary GROUP BY (atomic adds in scheduling order) is not
    guaranteed to equal it; WX_F_ROW_ORDER must."""
    cols, _ = table("c3o")
    f = fixture("c3o")
    v = cols["price"].astype(np.float64)
    q = cols["quantity"]
    rev = srt = 0
    for key, ref in zip(f["keys"], f["sums"]):
        rows = np.nonzero(q == key)[0]
        vals = v[rows]
        assert _fold(vals, np.arange(len(rows))) == ref  # row order: the fixture itself
        rev += _fold(vals, np.arange(len(rows))[::-1]) != ref
        srt += _fold(vals, np.argsort(vals, kind="stable")) != ref
    assert len(f["keys"]) == 200 and f["counts"].min() >= 400
    assert rev > 50 and srt > 50, (rev, srt)


def test_oracle_equals_reference_topk():
    cols, _ = table("c5")
    keys, idx, _ = ora.topk(ora.HostTable(cols), "price", 32, True)
    f = fixture("c5")
    assert np.array_equal(idx, f["rows"]) and np.array_equal(keys.view(np.uint32), f["bits"])


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c2", "c4"])
@pytest.mark.parametrize("idx_bytes", [4, 8])
def test_hip_compaction_equals_reference(name, idx_bytes):
    torch = pytest.importorskip("torch")
    from test_gpu_parity import dev_table, gpu_compact

    cols, _ = table(name)
    t, _ = dev_table(cols)
    e, c = ora.split_where(META["cases"][name]["query"])
    vals, idx = gpu_compact(t, ora.lower(e), ora.lower(c), idx_bytes=idx_bytes)
    ridx, rbits = compaction_fixture(name)
    assert np.array_equal(idx.astype(np.int64), ridx)
    assert np.array_equal(vals.view(np.uint32), rbits)
    del torch


@pytest.mark.gpu
def test_hip_dense_equals_reference():
    torch = pytest.importorskip("torch")
    from test_gpu_parity import dev_table, launch
    from warpdb_amd import _warpexec as wx

    cols, _ = table("c2")
    t, _ = dev_table(cols)
    out = torch.full((N,), float("nan"), dtype=torch.float32, device="cuda")
    wx.project_filter(t, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", launch(), wx.MODE_DENSE_FILL,
                      out.data_ptr(), 0, 4, 0)
    ridx, rbits = compaction_fixture("c2")
    o = out.cpu().numpy()
    assert np.array_equal(o[ridx].view(np.uint32), rbits)
    rest = np.ones(N, bool)
    rest[ridx] = False
    assert np.all(o[rest] == 0.0)


@pytest.mark.gpu
def test_hip_group_by_equals_reference():
    torch = pytest.importorskip("torch")
    from test_gpu_parity import dev_table, launch
    from warpdb_amd import _warpexec as wx

    cols, _ = table("c3")
    t, _ = dev_table(cols)
    cap = 4096
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    g = wx.group_sum(t, "price[idx]", "quantity[idx]", None, launch(), 0, cap, keys.data_ptr(), sums.data_ptr(),
                     cnts.data_ptr())
    f = fixture("c3")
    assert g == len(f["keys"])
    assert np.array_equal(keys[:g].cpu().numpy(), f["keys"]) and np.array_equal(cnts[:g].cpu().numpy(), f["counts"])
    assert np.array_equal(sums[:g].cpu().numpy(), f["sums"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["window+hash", "partitioned"])
def test_hip_many_key_group_by_equals_reference(path, monkeypatch):
    """55 313 groups over 100 000 rows (keys 0..74 999), the reference's
    std::map sums: the window + global-hash path (device-wide key sort of the
    out-of-window groups) and the range-partitioned kernels (forced at this
    size by the WARPDB_GP_MIN_ROWS test hook)."""
    torch = pytest.importorskip("torch")
    from test_gpu_parity import dev_table, launch
    from warpdb_amd import _warpexec as wx

    if path == "partitioned":
        monkeypatch.setenv("WARPDB_GP_MIN_ROWS", "0")
    cols, _ = table("c3w")
    t, _ = dev_table(cols)
    cap = 1 << 17
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    g = wx.group_sum(t, "price[idx]", "quantity[idx]", None, launch(), 0, cap, keys.data_ptr(), sums.data_ptr(),
                     cnts.data_ptr())
    f = fixture("c3w")
    assert g == len(f["keys"]) == 55_313
    assert np.array_equal(keys[:g].cpu().numpy(), f["keys"]) and np.array_equal(cnts[:g].cpu().numpy(), f["counts"])
    assert np.array_equal(sums[:g].cpu().numpy(), f["sums"])  # few rows per key: exact in any order


@pytest.mark.gpu
@pytest.mark.parametrize("path,rows", [("window", "span")] + [(p, r) for r in ("ordinary", "general")
                                                                for p in ("window", "window+hash", "hash", "partitioned")])
def test_hip_row_order_group_by_equals_reference(path, rows, monkeypatch):
    """WX_F_ROW_ORDER against the reference's own row-order fold on a table
    where the order shows in the bits (workload_c3o.npz), by every row-order
    route (WARPDB_GROUP_ROWS): the key-span path straight from the table
    ("span", the default), the key-span path after the ordinary call
    ("ordinary") and the general compaction + radix-sort path ("general");
    the ordinary call itself by the LDS window (key_lo 0), half the keys in
    the general-key hash (key_lo 100), all of them there (key_lo 10^6), and
    the range-partitioned first step (forced by the WARPDB_GP_MIN_ROWS test
    hook)."""
    torch = pytest.importorskip("torch")
    from test_gpu_parity import dev_table
    from warpdb_amd import _warpexec as wx

    # (the direct key-span path makes no ordinary call: key_lo and the ordinary paths do not apply to it)
    monkeypatch.setenv("WARPDB_GROUP_ROWS", rows)
    key_lo = {"window": 0, "window+hash": 100, "hash": 1_000_000, "partitioned": 0}[path]
    if path == "partitioned":
        monkeypatch.setenv("WARPDB_GP_MIN_ROWS", "0")
    cols, _ = table("c3o")
    t, _ = dev_table(cols)
    cap = 1 << 17 if path == "partitioned" else 4096
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    L = wx.make_launch(device=0, stream=torch.cuda.current_stream().cuda_stream, flags=wx.F_ROW_ORDER)
    g = wx.group_sum(t, "price[idx]", "quantity[idx]", None, L, key_lo, cap, keys.data_ptr(), sums.data_ptr(),
                     cnts.data_ptr())
    f = fixture("c3o")
    assert g == len(f["keys"]) == 200
    assert np.array_equal(keys[:g].cpu().numpy(), f["keys"]) and np.array_equal(cnts[:g].cpu().numpy(), f["counts"])
    assert np.array_equal(sums[:g].cpu().numpy().view(np.uint64), f["sums"].view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("k", [5, 32])
def test_hip_topk_equals_reference(k):
    torch = pytest.importorskip("torch")
    from test_gpu_parity import dev_table, launch
    from warpdb_amd import _warpexec as wx

    cols, _ = table("c5")
    t, _ = dev_table(cols)
    tk = torch.empty(k, dtype=torch.float32, device="cuda")
    ti = torch.empty(k, dtype=torch.int64, device="cuda")
    m = wx.topk(t, "price[idx]", None, None, k, True, launch(), tk.data_ptr(), ti.data_ptr(), 0)
    f = fixture("c5")
    assert m == k
    assert np.array_equal(ti.cpu().numpy(), f["rows"][:k])
    assert np.array_equal(tk.cpu().numpy().view(np.uint32), f["bits"][:k])
