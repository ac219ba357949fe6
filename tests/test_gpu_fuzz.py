"""Randomised parity: generated queries on the HIP path against the oracle.

Each case draws a nested arithmetic expression over float32, int32 and
float64 columns and constants, and a WHERE of comparisons joined by AND / OR,
lowers both with the reference's lowering (oracle `lower`, the restatement of
include/expression.hpp:32-78), and runs the lowered strings through the C ABI
exactly as `jit_compile_and_launch` receives them (src/jit.cpp:48-174).  The
compaction must match the oracle's JIT semantics bit for bit (ascending row
list of src/warpdb.cpp:336-344, value bits); SUM over the same rows within
1e-12 relative (double accumulation in another order), its count exactly;
the dense contract (src/warpdb.cpp:243-256) bit for bit; GROUP BY (the
ascending-key result of tests/sql_features_test.cpp:11-22) with keys and
counts exact and sums within 1e-12 relative, windows placed so that some keys
fall outside the dense window and take the general-key table.

Division only ever has a float operand on its right (a column of float type or
a constant, which lowers to a float literal), so no case divides integers by
zero on either side.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle_lib as ora
from test_gpu_parity import bits, dev_table, gpu_compact, launch

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from warpdb_amd import _warpexec as wx  # noqa: E402

N = 300_001
FLOAT_ATOMS = ["price", "quantity", "w", "2.5", "0.9", "10", "0.125", "3"]
ANY_ATOMS = FLOAT_ATOMS + ["qi", "qi"]
OPS = ["+", "-", "*", "/"]
CMPS = [">", "<", ">=", "<=", "==", "!="]


def table_cols():
    rng = np.random.default_rng(2024)
    return {
        "price": rng.uniform(0, 40, N).astype(np.float32),
        "quantity": rng.integers(1, 101, N).astype(np.float32),
        "qi": rng.integers(-50, 51, N).astype(np.int32),
        "w": rng.normal(0, 100, N).astype(np.float64),
    }


def gen_expr(rng, depth):
    if depth == 0 or rng.random() < 0.3:
        return str(rng.choice(ANY_ATOMS))
    op = str(rng.choice(OPS))
    left = gen_expr(rng, depth - 1)
    right = str(rng.choice(FLOAT_ATOMS)) if op == "/" else gen_expr(rng, depth - 1)
    return f"({left} {op} {right})"


def gen_cond(rng):
    parts = [f"{gen_expr(rng, 1)} {rng.choice(CMPS)} {gen_expr(rng, 1)}" for _ in range(int(rng.integers(1, 4)))]
    out = parts[0]
    for p in parts[1:]:
        out = f"{out} {rng.choice(['AND', 'OR'])} {p}"
    return out


def cases(count, seed):
    rng = np.random.default_rng(seed)
    return [(gen_expr(rng, 3), gen_cond(rng)) for _ in range(count)]


@pytest.fixture(scope="module")
def fuzz_table():
    cols = table_cols()
    table, tensors = dev_table(cols)
    return cols, table, tensors


@pytest.mark.parametrize("case", range(48))
def test_random_compaction_vs_oracle(fuzz_table, case):
    cols, table, _ = fuzz_table
    e, c = cases(48, 11)[case]
    vals, idx = gpu_compact(table, ora.lower(e), ora.lower(c))
    rv, ri = ora.project_filter(ora.HostTable(cols), e, c, sem=ora.SEM_JIT)
    assert np.array_equal(idx, ri), (e, c)
    assert np.array_equal(bits(vals), bits(rv)), (e, c)


@pytest.mark.parametrize("case", range(16))
def test_random_sum_and_dense_vs_oracle(fuzz_table, case):
    cols, table, _ = fuzz_table
    e, c = cases(16, 23)[case]
    ec, cc = ora.lower(e), ora.lower(c)
    s, cnt = wx.reduce_sum(table, ec, cc, launch())
    rs, rc = ora.reduce_sum(ora.HostTable(cols), e, c, sem=ora.SEM_JIT)
    assert cnt == rc, (e, c)
    assert s == rs or abs(s - rs) <= 1e-12 * max(abs(rs), 1e-300) or (np.isnan(s) and np.isnan(rs)), (e, c, s, rs)
    out = torch.full((N,), 7.0, dtype=torch.float32, device="cuda")
    wx.project_filter(table, ec, cc, launch(), wx.MODE_DENSE_FILL, out.data_ptr(), 0, 4, 0)
    want = ora.dense(ora.HostTable(cols), e, c, np.zeros(N, np.float32), sem=ora.SEM_JIT)
    assert np.array_equal(bits(out.cpu().numpy()), bits(want)), (e, c)


KEYS = ["qi", "(qi * 3)", "(qi - 40)", "quantity", "(quantity + qi)", "(price / 2.5)"]


@pytest.mark.parametrize("case", range(12))
def test_random_group_by_vs_oracle(fuzz_table, case):
    cols, table, _ = fuzz_table
    rng = np.random.default_rng(100 + case)
    val = gen_expr(rng, 2)
    key = KEYS[case % len(KEYS)]
    cond = gen_cond(rng) if case % 3 else None
    lo = int(rng.choice([-64, 0, 30, -2000]))
    cap = 4096
    keys = torch.empty(cap, dtype=torch.int32, device="cuda")
    sums = torch.empty(cap, dtype=torch.float64, device="cuda")
    cnts = torch.empty(cap, dtype=torch.int64, device="cuda")
    g = wx.group_sum(table, ora.lower(val), ora.lower(key), ora.lower(cond) if cond else None, launch(), lo, cap,
                     keys.data_ptr(), sums.data_ptr(), cnts.data_ptr())
    rk, rs, rc = ora.group_sum(ora.HostTable(cols), val, key, cond)
    assert g == len(rk), (val, key, cond)
    assert np.array_equal(keys[:g].cpu().numpy(), rk), (val, key, cond)
    assert np.array_equal(cnts[:g].cpu().numpy(), rc), (val, key, cond)
    got = sums[:g].cpu().numpy()
    assert np.all((got == rs) | (np.abs(got - rs) <= 1e-12 * np.maximum(np.abs(rs), 1e-300))), (val, key, cond)


@pytest.mark.parametrize("case", range(12))
def test_random_topk_vs_oracle(fuzz_table, case):
    # ORDER BY <expr> [DESC] LIMIT k with a random WHERE and SELECT expression
    # (src/warpdb.cpp:453-495 semantics: the stable order, ties by row): keys,
    # row ids and selected values bit for bit against the oracle
    cols, table, _ = fuzz_table
    rng = np.random.default_rng(300 + case)
    order = gen_expr(rng, 2)
    cond = gen_cond(rng) if case % 2 else None
    sel = gen_expr(rng, 2)
    k = int(rng.choice([1, 2, 5, 17, 32]))
    desc = bool(case % 3)
    keys = torch.empty(k, dtype=torch.float32, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    vals = torch.empty(k, dtype=torch.float32, device="cuda")
    m = wx.topk(table, ora.lower(order), ora.lower(cond) if cond else None, ora.lower(sel), k, desc, launch(),
                keys.data_ptr(), idx.data_ptr(), vals.data_ptr())
    rk, ri, rv = ora.topk(ora.HostTable(cols), order, k, desc, cond, sel)
    assert m == len(ri), (order, cond, sel, k, desc)
    assert np.array_equal(idx[:m].cpu().numpy(), ri), (order, cond, sel, k, desc)
    assert np.array_equal(bits(keys[:m].cpu().numpy()), bits(rk)), (order, cond, sel, k, desc)
    assert np.array_equal(bits(vals[:m].cpu().numpy()), bits(rv)), (order, cond, sel, k, desc)
