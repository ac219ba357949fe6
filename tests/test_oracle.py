"""CPU tests: the oracle pinned against the reference's own outputs.

golden.json was produced by tests/golden/make_golden.py from oracle/_ref
(the reference's tokenizer / parser / evaluator compiled from
/root/reference).  When oracle/_ref is present (build container) the oracle
is also cross-checked against it live on randomised queries.
"""
from __future__ import annotations

import json
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as ora
import synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def read_csv(path, schema=None):
    import csv

    with open(path) as f:
        rows = list(csv.reader(f))
    dt = {0: np.int32, 1: np.int64, 2: np.float32, 3: np.float64}
    cols = {}
    for i, name in enumerate(rows[0]):
        t = dt[int(schema[i])] if schema else np.float32
        vals = [row[i] for row in rows[1:]]
        cols[name] = np.array([int(v) for v in vals] if t in (np.int32, np.int64) else [float(v) for v in vals], t)
    return cols


@pytest.mark.parametrize("case", golden()["lower"], ids=lambda c: c["expr"])
def test_lowering_matches_reference(case):
    assert ora.lower(case["expr"]) == case["lowered"]


@pytest.mark.parametrize("case", golden()["errors"], ids=lambda c: repr(c["expr"]))
def test_parse_errors_match_reference(case):
    with pytest.raises(ora.OracleError) as ei:
        ora.lower(case["expr"])
    assert str(ei.value) == case["message"].replace("ERROR: ", "")


@pytest.mark.parametrize("case", golden()["project"], ids=lambda c: c["query"])
def test_project_matches_reference_evaluator(case):
    cols = read_csv(os.path.join(GOLDEN, case["csv"]), case["schema"])
    e, c = ora.split_where(case["query"])
    vals, idx = ora.project_filter(ora.HostTable(cols), e, c if c.strip() else None, sem=ora.SEM_CPU)
    assert idx.tolist() == case["idx"]
    assert [float(v) for v in vals] == [float.fromhex(x) for x in case["vals"]]


def test_reference_unit_expectations():
    # tests/test_expression.cpp, precedence_tests.cpp, expression_tests.cpp
    assert ora.lower("price > 10") == "(price[idx] > 10.0f)"
    assert ora.lower("quantity <= 5") == "(quantity[idx] <= 5.0f)"
    assert ora.lower("discount(price, 0.9)") == "discount(price[idx], 0.9f)"
    assert ora.lower("price > 10 AND quantity < 5") == "((price[idx] > 10.0f) && (quantity[idx] < 5.0f))"
    assert ora.lower("price > 10 OR quantity < 5") == "((price[idx] > 10.0f) || (quantity[idx] < 5.0f))"
    assert ora.lower("price + quantity * 2") == "(price[idx] + (quantity[idx] * 2.0f))"
    assert ora.lower("(price + quantity) * 2") == "((price[idx] + quantity[idx]) * 2.0f)"
    with pytest.raises(ora.OracleError, match="Unexpected token"):
        ora.lower("1 2")
    with pytest.raises(ora.OracleError, match="Expected '\\)'"):
        ora.lower("(price + 5")
    with pytest.raises(ora.OracleError, match="Unknown character"):
        ora.lower("price & 5")
    with pytest.raises(ora.OracleError, match="line 1"):
        ora.lower("price # 1\n")


def test_sql_features_expectations():
    # tests/sql_features_test.cpp:11-37 on data/test.csv
    cols = read_csv(os.path.join(GOLDEN, "test.csv"))
    t = ora.HostTable(cols)
    k, s, c = ora.group_sum(t, "price", "quantity", sem=ora.SEM_CPU)
    assert k.tolist() == [2, 3, 4, 5]
    assert s.tolist() == [15.25, 10.5, 20.0, 30.0]
    assert int((s > 15).sum()) == 3  # HAVING SUM(price) > 15 -> 3 groups
    keys, idx, vals = ora.topk(t, "price", 2, True, sem=ora.SEM_CPU)
    assert keys.tolist() == [30.0, 20.0]
    keys, idx, vals = ora.topk(t, "price", 5, True, sem=ora.SEM_CPU)
    assert keys.tolist() == [30.0, 20.0, 15.25, 10.5]
    keys, idx, _ = ora.topk(t, "price", 3, True, sem=ora.SEM_CPU)
    assert keys[1:3].tolist() == [20.0, 15.25]  # OFFSET 1 LIMIT 2


def test_extended_types_expectation():
    # tests/extended_types_test.cpp:5-13: schema {F32, I32, F32}, price * discount
    cols = read_csv(os.path.join(GOLDEN, "extended.csv"), "202")
    vals, idx = ora.project_filter(ora.HostTable(cols), "price * discount", None, sem=ora.SEM_CPU)
    assert len(vals) == 4 and int(vals[0]) == 1


def test_semantics_agree_on_float32_tables():
    cols = synth.c2_table(20_000)
    t = ora.HostTable(cols)
    for q in ["price * quantity WHERE price > 15", "price * 0.9 WHERE price > 20", "price / quantity - 1",
              "(price + quantity) * 2 WHERE quantity <= 4 OR price > 39"]:
        e, c = ora.split_where(q)
        a = ora.project_filter(t, e, c or None, sem=ora.SEM_CPU)
        b = ora.project_filter(t, e, c or None, sem=ora.SEM_JIT)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))


def test_jit_semantics_integer_division():
    t = ora.HostTable({"a": np.array([7, -7, 9], np.int32), "b": np.array([2, 2, 4], np.int32)})
    v, _ = ora.project_filter(t, "a / b", None, sem=ora.SEM_JIT)
    assert v.tolist() == [3.0, -3.0, 2.0]  # C integer division in the JIT kernel
    v, _ = ora.project_filter(t, "a / b", None, sem=ora.SEM_CPU)
    assert v.tolist() == [3.5, -3.5, 2.25]  # the CPU evaluator casts to float first


def test_topk_ties_use_row_order():
    t = ora.HostTable({"p": np.array([5, 9, 9, 1, 9, 5], np.float32)})
    k, i, _ = ora.topk(t, "p", 4, True)
    assert k.tolist() == [9, 9, 9, 5] and i.tolist() == [1, 2, 4, 0]
    k, i, _ = ora.topk(t, "p", 3, False)
    assert k.tolist() == [1, 5, 5] and i.tolist() == [3, 0, 5]


def test_group_sum_general_keys():
    rng = np.random.default_rng(3)
    keys = rng.integers(-(1 << 31), 1 << 31, 5000, dtype=np.int64).astype(np.int32)
    vals = rng.uniform(0, 1, 5000).astype(np.float32)
    t = ora.HostTable({"k": keys, "v": vals})
    k, s, c = ora.group_sum(t, "v", "k")
    order = np.argsort(keys, kind="stable")
    uk, first = np.unique(keys[order], return_index=True)
    assert np.array_equal(k, uk)
    assert c.sum() == 5000


def test_stats_and_group_minmax_vs_numpy():
    # AggData min / max (src/warpdb.cpp:375-385), stated NaN-skipping
    rng = np.random.default_rng(8)
    v = np.round(rng.uniform(-9, 9, 3000), 1).astype(np.float32)
    v[rng.uniform(size=3000) < 0.05] = np.nan
    k = rng.integers(0, 40, 3000).astype(np.int32)
    t = ora.HostTable({"v": v, "k": k})
    s, c, mn, mx = ora.stats(t, "v", "v > 2")
    sel = v[v > 2]
    assert c == len(sel) and mn == np.nanmin(sel) and mx == np.nanmax(sel)
    keys, sums, cnts, mins, maxs = ora.group_agg(t, "v", "k")
    for j, key in enumerate(keys):
        g = v[k == key]
        assert cnts[j] == len(g)
        assert mins[j] == np.nanmin(g) and maxs[j] == np.nanmax(g)
    # empty set -> NaN; -0.0 folds to +0.0
    _, c0, mn0, mx0 = ora.stats(t, "v", "v > 100")
    assert c0 == 0 and np.isnan(mn0) and np.isnan(mx0)
    z = ora.HostTable({"z": np.array([-0.0, 0.0, -0.0], np.float32)})
    _, _, zmn, zmx = ora.stats(z, "z")
    assert not np.signbit(zmn) and not np.signbit(zmx)


REF = ora.REF_HARNESS


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_vs_reference_live():
    rng = np.random.default_rng(1)
    atoms = ["price", "quantity", "1", "2.5", "0.9", "10", "(price + 1)"]
    ops = ["+", "-", "*", "/"]
    cmps = [">", "<", ">=", "<=", "==", "!="]
    csv = os.path.join(GOLDEN, "test.csv")
    cols = read_csv(csv)
    t = ora.HostTable(cols)
    for _ in range(60):
        e = " ".join([rng.choice(atoms), rng.choice(ops), rng.choice(atoms), rng.choice(ops), rng.choice(atoms)])
        c = f"{rng.choice(atoms)} {rng.choice(cmps)} {rng.choice(atoms)}"
        q = f"{e} WHERE {c}"
        assert ora.lower(e) == subprocess.run([REF, "lower", e], capture_output=True, text=True).stdout.strip()
        out = subprocess.run([REF, "eval", csv, q], capture_output=True, text=True).stdout.split("\n")
        rows = [l.split() for l in out if l.strip()]
        vals, idx = ora.project_filter(t, e, c, sem=ora.SEM_CPU)
        assert idx.tolist() == [int(r[0]) for r in rows], q
        assert [float(v) for v in vals] == [float.fromhex(r[1]) for r in rows], q
