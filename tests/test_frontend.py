"""CPU tests of the product front end (libwarpdb via pywarpdb): lowering,
tokenizer and error messages against the reference's goldens
(tests/golden/golden.json, produced from the reference's own parser) and the
expectations of the reference's unit tests."""
from __future__ import annotations

import json
import os

import pytest

from warpdb_amd import pywarpdb as pw

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", golden()["lower"], ids=lambda c: c["expr"])
def test_lowering_matches_reference(case):
    assert pw.lower_expression(case["expr"]) == case["lowered"]


@pytest.mark.parametrize("case", golden()["errors"], ids=lambda c: repr(c["expr"]))
def test_errors_match_reference(case):
    with pytest.raises(RuntimeError) as ei:
        pw.lower_expression(case["expr"])
    assert str(ei.value) == case["message"].replace("ERROR: ", "")


def test_tokenizer_expectations():
    # tests/tokenizer_tests.cpp
    toks = pw.tokenize("price > 10")
    assert [(t[0], t[1]) for t in toks] == [(0, "price"), (2, ">"), (1, "10"), (4, "")]
    kinds = [t[0] for t in pw.tokenize("(price + 5) * quantity")]
    assert kinds == [2, 0, 2, 1, 2, 2, 0, 4]
    vals = [t[1] for t in pw.tokenize("price > 10 AND quantity < 5") if t[0] == 3]
    assert vals == ["AND"]
    toks = pw.tokenize("a >= 1 != 2\n  b")
    assert [t[1] for t in toks][:5] == ["a", ">=", "1", "!=", "2"]
    assert toks[5][2:] == (2, 3)  # line / column tracking


def test_equality_is_not_assignment():
    # deviation: the reference lowers '=' to a C assignment
    assert pw.lower_expression("quantity = 7") == "(quantity[idx] == 7.0f)"


def test_split_where():
    assert pw.split_where("price * quantity WHERE price > 10") == ("price * quantity ", " price > 10")
    assert pw.split_where("price where price > 1") == ("price ", " price > 1")
    assert pw.split_where("price") == ("price", "")


def test_parse_query_reference_cases():
    # tests/query_parser_test.cpp
    q = pw.parse_query_summary("SELECT SUM(price), quantity FROM sales JOIN items ON sales.id = items.id "
                               "WHERE price > 10 GROUP BY quantity ORDER BY price DESC LIMIT 5")
    assert len(q["select"]) == 2 and q["joins"] == 1 and q["where"] and q["group_by"] == 1
    assert q["order_by"] == ("price[idx]", False) and q["limit"] == 5
    # tests/parse_query_error_test.cpp: message carries line and column
    with pytest.raises(RuntimeError, match="line 1 column"):
        pw.parse_query_summary("SELECT price")
    # tests/parsing_error_tests.cpp
    with pytest.raises(RuntimeError, match="Unexpected token"):
        pw.parse_query_summary("SELECT price FROM test EXTRA")
    # tests/sql_features_test.cpp shapes
    q = pw.parse_query_summary("SELECT price FROM test ORDER BY price DESC OFFSET 1 LIMIT 2")
    assert q["offset"] == 1 and q["limit"] == 2
    q = pw.parse_query_summary("SELECT SUM(price) FROM test GROUP BY quantity HAVING SUM(price) > 15 "
                               "ORDER BY quantity ASC")
    assert q["having"] == "(price[idx] > 15.0f)" and q["order_by"] == ("quantity[idx]", True)
    q = pw.parse_query_summary("SELECT DISTINCT quantity FROM test ORDER BY quantity DESC")
    assert q["distinct"]
    q = pw.parse_query_summary("SELECT COUNT(*) FROM t WHERE price > 1")
    assert q["select"] == ["1.0f"]


def test_plan_shards_matches_reference_partition():
    # ceil(N / devices) contiguous rows (src/multi_gpu_utils.cpp:24-32)
    assert pw.plan_shards(10, 4) == [(0, 0, 3), (1, 3, 6), (2, 6, 9), (3, 9, 10)]
    assert pw.plan_shards(3, 8) == [(0, 0, 1), (1, 1, 2), (2, 2, 3)]
    assert pw.plan_shards(0, 8) == []
    n = 8_000_000_000
    s = pw.plan_shards(n, 8)
    assert len(s) == 8 and s[-1][2] == n and all(e - b == 1_000_000_000 for _, b, e in s)


def test_optimizer_verdicts():
    # the reference's analyze_condition never decides (src/optimizer.cpp:13-17)
    st = {"price": (0.0, 39.99, 0, False), "quantity": (1.0, 100.0, 0, True)}
    cases = {"price > 40": "always_false", "price >= 0": "always_true", "price > 15": "unknown",
             "price > 10 AND quantity > 200": "always_false", "price > 50 OR quantity >= 1": "always_true",
             "price * 2 > 80": "always_false", "quantity / quantity > 2": "unknown", "price != 100": "always_true",
             "discount(price, 0.9) > 1000": "unknown", "missing > 1": "unknown"}
    for w, v in cases.items():
        assert pw.analyze_condition(w, st) == v, w
    # NaN rows fail every comparison but pass !=
    nan = {"price": (0.0, 39.99, 3, False)}
    assert pw.analyze_condition("price >= 0", nan) == "unknown"
    assert pw.analyze_condition("price < 0", nan) == "always_false"
    assert pw.analyze_condition("price != 100", nan) == "always_true"


def test_optimizer_is_sound_against_oracle():
    # whenever the interval analysis decides, every row must agree (JIT semantics)
    import numpy as np

    import oracle_lib as ora

    rng = np.random.default_rng(21)
    atoms = ["a", "b", "k", "1", "2.5", "0.9", "10", "40", "(a + 1)", "(k * 3)", "(a * b)", "(a / 7)", "(k / 3)"]
    cmps = [">", "<", ">=", "<=", "==", "!="]
    decided = 0
    for trial in range(40):
        n = 400
        a = rng.uniform(rng.uniform(-50, 0), rng.uniform(0, 50), n).astype(np.float32)
        b = np.round(rng.uniform(-3, 3, n), 1).astype(np.float32)
        k = rng.integers(-20, 20, n).astype(np.int32)
        if trial % 4 == 0:
            a[rng.uniform(size=n) < 0.1] = np.nan
        cols = {"a": a, "b": b, "k": k}
        stats = {}
        for name, v in cols.items():
            ok = v[~np.isnan(v)] if v.dtype == np.float32 else v
            stats[name] = (float(ok.min()), float(ok.max()), int(np.isnan(v).sum()) if v.dtype == np.float32 else 0,
                           v.dtype == np.int32)
        t = ora.HostTable(cols)
        for _ in range(25):
            def cmp():
                return f"{rng.choice(atoms)} {rng.choice(cmps)} {rng.choice(atoms)}"
            w = cmp()
            if rng.uniform() < 0.4:
                w = f"{w} {rng.choice(['AND', 'OR'])} {cmp()}"
            v = pw.analyze_condition(w, stats)
            if v == "unknown":
                continue
            decided += 1
            _, idx = ora.project_filter(t, "a", w)
            assert len(idx) == (n if v == "always_true" else 0), (w, v, len(idx))
    assert decided > 50


def test_cpp_frontend_binary():
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "-C", os.path.join(root, "tests", "cpp"), "frontend_test"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([os.path.join(root, "tests", "cpp", "bin", "frontend_test")], capture_output=True,
                       text=True, cwd=root)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "frontend_test: all passed" in r.stdout


def test_boundary_layout_static_asserts():
    # tests/cpp/layout_test.cpp: the source-level compatibility INTEGRATION.md
    # 1.1 states (64-bit row counts, DataType == wx_dtype numbering, the
    # reference's constructor calls) pinned by static_assert; building it is the test
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "-C", os.path.join(root, "tests", "cpp"), "layout_test"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([os.path.join(root, "tests", "cpp", "bin", "layout_test")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_host_code_under_asan_ubsan():
    # tests/cpp/sanitize_test.cpp: the front end on random token soup and deep
    # nesting, the parallel CSV parser against a sequential reading, built with
    # -fsanitize=address,undefined (any report fails the run)
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "-C", os.path.join(root, "tests", "cpp"), "sanitize_test"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(root, "tests", "cpp", "bin", "sanitize_test")], capture_output=True, text=True,
                       cwd=root, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize_test: all passed" in r.stdout


def test_parser_limits():
    with pytest.raises(RuntimeError, match="nested too deeply"):
        pw.lower_expression("(" * 10_000 + "1" + ")" * 10_000)
    assert pw.lower_expression("(" * 100 + "price" + ")" * 100) == "price[idx]"
    with pytest.raises(RuntimeError, match="LIMIT value out of range"):
        pw.parse_query_summary("SELECT price FROM t LIMIT 99999999999")


def _libc():
    import ctypes

    c = ctypes.CDLL(None)
    c.strtof.restype = ctypes.c_float
    c.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]
    c.strtoll.restype = ctypes.c_longlong
    c.strtoll.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int]
    return c


def test_parallel_csv_parser_matches_strtof(tmp_path):
    # the loader keeps the sequential std::strto* meaning of every cell
    # (src/csv_loader.cpp:49-124) while parsing line ranges in parallel
    import numpy as np

    rng = np.random.default_rng(5)
    odd = ["+1.5", " 2", "0x10", "1e3", "inf", "-inf", "-0", ".5", "7.", "3.4028236e38", "1e-46", "12abc",
           "  -4.25", "1E+2"]
    n = 60_000
    vals = []
    for i in range(n):
        if i % 97 == 0:
            vals.append(odd[(i // 97) % len(odd)])
        else:
            vals.append(repr(float(np.float32(rng.uniform(-1e4, 1e4)))))
    ints = rng.integers(-(1 << 40), 1 << 40, n)
    path = tmp_path / "p.csv"
    with open(path, "w", newline="") as f:
        f.write("a,b,s\r\n")
        for i in range(n):
            if i % 1000 == 0:
                f.write("\r\n")  # blank lines are skipped
            f.write(f"{vals[i]},{ints[i]},w{i}\r\n" if i % 3 else f"{vals[i]},{ints[i]},w{i}\n")
    schema = [pw.DataType.Float32, pw.DataType.Int64, pw.DataType.String]
    c = _libc()
    want_a = np.array([c.strtof(v.encode(), None) for v in vals], np.float32)
    for threads in (1, 3, 16):
        d = pw.load_csv_columns(str(path), schema, threads)
        assert np.array_equal(d["a"].view(np.uint32), want_a.view(np.uint32)), threads
        assert np.array_equal(d["b"], ints)
        assert d["s"][:3] == ["w0", "w1", "w2"] and len(d["s"]) == n


def test_csv_parser_errors(tmp_path):
    p = tmp_path / "bad.csv"
    p.write_text("a,b\n1,2\n3,abc\n")
    with pytest.raises(RuntimeError, match="Invalid numeric value in CSV: 'abc'"):
        pw.load_csv_columns(str(p))
    p.write_text("a,b\n1,2\n3\n")  # a missing cell is an empty cell
    with pytest.raises(RuntimeError, match="Invalid numeric value in CSV: ''"):
        pw.load_csv_columns(str(p))
    p.write_text("a,b\n1,2,9\n")  # extra cells are ignored
    d = pw.load_csv_columns(str(p))
    assert d["a"].tolist() == [1.0] and d["b"].tolist() == [2.0]
    # golden data files load as the reference does (default schema: all Float32)
    d = pw.load_csv_columns(os.path.join(GOLDEN, "test.csv"))
    assert d["price"].tolist() == [10.5, 20.0, 15.25, 30.0] and d["quantity"].tolist() == [3, 4, 2, 5]
