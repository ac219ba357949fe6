"""GPU tests of the reference-compatible API surface: the C++ engine test
binary (WarpDB facade + legacy jit_* entry points) and pywarpdb, checked
against the oracle and the reference's fixtures."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as ora
import synth

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
TEST_CSV = os.path.join(GOLDEN, "test.csv")


def pw():
    from warpdb_amd import pywarpdb

    return pywarpdb


def test_cpp_engine_binary():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "engine_test"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "bin", "engine_test")], capture_output=True, text=True,
                       cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "engine_test: all passed" in r.stdout


def test_python_smoke_like_reference():
    # tests/test_python.py
    db = pw().WarpDB(TEST_CSV)
    res = db.query("price + 1")
    assert len(res) == 4 and res == [11.5, 21.0, 16.25, 31.0]


def test_query_dense_and_compact_vs_oracle(tmp_path):
    n = 50_000
    cols = synth.c2_table(n)
    path = tmp_path / "t.csv"
    with open(path, "w") as f:
        f.write("price,quantity\n")
        for p, q in zip(cols["price"], cols["quantity"]):
            f.write(f"{float(p)!r},{int(q)}\n")
    db = pw().WarpDB(str(path))
    dense = np.array(db.query("price * quantity WHERE price > 15"), np.float32)
    rv, ri = ora.project_filter(ora.HostTable(cols), "price * quantity", "price > 15")
    ref = np.zeros(n, np.float32)
    ref[ri] = rv
    assert np.array_equal(dense.view(np.uint32), ref.view(np.uint32))
    vals, idx = db.query_compact("price * quantity WHERE price > 15")
    assert np.array_equal(np.array(idx), ri) and np.array_equal(np.array(vals, np.float32).view(np.uint32),
                                                                rv.view(np.uint32))
    s, c = db.query_sum("price * 0.9 WHERE price > 20")
    rs, rc = ora.reduce_sum(ora.HostTable(cols), "price * 0.9", "price > 20")
    assert c == rc and s == rs
    # multi-GPU paths (every visible GPU; one on the test box), also with the
    # host pipeline cut into many ragged chunks
    assert db.query_multi_gpu("price * quantity WHERE price > 15") == dense.tolist()
    os.environ["WARPDB_HOST_CHUNK_ROWS"] = "4097"
    try:
        assert db.query_multi_gpu("price * quantity WHERE price > 15") == dense.tolist()
    finally:
        del os.environ["WARPDB_HOST_CHUNK_ROWS"]
    ms, mc = db.query_multi_gpu_sum("price * 0.9 WHERE price > 20")
    assert mc == rc and ms == rs
    chunked = pw().WarpDB.query_multi_gpu_csv(str(path), "price * quantity WHERE price > 15", 7_777)
    assert np.array_equal(np.array(chunked, np.float32).view(np.uint32), ref.view(np.uint32))


def test_query_multi_gpu_csv_line_endings(tmp_path):
    # the streaming chunker cuts blocks at the rows_per_chunk-th non-empty
    # line: CRLF, blank lines and a last line without a newline must give the
    # same rows as the whole-file loader
    n = 30_011
    cols = synth.c2_table(n)
    path = tmp_path / "crlf.csv"
    with open(path, "wb") as f:
        f.write(b"price,quantity\r\n")
        for i, (p, q) in enumerate(zip(cols["price"], cols["quantity"])):
            if i % 97 == 0:
                f.write(b"\r\n" if i % 2 else b"\n")  # blank lines
            end = b"" if i == n - 1 else (b"\r\n" if i % 3 == 0 else b"\n")
            f.write(f"{float(p)!r},{int(q)}".encode() + end)
    db = pw().WarpDB(str(path))
    whole = db.query("price * quantity WHERE price > 15")
    assert len(whole) == n
    for rpc in (1, 333, 30_011, 1_000_000):
        got = pw().WarpDB.query_multi_gpu_csv(str(path), "price * quantity WHERE price > 15", rpc)
        assert got == whole, rpc


def test_query_errors():
    db = pw().WarpDB(TEST_CSV)
    with pytest.raises(RuntimeError, match="Unknown column: nope"):
        db.query("nope * 2")
    with pytest.raises(RuntimeError, match="Failed to parse expression"):
        db.query("price +")
    with pytest.raises(RuntimeError, match="Failed to parse WHERE clause"):
        db.query("price WHERE (")
    with pytest.raises(RuntimeError, match="Empty query expression"):
        db.query("")
    with pytest.raises(RuntimeError, match="Unsupported file format"):
        pw().WarpDB(os.path.join(GOLDEN, "golden.json.bak"))


def test_query_sql_reference_expectations():
    db = pw().WarpDB(TEST_CSV)
    assert db.query_sql("SELECT SUM(price) FROM test GROUP BY quantity ORDER BY quantity ASC") == \
        [15.25, 10.5, 20.0, 30.0]
    assert db.query_sql("SELECT price FROM test ORDER BY price DESC LIMIT 2") == [30.0, 20.0]
    assert db.query_sql("SELECT price FROM test ORDER BY price DESC OFFSET 1 LIMIT 2") == [20.0, 15.25]
    assert len(db.query_sql("SELECT SUM(price) FROM test GROUP BY quantity HAVING SUM(price) > 15 "
                            "ORDER BY quantity ASC")) == 3
    assert db.query_sql("SELECT SUM(price) FROM test GROUP BY quantity HAVING COUNT(price) > 1") == []
    d = db.query_sql("SELECT DISTINCT quantity FROM test ORDER BY quantity DESC")
    assert d == [5.0, 4.0, 3.0, 2.0]
    assert db.query_sql("SELECT COUNT(*) FROM test WHERE price > 12") == [3.0]
    assert db.query_sql("SELECT AVG(price) FROM test GROUP BY quantity ORDER BY quantity DESC LIMIT 1") == [30.0]
    assert db.query_sql("SELECT price * 2 FROM test WHERE quantity > 3") == [40.0, 60.0]


def test_query_sql_order_by_other_expression(tmp_path):
    # ORDER BY an expression other than the SELECT one, any LIMIT / OFFSET:
    # keyed device sort (src/warpdb.cpp:470-476), ties by row order, against
    # the oracle's stable ORDER BY (ora_topk with k = every row)
    n = 20_011
    cols = synth.c2_table(n)
    cols["price"] = (np.floor(cols["price"] * 4) / 4).astype(np.float32)  # ties
    path = tmp_path / "o.csv"
    with open(path, "w") as f:
        f.write("price,quantity\n")
        for p, q in zip(cols["price"], cols["quantity"]):
            f.write(f"{float(p)!r},{int(q)}\n")
    db = pw().WarpDB(str(path))
    ht = ora.HostTable(cols)
    for desc in (True, False):
        d = "DESC" if desc else "ASC"
        _, _, rv = ora.topk(ht, "price", n, desc, cond="price > 15", select_expr="quantity * 2")
        got = db.query_sql(f"SELECT quantity * 2 FROM t WHERE price > 15 ORDER BY price {d}")
        assert np.array_equal(np.array(got, np.float32), rv)
        got = db.query_sql(f"SELECT quantity * 2 FROM t WHERE price > 15 ORDER BY price {d} OFFSET 7 LIMIT 100")
        assert np.array_equal(np.array(got, np.float32), rv[7:107])
        # ORDER BY the bare column, no WHERE / LIMIT: the sort reads the column
        # directly (wx_sort_float_from); the table must be left unchanged
        _, _, rv = ora.topk(ht, "price", n, desc)
        assert np.array_equal(np.array(db.query_sql(f"SELECT price FROM t ORDER BY price {d}"), np.float32), rv)
    assert np.array_equal(np.array(db.query("price"), np.float32), cols["price"])
    # same expression, LIMIT beyond the top-K kernel's 32: full sort + slice
    _, _, rv = ora.topk(ht, "price", 100, True)
    assert np.array_equal(np.array(db.query_sql("SELECT price FROM t ORDER BY price DESC LIMIT 100"), np.float32), rv)


def test_query_sql_min_max():
    # AggData min / max (src/warpdb.cpp:375-385, 387-418) on data/test.csv:
    # price [10.5, 20, 15.25, 30], quantity [3, 4, 2, 5]
    db = pw().WarpDB(TEST_CSV)
    assert db.query_sql("SELECT MIN(price) FROM test") == [10.5]
    assert db.query_sql("SELECT MAX(price) FROM test WHERE quantity < 5") == [20.0]
    assert db.query_sql("SELECT MAX(price) FROM test GROUP BY quantity ORDER BY quantity ASC") == \
        [15.25, 10.5, 20.0, 30.0]
    assert db.query_sql("SELECT SUM(price) FROM test GROUP BY quantity HAVING MIN(price) > 12 "
                        "ORDER BY quantity ASC") == [15.25, 20.0, 30.0]
    assert db.query_sql("SELECT MIN(price * quantity) FROM test GROUP BY quantity ORDER BY MIN(price * quantity) "
                        "DESC LIMIT 2") == [150.0, 80.0]
    r = db.query_sql("SELECT MIN(price) FROM test WHERE price > 100")
    assert len(r) == 1 and r[0] != r[0]  # empty -> NaN (SQL NULL)


def test_optimizer_stats_pushdown(tmp_path):
    db = pw().WarpDB(TEST_CSV)
    st = db.column_stats()
    assert st["price"] == (10.5, 30.0, 0, False) and st["quantity"] == (2.0, 5.0, 0, False)
    r, v = db.query_optimized("price * quantity WHERE price > 100")
    assert v == "always_false" and r == [0.0, 0.0, 0.0, 0.0]
    r, v = db.query_optimized("price * quantity WHERE price > 10")
    assert v == "always_true" and r == [31.5, 80.0, 30.5, 150.0]
    r, v = db.query_optimized("price * quantity WHERE price > 15")
    assert v == "unknown" and r == db.query("price * quantity WHERE price > 15")
    # statistics of a larger table (with NaN) against numpy
    n = 100_003
    cols = synth.c2_table(n)
    cols["price"][::97] = np.nan
    path = tmp_path / "s.csv"
    with open(path, "w") as f:
        f.write("price,quantity\n")
        for p, q in zip(cols["price"], cols["quantity"]):
            f.write(f"{float(p)!r},{int(q)}\n")
    big = pw().WarpDB(str(path))
    st = big.column_stats()
    p = cols["price"]
    assert st["price"] == (float(np.nanmin(p)), float(np.nanmax(p)), int(np.isnan(p).sum()), False)
    r, v = big.query_optimized("price WHERE price >= 0", st)
    assert v == "unknown"  # NaN rows fail the comparison
    r, v = big.query_optimized("price WHERE quantity >= 1", st)
    assert v == "always_true"


def test_query_arrow_roundtrip():
    pa = pytest.importorskip("pyarrow")
    db = pw().WarpDB(TEST_CSV)
    get = ctypes.pythonapi.PyCapsule_GetPointer
    get.restype = ctypes.c_void_p
    get.argtypes = [ctypes.py_object, ctypes.c_char_p]
    for shm in (False, True):
        arr_cap, sch_cap = db.query_arrow("price * quantity", shm)
        a = pa.Array._import_from_c(get(arr_cap, None), get(sch_cap, None))
        assert a.type == pa.float32() and a.to_pylist() == [31.5, 80.0, 30.5, 150.0]


def test_sharded_query_single_rank():
    import torch.distributed as dist

    from warpdb_amd import distributed as wd

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    if not dist.is_initialized():
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    n = 300_001
    cols2, cols3 = synth.c2_table(n), synth.c3_table(n)
    shard = wd.Shard({k: torch.from_numpy(v).cuda() for k, v in cols2.items()}, 0, n)
    q = wd.ShardedQuery(shard, custom_src="__device__ float discount(float p, float r) { return p * r; }\n")
    v, i, off, total = q.compact("(price[idx] * quantity[idx])", "(price[idx] > 15.0f)")
    rv, ri = ora.project_filter(ora.HostTable(cols2), "price * quantity", "price > 15")
    assert off == 0 and total == len(ri) and np.array_equal(i.cpu().numpy(), ri)
    s, c = q.sum("(price[idx] * 0.9f)", "(price[idx] > 20.0f)")
    rs, rc = ora.reduce_sum(ora.HostTable(cols2), "price * 0.9", "price > 20")
    assert (s, c) == (rs, rc)
    tk, ti, tv = q.topk("price[idx]", None, "discount(price[idx], 0.9f)", 5, True)
    rk, rix, rvv = ora.topk(ora.HostTable(cols2), "price", 5, True, select_expr="discount(price, 0.9)")
    assert np.array_equal(ti.cpu().numpy(), rix) and np.array_equal(tv.cpu().numpy(), rvv)
    shard3 = wd.Shard({k: torch.from_numpy(v).cuda() for k, v in cols3.items()}, 0, n)
    gk, gs, gc = wd.ShardedQuery(shard3).group_sum("price[idx]", "quantity[idx]", None)
    rk3, rs3, rc3 = ora.group_sum(ora.HostTable(cols3), "price", "quantity")
    assert np.array_equal(gk.cpu().numpy(), rk3) and np.array_equal(gs.cpu().numpy(), rs3)
    dist.destroy_process_group()


@pytest.mark.parametrize("workload,extra", [
    ("project", ["--rows", "1e7", "--c4-rows", "20000001", "--c3-rows", "10000001"]),
    ("sum", ["--total-rows", "20000001"]),  # C4's strong-scaling form, ragged shards
    ("group", ["--rows", "5e6"]),           # the one-collective window + slots all-reduce
    ("group", ["--rows", "2e6", "--keys", "3000"]),  # many keys: list records, one all-gather, the device merge
    ("group", ["--rows", "4e6", "--keys", "100000"]),  # the same over each rank's range-partitioned GROUP BY
    ("topk", ["--rows", "5e6"]),
])
def test_bench_two_ranks_on_one_gpu(workload, extra):
    # the multi-rank bench path (torchrun rendezvous, shards, the product's
    # exchanges, max-over-ranks timing) with two ranks sharing the GPU over
    # gloo; RCCL on the 8-GPU node
    import json
    import socket
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, WARPDB_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--workload", workload, "--steps", "3", "--warmup", "1", *extra],
                       capture_output=True, text=True, cwd=ROOT, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["cpu_baseline"] is None
    assert str(d["check"]).startswith("ok"), d["check"]
    if workload == "project":
        assert d["config"]["total_rows"] == 2 * 10**7 and d["scaling"] == "weak"
        assert d["config"]["passing_rows_per_gpu"] > 0.6 * 10**7
        c4 = d["secondary"]["c4_sum_strong"]  # C4's strong-scaled SUM beside the headline
        assert c4["total_rows"] == 20000001 and c4["rows_per_gpu"] == 10000001 and str(c4["check"]).startswith("ok")
        c3 = d["secondary"]["c3_group_strong"]  # C3's strong-scaled GROUP BY beside it
        assert c3["total_rows"] == 10000001 and c3["rows_per_gpu"] == 5000001 and str(c3["check"]).startswith("ok")
    if workload == "sum":
        assert d["config"]["total_rows"] == 20000001 and d["scaling"] == "strong"
        assert d["config"]["rows_per_gpu"] == 10000001
