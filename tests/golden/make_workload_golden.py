"""Reference-generated fixtures at workload scale (BASELINE.json C2-C5 shapes).

TEST INFRASTRUCTURE.  Writes each synthetic table as CSV (the generator is
tests/synth.py, the same one wx_fill_synthetic runs on the device), runs the
reference's own CPU path on it through oracle/_ref/ref_harness (built by
oracle/build_ref.sh from /root/reference: load_csv_to_host with std::stof,
tokenize / parse_expression, eval_node), and stores what the reference
computed:

  workload_c2.npz  'price * quantity WHERE price > 15', 100 000 rows:
                   passing-row mask (packed bits) + result float bits
  workload_c4.npz  'price * 0.9 WHERE price > 20', 100 000 rows: same
  workload_c3.npz  SUM(price) GROUP BY quantity (int32 keys 0..1023),
                   100 000 rows: the reference query_sql's std::map
                   aggregation in double (src/warpdb.cpp:375-385)
  workload_c3w.npz SUM(price) GROUP BY quantity with int32 keys over
                   0..74 999 (about 55 000 distinct in 100 000 rows): the
                   many-key GROUP BY, same std::map aggregation
  workload_c3o.npz SUM(price) GROUP BY quantity where the fold order
                   matters: int32 keys 0..199 (about 500 rows each), prices
                   of 1e7, 1 and 1e-3 scales mixed within every key (a
                   group's values span more than a double's 53 bits), so
                   only the reference's own row-order std::map fold gives
                   these bits -- the fixture of WX_F_ROW_ORDER
  workload_c5.npz  ORDER BY price DESC LIMIT 32 over 100 000 rows of
                   price rounded to 0.25 (heavy ties): rows + key bits of a
                   stable sort by the reference's eval_node value
  workload_golden.json  queries, generator parameters, row counts and the
                   sha256 of each CSV text (the tests regenerate the table
                   and check the hash, so the fixture is tied to the data)

Run in the build container:
    ./oracle/build_ref.sh && python tests/golden/make_workload_golden.py [case ...]
(with case names, only those fixtures are rewritten and their entries in
workload_golden.json replaced; the others stay byte for byte)
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
N = 100_000


def csv_text(cols: dict, int_cols=()) -> str:
    """Header + rows; floats with 9 significant digits (std::stof reads them back exactly)."""
    names = list(cols)
    lines = [",".join(names)]
    cells = []
    for nm in names:
        v = cols[nm]
        cells.append([str(int(x)) for x in v] if nm in int_cols or v.dtype.kind == "i" else
                     ["%.9g" % float(x) for x in v])
    lines += [",".join(row) for row in zip(*cells)]
    return "\n".join(lines) + "\n"


def c3w_table(n: int):
    """price f32 U[0,40), quantity int32 U{0..74999}: many distinct keys."""
    return {"price": synth.uniform_f32(n, synth.SEED_PRICE, 0.0, 40.0),
            "quantity": synth.uniform_int(n, synth.SEED_KEY, 0, 74_999).astype(np.int32)}


def c3o_table(n: int):
    """price = U[0,1) x one of {1e7, 1, 1e-3} per row, quantity int32 U{0..199}:
    every group mixes values 2^33 apart in magnitude, so its double sum
    depends on the order of the adds."""
    u = synth.uniform_f32(n, synth.SEED_PRICE, 0.0, 1.0)
    scale = np.array([1e7, 1.0, 1e-3], np.float32)[synth.uniform_int(n, 4, 0, 2)]
    return {"price": (u * scale).astype(np.float32),
            "quantity": synth.uniform_int(n, synth.SEED_KEY, 0, 199).astype(np.int32)}


def c5_table(n: int):
    """price U[0,40) rounded to multiples of 0.25: ~160 distinct keys, heavy ties."""
    p = synth.uniform_f32(n, synth.SEED_PRICE, 0.0, 40.0)
    return {"price": (np.floor(p * np.float32(4.0)) / np.float32(4.0)).astype(np.float32)}


def run(*args) -> str:
    r = subprocess.run([HARNESS, *args], capture_output=True, text=True, check=True)
    return r.stdout


def main():
    if not os.path.exists(HARNESS):
        raise SystemExit("build oracle/_ref first: ./oracle/build_ref.sh")
    only = set(sys.argv[1:])
    meta = {"source": "oracle/_ref/ref_harness over the reference's load_csv_to_host / eval_node "
                      "(src/csv_loader.cpp:49-124, src/warpdb.cpp:109-157)", "rows": N, "cases": {}}
    if only:
        with open(os.path.join(HERE, "workload_golden.json")) as f:
            meta = json.load(f)
    with tempfile.TemporaryDirectory() as tmp:
        tables = {
            "c2": (synth.c2_table(N), (), None, "price * quantity WHERE price > 15"),
            "c4": (synth.c2_table(N), (), None, "price * 0.9 WHERE price > 20"),
            "c3": (synth.c3_table(N), ("quantity",), "20", None),
            "c3w": (c3w_table(N), ("quantity",), "20", None),
            "c3o": (c3o_table(N), ("quantity",), "20", None),
            "c5": (c5_table(N), (), None, None),
        }
        for name, (cols, ints, schema, query) in tables.items():
            if only and name not in only:
                continue
            text = csv_text(cols, ints)
            path = os.path.join(tmp, f"{name}.csv")
            with open(path, "w") as f:
                f.write(text)
            case = {"csv_sha256": hashlib.sha256(text.encode()).hexdigest(), "schema": schema}
            if name in ("c2", "c4"):
                rows = [ln.split() for ln in run("eval", path, query).splitlines() if ln.strip()]
                idx = np.array([int(r[0]) for r in rows], np.int64)
                vals = np.array([float.fromhex(r[1]) for r in rows], np.float32)
                mask = np.zeros(N, bool)
                mask[idx] = True
                np.savez_compressed(os.path.join(HERE, f"workload_{name}.npz"), mask=np.packbits(mask),
                                    bits=vals.view(np.uint32))
                case.update(query=query, generator="synth.c2_table", passing=int(len(idx)))
            elif name in ("c3", "c3w", "c3o"):
                rows = [ln.split() for ln in run("groupsum", path, "price", "quantity", schema).splitlines()]
                np.savez_compressed(os.path.join(HERE, f"workload_{name}.npz"),
                                    keys=np.array([int(r[0]) for r in rows], np.int32),
                                    sums=np.array([float.fromhex(r[1]) for r in rows], np.float64),
                                    counts=np.array([int(r[2]) for r in rows], np.int64))
                case.update(query="SELECT SUM(price) FROM t GROUP BY quantity",
                            generator="synth.c3_table" if name == "c3" else f"make_workload_golden.{name}_table",
                            groups=len(rows))
            else:
                rows = [ln.split() for ln in run("topk", path, "price", "32", "1").splitlines()]
                np.savez_compressed(os.path.join(HERE, "workload_c5.npz"),
                                    rows=np.array([int(r[0]) for r in rows], np.int64),
                                    bits=np.array([float.fromhex(r[1]) for r in rows], np.float32).view(np.uint32))
                case.update(query="SELECT price FROM t ORDER BY price DESC LIMIT 32",
                            generator="floor(synth.uniform_f32(n, 1, 0, 40) * 4) / 4", k=32)
            meta["cases"][name] = case
    with open(os.path.join(HERE, "workload_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
