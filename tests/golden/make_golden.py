"""Regenerate tests/golden/golden.json from the reference's own code.

Runs oracle/_ref/ref_harness (built by oracle/build_ref.sh from the
reference's tokenizer/parser/evaluator sources in /root/reference) on the
reference's data fixtures and records, per query, the passing row indices and
the exact float results (hex).  Run in the build container:
    ./oracle/build_ref.sh && python tests/golden/make_golden.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")

PROJECT = [
    ("test.csv", "price * quantity WHERE price > 10", None),
    ("test.csv", "price * quantity WHERE price > 15", None),
    ("test.csv", "price WHERE price > 15", None),
    ("test.csv", "price * 0.9 WHERE price > 20", None),
    ("test.csv", "price * 0.9", None),
    ("test.csv", "price * quantity * 1.08", None),
    ("test.csv", "price + 1", None),
    ("test.csv", "(price + quantity) * 2 WHERE quantity <= 4", None),
    ("test.csv", "price / quantity - 1 WHERE price != 20", None),
    ("extended.csv", "price * discount", "202"),
    ("extended.csv", "price * discount WHERE discount >= 0.1", "202"),
]
LOWER = [
    "price > 10", "quantity <= 5", "discount(price, 0.9)", "price > 10 AND quantity < 5",
    "price > 10 OR quantity < 5", "price + quantity * 2", "(price + quantity) * 2",
    "price * quantity", "price * 0.9", ".5 + price", "a.b + 1",
]
ERRORS = ["1 2", "(price + 5", "price & 5", "price # 1\n", "price +", ""]


def run(*args):
    return subprocess.run([HARNESS, *args], capture_output=True, text=True).stdout


def main():
    out = {"source": "oracle/_ref/ref_harness (reference src/expression.cpp:1-268, src/warpdb.cpp:109-157, "
                     "src/csv_loader.cpp:49-124)", "project": [], "lower": [], "errors": []}
    for csv, q, schema in PROJECT:
        args = ["eval", os.path.join(HERE, csv), q] + ([schema] if schema else [])
        rows = [l.split() for l in run(*args).strip().splitlines() if l.strip()]
        out["project"].append({"csv": csv, "query": q, "schema": schema,
                               "idx": [int(r[0]) for r in rows], "vals": [r[1] for r in rows]})
    for e in LOWER:
        out["lower"].append({"expr": e, "lowered": run("lower", e).strip()})
    for e in ERRORS:
        out["errors"].append({"expr": e, "message": run("lower", e).strip()})
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
