#!/usr/bin/env python3
"""Write profiles/pmc_<workload>.json from a tools/pmc_summary.py summary.

usage: pmc_record.py WORKLOAD ROWS SUMMARY_JSON [NOTE]
The record carries the collection date and the sha of the kernel sources it
was collected against (bench.kernel_src_sha16); bench.py reports a profile
whose sources have changed since as stale (traffic null), so every bench
line's `roofline.traffic` names a profile that matches the tree.
Per query: the dominant kernels of bench.PMC_FAMILIES, each kernel's
per-dispatch average times its dispatches per query (None: every kernel of
that prefix once -- a pipeline).  Read bytes are FETCH_SIZE x 2 (gfx950 counts
half of a 16 B/lane stream, MI355X_MICROARCH.md HBM section), written bytes
WRITE_SIZE; both reported in KB.
"""
import datetime
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

workload, rows, summary = sys.argv[1], int(float(sys.argv[2])), sys.argv[3]
note = sys.argv[4] if len(sys.argv) > 4 else ""
with open(summary) as f:
    per_kernel = json.load(f)
kernels, _ = bench.PMC_FAMILIES[workload]
fetch = write = 0.0
used = {}
for prefix, mult in kernels.items():
    hits = {k: v for k, v in per_kernel.items() if k.startswith(prefix)}
    if not hits:
        sys.exit(f"no kernel named {prefix}* in {summary}")
    if mult is None:
        for k, v in hits.items():
            fetch += v.get("fetch_bytes_corrected_x2", 0.0)
            write += v.get("write_bytes", 0.0)
            used[k] = 1
    else:
        # the busiest variant of the prefix (one query runs one of them)
        k, v = max(hits.items(), key=lambda kv: kv[1].get("fetch_bytes_corrected_x2", 0.0))
        fetch += mult * v.get("fetch_bytes_corrected_x2", 0.0)
        write += mult * v.get("write_bytes", 0.0)
        used[k] = mult
out = {
    "kernel": " + ".join(f"{m} x {k}" if m != 1 else k for k, m in used.items()),
    "rows": rows,
    "collected": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%MZ"),
    "kernel_src_sha16": bench.kernel_src_sha16(workload),
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/pmc_run.sh " + workload + ")"
              + (f"; {note}" if note else ""),
    "fetch_bytes_corrected": fetch,
    "write_bytes": write,
    "hbm_bytes_per_launch": fetch + write,
    "note": "FETCH_SIZE x1024 x2 (gfx950 counts half of a 16 B/lane stream, MI355X_MICROARCH.md HBM section); "
            "WRITE_SIZE x1024; per query: per-dispatch averages x dispatches per query",
}
path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
with open(path, "w") as f:
    json.dump(out, f, indent=1)
    f.write("\n")
print(json.dumps(out))
