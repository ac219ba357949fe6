#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs into per-kernel average counters.

usage: pmc_summary.py <counter_collection.csv>... > summary.json
FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KB; on gfx950 FETCH_SIZE
counts half the bytes of a wide (16 B/lane) coalesced stream
(MI355X_MICROARCH.md, HBM section), so both the raw and the x2 corrected read
bytes are given.
"""
import csv
import json
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?")
            cname = row.get("Counter_Name")
            val = float(row.get("Counter_Value", 0) or 0)
            disp = row.get("Dispatch_Id")
            acc[name][(cname, disp)].append(val)
out = {}
for kname, d in acc.items():
    per = defaultdict(list)
    for (cname, disp), vals in d.items():
        per[cname].append(sum(vals))  # sum over agent/XCC dimensions of one dispatch
    out[kname] = {c: {"dispatches": len(v), "avg": sum(v) / len(v)} for c, v in per.items()}
    if "FETCH_SIZE" in per:
        f = out[kname]["FETCH_SIZE"]["avg"] * 1024
        out[kname]["fetch_bytes_raw"] = f
        out[kname]["fetch_bytes_corrected_x2"] = 2 * f
    if "WRITE_SIZE" in per:
        out[kname]["write_bytes"] = out[kname]["WRITE_SIZE"]["avg"] * 1024
json.dump(out, sys.stdout, indent=1)
