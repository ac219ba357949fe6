#!/usr/bin/env python3
"""Per-kernel (and per-position-in-step) durations from a rocprofv3
--kernel-trace CSV.

usage: kernel_trace_summary.py TRACE.csv [PREFIX ...]
For every kernel name starting with one of the prefixes (default wx_), the
dispatch count and average / min / max duration in microseconds.  Kernels
that run several times per step in a fixed order (the radix sort's tile
passes) are also split by their index within each run of consecutive
dispatches of the same family, so pass 0..3 of every sort get their own line
("wx_radix_tile_k_fp_a #2" = the third tile pass of each sort).
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    prefixes = tuple(sys.argv[2:]) or ("wx_",)
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if not name.startswith(prefixes):
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    by_name = defaultdict(list)
    by_pos = defaultdict(list)
    prev, pos = None, 0
    for s, e, name in rows:
        us = (e - s) / 1e3
        by_name[name].append(us)
        pos = pos + 1 if name == prev else 0
        prev = name
        by_pos[(name, pos)].append(us)

    def line(label, v):
        print(f"{label:48s} n={len(v):5d} avg={sum(v) / len(v):10.2f} us  min={min(v):10.2f}  max={max(v):10.2f}")

    for name in sorted(by_name):
        line(name, by_name[name])
        keys = sorted(k for k in by_pos if k[0] == name)
        if len(keys) > 1:
            for k in keys:
                line(f"  {name} #{k[1]}", by_pos[k])


if __name__ == "__main__":
    main()
