"""bench.py host logic on the CPU: the PMC traffic field's provenance."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _write(root, workload, sha, rows=1_000_000_000, hbm=13.0e9):
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    with open(os.path.join(root, "profiles", f"pmc_{workload}.json"), "w") as f:
        json.dump({"rows": rows, "hbm_bytes_per_launch": hbm, "collected": "2026-10-18T00:00Z",
                   "kernel_src_sha16": sha}, f)


def test_traffic_names_its_profile_and_drops_stale_ones(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "kernel_src_sha16", lambda w: "feedfacecafebeef")
    # current profile: scaled bytes + where they came from
    _write(str(tmp_path), "project", "feedfacecafebeef")
    t, src = bench.pmc_traffic("project", 500_000_000)
    assert t == round(13.0e9 / 2)
    assert src["file"] == "profiles/pmc_project.json" and src["current"] and src["collected"]
    # collected against other kernel sources: no bytes, and it says why
    _write(str(tmp_path), "project", "0123456789abcdef")
    t, src = bench.pmc_traffic("project", 1_000_000_000)
    assert t is None and not src["current"] and "stale_reason" in src
    # many-key GROUP BY reads its own profile; a missing one is null
    t, src = bench.pmc_traffic("group", 1_000_000_000, keys=1_000_000)
    assert t is None and src["file"] is None
    r = bench.roofline(13e9, 2.0, 8e9, "k", (None, {"file": None}), "t")
    assert r["traffic"] is None and r["traffic_source"] == {"file": None} and r["frac"] == round(6500 / 8000, 4)


def test_kernel_src_sha_covers_every_family():
    shas = {w: bench.kernel_src_sha16(w) for w in bench.PMC_FAMILIES}
    assert all(len(s) == 16 for s in shas.values())
    assert len(set(shas.values())) == len(shas)  # each family hashes its own source
