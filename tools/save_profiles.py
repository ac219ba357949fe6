"""Copy a gpu_refresh.sh run into profiles/: per-workload PMC traffic
(profiles/pmc_<w>.json, read by bench.py), kernel-trace stats, PMC summaries
and the bench lines (with the PMC traffic filled in) under profiles/<round>/.

usage: python tools/save_profiles.py r01 [project sum group topk]
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = {"project": "wx_project_compact_deep", "sum": "wx_reduce_sum", "group": "wx_group_sum", "topk": "wx_topk_scan", "dense": "wx_project_dense",
     "sort": "wx_radix_tile_k_f_a"}
rnd = sys.argv[1]
wls = sys.argv[2:] or list(K)
out = os.path.join(ROOT, "profiles", rnd)
os.makedirs(out, exist_ok=True)
go = os.path.join(ROOT, "gpurun_out")
for w in wls:
    k = K[w]
    b = [json.loads(line) for line in open(os.path.join(go, "refresh", f"bench_{w}.log")) if line.startswith("{")][0]
    pmc_sum = os.path.join(go, f"pmc_{w}", "summary.json")
    if os.path.exists(pmc_sum) and w != "sort":  # sort: several kernels per step, no per-launch traffic
        s = json.load(open(pmc_sum))
        k = b["roofline"]["kernel"] if b["roofline"]["kernel"] in s else k
        s = s[k]
        d = {"kernel": k, "rows": b["config"]["rows_per_gpu"],
             "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/pmc_run.sh {w}), {rnd}",
             "fetch_size_kb_avg": s["FETCH_SIZE"]["avg"], "write_size_kb_avg": s["WRITE_SIZE"]["avg"],
             "fetch_bytes_corrected": s["fetch_bytes_corrected_x2"], "write_bytes": s["write_bytes"],
             "hbm_bytes_per_launch": s["fetch_bytes_corrected_x2"] + s["write_bytes"],
             "algorithmic_bytes_per_launch": b["roofline"]["bytes_per_launch"],
             "note": "FETCH_SIZE x1024 x2 (gfx950 counts half of a 16 B/lane stream, MI355X_MICROARCH.md HBM "
                     "section); WRITE_SIZE x1024"}
        json.dump(d, open(os.path.join(ROOT, "profiles", f"pmc_{w}.json"), "w"), indent=1)
        shutil.copy(pmc_sum, os.path.join(out, f"pmc_{w}_summary.json"))
        b["roofline"]["traffic"] = round(d["hbm_bytes_per_launch"])
    st = glob.glob(os.path.join(go, "refresh", f"prof_{w}", "**", "*kernel_stats.csv"), recursive=True)
    if st:
        shutil.copy(st[0], os.path.join(out, f"{w}_kernel_stats.csv"))
    json.dump(b, open(os.path.join(out, f"bench_{w}.json"), "w"), indent=1)
    print(w, b["ms_per_step"], b["roofline"]["kernel_ms"], b["roofline"]["traffic"])
