"""Dump the gfx950 assembly + resource usage of one generated kernel family.

usage: python tools/isa_dump.py {compact,sum,group,topk,util} [EXTRA_DEFINES]
Writes /tmp/wx_<op>.hip and /tmp/wx_<op>.s and prints vgpr/sgpr/scratch/LDS
per kernel (offline hipcc compile of the exact source the runtime builds).
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from warpdb_amd import _warpexec as wx  # noqa: E402

op = sys.argv[1]
if len(sys.argv) > 2:
    os.environ["WARPDB_EXTRA_DEFINES"] = sys.argv[2]
t = wx.Table(1 << 20, [wx.Column("price", wx.FLOAT32, 1 << 20), wx.Column("quantity", wx.FLOAT32, 2 << 20)])
t_int = wx.Table(1 << 20, [wx.Column("price", wx.FLOAT32, 1 << 20), wx.Column("quantity", wx.INT32, 2 << 20)])
jobs = {
    "dense": (t, wx.OP_DENSE, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", None, 0),
    "compact": (t, wx.OP_COMPACT, "(price[idx] * quantity[idx])", "(price[idx] > 15.0f)", None, 0),
    "sum": (t, wx.OP_SUM, "(price[idx] * 0.9f)", "(price[idx] > 20.0f)", None, 0),
    "group": (t_int, wx.OP_GROUP, "price[idx]", None, "quantity[idx]", 0),
    "topk": (t, wx.OP_TOPK, "price[idx]", None, "(price[idx] * 0.9f)", 5),
    "util": (None, wx.OP_UTIL, None, None, None, 0),
}
table, o, e, c, aux, k = jobs[op]
src = wx.prepare(table, o, e, c, aux, k, want_source=True)
hip = f"/tmp/wx_{op}.hip"
with open(hip, "w") as f:
    f.write(src)
asm = f"/tmp/wx_{op}.s"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-munsafe-fp-atomics",
                "--cuda-device-only", "-S", "-o", asm, hip], check=True)
text = open(asm).read()
for kern in re.findall(r"\.amdhsa_kernel (\w+)", text):
    blk = text.split(f".amdhsa_kernel {kern}\n", 1)
    if len(blk) < 2:
        continue
    meta = blk[1].split(".end_amdhsa_kernel", 1)[0]
    get = lambda key: (re.search(rf"{key}\s+(\S+)", meta) or [None, "?"])[1]
    print(f"{kern:28s} vgpr {get('.amdhsa_next_free_vgpr'):>4} sgpr {get('.amdhsa_next_free_sgpr'):>4} "
          f"scratch {get('.amdhsa_private_segment_fixed_size'):>5} lds {get('.amdhsa_group_segment_fixed_size'):>6}")
print("asm:", asm)
