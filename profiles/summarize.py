"""Summarize a rocprofv3 --kernel-trace --stats run: per-kernel, per-grid-size averages.
Usage: python profiles/summarize.py <dir with run_kernel_trace.csv> > summary.json"""
import csv
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
tr = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
acc = defaultdict(list)
meta = {}
for t in tr:
    key = (t["Kernel_Name"], int(t["Grid_Size_X"]) // max(1, int(t["Workgroup_Size_X"])))
    acc[key].append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3)
    meta[key] = {"vgpr": int(t["VGPR_Count"]), "agpr": int(t["Accum_VGPR_Count"]), "sgpr": int(t["SGPR_Count"]),
                 "lds_bytes": int(t["LDS_Block_Size"]), "scratch": int(t["Scratch_Size"]),
                 "wg": int(t["Workgroup_Size_X"])}
out = []
for (name, grid), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    out.append({"kernel": name, "workgroups": grid, "launches": len(v), "avg_us": sum(v) / len(v),
                "min_us": min(v), "max_us": max(v), "total_us": sum(v), **meta[(name, grid)]})
print(json.dumps(out, indent=1))
