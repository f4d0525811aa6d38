"""Summarize a rocprofv3 --kernel-trace --stats run: per-kernel, per-grid-size averages.
Usage: python profiles/summarize.py <dir with run_kernel_trace.csv | *_results.db> > summary.json
(rocprofv3 7.x writes an SQLite database by default; --output-format csv writes the CSV trace.)"""
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    dbs = [path] if path.endswith(".db") else sorted(glob.glob(os.path.join(path, "*.db")))
    if dbs:
        c = sqlite3.connect(dbs[0])
        for r in c.execute("select name, grid_x, workgroup_x, duration, vgpr_count, accum_vgpr_count, "
                           "sgpr_count, lds_size, scratch_size from kernels"):
            yield (r[0], int(r[1]) // max(1, int(r[2])), r[3] / 1e3,
                   {"vgpr": r[4], "agpr": r[5], "sgpr": r[6], "lds_bytes": r[7], "scratch": r[8], "wg": r[2]})
        return
    for t in csv.DictReader(open(os.path.join(path, "run_kernel_trace.csv"))):
        yield (t["Kernel_Name"], int(t["Grid_Size_X"]) // max(1, int(t["Workgroup_Size_X"])),
               (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3,
               {"vgpr": int(t["VGPR_Count"]), "agpr": int(t["Accum_VGPR_Count"]), "sgpr": int(t["SGPR_Count"]),
                "lds_bytes": int(t["LDS_Block_Size"]), "scratch": int(t["Scratch_Size"]),
                "wg": int(t["Workgroup_Size_X"])})


acc = defaultdict(list)
meta = {}
for name, grid, us, m in rows(sys.argv[1]):
    acc[(name, grid)].append(us)
    meta[(name, grid)] = m
out = []
for (name, grid), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    out.append({"kernel": name[:160], "workgroups": grid, "launches": len(v), "avg_us": sum(v) / len(v),
                "min_us": min(v), "max_us": max(v), "total_us": sum(v), **meta[(name, grid)]})
print(json.dumps(out, indent=1))
