"""Summarise rocprofv3 --pmc counter CSVs per kernel (per wave and per dispatch).
usage: python profiles/pmc_summary.py <dir-with-pass-subdirs> [pass ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    files = sorted(glob.glob(os.path.join(root, "*", "*_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in files:
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"][:48], int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[key][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    for key, d in agg.items():
        waves = d.get("SQ_WAVES")
        print(f"{key[0]}  workgroups={key[1]}")
        for c, v in sorted(d.items()):
            n = len(disp[key][c])
            pw = f"  per-wave {v / waves:10.1f}" if waves else ""
            print(f"   {c:26s} per-dispatch {v / n:12.4g}{pw}")


if __name__ == "__main__":
    main()
