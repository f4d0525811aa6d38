"""Summarise the rocprofv3 PMC passes of the bench's side measurements (tools/gpu_side_prof.sh: one
process per side configuration, run by tools/side_loop.py, one counter group per pass) into the
JSON bench.py reads (profiles/pmc_side_rNN.json), stamped with the library's SHA-256 prefix.

HBM bytes per MI355X_MICROARCH.md: FETCH_SIZE (KB) counts half of the bytes of wide coalesced reads
on gfx950 -> x2; WRITE_SIZE (KB) as counted.  Per dispatch means over every dispatch of the kernel.

usage: python profiles/pmc_side.py <out dir> <lib sha16>  > profiles/pmc_side_rNN.json"""
import collections
import csv
import glob
import json
import os
import sys

# side configuration -> (dominant kernel(s) whose per-launch counters the bench's roofline uses)
SIDES = {
    "ecp_c": ["k_quad_value<float, 4, 1>"],
    "ecp_c2": ["k_quad_value<float, 8, 2>"],
    "adam_be": ["k_quad_grad<float, 4, 1, false>"],
    "dmc_ne": ["k_walker_rev<float, 10, 1, true, false", "k_walker_lap<float, 10, 1, 1, false>"],
}
PASSES = ("fetch", "write", "mix")


def per_pass(root, side, name):
    """{kernel pattern: {counter: mean per dispatch, 'dispatches': n}} for one pass directory."""
    out = {}
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, side, name, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            pat = next((p for p in SIDES[side] if p in r["Kernel_Name"]), None)
            if pat is not None:
                acc[pat][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[pat].add(r["Dispatch_Id"])
    for pat, d in acc.items():
        n = max(len(disp[pat]), 1)
        out[pat] = {c: v / n for c, v in d.items()}
        out[pat]["dispatches"] = n
    return out


def summarise(root):
    res = {}
    for side, pats in SIDES.items():
        p = {n: per_pass(root, side, n) for n in PASSES}
        ks = {}
        tot = 0.0
        ok = True
        for pat in pats:
            g = lambda n, c: p.get(n, {}).get(pat, {}).get(c)
            f, w = g("fetch", "FETCH_SIZE"), g("write", "WRITE_SIZE")
            waves = g("mix", "SQ_WAVES") or g("fetch", "SQ_WAVES")
            k = {"dispatches": g("fetch", "dispatches"), "waves": waves}
            if f is not None and w is not None:
                k["hbm_read_bytes_per_launch"] = 2.0 * f * 1024
                k["hbm_write_bytes_per_launch"] = w * 1024
                k["hbm_bytes_per_launch"] = 2.0 * f * 1024 + w * 1024
                tot += k["hbm_bytes_per_launch"]
            else:
                ok = False
            if g("mix", "SQ_INSTS_VALU") is not None and waves:
                k["valu_insts_per_wave"] = g("mix", "SQ_INSTS_VALU") / waves
                fp = sum((g("mix", c) or 0.0) for c in ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32",
                                                        "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_TRANS_F32"))
                k["fp_valu_insts_per_wave"] = fp / waves
            ks[pat] = k
        res[side] = {"kernels": ks, "hbm_bytes_per_launch": tot if ok else None}
    return res


def main():
    root, sha = sys.argv[1], sys.argv[2]
    out = {"source": "tools/gpu_side_prof.sh: rocprofv3 --pmc, one side configuration per process "
                     "(tools/side_loop.py), one counter group per pass; per-dispatch means",
           "correction": "gfx950: FETCH_SIZE x2 (wide coalesced reads counted at half), WRITE_SIZE as counted",
           "lib_sha16": sha, "walkers": 4096, "sides": summarise(root)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
