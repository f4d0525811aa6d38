"""Summarize a rocprofv3 --kernel-trace --stats run: per-kernel, per-grid-size averages, with the
kernels' resources taken from the code objects, not from the trace.

Usage: python profiles/summarize.py <dir with run_kernel_trace.csv | *_results.db> [lib.so] > summary.json
(rocprofv3 7.x writes an SQLite database by default; --output-format csv writes the CSV trace.)

Resource columns: rocprofv3's VGPR_Count on gfx950 is the granule-encoded
arch-VGPR field decoded with the wrong granule (the N2 proposal instantiation reads 48; its code
object says 86-96) and LDS_Block_Size is the static group segment only (0 for every kernel here that
sizes its LDS at launch).  So:
  vgpr / agpr / sgpr / scratch_bytes_per_lane / lds_static_bytes / vgpr_spill: the AMDGPU metadata
    notes of the library's gfx950 code objects (tools/isa_resources.py);
  lds_dynamic_bytes_per_wg: the library's own launch sizes (aiqmc_debug_launch_lds, host only);
  waves_per_wg: workgroup size / 64 from the trace;
  occupancy_waves_per_simd: min(VGPR limit 512 // ceil8(vgpr) (.vgpr_count is the unified arch +
    acc allocation on gfx950), LDS limit
    160 KiB // (static + dynamic LDS per workgroup) * waves_per_wg / 4, 8);
  rocprof_raw: the trace's own fields, for reference.
"""
import csv
import glob
import json
import os
import re
import sqlite3
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd"))


def rows(path):
    dbs = [path] if path.endswith(".db") else sorted(glob.glob(os.path.join(path, "*.db")))
    if dbs:
        c = sqlite3.connect(dbs[0])
        for r in c.execute("select name, grid_x, workgroup_x, duration, vgpr_count, accum_vgpr_count, "
                           "sgpr_count, lds_size, scratch_size from kernels"):
            yield (r[0], int(r[1]) // max(1, int(r[2])), r[3] / 1e3, int(r[2]),
                   {"vgpr": r[4], "agpr": r[5], "sgpr": r[6], "lds_bytes": r[7], "scratch": r[8]})
        return
    traces = sorted(glob.glob(os.path.join(path, "*kernel_trace.csv")))
    for t in csv.DictReader(open(traces[0])):
        yield (t["Kernel_Name"], int(t["Grid_Size_X"]) // max(1, int(t["Workgroup_Size_X"])),
               (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3, int(t["Workgroup_Size_X"]),
               {"vgpr": int(t["VGPR_Count"]), "agpr": int(t["Accum_VGPR_Count"]), "sgpr": int(t["SGPR_Count"]),
                "lds_bytes": int(t["LDS_Block_Size"]), "scratch": int(t["Scratch_Size"])})


KIND = {  # template pattern -> AIQMC_LDS_* kind (the launches that size their LDS at launch time)
    r"k_walker_rev<(float|double), (\d+), (\d+), false, true,": "proposal",
    r"k_walker_rev<(float|double), (\d+), (\d+), false, false,": "walker",
    r"k_walker_rev<(float|double), (\d+), (\d+), true,": "adjoint",
    r"k_walker_lap<(float|double), (\d+), (\d+),": "lap",
    r"k_param_grad<(float|double), (\d+), (\d+)": "pgrad",
    r"k_walker<(float|double), (\d+), (\d+), 1>": "fwdlap",
}


def dynamic_lds(name, cache={}):
    for pat, kind in KIND.items():
        m = re.search(pat, name)
        if not m:
            continue
        key = (m.group(1), int(m.group(2)), int(m.group(3)))
        if key not in cache:
            try:
                import torch
                from aiqmc import _lib
                cache[key] = _lib.launch_lds(key[1], key[2], torch.float32 if key[0] == "float" else torch.float64)
            except Exception as e:   # a library without the query: say so rather than guess
                cache[key] = {"error": repr(e)}
        t = cache[key]
        return t[kind]["dyn_lds_bytes_per_wg"] if kind in t else None
    return 0


def occupancy(res, lds_total, waves_per_wg):
    regs = res["vgpr"]   # gfx950: unified file, .vgpr_count includes the acc VGPRs
    by_vgpr = 512 // max(8, -(-regs // 8) * 8)
    if lds_total:
        wgs = (160 * 1024) // lds_total
        by_lds = wgs * waves_per_wg / 4.0
    else:
        by_lds = 8
    return min(by_vgpr, by_lds, 8)


def main():
    lib = sys.argv[2] if len(sys.argv) > 2 else None
    try:
        import isa_resources
        isa = isa_resources.resources(lib) if lib else isa_resources.resources()
    except Exception as e:
        isa, isa_err = {}, repr(e)
    else:
        isa_err = None
    acc = defaultdict(list)
    meta = {}
    for name, grid, us, wg, raw in rows(sys.argv[1]):
        acc[(name, grid)].append(us)
        meta[(name, grid)] = (wg, raw)
    out = []
    for (name, grid), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        wg, raw = meta[(name, grid)]
        rec = {"kernel": name[:160], "workgroups": grid, "launches": len(v), "avg_us": sum(v) / len(v),
               "min_us": min(v), "max_us": max(v), "total_us": sum(v), "waves_per_wg": wg // 64}
        r = isa.get(name)
        if r:
            dyn = dynamic_lds(name)
            rec.update({k: r[k] for k in ("vgpr", "agpr", "sgpr", "scratch_bytes_per_lane", "lds_static_bytes",
                                          "vgpr_spill")})
            rec["lds_dynamic_bytes_per_wg"] = dyn
            if dyn is not None:
                rec["occupancy_waves_per_simd"] = occupancy(r, r["lds_static_bytes"] + dyn, max(1, wg // 64))
        else:
            rec["resources"] = "not in the library's code objects" + (f" ({isa_err})" if isa_err else "")
        rec["rocprof_raw"] = raw
        out.append(rec)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
