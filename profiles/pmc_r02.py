"""Per-launch PMC figures of the Metropolis kernels from the rocprofv3 --pmc passes of
tools/gpu_pmc2.sh (one pass per counter group over tools/mc_loop.py), as the JSON bench.py reads
(profiles/pmc_r02.json).  HBM bytes per MI355X_MICROARCH.md: FETCH_SIZE (KB) counts half of the
bytes of wide coalesced reads on gfx950 -> x2; WRITE_SIZE (KB) as counted.
usage: python profiles/pmc_r02.py <gpurun_out/pmc>"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {
    "proposal": "k_walker_rev<float, 14, 2, false, true>",
    "walker": "k_walker_rev<float, 14, 2, false, false>",
    "moved_electron": "k_moved_electron<float, 14, 2>",
}
PROPOSAL_WAVES = 4096 * 14   # reuse off: the proposals run in the general instantiation


def classify(name, grid, wg):
    """Kernel key of one dispatch (by name; the general instantiation by its grid)."""
    for key, pat in KERNELS.items():
        if pat in name:
            if key == "walker" and grid // wg == PROPOSAL_WAVES:
                return "proposal"
            return key
    return None


def per_pass(root, name):
    """{kernel key: {counter: mean per dispatch}} for one pass directory."""
    out = {}
    for f in glob.glob(os.path.join(root, name, "*_counter_collection.csv")):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            key = classify(r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]))
            if key is not None:
                acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[key].add(r["Dispatch_Id"])
        for key, d in acc.items():
            n = max(len(disp[key]), 1)
            out[key] = {c: v / n for c, v in d.items()}
    return out


def summarise(root, prefix=""):
    p = {n: per_pass(root, prefix + n) for n in ("mix", "stall", "misc", "mem", "fetch", "write")}
    res = {}
    for key in KERNELS:
        get = lambda n, c: p.get(n, {}).get(key, {}).get(c)
        waves = get("mix", "SQ_WAVES") or get("fetch", "SQ_WAVES")
        d = {"waves": waves}
        if get("mix", "SQ_INSTS_VALU") is not None and waves:
            d["valu_insts_per_wave"] = get("mix", "SQ_INSTS_VALU") / waves
            for c in ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32",
                      "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_LDS"):
                if get("mix", c) is not None:
                    d[c.lower() + "_per_wave"] = get("mix", c) / waves
        if get("stall", "SQ_WAVE_CYCLES") is not None and waves:
            for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                d[c.lower() + "_per_wave"] = get("stall", c) / waves
        if get("misc", "SQ_INSTS_MFMA") is not None:
            d["mfma_insts_per_launch"] = get("misc", "SQ_INSTS_MFMA")
            d["mfma_busy_cycles_per_launch"] = get("misc", "SQ_VALU_MFMA_BUSY_CYCLES")
            d["mfma_util"] = 0.0 if not get("misc", "SQ_INSTS_MFMA") else None
            if waves:
                d["lds_bank_conflict_cycles_per_wave"] = (get("misc", "SQ_LDS_BANK_CONFLICT") or 0) / waves
        if get("mem", "SQ_INSTS_VMEM_RD") is not None and waves:
            d["vmem_rd_per_wave"] = get("mem", "SQ_INSTS_VMEM_RD") / waves
            d["vmem_wr_per_wave"] = get("mem", "SQ_INSTS_VMEM_WR") / waves
        f, w = get("fetch", "FETCH_SIZE"), get("write", "WRITE_SIZE")
        if f is not None:
            d["fetch_size_kb_per_launch"] = f
            d["hbm_read_bytes_per_launch"] = 2.0 * f * 1024
        if w is not None:
            d["write_size_kb_per_launch"] = w
            d["hbm_write_bytes_per_launch"] = w * 1024
        if f is not None and w is not None:
            d["hbm_bytes_per_launch"] = 2.0 * f * 1024 + w * 1024
        res[key] = d
    return res


def main():
    root = sys.argv[1]
    reuse = summarise(root)
    noreuse = summarise(root, "noreuse_")
    prop = reuse.get("proposal", {})
    out = {
        "source": "tools/gpu_pmc2.sh: rocprofv3 --pmc, one counter group per run, tools/mc_loop.py 2 "
                  "(N2, 4096 walkers, fp32, 10 sweeps per iteration); per-launch means over the run's dispatches",
        "correction": "gfx950: FETCH_SIZE x2 (wide coalesced reads counted at half), WRITE_SIZE as counted",
        "proposal_hbm_bytes_per_launch": prop.get("hbm_bytes_per_launch"),
        "proposal_valu_insts_per_wave": prop.get("valu_insts_per_wave"),
        "proposal_mfma_util": prop.get("mfma_util"),
        "reuse": reuse,
        "recompute": {k: v for k, v in noreuse.items() if k == "proposal"},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
