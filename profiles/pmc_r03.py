"""Per-launch PMC figures of the N2 VMC kernels from the rocprofv3 --pmc passes of
tools/gpu_pmc3.sh (one counter group per run over tools/mc_loop.py), as the JSON bench.py reads
(profiles/pmc_r03.json).  Stamped with the SHA-256 (16 hex) of the library the passes ran on:
bench.py reports the counters only when it loads the same library.
HBM bytes per MI355X_MICROARCH.md: FETCH_SIZE (KB) counts half of the bytes of wide coalesced
reads on gfx950 -> x2; WRITE_SIZE (KB) as counted.
Non-FP VALU = SQ_INSTS_VALU - (FMA_F32 + MUL_F32 + ADD_F32 + TRANS_F32): integer, move, select,
compare, conversion and lane-permute instructions.
usage: python profiles/pmc_r03.py <gpurun_out/pmc> <lib_sha16> <walkers>"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {
    "proposal": "k_walker_rev<float, 14, 2, false, true",   # (a trailing PW7 template flag since round 4)
    "walker": "k_walker_rev<float, 14, 2, false, false",
    "prep": "k_walker_rev<float, 14, 2, true, false",
    "lap": "k_walker_lap<float, 14, 2",
    "moved_electron": "k_moved_electron<float, 14, 2>",
}
PASSES = ("mix", "stall", "misc", "mem", "fetch", "write")


def per_pass(root, name):
    """{kernel key: {counter: mean per dispatch}} for one pass directory."""
    out = {}
    for f in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            key = next((k for k, pat in KERNELS.items() if pat in r["Kernel_Name"]), None)
            if key is not None:
                acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[key].add(r["Dispatch_Id"])
        for key, d in acc.items():
            n = max(len(disp[key]), 1)
            out[key] = {c: v / n for c, v in d.items()}
    return out


def summarise(root):
    p = {n: per_pass(root, n) for n in PASSES}
    res = {}
    for key in KERNELS:
        get = lambda n, c: p.get(n, {}).get(key, {}).get(c)
        waves = get("mix", "SQ_WAVES") or get("fetch", "SQ_WAVES")
        d = {"waves": waves}
        if get("mix", "SQ_INSTS_VALU") is not None and waves:
            d["valu_insts_per_wave"] = get("mix", "SQ_INSTS_VALU") / waves
            fp = 0.0
            for c in ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32",
                      "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_CVT"):
                v = get("mix", c)
                if v is not None:
                    d[c.lower() + "_per_wave"] = v / waves
                    if c in ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32",
                             "SQ_INSTS_VALU_TRANS_F32"):
                        fp += v / waves
            d["fp_valu_insts_per_wave"] = fp
            d["nonfp_valu_insts_per_wave"] = d["valu_insts_per_wave"] - fp
        if get("stall", "SQ_WAVE_CYCLES") is not None and waves:
            for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if get("stall", c) is not None:
                    d[c.lower() + "_per_wave"] = get("stall", c) / waves
        if get("misc", "SQ_INSTS_MFMA") is not None:
            d["mfma_insts_per_launch"] = get("misc", "SQ_INSTS_MFMA")
            d["mfma_busy_cycles_per_launch"] = get("misc", "SQ_VALU_MFMA_BUSY_CYCLES")
            if waves:
                d["lds_bank_conflict_cycles_per_wave"] = (get("misc", "SQ_LDS_BANK_CONFLICT") or 0) / waves
                d["lds_insts_per_wave"] = (get("misc", "SQ_INSTS_LDS") or 0) / waves
                d["salu_insts_per_wave"] = (get("misc", "SQ_INSTS_SALU") or 0) / waves
                d["smem_insts_per_wave"] = (get("misc", "SQ_INSTS_SMEM") or 0) / waves
            gui = get("fetch", "GRBM_GUI_ACTIVE")
            busy = get("misc", "SQ_VALU_MFMA_BUSY_CYCLES")
            # MFMA busy cycles are summed over the 1024 SIMDs; utilisation against the launch's
            # GPU-active cycles (GRBM_GUI_ACTIVE) x SIMDs
            d["mfma_util"] = (busy / (gui * 1024) if (busy and gui) else 0.0)
            d["gui_active_per_launch"] = gui
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
    root, lib_sha, walkers = sys.argv[1], sys.argv[2], int(sys.argv[3])
    k = summarise(root)
    prop, prep, lap = k.get("proposal", {}), k.get("prep", {}), k.get("lap", {})
    el_bytes = None
    if prep.get("hbm_bytes_per_launch") is not None and lap.get("hbm_bytes_per_launch") is not None:
        el_bytes = prep["hbm_bytes_per_launch"] + lap["hbm_bytes_per_launch"]
    # the local-energy pair's MFMA utilisation: both launches' MFMA busy cycles over both launches'
    # active cycles (the adjoint pass forms Q_f on the matrix cores)
    el_mfma = None
    if prep.get("gui_active_per_launch") and lap.get("gui_active_per_launch"):
        el_mfma = ((prep.get("mfma_busy_cycles_per_launch") or 0) + (lap.get("mfma_busy_cycles_per_launch") or 0)) / (
            (prep["gui_active_per_launch"] + lap["gui_active_per_launch"]) * 1024)
    out = {
        "source": "tools/gpu_pmc3.sh: rocprofv3 --pmc, one counter group per run, tools/mc_loop.py "
                  f"(N2, {walkers} walkers, fp32, 10 sweeps + local energy per iteration); per-launch means",
        "correction": "gfx950: FETCH_SIZE x2 (wide coalesced reads counted at half), WRITE_SIZE as counted",
        "lib_sha16": lib_sha,
        "walkers": walkers,
        "proposal_hbm_bytes_per_launch": prop.get("hbm_bytes_per_launch"),
        "proposal_valu_insts_per_wave": prop.get("valu_insts_per_wave"),
        "proposal_nonfp_valu_insts_per_wave": prop.get("nonfp_valu_insts_per_wave"),
        "proposal_mfma_util": prop.get("mfma_util"),
        "local_energy_hbm_bytes_per_pair": el_bytes,
        "local_energy_mfma_util": el_mfma if el_mfma is not None else lap.get("mfma_util"),
        "kernels": k,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
