"""Static per-phase VALU opcode histogram of one kernel in a gfx950 assembly file compiled with
-DAQ_PHASE_MARK (walker_rev.h AQ_PH markers become ';AQMARK k' comments).

usage: python tools/isa_phases.py <file.s> <kernel-symbol-regex> [--ops]
Classes follow the SQ_INSTS_VALU_* counters: fma/mul/add/trans fp32 (v_pk_* counted as one
instruction each, listed separately), int32, and 'other' (moves incl. DPP, selects, compares,
lane ops, conversions).  Static counts: loops are reported (backward branches), not unrolled."""
import collections
import re
import sys

# AQ_PH(k) marks the END of a phase: code after marker k belongs to the next phase
PHASE_NAMES = {None: "F0 positions", "0": "F1 stage/cache", "1": "F2 pair patch", "2": "F4 h layers",
               "3": "F5 Phi+GJ", "4": "B1 H/Yt adj", "5": "B2 layers back", "6": "B3 pair adj (+B4 loads)",
               "7": "B4 gradient", "8": "outputs", "9": "epilogue",
               "10": "F5 fallback (pivoted GJ, rare)", "11": "F5 after fallback"}


def classify(op):
    if op.startswith("v_pk_"):
        if "fma" in op: return "pk_fma"
        if "mul" in op: return "pk_mul"
        if "add" in op: return "pk_add"
        return "pk_other"
    if re.match(r"v_(fma|fmac|fmaak|fmamk|mad|mac)_f32", op) or op.startswith("v_fma_mix") or op.startswith("v_dot"):
        return "fma"
    if re.match(r"v_mul_f32|v_mul_legacy_f32", op): return "mul"
    if re.match(r"v_(add|sub|subrev)_f32", op): return "add"
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", op): return "trans"
    if re.match(r"v_(max|min|med3)_f32|v_ldexp_f32|v_frexp|v_div_|v_fract_f32|v_floor_f32|v_trunc_f32|v_rndne_f32|v_ceil_f32", op):
        return "fp_misc"
    if re.match(r"v_cmp|v_cmpx", op): return "cmp"
    if re.match(r"v_cndmask", op): return "cndmask"
    if re.match(r"v_mov_b32|v_mov_b64", op): return "mov"
    if re.match(r"v_readlane|v_readfirstlane|v_writelane|v_permlane|v_swap", op): return "lane"
    if re.match(r"v_cvt", op): return "cvt"
    if re.match(r"v_(add|sub|subrev|mul_lo|mul_hi|mad_u|mad_i|mad_u32|lshl|lshr|ashr|and|or|xor|not|bfe|bfi|alignbit|lshl_add|add3|lshl_or|and_or|or3|xad|mbcnt|bcnt|ffbh|ffbl|max_i|max_u|min_i|min_u|cndmask_b16)", op):
        return "int"
    if op.startswith("v_accvgpr"): return "acc"
    if op.startswith("v_mfma"): return "mfma"
    if op.startswith("v_"): return "v_other:" + op
    if op.startswith("ds_"): return "LDS"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_") or op.startswith("scratch_"):
        return "VMEM"
    if op.startswith("s_load") or op.startswith("s_buffer_load"): return "SMEM"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"): return "wait/nop"
    if op.startswith("s_"): return "SALU"
    return "other:" + op


def main():
    path, pat = sys.argv[1], sys.argv[2]
    show_ops = "--ops" in sys.argv
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"^([A-Za-z0-9_.$]+):\s*(;.*)?$", l)
        if m and re.search(pat, m.group(1)) and not m.group(1).startswith("."):
            start = i
            name = m.group(1)
            break
    if start is None:
        sys.exit("kernel not found")
    phase = None
    hist = collections.OrderedDict()
    ops = collections.defaultdict(collections.Counter)
    labels = {}
    loops = collections.Counter()
    order = [None]
    for l in lines[start + 1:]:
        if re.match(r"^\.Lfunc_end", l):
            break
        m = re.search(r";AQMARK (\d+)", l)
        if m:
            phase = m.group(1)
            if phase not in order:
                order.append(phase)
            continue
        lm = re.match(r"^(\.LBB[0-9_]+):", l)
        if lm:
            labels[lm.group(1)] = phase
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        c = classify(op)
        hist.setdefault(phase, collections.Counter())[c] += 1
        ops[phase][op] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in labels:
                loops[phase] += 1
    fp = ("fma", "mul", "add", "trans", "pk_fma", "pk_mul", "pk_add")
    nonfp = ("int", "cmp", "cndmask", "mov", "lane", "cvt", "fp_misc", "pk_other")
    print(f"kernel {name}")
    hdr = ["phase", "VALU", "fp", "non-fp", "int", "cmp", "cndmask", "mov", "lane", "fp_misc", "pk*", "LDS", "VMEM", "SMEM", "SALU", "loops"]
    print(" | ".join(hdr))
    tot = collections.Counter()
    for ph in order:
        h = hist.get(ph, collections.Counter())
        valu = sum(v for k, v in h.items() if k in fp + nonfp or k.startswith("v_other") or k in ("acc", "mfma"))
        f = sum(h[k] for k in fp)
        nf = valu - f
        pk = h["pk_fma"] + h["pk_mul"] + h["pk_add"]
        row = [PHASE_NAMES.get(ph, ph), valu, f, nf, h["int"], h["cmp"], h["cndmask"], h["mov"], h["lane"], h["fp_misc"], pk,
               h["LDS"], h["VMEM"], h["SMEM"], h["SALU"], loops[ph]]
        for k, v in zip(hdr[1:], row[1:]):
            tot[k] += v
        print(" | ".join(str(x) for x in row))
    print(" | ".join(["total"] + [str(tot[k]) for k in hdr[1:]]))
    if show_ops:
        for ph in order:
            print(f"--- {PHASE_NAMES.get(ph, ph)}")
            print(", ".join(f"{o}:{n}" for o, n in ops[ph].most_common() if o.startswith("v_")))


if __name__ == "__main__":
    main()
