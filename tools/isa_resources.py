"""Per-kernel resources from the gfx950 code objects of a built library: the AMDGPU metadata notes
(.vgpr_count, .agpr_count, .sgpr_count, .private_segment_fixed_size, .group_segment_fixed_size,
.vgpr_spill_count), keyed by the demangled kernel name as rocprofv3 prints it.  On gfx950 the
register file is unified: .vgpr_count is the whole allocation (arch + acc VGPRs), which is what
bounds occupancy (512 per lane per SIMD).

rocprofv3's kernel-trace VGPR_Count is the dispatch's granule-encoded arch-VGPR field decoded with
the wrong granule on gfx950 (k_walker_rev's proposal instantiation shows 48, the ISA says 86-96),
and its LDS_Block_Size is the static group segment only (0 for the kernels that size their LDS
at launch); profiles/summarize.py uses this table instead, plus the library's own dynamic-LDS
figures (aiqmc_debug_launch_lds).

usage: python tools/isa_resources.py [lib.so] > resources.json   (library default: the in-tree one)
"""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd",
                           "aiqmc", "libaiqmc_hip.so")


def bundles(data):
    """The offload bundles a .hip_fatbin section concatenates (one per TU): plain
    (__CLANG_OFFLOAD_BUNDLE__) or zstd-compressed (--offload-compress: "CCOB" + version, method,
    total size, ...; each cut to its total size -- the section pads between them)."""
    import struct
    plain = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = sorted([m.start() for m in re.finditer(re.escape(plain), data)] +
                    [m.start() for m in re.finditer(b"CCOB", data)])
    out = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        if data[s:s + 4] == b"CCOB":
            ver = struct.unpack_from("<H", data, s + 4)[0]
            tot = struct.unpack_from("<I", data, s + 8)[0] if ver == 2 else struct.unpack_from("<Q", data, s + 8)[0]
            if not 0 < tot <= e - s:
                continue   # "CCOB" bytes inside another bundle's payload
            e = s + tot
        out.append(data[s:e])
    return out


def code_objects(lib):
    """The gfx950 code objects bundled in lib's .hip_fatbin section (one per translation unit)."""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        out = []
        for i, piece in enumerate(bundles(data)):
            bpath = os.path.join(d, f"b{i}")
            open(bpath, "wb").write(piece)
            lst = subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={bpath}"],
                                 capture_output=True, text=True)
            tgts = [t for t in lst.stdout.split() if "gfx950" in t]
            if not tgts:
                continue
            co = os.path.join(d, f"co{i}")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={bpath}",
                                f"--targets={tgts[0]}", f"--output={co}", "--unbundle"], capture_output=True)
            if r.returncode == 0 and os.path.getsize(co):
                out.append(open(co, "rb").read())
        return out


def kernel_notes(co_bytes):
    import yaml
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co_bytes)
        f.flush()
        txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
    doc = txt[txt.index("---"):]
    doc = doc[:doc.index("\n...")] if "\n..." in doc else doc
    meta = yaml.safe_load(doc)
    res = {}
    for k in meta.get("amdhsa.kernels", []):
        # .vgpr_count is the whole unified register allocation on gfx950 (arch + acc VGPRs)
        res[k[".name"]] = {"vgpr": int(k[".vgpr_count"]), "agpr": int(k.get(".agpr_count", 0)),
                           "sgpr": int(k[".sgpr_count"]),
                           "scratch_bytes_per_lane": int(k[".private_segment_fixed_size"]),
                           "lds_static_bytes": int(k[".group_segment_fixed_size"]),
                           "vgpr_spill": int(k.get(".vgpr_spill_count", 0)),
                           "sgpr_spill": int(k.get(".sgpr_spill_count", 0))}
    return res


def demangle(names):
    tool = f"{LLVM}/llvm-cxxfilt" if os.path.exists(f"{LLVM}/llvm-cxxfilt") else "c++filt"
    out = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True).stdout
    return out.split("\n")[:len(names)]


def resources(lib=DEFAULT_LIB):
    table = {}
    for co in code_objects(lib):
        table.update(kernel_notes(co))
    names = sorted(table)
    return {d: dict(table[m], symbol=m) for m, d in zip(names, demangle(names))}


if __name__ == "__main__":
    print(json.dumps(resources(sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB), indent=1))
