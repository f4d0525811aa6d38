#!/bin/bash
# kres.sh OBJ PATTERN -- register / LDS / scratch usage of the gfx950 kernels in a hipcc object
# whose symbol matches PATTERN (reads the code object's metadata notes).
B=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
$B/llvm-objcopy --dump-section .hip_fatbin=$tmp/fb "$1" /dev/null 2>/dev/null || { echo "no .hip_fatbin in $1"; exit 1; }
tgt=$($B/clang-offload-bundler --list --type=o --input=$tmp/fb | grep gfx950 | head -1)
$B/clang-offload-bundler --type=o --input=$tmp/fb --targets=$tgt --output=$tmp/co --unbundle
$B/llvm-readelf --notes $tmp/co | python3 -c "
import sys,re
txt=sys.stdin.read()
for blk in txt.split('.name:')[1:]:
    name=blk.split()[0]
    if re.search(sys.argv[1], name):
        g=lambda k: (re.search(r'\.'+k+r':\s+(\S+)',blk) or [None,None])[1]
        print(name, 'vgpr', g('vgpr_count'), 'agpr', g('agpr_count'), 'sgpr', g('sgpr_count'), 'scratch', g('private_segment_fixed_size'), 'lds', g('group_segment_fixed_size'), 'vspill', g('vgpr_spill_count'))
" "$2"
rm -rf $tmp
