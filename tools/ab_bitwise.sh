#!/bin/bash
# Interleaved A/B timing of dev variants (tools/ab_variants.sh) + bitwise comparison of their
# walker positions / local energies after three N2 steps against the first variant.
# usage: tools/ab_bitwise.sh tag1 tag2 ...
set -o pipefail
mkdir -p gpurun_out/ab
for t in "$@"; do
  AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/pos_dump.py gpurun_out/ab/pos_$t.npy > /dev/null 2>&1 || { echo "$t pos_dump FAILED"; exit 1; }
done
python3 - "$@" <<'PY'
import sys, numpy as np
ref = np.load(f"gpurun_out/ab/pos_{sys.argv[1]}.npy")
for t in sys.argv[2:]:
    x = np.load(f"gpurun_out/ab/pos_{t}.npy")
    print(f"{t} vs {sys.argv[1]}: bitwise equal {np.array_equal(x, ref)}, max |diff| {np.max(np.abs(x - ref)):.3e}")
PY
bash tools/ab_variants.sh "$@"
