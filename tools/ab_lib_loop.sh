#!/bin/bash
# Interleaved A/B of dev library variants on the N2 VMC loop: AB_VARIANTS="a b" AB_WALKERS="4096" [AB_REPS=3]
# positions after three mc_step calls compared bytewise against the first variant, then
# tools/mc_loop.py (20 iterations) per variant, batch size and rep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
set -- $AB_VARIANTS
base=$1
for v in $AB_VARIANTS; do
  AIQMC_LIB_VARIANT=$v timeout -k 10 120 python tools/pos_dump.py gpurun_out/ab/pos_$v.npy N2 ${AB_POS_WALKERS:-4096} > /dev/null 2>&1 || { echo "pos_dump $v FAILED"; exit 1; }
  python3 -c "
import numpy as np
a, b = np.load('gpurun_out/ab/pos_$base.npy'), np.load('gpurun_out/ab/pos_$v.npy')
print('$v vs $base: bitwise equal', np.array_equal(a, b), 'max |diff|', float(np.max(np.abs(a - b))))"
done
for rep in $(seq 1 ${AB_REPS:-3}); do
  for B in $AB_WALKERS; do
    for v in $AB_VARIANTS; do
      r=$(AIQMC_LIB_VARIANT=$v timeout -k 10 120 python tools/mc_loop.py 20 N2 $B 2>&1 | grep -v amdgpu.ids) || { echo "loop $v $B FAILED"; exit 1; }
      echo "$v rep$rep $r"
    done
  done
done
