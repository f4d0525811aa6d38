#!/bin/bash
# Interleaved A/B of two dev libraries (N2 and Be shapes): bytewise positions after N2 sweeps
# (tools/pos_dump.py), E_L agreement, N2 loops at 4096 and 512 walkers, Be loops at 4096.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_yt.txt
: > $out
A=$1; B=$2
for t in $A $B; do
  AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/el_dump.py gpurun_out/el_$t.npz >> $out 2>&1 || { echo "$t dump FAILED" >> $out; exit 1; }
done
python tools/el_dump.py --compare gpurun_out/el_$A.npz gpurun_out/el_$B.npz | tee -a $out
for t in $A $B; do AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/pos_dump.py gpurun_out/pos_$t.npy N2 4096 > /dev/null 2>&1 || { echo "$t pos FAILED" >> $out; exit 1; }; done
python -c "import numpy as np, sys; a=np.load('gpurun_out/pos_$A.npy'); b=np.load('gpurun_out/pos_$B.npy'); print('positions bitwise equal', a.tobytes()==b.tobytes(), 'max diff', float(abs(a-b).max()))" | tee -a $out
for rep in 1 2 3; do
  for t in $A $B; do
    for cfg in "N2 4096" "N2 512" "Be 4096"; do
      r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 $cfg 2>&1 | grep -v amdgpu.ids) || { echo "$t FAILED" >> $out; exit 1; }
      echo "$t rep$rep $r" | tee -a $out
    done
  done
done
