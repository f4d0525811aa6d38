#!/bin/bash
# Local energy with the pair tanh's from the adjoint pass (variant lpt) vs base: E_L / gradient
# agreement (fp32, fp64) and interleaved N2 loop timing.  Output under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/lap_pt_ab.txt
: > $out
for t in base lpt lpt2; do
  AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/el_dump.py gpurun_out/el_$t.npz >> $out 2>&1 || { echo "$t dump FAILED" >> $out; exit 1; }
done
for t in lpt lpt2; do python tools/el_dump.py --compare gpurun_out/el_base.npz gpurun_out/el_$t.npz | tee -a $out; done
for rep in 1 2 3; do
  for t in base lpt lpt2; do
    r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20) || { echo "$t FAILED" >> $out; exit 1; }
    echo "$t rep$rep $r" | tee -a $out
  done
done
