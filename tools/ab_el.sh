#!/bin/bash
# Interleaved A/B of N2 dev library variants (usage: tools/ab_el.sh REF V1 V2 ...): E_L / gradient agreement
# of each variant with REF (fp32, fp64; tools/el_dump.py) and three interleaved N2 loop timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_el.txt
: > $out
for t in "$@"; do
  AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/el_dump.py gpurun_out/el_$t.npz >> $out 2>&1 || { echo "$t dump FAILED" >> $out; exit 1; }
done
ref=$1; shift
for t in "$@"; do echo "== $t vs $ref" | tee -a $out; python tools/el_dump.py --compare gpurun_out/el_$ref.npz gpurun_out/el_$t.npz | tee -a $out; done
for rep in 1 2 3; do
  for t in $ref "$@"; do
    r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20) || { echo "$t FAILED" >> $out; exit 1; }
    echo "$t rep$rep $r" | tee -a $out
  done
done
