#!/bin/bash
# round 3, third session: pp local-energy A/B (variant $1 vs in-tree), then the full measurement
# pass (tools/gpu_r3_full.sh: suite, fp32 tail, bench, rocprof, PMC stamped with the library).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=${1:-head}
mkdir -p gpurun_out
for sys in C2_ecp C_ecp; do
  for rep in 1 2; do
    for tag in $V main; do
      if [ $tag = main ]; then unset AIQMC_LIB_VARIANT; else export AIQMC_LIB_VARIANT=$tag; fi
      echo "$tag rep$rep $(timeout -k 10 180 python tools/ecp_ab.py $sys 4096)" || exit 1
    done
  done
done > gpurun_out/ab_ecp.txt
cat gpurun_out/ab_ecp.txt
unset AIQMC_LIB_VARIANT
bash tools/gpu_r3_full.sh
