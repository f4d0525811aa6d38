#!/bin/bash
# GPU: A/B of the C2 ccECP quadrature (k_quad_value<float,8,2>) between the in-tree library and
# a variant (AIQMC_LIB_VARIANT=$1), then the -m gpu suite on the variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=${1:-q8}
mkdir -p gpurun_out
for rep in 1 2; do
  for tag in base $V; do
    if [ $tag = base ]; then unset AIQMC_LIB_VARIANT; else export AIQMC_LIB_VARIANT=$tag; fi
    echo "$tag rep$rep $(timeout -k 10 180 python tools/ecp_ab.py C2_ecp 4096)" || exit 1
  done
done
unset AIQMC_LIB_VARIANT
export AIQMC_LIB_VARIANT=$V
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python tools/ecp_ab.py C2_ecp 4096 > gpurun_out/prof_$V.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_$V.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_$V.log
exit $rc
