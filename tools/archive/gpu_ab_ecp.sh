#!/bin/bash
# GPU: interleaved A/B of the pp local energy (tools/ecp_ab.py) between a variant library
# (AIQMC_LIB_VARIANT=$1) and the in-tree one, for C2_ecp and C_ecp; then the -m gpu suite and
# the default bench on the in-tree library.
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
done
unset AIQMC_LIB_VARIANT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/b_main.json 2> gpurun_out/b_main.err || { tail -20 gpurun_out/b_main.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_main.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_local_energy']['avg_launch_ms'], d['ecp_c2']['ms_per_eval_batch'], d['ecp_c_atom']['ms_per_eval_batch'])"
