set -o pipefail
cd $GRAFT_REPO_ROOT
for hp in 1 0; do
  if [ $hp = 1 ]; then export AIQMC_HOST_PARAMS=1; else unset AIQMC_HOST_PARAMS; fi
  AIQMC_PP=1 timeout -k 10 200 python -m cProfile -s tottime tools/adam_only.py > gpurun_out/cprof_pp_hp$hp.txt 2>&1 || exit 1
  echo "== host_params=$hp"; grep -A25 "Ordered by" gpurun_out/cprof_pp_hp$hp.txt | head -28
done
