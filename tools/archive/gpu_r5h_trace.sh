# round 5: kernel traces of the C-atom ccECP Adam side measurement, parameters round-tripped
# through the host (AIQMC_HOST_PARAMS=1) vs kept on the device
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for hp in 1 0; do
  rm -rf gpurun_out/tr_hp$hp
  cd /tmp
  if [ $hp = 1 ]; then export AIQMC_HOST_PARAMS=1; else unset AIQMC_HOST_PARAMS; fi
  AIQMC_PP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_hp$hp -o run -- python3 $GRAFT_REPO_ROOT/tools/adam_only.py > $GRAFT_REPO_ROOT/gpurun_out/tr_hp$hp.txt 2>&1 || { echo FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/tr_hp$hp.txt; exit 1; }
  cd $GRAFT_REPO_ROOT
  echo "== host_params=$hp"; tail -1 gpurun_out/tr_hp$hp.txt | cut -c1-200
  head -25 gpurun_out/tr_hp$hp/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
done
