# round 5: walker launch at 4096 / 512 walkers with the sweep's Philox draws generated inside it
# (default) vs device-resident draws passed in (AIQMC_HOST_DRAWS): is the draw generation on the
# walker launch's path?
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for W in 4096 512; do for hd in 0 1; do
  if [ $hd = 1 ]; then export AIQMC_HOST_DRAWS=1; else unset AIQMC_HOST_DRAWS; fi
  r=$(timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo FAIL; exit 1; }
  echo "host_draws=$hd W=$W rep$rep $r"
done; done; done
