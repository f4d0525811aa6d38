# round 5: walker launch without its pair stream F2 (timing probe only; the sweep's values are wrong)
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for W in 4096 512; do for t in base wnof2; do
  r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo FAIL; exit 1; }
  echo "$t W=$W rep$rep $r"
done; done; done
