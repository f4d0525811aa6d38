# round 5: walker launch at 4096 / 512 walkers without its walker-cache stores (timing probe only:
# proposals then read a stale cache) -- is the launch's F1/F2 time the cache writes?
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for W in 4096 512; do for t in base nolocst noptst nost; do
  r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t FAILED"; exit 1; }
  echo "$t W=$W rep$rep $r"
done; done; done
