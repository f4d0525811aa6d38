# round 5: walker launch with the previous sweep's acceptance fused in (mc_step of 10 sweeps: 9 of
# 10 launches carry it) vs without (mc_step of 1 sweep: none does; k_accept applies it)
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for W in 4096 512; do for ns in 10 1; do
  r=$(AIQMC_NSTEPS=$ns timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo FAIL; exit 1; }
  echo "nsteps=$ns W=$W rep$rep $r"
done; done; done
