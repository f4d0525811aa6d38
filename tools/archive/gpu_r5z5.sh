# round 5: counters of the packed ccECP kernels on the shipped library (after the F2 change):
# C atom (k_quad_value<float,4,1>) and C2 (k_quad_value<float,8,2>)
set -o pipefail
cd $GRAFT_REPO_ROOT
unset AIQMC_LIB_VARIANT
PMC_TAG=_c ECP_SYSTEM=C_ecp bash tools/gpu_r5r.sh > gpurun_out/pmc_ecp_c.txt 2>&1 || { tail -5 gpurun_out/pmc_ecp_c.txt; exit 1; }
PMC_TAG=_c2 ECP_SYSTEM=C2_ecp bash tools/gpu_r5r.sh > gpurun_out/pmc_ecp_c2.txt 2>&1 || { tail -5 gpurun_out/pmc_ecp_c2.txt; exit 1; }
cat gpurun_out/pmc_ecp_c.txt gpurun_out/pmc_ecp_c2.txt
