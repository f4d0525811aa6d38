set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_ecp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --kernel-include-regex "k_walker_rev" -d $R/gpurun_out/pmc_ecp/sq -o sq -f csv -- python3 $R/tools/ecp_only.py > $R/gpurun_out/pmc_ecp/sq.log 2>&1 || { echo PMC_FAIL; tail -5 $R/gpurun_out/pmc_ecp/sq.log; exit 1; }
cd $R && python3 profiles/pmc_summary.py gpurun_out/pmc_ecp > gpurun_out/pmc_ecp_summary.txt && cat gpurun_out/pmc_ecp_summary.txt
