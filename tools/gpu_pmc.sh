# PMC passes (one counter group per rocprofv3 run) + phase/fallback diagnostics.
set -o pipefail
cd $GRAFT_REPO_ROOT
AIQMC_LIB_VARIANT=phaseprof timeout -k 10 200 python -u profiles/phase_prof.py > gpurun_out/phase.json 2> gpurun_out/phase.err || { echo PHASE_FAIL; tail gpurun_out/phase.err; exit 1; }
bash profiles/pmc_passes.sh gpurun_out/pmc sq1=SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY fetch=FETCH_SIZE write=WRITE_SIZE || exit 1
python3 profiles/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt && echo PMC_OK
