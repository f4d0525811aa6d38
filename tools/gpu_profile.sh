# rocprofv3 kernel-trace summary of the default bench + PMC passes (one counter group per run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-ecp --no-adam --no-dmc > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof.err; exit 1; }
echo PROF_OK
python3 $R/profiles/summarize.py $R/gpurun_out/prof > $R/gpurun_out/prof_summary.json || true
bash $R/profiles/pmc_passes.sh gpurun_out/pmc fetch=FETCH_SIZE && bash $R/profiles/pmc_passes.sh gpurun_out/pmc write=WRITE_SIZE && bash $R/profiles/pmc_passes.sh gpurun_out/pmc sq=SQ_WAVES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAIT_INST_ANY || { echo PMC_FAIL; exit 1; }
python3 $R/profiles/pmc_summary.py $R/gpurun_out/pmc > $R/gpurun_out/pmc_summary.txt
echo PMC_OK
