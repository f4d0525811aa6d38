# round 5: rocprofv3 kernel stats of the default bench on the shipped library (4fbb6bf3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
unset AIQMC_LIB_VARIANT
mkdir -p gpurun_out
rm -rf gpurun_out/prof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo PROF_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/prof > gpurun_out/prof_summary.json && echo PROF_OK
