# round 6 measurement pass, part B: the default bench (reads the stamped PMC files under profiles/) and the
# rocprofv3 kernel-trace summary of the same command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r6g_bench.json 2> gpurun_out/r6g_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r6g_bench.err; exit 1; }
head -c 1200 gpurun_out/r6g_bench.json; echo
rm -rf gpurun_out/r6g_prof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6g_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r6g_bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r6g_prof.err || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/r6g_prof > gpurun_out/r6g_prof_summary.json && cp gpurun_out/r6g_prof/run_kernel_stats.csv gpurun_out/r6g_kernel_stats.csv && echo PROF_OK
