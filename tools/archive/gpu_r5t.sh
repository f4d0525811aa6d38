# round 5: kernel trace of the DMC side measurements (C ccECP and Ne all-electron DMC steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/prof_dmc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-ecp --no-adam --no-cpu-baseline --no-per-rank > $GRAFT_REPO_ROOT/gpurun_out/prof_dmc.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_dmc.err || { echo PROF_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_dmc.err; exit 1; }
cd $GRAFT_REPO_ROOT
head -30 gpurun_out/prof_dmc/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
