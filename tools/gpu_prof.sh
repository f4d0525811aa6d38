# GPU: parity tests, bench, rocprofv3 kernel-trace stats (CSV) of a bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/prof > gpurun_out/prof_summary.json && echo PROF_OK
