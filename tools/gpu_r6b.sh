# round 6: the new RCCL / fused-loss / shape tests, the full -m gpu suite, smoke, the bench and its rocprofv3 kernel summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_shapes.py -k "rccl or adam or partial_last_wave or set_params_device" -x -v --timeout 240 --timeout-method thread > gpurun_out/r6b_new_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r6b_new_tests.log; [ $rc -eq 0 ] || exit $rc
SUITE_TIMEOUT=1500 bash tools/gpu_tests.sh > gpurun_out/r6b_suite_tail.txt 2>&1; rc=$?; tail -15 gpurun_out/r6b_suite_tail.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6b_smoke.txt 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/r6b_smoke.txt; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r6b_bench.err; exit 1; }
head -c 1500 gpurun_out/r6b_bench.json; echo
rm -rf gpurun_out/r6b_prof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6b_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r6b_bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r6b_prof.err || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/r6b_prof > gpurun_out/r6b_prof_summary.json && echo PROF_OK
