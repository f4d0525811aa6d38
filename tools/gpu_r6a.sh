# round 6, first pass: VALU issue rates, the new RCCL / fused-loss / shape tests, the full -m gpu suite, the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o /tmp/valu_rate && timeout -k 10 60 /tmp/valu_rate > gpurun_out/valu_rate.txt 2>&1; cat gpurun_out/valu_rate.txt | head -40
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_shapes.py -k "rccl or adam or partial_last_wave or set_params_device" -x -v --timeout 240 --timeout-method thread > gpurun_out/r6a_new_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r6a_new_tests.log; [ $rc -eq 0 ] || exit $rc
SUITE_TIMEOUT=1500 bash tools/gpu_tests.sh > gpurun_out/r6a_suite_tail.txt 2>&1; rc=$?; tail -15 gpurun_out/r6a_suite_tail.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r6a_bench.err; exit 1; }
head -c 2500 gpurun_out/r6a_bench.json; echo
