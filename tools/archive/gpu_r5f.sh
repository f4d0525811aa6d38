# round 5: fused limdrift accumulators in two banks (the last k_accept of an mc_step call zeroes
# the other bank: no memset launch per call) -- Metropolis parity tests, then the N2 loop at 4096
# and 512 walkers and a kernel trace at 512 (no fillBuffer per iteration expected)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mc_fp32.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_fp32_statistics.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5f_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
for B in 4096 512; do
  for rep in 1 2 3; do
    r=$(AIQMC_NOPROF=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "rep$rep $r" | tee -a gpurun_out/r5f_loop.txt
  done
done
rm -rf gpurun_out/prof512f
cd /tmp
AIQMC_NOPROF=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof512f -o run -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py 10 N2 512 > $GRAFT_REPO_ROOT/gpurun_out/r5f_loop512.txt 2>&1 || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT && head -12 gpurun_out/prof512f/run_kernel_stats.csv | cut -c1-150
