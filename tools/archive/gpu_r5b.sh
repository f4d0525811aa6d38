# round 5: range-safe pivots -- the new tests on the shipped library, the old library (HEAD~ headers,
# N2-only variant "base") failing them, then interleaved N2 loop A/B base vs new (dev variants)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32_pivot_range.py tests/test_gpu_fp32_statistics.py tests/test_gpu_fullsize.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "pivot or far_electron" > gpurun_out/r5b_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r5b_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AIQMC_LIB_VARIANT=base timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32_pivot_range.py -m gpu -q -rf --timeout 120 --timeout-method thread -k N2 > gpurun_out/r5b_tests_oldlib.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5b_tests_oldlib.log | tail -3; grep FAILED gpurun_out/r5b_tests_oldlib.log | head -20; echo "oldlib rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
out=gpurun_out/ab_r5b.txt
: > $out
for B in 4096 512; do
  for rep in 1 2 3; do
    for v in base new; do
      r=$(AIQMC_LIB_VARIANT=$v AIQMC_NOPROF=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "$v rep$rep $r" | tee -a $out
    done
  done
  for v in base new; do
    r=$(AIQMC_LIB_VARIANT=$v timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "$v events $r" | tee -a $out
  done
done
