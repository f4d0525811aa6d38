# round 5: 3-5 atom shapes (development library with A >= 3 instantiations) against the fp64 oracle
set -o pipefail
cd $GRAFT_REPO_ROOT
export AIQMC_LIB_VARIANT=atest
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_shapes.py > gpurun_out/r5k_tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r5k_tests.txt | grep -v SKIP | tail -40
exit $rc
