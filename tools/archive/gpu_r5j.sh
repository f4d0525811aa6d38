# round 5: every (N, A) shape with 2 <= N <= 16, A <= 2 against the fp64 oracle, plus the golden parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_shapes.py tests/test_gpu_parity.py > gpurun_out/r5j_tests.txt 2>&1 \
  || { tail -60 gpurun_out/r5j_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/r5j_tests.txt | tail -3
