set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ecp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ecp.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_ecp.log; exit 1; }
tail -8 gpurun_out/pytest_ecp.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
